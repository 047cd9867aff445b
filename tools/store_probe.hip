// Store-burst probe (diagnostic, not product): what limits a GEMM epilogue's store burst on gfx950?
// Each workgroup (512 threads = 8 waves, one per CU as in the 8-phase GEMM) writes TILE bytes
// (192 KB: an FF1 tile's h + g) from registers with 16-B stores in one of four address patterns:
//   0: 16 rows x 64 B per wave instruction (the transposed-accumulator epilogue_t layout)
//   1: 8 rows x 128 B (full cache lines per row)
//   2: 4 rows x 256 B
//   3: 1 KB contiguous
//   4: 8 rows x 128 B, consecutive lanes on consecutive 16 B of a row (row = lane / 8)
//   5: 16 rows x 64 B, lane-contiguous (row = lane / 4)
//   6: 4 rows x 256 B, lane-contiguous (row = lane / 16)
// Grid: `active` workgroups store, one per CU (256 = every CU at once; fewer = a partial burst),
// each `reps` tiles back to back into disjoint memory.  Reports device time, GB/s and the per-CU
// bytes per cycle (s_memtime, median over workgroups).
// build: hipcc --offload-arch=gfx950 -O3 -o /tmp/store_probe tools/store_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>

constexpr int TILE = 192 * 1024;           // bytes per workgroup tile
constexpr int NTH = 512;
constexpr int PER_THREAD = TILE / NTH / 16;  // 16-B stores per thread per tile = 24

__global__ __launch_bounds__(NTH, 1) void probe(uint4* out, int pattern, int reps, unsigned long long* cyc) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint4 v = make_uint4(lane, w, blockIdx.x, 7);
  char* base = (char*)out + (size_t)blockIdx.x * reps * TILE;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < reps; ++r) {
    char* tb = base + (size_t)r * TILE;
#pragma unroll
    for (int i = 0; i < PER_THREAD; ++i) {
      const int inst = w * PER_THREAD + i;          // wave instruction index: 1 KB each
      size_t off;
      if (pattern == 0) {        // 16 rows x 64 B, row pitch 512 B (a 256-column bf16 tile row)
        const int row = (inst / 8) * 16 + (lane & 15), cb = (inst % 8) * 64 + (lane >> 4) * 16;
        off = (size_t)row * 512 + cb;
      } else if (pattern == 1) { // 8 rows x 128 B
        const int row = (inst / 4) * 8 + (lane & 7), cb = (inst % 4) * 128 + (lane >> 3) * 16;
        off = (size_t)row * 512 + cb;
      } else if (pattern == 2) { // 4 rows x 256 B
        const int row = (inst / 2) * 4 + (lane & 3), cb = (inst % 2) * 256 + (lane >> 2) * 16;
        off = (size_t)row * 512 + cb;
      } else if (pattern == 3) { // 1 KB contiguous
        off = (size_t)inst * 1024 + lane * 16;
      } else if (pattern == 4) {
        const int row = (inst / 4) * 8 + (lane >> 3), cb = (inst % 4) * 128 + (lane & 7) * 16;
        off = (size_t)row * 512 + cb;
      } else if (pattern == 5) {
        const int row = (inst / 8) * 16 + (lane >> 2), cb = (inst % 8) * 64 + (lane & 3) * 16;
        off = (size_t)row * 512 + cb;
      } else {
        const int row = (inst / 2) * 4 + (lane >> 4), cb = (inst % 2) * 256 + (lane & 15) * 16;
        off = (size_t)row * 512 + cb;
      }
      *(uint4*)(tb + off) = v;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) cyc[blockIdx.x] = __builtin_amdgcn_s_memtime() - t0;
}

int main() {
  const int reps = 8;
  uint4* out;
  unsigned long long* cyc;
  hipMalloc(&out, (size_t)256 * reps * TILE);
  hipMalloc(&cyc, 256 * sizeof(unsigned long long));
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  printf("pattern active  ms      GB/s   B/cyc/CU(median)\n");
  for (int active : {256, 128, 32}) {
    for (int pat = 0; pat < 7; ++pat) {
      for (int it = 0; it < 2; ++it) {
        hipEventRecord(a);
        hipLaunchKernelGGL(probe, dim3(active), dim3(NTH), 0, 0, out, pat, reps, cyc);
        hipEventRecord(b);
        hipEventSynchronize(b);
        if (it == 0) continue;
        float ms;
        hipEventElapsedTime(&ms, a, b);
        std::vector<unsigned long long> h(active);
        hipMemcpy(h.data(), cyc, active * sizeof(unsigned long long), hipMemcpyDeviceToHost);
        std::sort(h.begin(), h.end());
        const double bytes = (double)active * reps * TILE;
        printf("%7d %6d %7.3f %8.1f %8.2f\n", pat, active, ms, bytes / ms / 1e6,
               (double)reps * TILE / (double)h[active / 2]);
      }
    }
  }
  hipFree(out);
  hipFree(cyc);
  return 0;
}
