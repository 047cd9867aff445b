// Store-burst probe (diagnostic, not product): what limits a GEMM epilogue's store burst on gfx950?
// Each workgroup (512 threads = 8 waves, one per CU as in the 8-phase GEMM) writes TILE bytes
// (192 KB: an FF1 tile's h + g) from registers, in one of these per-wave-instruction address
// patterns (tile rows 512 B apart, a 256-column bf16 tile row):
//   0: 16 rows x 64 B, 16-B lanes, row = lane % 16 (the transposed-accumulator epilogue_t layout)
//   1: 8 rows x 128 B, 16-B lanes, row = lane % 8
//   2: 4 rows x 256 B, 16-B lanes, row = lane % 4
//   3: 1 KB contiguous, 16-B lanes
//   4: 8 rows x 128 B, 16-B lanes, lane-contiguous (row = lane / 8)
//   5: 16 rows x 64 B, 16-B lanes, lane-contiguous (row = lane / 4)
//   6: 4 rows x 256 B, 16-B lanes, lane-contiguous (row = lane / 16)
//   7: 4 rows x 128 B, 8-B lanes, lane-contiguous (row = lane / 16)
//   8: 16 rows x 32 B, 8-B lanes, row = lane % 16
//   9: 4 rows x 64 B, 4-B lanes, lane-contiguous (row = lane / 16)
// Grid: `active` workgroups store, one per CU (256 = every CU at once; fewer = a partial burst),
// each `reps` tiles back to back into disjoint memory.  Reports device time, GB/s and the per-CU
// bytes per cycle (s_memtime, median over workgroups).
// build: hipcc --offload-arch=gfx950 -O3 -Wno-unused-result -o tools/store_probe tools/store_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>

constexpr int TILE = 192 * 1024;           // bytes per workgroup tile
constexpr int NTH = 512;

template <int PAT>
__device__ __forceinline__ size_t offset_of(int inst, int lane) {
  if constexpr (PAT == 0) return (size_t)((inst / 8) * 16 + (lane & 15)) * 512 + (inst % 8) * 64 + (lane >> 4) * 16;
  if constexpr (PAT == 1) return (size_t)((inst / 4) * 8 + (lane & 7)) * 512 + (inst % 4) * 128 + (lane >> 3) * 16;
  if constexpr (PAT == 2) return (size_t)((inst / 2) * 4 + (lane & 3)) * 512 + (inst % 2) * 256 + (lane >> 2) * 16;
  if constexpr (PAT == 3) return (size_t)inst * 1024 + lane * 16;
  if constexpr (PAT == 4) return (size_t)((inst / 4) * 8 + (lane >> 3)) * 512 + (inst % 4) * 128 + (lane & 7) * 16;
  if constexpr (PAT == 5) return (size_t)((inst / 8) * 16 + (lane >> 2)) * 512 + (inst % 8) * 64 + (lane & 3) * 16;
  if constexpr (PAT == 6) return (size_t)((inst / 2) * 4 + (lane >> 4)) * 512 + (inst % 2) * 256 + (lane & 15) * 16;
  if constexpr (PAT == 7) return (size_t)((inst / 4) * 4 + (lane >> 4)) * 512 + (inst % 4) * 128 + (lane & 15) * 8;
  if constexpr (PAT == 8) return (size_t)((inst / 16) * 16 + (lane & 15)) * 512 + (inst % 16) * 32 + (lane >> 4) * 8;
  return (size_t)((inst / 8) * 4 + (lane >> 4)) * 512 + (inst % 8) * 64 + (lane & 15) * 4;
}
template <int PAT> constexpr int width() { return PAT <= 6 ? 16 : PAT <= 8 ? 8 : 4; }

template <int PAT>
__global__ __launch_bounds__(NTH, 1) void probe(char* out, int reps, unsigned long long* cyc) {
  constexpr int W = width<PAT>();
  constexpr int PER_THREAD = TILE / NTH / W;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  char* base = out + (size_t)blockIdx.x * reps * TILE;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < reps; ++r) {
    char* tb = base + (size_t)r * TILE;
#pragma unroll
    for (int i = 0; i < PER_THREAD; ++i) {
      const int inst = w * PER_THREAD + i;
      char* p = tb + offset_of<PAT>(inst, lane);
      if constexpr (W == 16) *(uint4*)p = make_uint4(lane, w, blockIdx.x, i);
      else if constexpr (W == 8) *(uint2*)p = make_uint2(lane, i);
      else *(unsigned*)p = lane + i;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) cyc[blockIdx.x] = __builtin_amdgcn_s_memtime() - t0;
}

typedef void (*KFn)(char*, int, unsigned long long*);

int main() {
  const int reps = 8;
  char* out;
  unsigned long long* cyc;
  hipMalloc(&out, (size_t)256 * reps * TILE);
  hipMalloc(&cyc, 256 * sizeof(unsigned long long));
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const KFn fns[10] = {probe<0>, probe<1>, probe<2>, probe<3>, probe<4>, probe<5>, probe<6>, probe<7>, probe<8>, probe<9>};
  printf("pattern active  ms      GB/s   B/cyc/CU(median)\n");
  for (int active : {256, 128, 32}) {
    for (int pat = 0; pat < 10; ++pat) {
      for (int it = 0; it < 2; ++it) {
        hipEventRecord(a);
        hipLaunchKernelGGL(fns[pat], dim3(active), dim3(NTH), 0, 0, out, reps, cyc);
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
