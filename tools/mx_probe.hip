// Operand-layout probe for v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3 x e4m3, e8m0 scales):
// random small-integer A (16x128), B (128x16) and per-(row|col, 32-k block) scales, packed into
// lane registers under each candidate k-map, checked against a host f64 matmul.
//   map 0: lane l, byte j -> k = 32*(l>>4) + j
//   map 1: lane l, byte j -> k = 16*(l>>4) + (j & 15) + 64*(j >> 4)
// Result on gfx950 (this probe, gpurun_out/mx_probe.log): map 1 - lane group g = l>>4 holds k
// 16g..16g+15 in bytes 0-15 and 64+16g.. in bytes 16-31, and supplies the e8m0 scale of
// (row|col l&15, k block g) (the 32-block is split across two lane groups' registers).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstdint>
#include <cstring>

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void probe(const uint8_t* A, const uint8_t* B, const uint8_t* sa, const uint8_t* sb, float* C, int map,
                      const uint8_t* lane_sa, const uint8_t* lane_sb) {
  const int l = threadIdx.x;
  uint8_t a[32], b[32];
  const int blk = l >> 4;   // lane group g supplies the scale of k block g (probe result)
  for (int j = 0; j < 32; ++j) {
    const int k = map == 0 ? 32 * (l >> 4) + j : 16 * (l >> 4) + (j & 15) + 64 * (j >> 4);
    a[j] = A[(l & 15) * 128 + k];       // A row-major [16][128]
    b[j] = B[(l & 15) * 128 + k];       // B stored [n][k]
  }
  i32x8 ra, rb;
  for (int r = 0; r < 8; ++r) {
    ra[r] = a[4 * r] | (a[4 * r + 1] << 8) | (a[4 * r + 2] << 16) | (a[4 * r + 3] << 24);
    rb[r] = b[4 * r] | (b[4 * r + 1] << 8) | (b[4 * r + 2] << 16) | (b[4 * r + 3] << 24);
  }
  const int sca = lane_sa ? lane_sa[l] : sa[(l & 15) * 4 + blk], scb = lane_sb ? lane_sb[l] : sb[(l & 15) * 4 + blk];
  f32x4 c = {0.f, 0.f, 0.f, 0.f};
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(ra, rb, c, 0, 0, 0, sca, 0, scb);
  for (int r = 0; r < 4; ++r) C[((l >> 4) * 4 + r) * 16 + (l & 15)] = c[r];
}

static uint8_t e4m3_of_int(int v) {  // exact for |v| <= 2
  if (v == 0) return 0;
  const uint8_t s = v < 0 ? 0x80 : 0;
  const int a = abs(v);
  return s | (a == 1 ? 0x38 : 0x40);  // 1.0 = exp 7 (bias 7) -> 0x38; 2.0 -> 0x40
}


static int Ai[16][128], Bi[16][128], Sa[16][4], Sb[16][4];
static double ref[16][16];
static uint8_t *dA, *dB, *dsa, *dsb, *dla, *dlb;
static float* dC;

static void host_ref() {
  for (int i = 0; i < 16; ++i)
    for (int n = 0; n < 16; ++n) {
      double s = 0;
      for (int k = 0; k < 128; ++k) s += ldexp((double)Ai[i][k] * Bi[n][k], Sa[i][k >> 5] + Sb[n][k >> 5]);
      ref[i][n] = s;
    }
}

static void upload() {
  uint8_t hA[2048], hB[2048], hsa[64], hsb[64];
  for (int i = 0; i < 16; ++i)
    for (int k = 0; k < 128; ++k) { hA[i * 128 + k] = e4m3_of_int(Ai[i][k]); hB[i * 128 + k] = e4m3_of_int(Bi[i][k]); }
  for (int i = 0; i < 64; ++i) { hsa[i] = 127 + Sa[i / 4][i % 4]; hsb[i] = 127 + Sb[i / 4][i % 4]; }
  hipMemcpy(dA, hA, 2048, hipMemcpyHostToDevice); hipMemcpy(dB, hB, 2048, hipMemcpyHostToDevice);
  hipMemcpy(dsa, hsa, 64, hipMemcpyHostToDevice); hipMemcpy(dsb, hsb, 64, hipMemcpyHostToDevice);
}

static void run(int map, float* hC, const uint8_t* lsa, const uint8_t* lsb) {
  if (lsa) hipMemcpy(dla, lsa, 64, hipMemcpyHostToDevice);
  if (lsb) hipMemcpy(dlb, lsb, 64, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dA, dB, dsa, dsb, dC, map, lsa ? dla : nullptr, lsb ? dlb : nullptr);
  hipMemcpy(hC, dC, 1024, hipMemcpyDeviceToHost);
}

static int mism(const float* hC) {
  int bad = 0;
  for (int i = 0; i < 16; ++i)
    for (int n = 0; n < 16; ++n) bad += fabs(hC[i * 16 + n] - ref[i][n]) > 1e-6 * (1 + fabs(ref[i][n]));
  return bad;
}

int main() {
  srand(7);
  hipMalloc(&dA, 2048); hipMalloc(&dB, 2048); hipMalloc(&dsa, 64); hipMalloc(&dsb, 64); hipMalloc(&dC, 1024);
  hipMalloc(&dla, 64); hipMalloc(&dlb, 64);
  for (int i = 0; i < 16; ++i)
    for (int k = 0; k < 128; ++k) { Ai[i][k] = rand() % 5 - 2; Bi[i][k] = rand() % 5 - 2; }
  float hC[256];
  int ok_any = 0;
  // 1) unity scales: element maps
  memset(Sa, 0, sizeof Sa); memset(Sb, 0, sizeof Sb);
  host_ref(); upload();
  for (int map = 0; map < 2; ++map) { run(map, hC, nullptr, nullptr); printf("unity scales, map %d: %d mismatches\n", map, mism(hC)); }
  // 2) per-lane scale perturbation (2x on one lane's scale): for every row (A side) / column
  // (B side) it changed, the subset of 16-k chunks whose partial sums explain the change
  float base[256];
  run(0, base, nullptr, nullptr);
  for (int side = 0; side < 2; ++side) {
    printf("%s scale perturbation (lane: {row/col: 16-k chunk mask}):\n", side ? "B" : "A");
    for (int L = 0; L < 64; ++L) {
      uint8_t ls[64];
      for (int i = 0; i < 64; ++i) ls[i] = 127;
      ls[L] = 128;
      run(0, hC, side ? nullptr : ls, side ? ls : nullptr);
      printf(" %2d:", L);
      for (int r = 0; r < 16; ++r) {
        bool changed = false;
        for (int o = 0; o < 16; ++o) {
          const int idx = side ? o * 16 + r : r * 16 + o;
          if (fabs(hC[idx] - base[idx]) > 1e-6) changed = true;
        }
        if (!changed) continue;
        int found = -1;
        for (int mask = 1; mask < 256 && found < 0; ++mask) {
          bool ok = true;
          for (int o = 0; o < 16 && ok; ++o) {
            const int i = side ? o : r, n = side ? r : o;
            double ps = 0;
            for (int k = 0; k < 128; ++k)
              if (mask >> (k >> 4) & 1) ps += (double)Ai[i][k] * Bi[n][k];
            if (fabs(hC[i * 16 + n] - base[i * 16 + n] - ps) > 1e-6) ok = false;
          }
          if (ok) found = mask;
        }
        printf(" {%d:%02x}", r, found);
      }
      printf("\n");
    }
  }
  // 3) random (row, block) scales under the lane = row + 16*block hypothesis
  for (int i = 0; i < 16; ++i)
    for (int q = 0; q < 4; ++q) { Sa[i][q] = rand() % 7 - 3; Sb[i][q] = rand() % 7 - 3; }
  host_ref(); upload();
  for (int map = 0; map < 2; ++map) {
    run(map, hC, nullptr, nullptr);
    const int bad = mism(hC);
    printf("random scales, map %d: %d mismatches\n", map, bad);
    ok_any |= bad == 0;
  }
  return ok_any ? 0 : 1;
}
