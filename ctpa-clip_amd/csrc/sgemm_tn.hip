// Exact-f32 "TN" GEMM of the f32 image tower (functional.set_vit_precision('f32')):
//   C[m, n] = epilogue(alpha * sum_k A[m, k] * B[n, k])      A [M][K], B [N][K] row-major f32
// i.e. every nn.Linear of the 3D-ViT forward (ct_clip/attention.py:44-52,119-125; the patch
// embedding's Linear, ct_clip/ctvit.py:172) with the f32 operands the reference's fp32 run uses.
// Each output is ONE f32 fma chain in ascending k (v_mfma_f32_16x16x4_f32 is exact f32,
// MI355X_MICROARCH.md § Matrix cores), bit-identical to ctclip_sgemm on the same operands.
//
// 128 x 128 x 16 block tile, 256 threads = 4 waves (2 x 2) of 64 x 64 = 4 x 4 MFMA blocks; the
// f32 matrix pipe (64 FLOP/clk/SIMD, 1/16 of bf16) is the bound, so the structure is the simple
// one: operands register-staged with 16-B loads (4 consecutive k of a row), double-buffered LDS
// images [128 rows][16 k] with a 20-float row stride (16-B aligned writes; the 64 lanes' 4-byte
// fragment reads hit 64 distinct banks), one barrier per 16-deep K step, the next step's global
// loads in flight under the current step's 64 MFMAs.  MFMA operands are swapped (B fragment
// first) so each lane ends with one row and 4 consecutive columns of every 16 x 16 block: f32x4
// / bf16x4 stores.  Epilogues: act 0 -- C (f32) = alpha acc (+ bias[n]) (+ R f32), optional bf16
// copy C2; act 2 -- GEGLU over the packed [32 x | 32 gate] column pairs of the FF1 weight
// (functional.ff1_rowmap): C2 = h (bf16, the backward's saved pre-activation), C = g (f32),
// C3 = g (bf16), g = gelu_erf(gate) * x with libm erff on the f32 values.
#include "common.h"
#include "../../include/ctclip_hip.h"

namespace {

constexpr int BM = 128, BN = 128, KT = 16, LDR = 20, NTH = 256;
constexpr int TILE_FLOATS = BM * LDR;   // one operand image

struct FP {
  int64_t M, N, K;
  const float* A; int64_t lda;
  const float* B; int64_t ldb;
  float* C; int64_t ldc;
  u16* C2; int64_t ldc2;
  u16* C3; int64_t ldc3;
  const float* bias;
  const float* R; int64_t ldr;
  float alpha;
  int act;
};

// this thread's two 16-B chunks of a 128-row x 16-k operand tile: rows t/4 and 64 + t/4, k quad t%4
__device__ __forceinline__ void gload(f32x4 (&r)[2], const float* __restrict__ base, int64_t ld, int64_t rows,
                                      int64_t K, int64_t row0, int64_t k0) {
  const int t = threadIdx.x;
  const int64_t gk = k0 + (t & 3) * 4;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int64_t gr = row0 + (t >> 2) + 64 * i;
    r[i] = (gr < rows && gk < K) ? *(const f32x4*)(base + gr * ld + gk) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
}

__device__ __forceinline__ void swrite(float* img, const f32x4 (&r)[2]) {
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 2; ++i) *(f32x4*)(img + ((t >> 2) + 64 * i) * LDR + (t & 3) * 4) = r[i];
}

__device__ __forceinline__ void xcd_remap(int& tx, int& ty) {
  const int gx = gridDim.x, nwg = gridDim.x * gridDim.y;
  const int orig = blockIdx.y * gx + blockIdx.x;
  int id = orig;
  if (nwg >= 16) {
    const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
    id = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  }
  ty = id / gx;
  tx = id - ty * gx;
}

__device__ __forceinline__ uint2 pack4f(const float* v) { return make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3])); }

template <int ACT>
__global__ __launch_bounds__(NTH, 2) void sgemm_tn_kernel(FP p) {
  __shared__ __attribute__((aligned(16))) float smem[4 * TILE_FLOATS];   // [buf][A | B] images, 40 KB
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, wm = w >> 1, wn = w & 1;
  int tx, ty;
  xcd_remap(tx, ty);
  const int64_t m0 = (int64_t)ty * BM, n0 = (int64_t)tx * BN;
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = (int)((p.K + KT - 1) / KT);
  f32x4 ra[2], rb[2];
  gload(ra, p.A, p.lda, p.M, p.K, m0, 0);
  gload(rb, p.B, p.ldb, p.N, p.K, n0, 0);
  swrite(smem, ra);
  swrite(smem + TILE_FLOATS, rb);
  __syncthreads();
  const int r16 = lane & 15, g = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const float* As = smem + (kt & 1) * 2 * TILE_FLOATS;
    const float* Bs = As + TILE_FLOATS;
    if (kt + 1 < nk) {
      gload(ra, p.A, p.lda, p.M, p.K, m0, (int64_t)(kt + 1) * KT);
      gload(rb, p.B, p.ldb, p.N, p.K, n0, (int64_t)(kt + 1) * KT);
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) {          // k = 4 s + g: one 16 x 16 x 4 MFMA per block, ascending k
      float a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = As[(wm * 64 + i * 16 + r16) * LDR + 4 * s + g];
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = Bs[(wn * 64 + j * 16 + r16) * LDR + 4 * s + g];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(b[j], a[i], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) {
      float* nb = smem + ((kt + 1) & 1) * 2 * TILE_FLOATS;
      swrite(nb, ra);
      swrite(nb + TILE_FLOATS, rb);
    }
    __syncthreads();
  }
  // lane: row m0 + wm*64 + 16 i + r16, columns n0 + wn*64 + 16 j + 4 g + [0, 4)
  const int64_t wc0 = n0 + wn * 64;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t gm = m0 + wm * 64 + i * 16 + r16;
    if (gm >= p.M) continue;
    float v[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) v[j][r] = acc[i][j][r] * p.alpha;
    if constexpr (ACT == 2) {
      // the wave's 64 columns are one packed group: blocks 0, 1 = x, blocks 2, 3 = gate
      if (wc0 >= p.N) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        *(uint2*)(p.C2 + gm * p.ldc2 + wc0 + 16 * j + 4 * g) = pack4f(v[j]);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        float o[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float gt = v[j + 2][r];
          o[r] = gt * 0.5f * (1.f + erff(gt * 0.70710678118654752f)) * v[j][r];
        }
        const int64_t gc = (wc0 >> 1) + 16 * j + 4 * g;
        *(f32x4*)(p.C + gm * p.ldc + gc) = f32x4{o[0], o[1], o[2], o[3]};
        if (p.C3) *(uint2*)(p.C3 + gm * p.ldc3 + gc) = pack4f(o);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t gn = wc0 + 16 * j + 4 * g;
        if (gn >= p.N) continue;
        if (p.bias) {
          const f32x4 b = *(const f32x4*)(p.bias + gn);
#pragma unroll
          for (int r = 0; r < 4; ++r) v[j][r] += b[r];
        }
        if (p.R) {
          const f32x4 rr = *(const f32x4*)(p.R + gm * p.ldr + gn);
#pragma unroll
          for (int r = 0; r < 4; ++r) v[j][r] += rr[r];
        }
        *(f32x4*)(p.C + gm * p.ldc + gn) = f32x4{v[j][0], v[j][1], v[j][2], v[j][3]};
        if (p.C2) *(uint2*)(p.C2 + gm * p.ldc2 + gn) = pack4f(v[j]);
      }
    }
  }
}

}  // namespace

extern "C" int ctclip_sgemm_tn(const ctclip_sgemm_tn_args* a, void* stream) {
  if (!a) return CT_EINVAL;
  if (a->M == 0 || a->N == 0) return 0;
  CT_REQUIRE(a->M > 0 && a->N > 0 && a->K > 0 && a->C && a->A && a->B, CT_EINVAL);
  CT_REQUIRE(a->act == 0 || a->act == 2, CT_EINVAL);
  CT_REQUIRE(a->K % 4 == 0 && a->N % 4 == 0 && a->lda % 4 == 0 && a->ldb % 4 == 0 && a->ldc % 4 == 0, CT_EALIGN);
  CT_REQUIRE(aligned16(a->A) && aligned16(a->B) && aligned16(a->C), CT_EALIGN);
  if (a->C2) CT_REQUIRE(((uintptr_t)a->C2 & 7) == 0 && a->ldc2 % 4 == 0, CT_EALIGN);
  if (a->C3) CT_REQUIRE(((uintptr_t)a->C3 & 7) == 0 && a->ldc3 % 4 == 0, CT_EALIGN);
  if (a->bias) CT_REQUIRE(aligned16(a->bias) && a->act == 0, CT_EINVAL);
  if (a->R) CT_REQUIRE(aligned16(a->R) && a->ldr % 4 == 0 && a->act == 0, CT_EINVAL);
  if (a->act == 2) CT_REQUIRE(a->N % 64 == 0 && a->C2, CT_EINVAL);
  FP p{a->M, a->N, a->K, a->A, a->lda, a->B, a->ldb, a->C, a->ldc, (u16*)a->C2, a->ldc2, (u16*)a->C3, a->ldc3,
       a->bias, a->R, a->ldr, a->alpha, a->act};
  dim3 grid((unsigned)cdiv(a->N, BN), (unsigned)cdiv(a->M, BM));
  if (a->act == 2)
    hipLaunchKernelGGL(sgemm_tn_kernel<2>, grid, dim3(NTH), 0, (hipStream_t)stream, p);
  else
    hipLaunchKernelGGL(sgemm_tn_kernel<0>, grid, dim3(NTH), 0, (hipStream_t)stream, p);
  CT_CHECK_LAUNCH();
  return 0;
}
