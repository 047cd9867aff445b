// Exact-f32 GEMM with arbitrary strides (operands of any orientation), used where the reference
// computes in fp32 on small matrices: the continuous-position-bias MLP on the 2,209
// deduplicated offsets (ct_clip/attention.py:247-252,271-274) and its backward, and the
// text-latent projection (ct_clip.py:549,765).
//   C[m*scm + n*scn] (+)= epi( alpha * sum_k A[m*sam + k*sak] * B[k*sbk + n*sbn] + bias[n] )
//   act 0: none; 1: LeakyReLU(slope); 2: multiply by LeakyReLU'(aux[m*sxm + n*sxn]) (backward)
// On v_mfma_f32_16x16x4_f32 (exact f32: a k-ordered fmaf chain per output, CDNA4 f32-input
// MFMA): 64x64 block tile, 4 waves of 32x32, K tile 32 staged through LDS with a load mapping
// chosen by which operand stride is unit (coalesced either way).  Long-K / few-tile products
// (the weight gradients, K = 2,209 offsets) split K over gridDim.z into f32 slabs of a caller
// workspace, folded in a fixed order by a second kernel that applies the epilogue.
#include "common.h"
#include "../../include/ctclip_hip.h"

namespace {

constexpr int BT = 64, KT = 32, LDP = BT + 4;

struct SP {
  int64_t M, N, K;
  const float* A; int64_t sam, sak;
  const float* B; int64_t sbk, sbn;
  float* C; int64_t scm, scn;
  const float* bias; float alpha; int act; float slope;
  const float* aux; int64_t sxm, sxn;
  int accumulate;
  float* ws; int split; int64_t kper;
};

__device__ __forceinline__ float epi(const SP& p, int64_t m, int64_t n, float v) {
  v *= p.alpha;
  if (p.bias) v += p.bias[n];
  if (p.act == 1) v = v > 0.f ? v : v * p.slope;
  if (p.act == 2) v *= p.aux[m * p.sxm + n * p.sxn] > 0.f ? 1.f : p.slope;
  return v;
}

__global__ __launch_bounds__(256) void sgemm_mfma_kernel(SP p) {
  __shared__ float As[KT][LDP];   // [k][m]
  __shared__ float Bs[KT][LDP];   // [k][n]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wm = w >> 1, wn = w & 1;
  const int64_t m0 = (int64_t)blockIdx.y * BT, n0 = (int64_t)blockIdx.x * BT;
  const int64_t kb = (int64_t)blockIdx.z * p.kper, ke = min(p.K, kb + p.kper);
  const bool a_kc = p.sak == 1, b_kc = p.sbk == 1;
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int64_t k0 = kb; k0 < ke; k0 += KT) {
#pragma unroll
    for (int r = 0; r < KT * BT / 256; ++r) {
      const int e = tid + r * 256;
      int mm, kk;
      if (a_kc) { mm = e / KT; kk = e % KT; } else { mm = e % BT; kk = e / BT; }
      const int64_t gm = m0 + mm, gk = k0 + kk;
      As[kk][mm] = (gm < p.M && gk < ke) ? p.A[gm * p.sam + gk * p.sak] : 0.f;
      int nn, kk2;
      if (b_kc) { nn = e / KT; kk2 = e % KT; } else { nn = e % BT; kk2 = e / BT; }
      const int64_t gn = n0 + nn, gk2 = k0 + kk2;
      Bs[kk2][nn] = (gn < p.N && gk2 < ke) ? p.B[gk2 * p.sbk + gn * p.sbn] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < KT; ks += 4) {
      const int k = ks + (lane >> 4);
      float a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = As[k][wm * 32 + i * 16 + (lane & 15)];
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = Bs[k][wn * 32 + j * 16 + (lane & 15)];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t m = m0 + wm * 32 + i * 16 + (lane >> 4) * 4 + r;
        const int64_t n = n0 + wn * 32 + j * 16 + (lane & 15);
        if (m >= p.M || n >= p.N) continue;
        if (p.split > 1) {
          p.ws[((int64_t)blockIdx.z * p.M + m) * p.N + n] = acc[i][j][r];
        } else {
          const float v = epi(p, m, n, acc[i][j][r]);
          float* c = p.C + m * p.scm + n * p.scn;
          *c = p.accumulate ? *c + v : v;
        }
      }
}

// fold the split-K slabs in slab order, then the epilogue
__global__ __launch_bounds__(256) void sgemm_fold_kernel(SP p) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= p.M * p.N) return;
  const int64_t m = i / p.N, n = i - m * p.N;
  float s = 0.f;
  for (int z = 0; z < p.split; ++z) s += p.ws[(int64_t)z * p.M * p.N + i];
  const float v = epi(p, m, n, s);
  float* c = p.C + m * p.scm + n * p.scn;
  *c = p.accumulate ? *c + v : v;
}

}  // namespace

extern "C" int ctclip_sgemm(int64_t M, int64_t N, int64_t K, const float* A, int64_t sam, int64_t sak, const float* B,
                            int64_t sbk, int64_t sbn, float* C, int64_t scm, int64_t scn, const float* bias,
                            float alpha, int32_t act, float slope, const float* aux, int64_t sxm, int64_t sxn,
                            int32_t accumulate, float* workspace, int32_t split, void* stream) {
  if (M == 0 || N == 0) return 0;
  CT_REQUIRE(split >= 1 && (split == 1 || workspace != nullptr), CT_EINVAL);
  SP p{M, N, K, A, sam, sak, B, sbk, sbn, C, scm, scn, bias, alpha, act, slope, aux, sxm, sxn, accumulate,
       workspace, split, 0};
  p.kper = ((K + split - 1) / split + KT - 1) / KT * KT;
  if (p.kper == 0) p.kper = KT;
  dim3 grid(cdiv(N, BT), cdiv(M, BT), split);
  hipLaunchKernelGGL(sgemm_mfma_kernel, grid, dim3(256), 0, (hipStream_t)stream, p);
  CT_CHECK_LAUNCH();
  if (split > 1) {
    hipLaunchKernelGGL(sgemm_fold_kernel, dim3(cdiv(M * N, 256)), dim3(256), 0, (hipStream_t)stream, p);
    CT_CHECK_LAUNCH();
  }
  return 0;
}
