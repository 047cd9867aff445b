// Small exact-f32 GEMM with arbitrary strides (operands of any orientation), used where the
// reference computes in fp32 on small matrices: the continuous-position-bias MLP on the
// 2,209 deduplicated offsets (ct_clip/attention.py:247-252,271-274) and its backward, and the
// text-latent projection (ct_clip.py:549,765).  64x64 tile, 256 threads x (4x4) outputs.
//   C[m*scm + n*scn] (+)= epi( alpha * sum_k A[m*sam + k*sak] * B[k*sbk + n*sbn] + bias[n] )
//   act 0: none; 1: LeakyReLU(slope); 2: multiply by LeakyReLU'(aux[m*sam2 + n*san2]) (backward)
#include "common.h"
#include "../../include/ctclip_hip.h"

namespace {

__global__ __launch_bounds__(256) void sgemm_kernel(int64_t M, int64_t N, int64_t K, const float* __restrict__ A,
                                                    int64_t sam, int64_t sak, const float* __restrict__ B, int64_t sbk,
                                                    int64_t sbn, float* __restrict__ C, int64_t scm, int64_t scn,
                                                    const float* __restrict__ bias, float alpha, int act, float slope,
                                                    const float* __restrict__ aux, int64_t sxm, int64_t sxn,
                                                    int accumulate) {
  __shared__ float As[16][64 + 4];
  __shared__ float Bs[16][64 + 4];
  const int tid = threadIdx.x;
  const int tx = tid & 15, ty = tid >> 4;
  const int64_t m0 = (int64_t)blockIdx.y * 64, n0 = (int64_t)blockIdx.x * 64;
  float acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = 0.f;
  for (int64_t k0 = 0; k0 < K; k0 += 16) {
    for (int e = tid; e < 16 * 64; e += 256) {
      const int kk = e / 64, mm = e - kk * 64;
      const int64_t gk = k0 + kk;
      As[kk][mm] = (m0 + mm < M && gk < K) ? A[(m0 + mm) * sam + gk * sak] : 0.f;
      Bs[kk][mm] = (n0 + mm < N && gk < K) ? B[gk * sbk + (n0 + mm) * sbn] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) {
      float a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) { a[i] = As[kk][ty * 4 + i]; b[i] = Bs[kk][tx * 4 + i]; }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(a[i], b[j], acc[i][j]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t m = m0 + ty * 4 + i;
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t n = n0 + tx * 4 + j;
      if (n >= N) continue;
      float v = acc[i][j] * alpha;
      if (bias) v += bias[n];
      if (act == 1) v = v > 0.f ? v : v * slope;
      if (act == 2) v *= aux[m * sxm + n * sxn] > 0.f ? 1.f : slope;
      float* c = C + m * scm + n * scn;
      *c = accumulate ? *c + v : v;
    }
  }
}

}  // namespace

extern "C" int ctclip_sgemm(int64_t M, int64_t N, int64_t K, const float* A, int64_t sam, int64_t sak, const float* B,
                            int64_t sbk, int64_t sbn, float* C, int64_t scm, int64_t scn, const float* bias,
                            float alpha, int32_t act, float slope, const float* aux, int64_t sxm, int64_t sxn,
                            int32_t accumulate, void* stream) {
  if (M == 0 || N == 0) return 0;
  dim3 grid(cdiv(N, 64), cdiv(M, 64));
  hipLaunchKernelGGL(sgemm_kernel, grid, dim3(256), 0, (hipStream_t)stream, M, N, K, A, sam, sak, B, sbk, sbn, C, scm,
                     scn, bias, alpha, act, slope, aux, sxm, sxn, accumulate);
  CT_CHECK_LAUNCH();
  return 0;
}
