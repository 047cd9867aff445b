// Image x text similarity + symmetric InfoNCE (ct_clip/ct_clip.py:771,796,845-901), fused
// forward + backward in one workgroup.  Exactly the reference's formula: no max subtraction,
// log(x + 1e-20), mean over rows, both directions averaged.  Inputs are the RAW projected
// latents of the (all-gathered) global batch; the kernel l2-normalises them (F.normalize,
// eps 1e-12, ct_clip.py:771) and returns d(loss)/d(raw latents) for every row.
#include "common.h"
#include "../../include/ctclip_hip.h"

namespace {

constexpr int MAXB = 128;

// 1,024 threads: the per-row passes (2 Bg rows) and the Bg^2 dot products spread over 16 waves
// (with 4 waves each walked 4 rows / 16 dots in sequence: ~110 us in the step, on its critical path)
constexpr int CL_NT = 1024, CL_NW = CL_NT / 64;
__global__ __launch_bounds__(CL_NT) void clip_loss_kernel(const float* __restrict__ t_raw, const float* __restrict__ i_raw,
                                                        int Bg, int Dl, const float* __restrict__ log_temp,
                                                        float* __restrict__ tn, float* __restrict__ in_,
                                                        float* __restrict__ loss_out, float* __restrict__ dt_raw,
                                                        float* __restrict__ di_raw, float* __restrict__ dlogtemp,
                                                        float* __restrict__ sim_out) {
  __shared__ float S[MAXB][MAXB + 1];
  __shared__ float tnorm[MAXB], inorm[MAXB], rs[MAXB], cs[MAXB], red[CL_NW];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const float temp = __expf(log_temp[0]);
  // 1. norms (one wave per row)
  for (int r = w; r < 2 * Bg; r += CL_NW) {
    const float* src = r < Bg ? t_raw + (int64_t)r * Dl : i_raw + (int64_t)(r - Bg) * Dl;
    float s = 0.f;
    for (int k = lane; k < Dl; k += 64) s += src[k] * src[k];
    s = warp_sum(s);
    const float n = sqrtf(s);
    const float inv = 1.f / fmaxf(n, 1e-12f);
    float* dst = r < Bg ? tn + (int64_t)r * Dl : in_ + (int64_t)(r - Bg) * Dl;
    for (int k = lane; k < Dl; k += 64) dst[k] = src[k] * inv;
    if (lane == 0) { if (r < Bg) tnorm[r] = n; else inorm[r - Bg] = n; }
  }
  __syncthreads();
  // 2. S = temp * tn . in^T
  for (int e = w; e < Bg * Bg; e += CL_NW) {
    const int i = e / Bg, j = e - i * Bg;
    float s = 0.f;
    for (int k = lane; k < Dl; k += 64) s += tn[(int64_t)i * Dl + k] * in_[(int64_t)j * Dl + k];
    s = warp_sum(s);
    if (lane == 0) S[i][j] = s * temp;
  }
  __syncthreads();
  // 3. exp, row / column sums
  for (int e = tid; e < Bg * Bg; e += CL_NT) {
    const int i = e / Bg, j = e - i * Bg;
    if (sim_out) sim_out[e] = S[i][j];
  }
  __syncthreads();
  for (int e = tid; e < Bg * Bg; e += CL_NT) {
    const int i = e / Bg, j = e - i * Bg;
    S[i][j] = __expf(S[i][j]);
  }
  __syncthreads();
  if (tid < Bg) {
    float r = 0.f, c = 0.f;
    for (int j = 0; j < Bg; ++j) { r += S[tid][j]; c += S[j][tid]; }
    rs[tid] = r;
    cs[tid] = c;
  }
  __syncthreads();
  float part = 0.f;
  if (tid < Bg) {
    const float e = S[tid][tid];
    part = (-__logf(e + 1e-20f) + __logf(rs[tid] + 1e-20f)) + (-__logf(e + 1e-20f) + __logf(cs[tid] + 1e-20f));
  }
  const float tot = block_sum(part, red);
  if (tid == 0) loss_out[0] = 0.5f * tot / Bg;
  __syncthreads();
  // 4. dS (stored in place over exp(S)); dlogtemp = sum dS * S  (S = log(E))
  const float c0 = 0.5f / Bg;
  float dlt = 0.f;
  for (int e = tid; e < Bg * Bg; e += CL_NT) {
    const int i = e / Bg, j = e - i * Bg;
    const float E = S[i][j];
    float d = E / (rs[i] + 1e-20f) + E / (cs[j] + 1e-20f);
    if (i == j) d -= 2.f * E / (E + 1e-20f);
    d *= c0;
    dlt += d * __logf(E);
    S[i][j] = d;  // safe: every thread reads only its own elements after the sums
  }
  const float dltot = block_sum(dlt, red);
  if (tid == 0 && dlogtemp) dlogtemp[0] = dltot;
  __syncthreads();
  // 5. d tn_i = temp * sum_j dS_ij in_j ; d in_j = temp * sum_i dS_ij tn_i ; then through l2norm
  for (int r = w; r < 2 * Bg; r += CL_NW) {
    const bool is_t = r < Bg;
    const int a = is_t ? r : r - Bg;
    const float* self = is_t ? tn + (int64_t)a * Dl : in_ + (int64_t)a * Dl;
    const float* other = is_t ? in_ : tn;
    float* out = is_t ? dt_raw + (int64_t)a * Dl : di_raw + (int64_t)a * Dl;
    const float n = is_t ? tnorm[a] : inorm[a];
    // pass 1: dot(self, dn)
    float dotp = 0.f;
    for (int k = lane; k < Dl; k += 64) {
      float g = 0.f;
      for (int b = 0; b < Bg; ++b) g += (is_t ? S[a][b] : S[b][a]) * other[(int64_t)b * Dl + k];
      g *= temp;
      out[k] = g;
      dotp += g * self[k];
    }
    dotp = warp_sum(dotp);
    const float inv = 1.f / fmaxf(n, 1e-12f);
    for (int k = lane; k < Dl; k += 64) {
      const float g = out[k];
      out[k] = n > 1e-12f ? (g - self[k] * dotp) * inv : g * inv;
    }
  }
}

__global__ void clip_scores_kernel(const float* __restrict__ t_raw, const float* __restrict__ i_raw, int B, int Dl,
                                   const float* __restrict__ log_temp, float* __restrict__ out) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int b = w; b < B; b += 4) {
    float tt = 0.f, ii = 0.f, ti = 0.f;
    for (int k = lane; k < Dl; k += 64) {
      const float x = t_raw[(int64_t)b * Dl + k], y = i_raw[(int64_t)b * Dl + k];
      tt += x * x; ii += y * y; ti += x * y;
    }
    tt = warp_sum(tt); ii = warp_sum(ii); ti = warp_sum(ti);
    if (lane == 0) out[b] = ti / (fmaxf(sqrtf(tt), 1e-12f) * fmaxf(sqrtf(ii), 1e-12f)) * __expf(log_temp[0]);
  }
}

// Zero-shot scoring (ct_clip/ctclip_inference.py:305-315 over the eval branch ct_clip.py:805-807):
// one workgroup per image row n; the image latent is l2-normalised once, then every wave takes
// prompt pairs j: s = temp * <t_norm, i_norm> for "present" (row 2j) and "not present" (2j+1),
// prob = softmax over the pair, entry 0.  The image latent stays in LDS; F.normalize eps 1e-12.
__global__ __launch_bounds__(256) void zero_shot_kernel(const float* __restrict__ t_raw, const float* __restrict__ i_raw,
                                                        int P, int Dl, const float* __restrict__ log_temp,
                                                        float* __restrict__ scores, float* __restrict__ probs) {
  extern __shared__ float img[];
  __shared__ float red[4];
  const int n = blockIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float ii = 0.f;
  for (int k = threadIdx.x; k < Dl; k += 256) {
    const float y = i_raw[(int64_t)n * Dl + k];
    img[k] = y;
    ii += y * y;
  }
  ii = warp_sum(ii);
  if (lane == 0) red[w] = ii;
  __syncthreads();
  const float inorm = fmaxf(sqrtf(red[0] + red[1] + red[2] + red[3]), 1e-12f);
  const float temp = expf(log_temp[0]);
  for (int j = w; j < P; j += 4) {
    float s[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const float* t = t_raw + (int64_t)(2 * j + e) * Dl;
      float tt = 0.f, ti = 0.f;
      for (int k = lane; k < Dl; k += 64) {
        const float x = t[k];
        tt += x * x;
        ti += x * img[k];
      }
      tt = warp_sum(tt);
      ti = warp_sum(ti);
      s[e] = ti / (fmaxf(sqrtf(tt), 1e-12f) * inorm) * temp;
    }
    if (lane == 0) {
      const float m = fmaxf(s[0], s[1]), e0 = expf(s[0] - m), e1 = expf(s[1] - m);
      scores[((int64_t)n * P + j) * 2] = s[0];
      scores[((int64_t)n * P + j) * 2 + 1] = s[1];
      probs[(int64_t)n * P + j] = e0 / (e0 + e1);
    }
  }
}

}  // namespace

extern "C" int ctclip_zero_shot(const float* t_raw, const float* i_raw, int32_t P, int32_t N, int32_t Dl,
                                const float* log_temp, float* scores, float* probs, void* stream) {
  CT_REQUIRE(P >= 0 && N >= 0 && Dl > 0 && Dl <= 8192, CT_ESHAPE);
  if (P == 0 || N == 0) return 0;
  hipLaunchKernelGGL(zero_shot_kernel, dim3(N), dim3(256), (size_t)Dl * 4, (hipStream_t)stream, t_raw, i_raw, P, Dl,
                     log_temp, scores, probs);
  CT_CHECK_LAUNCH();
  return 0;
}

extern "C" int ctclip_clip_loss(const float* t_raw, const float* i_raw, int32_t Bg, int32_t Dl, const float* log_temp,
                                float* t_norm, float* i_norm, float* loss, float* dt_raw, float* di_raw,
                                float* dlogtemp, float* sim, void* stream) {
  CT_REQUIRE(Bg > 0 && Bg <= MAXB, CT_ESHAPE);
  hipLaunchKernelGGL(clip_loss_kernel, dim3(1), dim3(CL_NT), 0, (hipStream_t)stream, t_raw, i_raw, Bg, Dl, log_temp,
                     t_norm, i_norm, loss, dt_raw, di_raw, dlogtemp, sim);
  CT_CHECK_LAUNCH();
  return 0;
}

extern "C" int ctclip_clip_scores(const float* t_raw, const float* i_raw, int32_t B, int32_t Dl, const float* log_temp,
                                  float* out, void* stream) {
  hipLaunchKernelGGL(clip_scores_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, t_raw, i_raw, B, Dl, log_temp,
                     out);
  CT_CHECK_LAUNCH();
  return 0;
}
