// Optimizer step of CTClipTrainer.train_step (ct_clip/CTCLIPTrainer.py:347-353):
// clip_grad_norm_(max_norm) then Adam (ct_clip/optimizer.py:24, wd = 0 -> torch.optim.Adam),
// over ONE flat f32 parameter / gradient arena, with the bf16 working copy refreshed in the
// same pass.  Norm clip coefficient computed on device (no host sync).
#include "common.h"
#include "../../include/ctclip_hip.h"

namespace {

__global__ __launch_bounds__(256) void sumsq_kernel(const float* __restrict__ x, int64_t n, float* __restrict__ part) {
  __shared__ float red[8];
  float s = 0.f;
  const int64_t n4 = n / 4;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    const f32x4 v = ((const f32x4*)x)[i];
    s += v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3];
  }
  for (int64_t i = n4 * 4 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    s += x[i] * x[i];
  s = block_sum(s, red);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

__global__ __launch_bounds__(256) void clip_coef_kernel(const float* __restrict__ part, int nblk, float max_norm,
                                                        float* __restrict__ out) {
  __shared__ float red[8];
  float s = 0.f;
  for (int i = threadIdx.x; i < nblk; i += 256) s += part[i];
  s = block_sum(s, red);
  if (threadIdx.x == 0) {
    const float norm = sqrtf(s);
    out[0] = norm;
    out[1] = max_norm > 0.f ? fminf(1.f, max_norm / (norm + 1e-6f)) : 1.f;
  }
}

__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v, int64_t n, float lr,
                                                   float b1, float b2, float eps, float wd, float bc1, float bc2_sqrt,
                                                   const float* __restrict__ coef, u16* __restrict__ pb) {
  const float c = coef ? coef[1] : 1.f;
  const float step = lr / bc1;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float gi = g[i] * c;
    float pi = p[i];
    if (wd != 0.f) gi += wd * pi;
    const float mi = b1 * m[i] + (1.f - b1) * gi;
    const float vi = b2 * v[i] + (1.f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    pi -= step * mi / (sqrtf(vi) / bc2_sqrt + eps);
    p[i] = pi;
    if (pb) pb[i] = f2bf(pi);
  }
}

}  // namespace

extern "C" int ctclip_grad_norm(const float* g, int64_t n, float max_norm, float* part, int32_t nblk, float* out,
                                void* stream) {
  hipLaunchKernelGGL(sumsq_kernel, dim3(nblk), dim3(256), 0, (hipStream_t)stream, g, n, part);
  hipLaunchKernelGGL(clip_coef_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, part, nblk, max_norm, out);
  CT_CHECK_LAUNCH();
  return 0;
}

extern "C" int ctclip_adam(float* p, const float* g, float* m, float* v, int64_t n, float lr, float b1, float b2,
                           float eps, float wd, int32_t step, const float* coef, void* p_bf16, void* stream) {
  const float bc1 = 1.f - powf(b1, (float)step);
  const float bc2 = sqrtf(1.f - powf(b2, (float)step));
  const int blocks = (int)std::min<int64_t>(8192, (n + 255) / 256);
  hipLaunchKernelGGL(adam_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, p, g, m, v, n, lr, b1, b2, eps, wd,
                     bc1, bc2, coef, (u16*)p_bf16);
  CT_CHECK_LAUNCH();
  return 0;
}
