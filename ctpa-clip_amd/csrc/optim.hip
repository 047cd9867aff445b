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
                                                        float* __restrict__ out, int* skip) {
  __shared__ float red[8];
  float s = 0.f;
  for (int i = threadIdx.x; i < nblk; i += 256) s += part[i];
  s = block_sum(s, red);
  if (threadIdx.x == 0) {
    const float norm = sqrtf(s);
    out[0] = norm;
    out[1] = max_norm > 0.f ? fminf(1.f, max_norm / (norm + 1e-6f)) : 1.f;
    // a NaN / inf gradient would reach every parameter through Adam (torch's clip_grad_norm_ would
    // scale by a NaN coefficient): flag the step in the Adam kernels' skip word instead.  The norm is
    // taken after the SUM all-reduce, so every rank sees the same value and skips together.
    if (skip && !(norm <= 3.4e38f))
      __hip_atomic_fetch_or(skip, CT_STATUS_NONFINITE_GRAD, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__device__ __forceinline__ float adam_one(float& pi, float gi, float& mi, float& vi, float c, float b1, float b2,
                                          float eps, float wd, float step, float bc2_sqrt) {
  gi *= c;
  if (wd != 0.f) gi += wd * pi;
  mi = b1 * mi + (1.f - b1) * gi;
  vi = b2 * vi + (1.f - b2) * gi * gi;
  pi -= step * mi / (sqrtf(vi) / bc2_sqrt + eps);
  return pi;
}

// 16-B vector body over [head, head + 4*n4) (all five arenas share one element layout, so one
// alignment head serves every pointer); block 0 also does the <= 3-element head and the tail.
// The gradient is zeroed in the same pass (the trainer's zero_grad).
__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v, int64_t n, int head,
                                                   float lr, float b1, float b2, float eps, float wd, float bc1,
                                                   float bc2_sqrt, const float* __restrict__ coef,
                                                   u16* __restrict__ pb, u16* __restrict__ pbl, int zero_grad,
                                                   const int* __restrict__ skip) {
  const float c = coef ? coef[1] : 1.f;
  const float step = lr / bc1;
  const int64_t n4 = (n - head) >> 2;
  f32x4* p4 = (f32x4*)(p + head);
  f32x4* g4 = (f32x4*)(g + head);
  f32x4* m4 = (f32x4*)(m + head);
  f32x4* v4 = (f32x4*)(v + head);
  // the step's guard word (the LayerNorm-fused GEMM status): a step whose forward produced wrong
  // LayerNorm outputs is dropped -- parameters and moments stay as they are, its gradients are
  // cleared (zero_grad) so they do not leak into a later step
  if (skip && *skip) {
    if (!zero_grad) return;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x)
      g4[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (blockIdx.x == 0 && threadIdx.x < 8) {
      const int t = threadIdx.x;
      const int64_t i = t < 4 ? (t < head ? t : -1) : head + 4 * n4 + (t - 4);
      if (i >= 0 && i < n) g[i] = 0.f;
    }
    return;
  }
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    f32x4 pi = p4[i], gi = g4[i], mi = m4[i], vi = v4[i];
    float o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float pj = pi[j], mj = mi[j], vj = vi[j];
      o[j] = adam_one(pj, gi[j], mj, vj, c, b1, b2, eps, wd, step, bc2_sqrt);
      pi[j] = pj; mi[j] = mj; vi[j] = vj;
    }
    p4[i] = pi; m4[i] = mi; v4[i] = vi;
    if (zero_grad) g4[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (pb) {
      u16 h[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) h[j] = f2bf(o[j]);
      uint2 w;
      w.x = (unsigned)h[0] | ((unsigned)h[1] << 16);
      w.y = (unsigned)h[2] | ((unsigned)h[3] << 16);
      *(uint2*)(pb + head + 4 * i) = w;
      if (pbl) {          // lo = bf16(p - hi): the text tower's split weights (gemm.hip B2)
        w.x = (unsigned)f2bf(o[0] - bf2f(h[0])) | ((unsigned)f2bf(o[1] - bf2f(h[1])) << 16);
        w.y = (unsigned)f2bf(o[2] - bf2f(h[2])) | ((unsigned)f2bf(o[3] - bf2f(h[3])) << 16);
        *(uint2*)(pbl + head + 4 * i) = w;
      }
    }
  }
  if (blockIdx.x == 0 && threadIdx.x < 8) {
    const int t = threadIdx.x;
    const int64_t i = t < 4 ? (t < head ? t : -1) : head + 4 * n4 + (t - 4);
    if (i >= 0 && i < n) {
      float pj = p[i], mj = m[i], vj = v[i];
      adam_one(pj, g[i], mj, vj, c, b1, b2, eps, wd, step, bc2_sqrt);
      p[i] = pj; m[i] = mj; v[i] = vj;
      if (zero_grad) g[i] = 0.f;
      if (pb) pb[i] = f2bf(pj);
      if (pb && pbl) pbl[i] = f2bf(pj - bf2f(f2bf(pj)));
    }
  }
}

}  // namespace

extern "C" int ctclip_grad_norm(const float* g, int64_t n, float max_norm, float* part, int32_t nblk, float* out,
                                void* stream) {
  return ctclip_grad_norm_s(g, n, max_norm, part, nblk, out, nullptr, stream);
}

extern "C" int ctclip_grad_norm_s(const float* g, int64_t n, float max_norm, float* part, int32_t nblk, float* out,
                                  int32_t* skip, void* stream) {
  hipLaunchKernelGGL(sumsq_kernel, dim3(nblk), dim3(256), 0, (hipStream_t)stream, g, n, part);
  hipLaunchKernelGGL(clip_coef_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, part, nblk, max_norm, out,
                     (int*)skip);
  CT_CHECK_LAUNCH();
  return 0;
}

extern "C" int ctclip_adam(float* p, float* g, float* m, float* v, int64_t n, float lr, float b1, float b2,
                           float eps, float wd, int32_t step, const float* coef, void* p_bf16, void* p_bf16_lo,
                           int32_t zero_grad, const int32_t* skip, void* stream) {
  const float bc1 = 1.f - powf(b1, (float)step);
  const float bc2 = sqrtf(1.f - powf(b2, (float)step));
  if (n <= 0) return 0;
  // p, g, m, v are slices of arenas with one shared element layout: one alignment head for all
  const int head = (int)std::min<int64_t>(n, ((16 - ((uintptr_t)p & 15)) & 15) / 4);
  if (((uintptr_t)g & 15) != ((uintptr_t)p & 15) || ((uintptr_t)m & 15) != ((uintptr_t)p & 15) ||
      ((uintptr_t)v & 15) != ((uintptr_t)p & 15) || ((uintptr_t)p & 3))
    return CT_EALIGN;
  const int64_t n4 = (n - head) / 4;
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>(4096, (n4 + 255) / 256));
  hipLaunchKernelGGL(adam_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, p, g, m, v, n, head, lr, b1, b2,
                     eps, wd, bc1, bc2, coef, (u16*)p_bf16, (u16*)p_bf16_lo, zero_grad, skip);
  CT_CHECK_LAUNCH();
  return 0;
}
