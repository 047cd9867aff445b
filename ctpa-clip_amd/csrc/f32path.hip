// Exact-f32 forward kernels of the opt-in f32 image tower (ctclip_mi355x/precise.py,
// functional.set_vit_precision('f32')): the reference runs the 3D-ViT in fp32
// (ct_clip/CTCLIPTrainer.py:342 -- accelerator.autocast() is a no-op), and its VQ argmax
// (ct_clip/ctvit.py:427) flips on near-ties under the bf16 tower's ~1e-2 token error.  This mode
// keeps every activation f32 and every product an f32 fma, so the tokens entering the VQ carry
// only f32 summation-order differences.  The linears run on ctclip_sgemm (v_mfma_f32_16x16x4_f32,
// exact f32); the kernels here are the non-GEMM stages:
//   patch_ln_f32 : patchify (c pt p1 p2) + LayerNorm(pd) with affine   (ctvit.py:169-174)
//   peg_f32      : causal depthwise 3x3x3 conv + bias + residual       (attention.py:56-84, 324)
//   l2norm_f32   : l2norm per head * scale                             (attention.py:152-154)
//   attn_f32     : softmax(scale q.k^T + CPB bias) v per (sequence, head), online softmax
//                  (attention.py:156-181, CPB table of attention.py:229-276)
//   geglu_f32    : gelu(gate) * x on the un-interleaved FF1 output    (attention.py:39-42)
// Transcendentals use the libm forms (expf, erff, sqrtf), not the fast approximations of the
// bf16 path.  Index maps are the bf16 kernels' (peg.hip, attn.hip): canonical (b, t, h, w) rows.
#include "common.h"
#include "../../include/ctclip_hip.h"

namespace {

constexpr int MAXC = 64;  // patch_dim <= 64 * 64

__global__ __launch_bounds__(256) void patch_ln_f32_kernel(const void* __restrict__ video, int is_f32, int is_hu,
                                                           int64_t ntok, int T, int Hg, int Wg, int64_t vol_stride,
                                                           int64_t frame_elems, int W, int PT, int P,
                                                           const int32_t* __restrict__ offs, int pd, float eps,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ beta, float* __restrict__ out,
                                                           int64_t ldo) {
  const int lane = threadIdx.x & 63;
  const int64_t tok = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (tok >= ntok) return;
  int64_t r = tok;
  const int wg = (int)(r % Wg); r /= Wg;
  const int hg = (int)(r % Hg); r /= Hg;
  const int t = (int)(r % T);
  const int64_t b = r / T;
  const int64_t base = b * vol_stride + (int64_t)t * PT * frame_elems + (int64_t)hg * P * W + (int64_t)wg * P;
  float v[MAXC];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < MAXC; ++i) {
    const int e = lane + 64 * i;
    float x = 0.f;
    if (e < pd) {
      const int64_t a = base + offs[e];
      x = is_f32 ? ((const float*)video)[a] : (float)((const short*)video)[a];
      if (is_hu) x = fminf(fmaxf(x, -1000.f), 1000.f) / 1000.f;   // ct_clip/data.py:150-152 (exact divide)
    }
    v[i] = x;
    s += x;
  }
  const float mean = warp_sum(s) / (float)pd;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < MAXC; ++i) {
    const int e = lane + 64 * i;
    if (e < pd) { const float d = v[i] - mean; q += d * d; }
  }
  const float rstd = 1.f / sqrtf(warp_sum(q) / (float)pd + eps);
  float* o = out + tok * ldo;
#pragma unroll
  for (int i = 0; i < MAXC; ++i) {
    const int e = lane + 64 * i;
    if (e < pd) o[e] = (v[i] - mean) * rstd * gamma[e] + beta[e];
  }
}

// one thread per (token, 4 channels); out = x + bias + sum of the 27 taps in the reference's view
__global__ __launch_bounds__(256) void peg_f32_kernel(const float* __restrict__ x, int64_t ntok, int D,
                                                      const float* __restrict__ w, const float* __restrict__ bias,
                                                      int T, int H, int W, int mode, float* __restrict__ out) {
  const int dq = D / 4;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= ntok * dq) return;
  const int64_t v = i / dq;
  const int c = (int)(i - v * dq) * 4;
  const int hw = H * W, thw = T * hw;
  const int64_t b = v / thw;
  const int r = (int)(v - b * thw);
  // mode 1: canonical row r = (t, hw) sits at the reference's physical row hw*T + t of '(b h w) t d',
  // raw-reshaped to (b, t, h, w) (attention.py:69-70)
  const int pv = mode == 0 ? r : (r % hw) * T + r / hw;
  const int tv = pv / hw, hv = (pv / W) % H, wv = pv % W;
  float acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = bias ? bias[c + j] : 0.f;
  for (int kt = 0; kt < 3; ++kt) {
    const int tt = tv + kt - 2;
    if (tt < 0) continue;
    for (int kh = 0; kh < 3; ++kh) {
      const int hh = hv + kh - 1;
      if (hh < 0 || hh >= H) continue;
      for (int kw = 0; kw < 3; ++kw) {
        const int ww = wv + kw - 1;
        if (ww < 0 || ww >= W) continue;
        const int p2 = (tt * H + hh) * W + ww;
        const int r2 = mode == 0 ? p2 : (p2 % T) * hw + p2 / T;
        const f32x4 xv = *(const f32x4*)(x + (b * thw + r2) * (int64_t)D + c);
        const int tap = (kt * 3 + kh) * 3 + kw;
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = fmaf(w[(int64_t)(c + j) * 27 + tap], xv[j], acc[j]);
      }
    }
  }
  const f32x4 xr = *(const f32x4*)(x + v * (int64_t)D + c);
  *(f32x4*)(out + v * (int64_t)D + c) = f32x4{acc[0] + xr[0], acc[1] + xr[1], acc[2] + xr[2], acc[3] + xr[3]};
}

// one thread per (row, head): y = x / max(||x||, 1e-12) * scale  (F.normalize semantics)
__global__ __launch_bounds__(256) void l2norm_f32_kernel(const float* __restrict__ x, int64_t ldx, int64_t rows,
                                                         int H, int D, const float* __restrict__ scale,
                                                         float* __restrict__ y, int64_t ldy) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= rows * H) return;
  const int64_t row = i / H;
  const int h = (int)(i - row * H);
  const float* xp = x + row * ldx + h * D;
  float s = 0.f;
  for (int d = 0; d < D; ++d) s = fmaf(xp[d], xp[d], s);
  const float n = fmaxf(sqrtf(s), 1e-12f);
  float* yp = y + row * ldy + h * D;
  for (int d = 0; d < D; ++d) yp[d] = xp[d] / n * scale[d];
}

__global__ __launch_bounds__(256) void geglu_f32_kernel(const float* __restrict__ h, int64_t ldh, int64_t rows,
                                                        int inner, float* __restrict__ g, int64_t ldg) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= rows * inner) return;
  const int64_t r = i / inner;
  const int c = (int)(i - r * inner);
  const float x = h[r * ldh + c], gt = h[r * ldh + inner + c];
  g[r * ldg + c] = gt * 0.5f * (1.f + erff(gt * 0.70710678118654752f)) * x;
}

// one wave per (64 queries, head, sequence); keys / values staged through LDS 64 at a time
template <int D>
__global__ __launch_bounds__(64) void attn_f32_kernel(ctclip_attn_args a) {
  __shared__ float Ks[64][D + 1];
  __shared__ float Vs[64][D + 1];
  const int lane = threadIdx.x;
  const int h = blockIdx.y;
  const int64_t s = blockIdx.z;
  const int L = a.L;
  const int64_t rbase = (s / a.n_inner) * a.s_outer + (s % a.n_inner) * a.s_inner;
  const int qi = blockIdx.x * 64 + lane;
  const bool qv = qi < L;
  const float* Q = (const float*)a.q;
  const float* Kp = (const float*)a.k;
  const float* Vp = (const float*)a.v;
  float q[D], o[D];
#pragma unroll
  for (int d = 0; d < D; ++d) {
    q[d] = qv ? Q[(rbase + (int64_t)qi * a.s_pos) * a.ldq + h * D + d] : 0.f;
    o[d] = 0.f;
  }
  const bool bias = a.bias_u != nullptr;
  const int Wg = a.grid_w > 0 ? a.grid_w : 1;
  const int nb = (2 * a.grid_h - 1) * (2 * Wg - 1);
  const int hq = qi / Wg, wq = qi % Wg;
  float m = -INFINITY, l = 0.f;
  for (int k0 = 0; k0 < L; k0 += 64) {
    const int kj = k0 + lane;
    const int64_t krow = rbase + (int64_t)min(kj, L - 1) * a.s_pos;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      Ks[lane][d] = Kp[krow * a.ldk + h * D + d];
      Vs[lane][d] = Vp[krow * a.ldv + h * D + d];
    }
    __syncthreads();
    const int nk = min(64, L - k0);
    float sc[64];
    float cmax = -INFINITY;
#pragma unroll
    for (int j = 0; j < 64; ++j) {
      float dot = 0.f;
#pragma unroll
      for (int d = 0; d < D; ++d) dot = fmaf(q[d], Ks[j][d], dot);
      float v = dot * a.scale;
      if (bias) {
        const int kk = k0 + j;
        const int bin = (hq - kk / Wg + a.grid_h - 1) * (2 * Wg - 1) + (wq - kk % Wg + Wg - 1);
        v += (j < nk && qv) ? a.bias_u[(int64_t)h * nb + bin] : 0.f;
      }
      sc[j] = j < nk ? v : -INFINITY;
      cmax = fmaxf(cmax, sc[j]);
    }
    const float mn = fmaxf(m, cmax);
    const float corr = expf(m - mn);   // m = -inf on the first chunk -> 0
    l *= corr;
#pragma unroll
    for (int d = 0; d < D; ++d) o[d] *= corr;
#pragma unroll
    for (int j = 0; j < 64; ++j) {
      const float pj = expf(sc[j] - mn);
      l += pj;
#pragma unroll
      for (int d = 0; d < D; ++d) o[d] = fmaf(pj, Vs[j][d], o[d]);
    }
    m = mn;
    __syncthreads();
  }
  if (!qv) return;
  float* O = (float*)a.o + (rbase + (int64_t)qi * a.s_pos) * a.ldo + h * D;
#pragma unroll
  for (int d = 0; d < D; ++d) O[d] = o[d] / l;
}

inline unsigned blocks_for(int64_t n) { return (unsigned)((n + 255) / 256); }

}  // namespace

extern "C" int ctclip_patch_ln_f32(const void* video, int32_t is_f32, int32_t is_hu, int64_t B, int32_t C,
                                   int32_t F, int32_t H, int32_t W, int32_t PT, int32_t P, const int32_t* offs,
                                   float eps, const float* gamma, const float* beta, float* out, int64_t ldo,
                                   void* stream) {
  const int pd = C * PT * P * P;
  CT_REQUIRE(pd <= 64 * MAXC && ldo >= pd && gamma && beta, CT_ESHAPE);
  CT_REQUIRE(F % PT == 0 && H % P == 0 && W % P == 0, CT_ESHAPE);
  const int T = F / PT, Hg = H / P, Wg = W / P;
  const int64_t ntok = B * T * Hg * Wg;
  if (ntok == 0) return 0;
  hipLaunchKernelGGL(patch_ln_f32_kernel, dim3((unsigned)cdiv(ntok, 4)), dim3(256), 0, (hipStream_t)stream, video,
                     is_f32, is_hu, ntok, T, Hg, Wg, (int64_t)C * F * H * W, (int64_t)H * W, W, PT, P, offs, pd, eps,
                     gamma, beta, out, ldo);
  CT_CHECK_LAUNCH();
  return 0;
}

extern "C" int ctclip_peg_fwd_f32(const float* x, int64_t B, int32_t T, int32_t H, int32_t W, int32_t D,
                                  const float* weight, const float* bias, int32_t mode, float* out, void* stream) {
  CT_REQUIRE(D % 4 == 0 && aligned16(x) && aligned16(out) && (mode == 0 || mode == 1), CT_EINVAL);
  const int64_t ntok = B * T * H * W;
  if (ntok == 0) return 0;
  hipLaunchKernelGGL(peg_f32_kernel, dim3(blocks_for(ntok * (D / 4))), dim3(256), 0, (hipStream_t)stream, x, ntok, D,
                     weight, bias, T, H, W, mode, out);
  CT_CHECK_LAUNCH();
  return 0;
}

extern "C" int ctclip_l2norm_scale_fwd_f32(const float* x, int64_t ldx, int64_t rows, int32_t H, int32_t D,
                                           const float* scale, float* y, int64_t ldy, void* stream) {
  if (rows == 0) return 0;
  hipLaunchKernelGGL(l2norm_f32_kernel, dim3(blocks_for(rows * H)), dim3(256), 0, (hipStream_t)stream, x, ldx, rows,
                     H, D, scale, y, ldy);
  CT_CHECK_LAUNCH();
  return 0;
}

extern "C" int ctclip_geglu_f32(const float* h, int64_t ldh, int64_t rows, int32_t inner, float* g, int64_t ldg,
                                void* stream) {
  if (rows == 0) return 0;
  hipLaunchKernelGGL(geglu_f32_kernel, dim3(blocks_for(rows * inner)), dim3(256), 0, (hipStream_t)stream, h, ldh, rows,
                     inner, g, ldg);
  CT_CHECK_LAUNCH();
  return 0;
}

extern "C" int ctclip_attn_fwd_f32(const ctclip_attn_args* a, void* stream) {
  CT_REQUIRE(a && a->q && a->k && a->v && a->o && a->L > 0 && a->nseq >= 0 && a->n_inner > 0, CT_EINVAL);
  CT_REQUIRE(!a->kmask && a->dropout_p == 0.f, CT_EINVAL);
  if (a->bias_u) CT_REQUIRE(a->grid_h > 0 && a->grid_w > 0 && a->grid_h * a->grid_w == a->L, CT_ESHAPE);
  if (a->nseq == 0) return 0;
  dim3 grid((unsigned)cdiv(a->L, 64), (unsigned)a->H, (unsigned)a->nseq);
  if (a->D == 32)
    hipLaunchKernelGGL(attn_f32_kernel<32>, grid, dim3(64), 0, (hipStream_t)stream, *a);
  else if (a->D == 64)
    hipLaunchKernelGGL(attn_f32_kernel<64>, grid, dim3(64), 0, (hipStream_t)stream, *a);
  else
    return CT_ESHAPE;
  CT_CHECK_LAUNCH();
  return 0;
}
