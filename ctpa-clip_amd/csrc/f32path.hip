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

// the same with each lane on 4 consecutive patch elements (P % 4 == 0: one 4-voxel run of a patch
// row, an 8-B int16 / 16-B f32 read; 16-B f32 stores): one wave per token, quads lane + 64 i
__global__ __launch_bounds__(256) void patch_ln_f32_q_kernel(const void* __restrict__ video, int is_f32, int is_hu,
                                                             int64_t ntok, int T, int Hg, int Wg, int64_t vol_stride,
                                                             int64_t frame_elems, int W, int PT, int P,
                                                             const int32_t* __restrict__ offs, int pd, float eps,
                                                             const float* __restrict__ gamma,
                                                             const float* __restrict__ beta, float* __restrict__ out,
                                                             int64_t ldo) {
  constexpr int NQ = MAXC / 4;
  const int lane = threadIdx.x & 63;
  const int64_t tok = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (tok >= ntok) return;
  int64_t r = tok;
  const int wg = (int)(r % Wg); r /= Wg;
  const int hg = (int)(r % Hg); r /= Hg;
  const int t = (int)(r % T);
  const int64_t b = r / T;
  const int64_t base = b * vol_stride + (int64_t)t * PT * frame_elems + (int64_t)hg * P * W + (int64_t)wg * P;
  const int nq = pd / 4;
  f32x4 v[NQ];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NQ; ++i) {
    const int qd = lane + 64 * i;
    f32x4 x = {0.f, 0.f, 0.f, 0.f};
    if (qd < nq) {
      const int64_t a = base + offs[4 * qd];
      if (is_f32) {
        x = *(const f32x4*)((const float*)video + a);
      } else {
        const short4 h = *(const short4*)((const short*)video + a);
        x = f32x4{(float)h.x, (float)h.y, (float)h.z, (float)h.w};
      }
      if (is_hu) {
#pragma unroll
        for (int e = 0; e < 4; ++e) x[e] = fminf(fmaxf(x[e], -1000.f), 1000.f) / 1000.f;   // data.py:150-152
      }
    }
    v[i] = x;
    s += (x[0] + x[1]) + (x[2] + x[3]);
  }
  const float mean = warp_sum(s) / (float)pd;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NQ; ++i) {
    if (lane + 64 * i < nq) {
#pragma unroll
      for (int e = 0; e < 4; ++e) { const float d = v[i][e] - mean; q += d * d; }
    }
  }
  const float rstd = 1.f / sqrtf(warp_sum(q) / (float)pd + eps);
  float* o = out + tok * ldo;
#pragma unroll
  for (int i = 0; i < NQ; ++i) {
    const int qd = lane + 64 * i;
    if (qd < nq) {
      const f32x4 gm = *(const f32x4*)(gamma + 4 * qd), bt = *(const f32x4*)(beta + 4 * qd);
      f32x4 y;
#pragma unroll
      for (int e = 0; e < 4; ++e) y[e] = (v[i][e] - mean) * rstd * gm[e] + bt[e];
      *(f32x4*)(o + 4 * qd) = y;
    }
  }
}

// out = x + bias + sum of the 27 taps in the reference's view.  Thread = one 4-channel quad, its
// 4 x 27 weights held in registers (one contiguous 432-B read per thread, not a stride-27 gather
// per tap); a block = 256 / (D / 4) token slots x PEG_NT consecutive tokens, lanes of a token
// on consecutive quads (coalesced 16-B reads of each tap's row).
constexpr int PEG_NT = 16;

__global__ __launch_bounds__(256) void peg_f32_kernel(const float* __restrict__ x, int64_t ntok, int D,
                                                      const float* __restrict__ w, const float* __restrict__ bias,
                                                      int T, int H, int W, int mode, float* __restrict__ out) {
  const int dq = D / 4, slots = 256 / dq;
  if ((int)threadIdx.x >= slots * dq) return;
  const int slot = threadIdx.x / dq, c = (threadIdx.x - slot * dq) * 4;
  float wr[27][4];
#pragma unroll
  for (int i = 0; i < 27; ++i) {
    const f32x4 t = *(const f32x4*)(w + (int64_t)c * 27 + 4 * i);   // weights of channels c..c+3, taps in order
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int f = 4 * i + e;                                      // flat index (c + f / 27) * 27 + f % 27
      wr[f % 27][f / 27] = t[e];
    }
  }
  float bs[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) bs[j] = bias ? bias[c + j] : 0.f;
  const int hw = H * W, thw = T * hw;
  const int64_t v0 = (int64_t)blockIdx.x * slots * PEG_NT;
  for (int it = 0; it < PEG_NT; ++it) {
    const int64_t v = v0 + (int64_t)it * slots + slot;
    if (v >= ntok) return;
    const int64_t b = v / thw;
    const int r = (int)(v - b * thw);
    // mode 1: canonical row r = (t, hw) sits at the reference's physical row hw*T + t of
    // '(b h w) t d', raw-reshaped to (b, t, h, w) (attention.py:69-70)
    const int pv = mode == 0 ? r : (r % hw) * T + r / hw;
    const int tv = pv / hw, hv = (pv / W) % H, wv = pv % W;
    const float* xb = x + b * thw * (int64_t)D + c;
    float acc[4] = {bs[0], bs[1], bs[2], bs[3]};
#pragma unroll
    for (int kt = 0; kt < 3; ++kt) {
      const int tt = tv + kt - 2;
      if (tt < 0) continue;
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        const int hh = hv + kh - 1;
        if (hh < 0 || hh >= H) continue;
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
          const int ww = wv + kw - 1;
          if (ww < 0 || ww >= W) continue;
          const int p2 = (tt * H + hh) * W + ww;
          const int r2 = mode == 0 ? p2 : (p2 % T) * hw + p2 / T;
          const f32x4 xv = *(const f32x4*)(xb + (int64_t)r2 * D);
          const int tap = (kt * 3 + kh) * 3 + kw;
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[j] = fmaf(wr[tap][j], xv[j], acc[j]);
        }
      }
    }
    const f32x4 xr = *(const f32x4*)(x + v * (int64_t)D + c);
    *(f32x4*)(out + v * (int64_t)D + c) = f32x4{acc[0] + xr[0], acc[1] + xr[1], acc[2] + xr[2], acc[3] + xr[3]};
  }
}

// G = D / 4 lanes per (row, head), a 16-B quad each: y = x / max(||x||, 1e-12) * scale (F.normalize)
template <int G>
__global__ __launch_bounds__(256) void l2norm_f32_vec_kernel(const float* __restrict__ x, int64_t ldx, int64_t rows,
                                                             int H, const float* __restrict__ scale,
                                                             float* __restrict__ y, int64_t ldy,
                                                             u16* __restrict__ yb, int64_t ldyb) {
  const int64_t i = (int64_t)blockIdx.x * (256 / G) + threadIdx.x / G;
  const int q = threadIdx.x % G;
  const bool ok = i < rows * H;
  const int64_t row = ok ? i / H : 0;
  const int h = ok ? (int)(i - row * H) : 0;
  const int D = 4 * G;
  f32x4 v = ok ? *(const f32x4*)(x + row * ldx + h * D + 4 * q) : f32x4{0.f, 0.f, 0.f, 0.f};
  float s = v[0] * v[0];
#pragma unroll
  for (int e = 1; e < 4; ++e) s = fmaf(v[e], v[e], s);
#pragma unroll
  for (int o = 1; o < G; o <<= 1) s += __shfl_xor(s, o, 64);
  if (!ok) return;
  const float n = fmaxf(sqrtf(s), 1e-12f);
  const f32x4 sc = *(const f32x4*)(scale + 4 * q);
  float out[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) out[e] = v[e] / n * sc[e];
  *(f32x4*)(y + row * ldy + h * D + 4 * q) = f32x4{out[0], out[1], out[2], out[3]};
  if (yb) *(uint2*)(yb + row * ldyb + h * D + 4 * q) = pack4(out);   // the bf16 copy (the backward's operand)
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

// D = 32 on the f32 matrix pipe (v_mfma_f32_16x16x4_f32, exact f32 products): one block of 4 waves
// per (64 queries, head, sequence), each wave 16 queries; keys / values in chunks of 64 through LDS.
// QK^T is computed transposed (first MFMA operand = K rows) so a lane ends with 4 keys of ONE query
// (keys 16 j + 4 g + r of sub-block j, query lane & 15): the softmax needs only cross-lane max /
// sum over the 4 lane groups g.  PV reuses that layout with the keys of MFMA step s taken as
// {16 j + 4 g + s : g} -- the probability a lane holds in register s is exactly its B operand, and
// V is staged [key / 4][d][key % 4] so the matching A fragment is one 16-B LDS read.  K is staged
// with its head dims permuted (d = 4 s + g at g * 8 + s) so a lane's 8 QK fragments are 2 reads.
// The CPB bias row of the head and a key -> (h_k * (2 W - 1) + w_k) table sit in LDS.
constexpr int FA_KLD = 36, FA_MAXNB = 2304, FA_MAXL = 1024;

__global__ __launch_bounds__(256) void attn_f32_mfma_kernel(ctclip_attn_args a) {
  __shared__ __attribute__((aligned(16))) float Ks[64 * FA_KLD];
  __shared__ __attribute__((aligned(16))) float Vt[16 * 32 * 4];
  __shared__ float Bs[FA_MAXNB];
  __shared__ __attribute__((aligned(16))) int Kx[FA_MAXL + 64];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r16 = lane & 15, g = lane >> 4;
  const int h = blockIdx.y;
  const int64_t sq = blockIdx.z;
  const int L = a.L;
  const int64_t rbase = (sq / a.n_inner) * a.s_outer + (sq % a.n_inner) * a.s_inner;
  const float* Q = (const float*)a.q;
  const float* Kp = (const float*)a.k;
  const float* Vp = (const float*)a.v;
  const bool bias = a.bias_u != nullptr;
  const int Wg = bias ? a.grid_w : 1;
  const int nb = bias ? (2 * a.grid_h - 1) * (2 * Wg - 1) : 0;
  if (bias) {
    for (int i = tid; i < nb; i += 256) Bs[i] = a.bias_u[(int64_t)h * nb + i];
    for (int i = tid; i < L + 64; i += 256) Kx[i] = i < L ? (i / Wg) * (2 * Wg - 1) + i % Wg : 0;
  }
  const int qi = blockIdx.x * 64 + w * 16 + r16;
  const bool qv = qi < L;
  const int64_t qrow = rbase + (int64_t)min(qi, L - 1) * a.s_pos;
  float qf[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) qf[s] = qv ? Q[qrow * a.ldq + h * 32 + 4 * s + g] : 0.f;
  int qbase = 0;
  if (bias) qbase = (qi / Wg + a.grid_h - 1) * (2 * Wg - 1) + qi % Wg + Wg - 1;
  float m = -INFINITY, l = 0.f;
  f32x4 o[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  const int kk = tid >> 2, c = tid & 3;   // staging: key kk of the chunk, head dims 8 c .. 8 c + 7
  for (int k0 = 0; k0 < L; k0 += 64) {
    __syncthreads();
    {
      const int64_t krow = rbase + (int64_t)min(k0 + kk, L - 1) * a.s_pos;
      const f32x4 k_lo = *(const f32x4*)(Kp + krow * a.ldk + h * 32 + 8 * c);
      const f32x4 k_hi = *(const f32x4*)(Kp + krow * a.ldk + h * 32 + 8 * c + 4);
      const f32x4 v_lo = *(const f32x4*)(Vp + krow * a.ldv + h * 32 + 8 * c);
      const f32x4 v_hi = *(const f32x4*)(Vp + krow * a.ldv + h * 32 + 8 * c + 4);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int d = 8 * c + j;
        const float kv = j < 4 ? k_lo[j] : k_hi[j - 4];
        const float vv = j < 4 ? v_lo[j] : v_hi[j - 4];
        Ks[kk * FA_KLD + (d & 3) * 8 + (d >> 2)] = kv;
        Vt[(kk >> 2) * 128 + d * 4 + (kk & 3)] = vv;
      }
    }
    __syncthreads();
    float x[4][4];
    float cm = -INFINITY;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const f32x4 ka = *(const f32x4*)(Ks + (16 * j + r16) * FA_KLD + g * 8);
      const f32x4 kb = *(const f32x4*)(Ks + (16 * j + r16) * FA_KLD + g * 8 + 4);
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ka[s], qf[s], acc, 0, 0, 0);
#pragma unroll
      for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(kb[s], qf[4 + s], acc, 0, 0, 0);
      const int key0 = k0 + 16 * j + 4 * g;
      int kx[4] = {0, 0, 0, 0};
      if (bias) {
        const int4 t4 = *(const int4*)(Kx + key0);
        kx[0] = t4.x; kx[1] = t4.y; kx[2] = t4.z; kx[3] = t4.w;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = acc[r] * a.scale;
        if (bias) v += qv ? Bs[qbase - kx[r]] : 0.f;
        x[j][r] = key0 + r < L ? v : -INFINITY;
        cm = fmaxf(cm, x[j][r]);
      }
    }
    cm = fmaxf(cm, __shfl_xor(cm, 16, 64));
    cm = fmaxf(cm, __shfl_xor(cm, 32, 64));
    const float mn = fmaxf(m, cm);
    const float corr = expf(m - mn);   // m = -inf on the first chunk -> 0
    l *= corr;
#pragma unroll
    for (int r = 0; r < 4; ++r) { o[0][r] *= corr; o[1][r] *= corr; }
    m = mn;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float p[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        p[r] = expf(x[j][r] - mn);
        l += p[r];
      }
#pragma unroll
      for (int db = 0; db < 2; ++db) {
        const f32x4 vf = *(const f32x4*)(Vt + (4 * j + g) * 128 + (db * 16 + r16) * 4);
#pragma unroll
        for (int s = 0; s < 4; ++s) o[db] = __builtin_amdgcn_mfma_f32_16x16x4f32(vf[s], p[s], o[db], 0, 0, 0);
      }
    }
  }
  l += __shfl_xor(l, 16, 64);
  l += __shfl_xor(l, 32, 64);
  if (!qv) return;
  float* O = (float*)a.o + qrow * a.ldo + h * 32;
#pragma unroll
  for (int db = 0; db < 2; ++db)
    *(f32x4*)(O + db * 16 + 4 * g) = f32x4{o[db][0] / l, o[db][1] / l, o[db][2] / l, o[db][3] / l};
}

// The same attention on the 16-bit matrix pipe with split-fp16 operands (precise 'split' mode,
// round 6): q, k, v (f32) become fp16 (hi, lo) pairs, the probabilities too, and every product is the
// x3 sum hi.hi + hi.lo + lo.hi of v_mfma_f32_16x16x32_f16 (~22-bit operands, f32 accumulation) --
// 6 MFMAs of 16 cycles per 16 queries x 32 keys against 16 of 32 cycles on the f32 pipe.  Layouts
// follow the f32 kernel: S^T = K Q^T (a lane holds keys 16 j + 4 g + r of query lane & 15); for PV
// the k-slots of lane group g in key pair P are keys 32 P + 16 (i >> 2) + 4 g + (i & 3), i = 0..7,
// exactly the probabilities the lane holds, so V^T is staged in that key order.  Outputs: O as the
// fp16 pair of the x3 to_out GEMM (oh, ol), O in bf16 and the natural-log LSE (the bf16 backward's
// operands: it recomputes P from its bf16 q / k against this LSE).  The probabilities go through
// v_exp_f32 on log2-unit scores (scale log2 e folded into the score multiply, the bias table scaled
// at staging), not libm expf: ~1 ulp, and the kernel's VALU work per score roughly halves (round 6).
constexpr float X3_LOG2E = 1.4426950408889634f, X3_LN2 = 0.6931471805599453f;
constexpr int X3_KLD = 40;            // K image row: 32 d + 8 pad (fp16)
constexpr int X3_VLD = 72;            // V^T image row: 64 keys + 8 pad (fp16)

__device__ __forceinline__ void split2h(float x, _Float16& h, _Float16& l) {
  h = (_Float16)x;
  l = (_Float16)(x - (float)h);
}

__global__ __launch_bounds__(256) void attn_x3_fwd_kernel(ctclip_attn_args a, u16* __restrict__ oh,
                                                          u16* __restrict__ ol, u16* __restrict__ ob,
                                                          float* __restrict__ lse) {
  __shared__ __attribute__((aligned(16))) _Float16 Kh[64 * X3_KLD], Kl[64 * X3_KLD];
  __shared__ __attribute__((aligned(16))) _Float16 Vh[32 * X3_VLD], Vl[32 * X3_VLD];
  __shared__ float Bs[FA_MAXNB];
  __shared__ __attribute__((aligned(16))) int Kx[FA_MAXL + 64];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r16 = lane & 15, g = lane >> 4;
  const int h = blockIdx.y;
  const int64_t sq = blockIdx.z;
  const int L = a.L;
  const int64_t rbase = (sq / a.n_inner) * a.s_outer + (sq % a.n_inner) * a.s_inner;
  const float* Q = (const float*)a.q;
  const float* Kp = (const float*)a.k;
  const float* Vp = (const float*)a.v;
  const bool bias = a.bias_u != nullptr;
  const int Wg = bias ? a.grid_w : 1;
  const int nb = bias ? (2 * a.grid_h - 1) * (2 * Wg - 1) : 0;
  if (bias) {
    // (log2 units: the scores go through v_exp_f32 directly, round 6)
    for (int i = tid; i < nb; i += 256) Bs[i] = a.bias_u[(int64_t)h * nb + i] * X3_LOG2E;
    for (int i = tid; i < L + 64; i += 256) Kx[i] = i < L ? (i / Wg) * (2 * Wg - 1) + i % Wg : 0;
  }
  const int qi = blockIdx.x * 64 + w * 16 + r16;
  const bool qv = qi < L;
  const int64_t qrow = rbase + (int64_t)min(qi, L - 1) * a.s_pos;
  // B operand of S^T: query lane & 15, head dims 8 g .. 8 g + 7 as an fp16 pair
  f16x8 qh, ql;
  {
    const float* qp = Q + qrow * a.ldq + h * 32 + 8 * g;
    const f32x4 q0 = *(const f32x4*)qp, q1 = *(const f32x4*)(qp + 4);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      _Float16 hh, ll;
      split2h(qv ? (e < 4 ? q0[e] : q1[e - 4]) : 0.f, hh, ll);
      qh[e] = hh;
      ql[e] = ll;
    }
  }
  int qbase = 0;
  if (bias) qbase = (qi / Wg + a.grid_h - 1) * (2 * Wg - 1) + qi % Wg + Wg - 1;
  const float sc2 = a.scale * X3_LOG2E;
  float m = -INFINITY, l = 0.f;
  f32x4 o[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  const int kk = tid >> 2, c = tid & 3;   // staging: key kk of the chunk, head dims 8 c .. 8 c + 7
  // the key's position in the V^T image: pair P = kk >> 5, lane group gk = (kk >> 2) & 3, slot
  // i = 4 ((kk >> 4) & 1) + (kk & 3) (see above)
  const int vpos = (kk >> 5) * 32 + ((kk >> 2) & 3) * 8 + 4 * ((kk >> 4) & 1) + (kk & 3);
  // this thread's K / V slice of a chunk, loaded one chunk ahead (registers) so the global load
  // latency hides behind the previous chunk's MFMAs
  f32x4 k_lo, k_hi, v_lo, v_hi;
  auto fetch = [&](int c0) {
    const int64_t krow = rbase + (int64_t)min(c0 + kk, L - 1) * a.s_pos;
    k_lo = *(const f32x4*)(Kp + krow * a.ldk + h * 32 + 8 * c);
    k_hi = *(const f32x4*)(Kp + krow * a.ldk + h * 32 + 8 * c + 4);
    v_lo = *(const f32x4*)(Vp + krow * a.ldv + h * 32 + 8 * c);
    v_hi = *(const f32x4*)(Vp + krow * a.ldv + h * 32 + 8 * c + 4);
  };
  fetch(0);
  for (int k0 = 0; k0 < L; k0 += 64) {
    __syncthreads();
    {
      f16x8 kh8, kl8;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        _Float16 hh, ll;
        split2h(j < 4 ? k_lo[j] : k_hi[j - 4], hh, ll);
        kh8[j] = hh;
        kl8[j] = ll;
        split2h(j < 4 ? v_lo[j] : v_hi[j - 4], hh, ll);
        Vh[(8 * c + j) * X3_VLD + vpos] = hh;
        Vl[(8 * c + j) * X3_VLD + vpos] = ll;
      }
      *(f16x8*)(Kh + kk * X3_KLD + 8 * c) = kh8;
      *(f16x8*)(Kl + kk * X3_KLD + 8 * c) = kl8;
    }
    if (k0 + 64 < L) fetch(k0 + 64);
    __syncthreads();
    float x[4][4];
    float cm = -INFINITY;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const f16x8 kah = *(const f16x8*)(Kh + (16 * j + r16) * X3_KLD + 8 * g);
      const f16x8 kal = *(const f16x8*)(Kl + (16 * j + r16) * X3_KLD + 8 * g);
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(kah, qh, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(kah, ql, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(kal, qh, acc, 0, 0, 0);
      const int key0 = k0 + 16 * j + 4 * g;
      int kx[4] = {0, 0, 0, 0};
      if (bias) {
        const int4 t4 = *(const int4*)(Kx + key0);
        kx[0] = t4.x; kx[1] = t4.y; kx[2] = t4.z; kx[3] = t4.w;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = acc[r] * sc2;
        if (bias) v += qv ? Bs[qbase - kx[r]] : 0.f;
        x[j][r] = key0 + r < L ? v : -INFINITY;
        cm = fmaxf(cm, x[j][r]);
      }
    }
    cm = fmaxf(cm, __shfl_xor(cm, 16, 64));
    cm = fmaxf(cm, __shfl_xor(cm, 32, 64));
    const float mn = fmaxf(m, cm);
    const float corr = __builtin_amdgcn_exp2f(m - mn);   // m = -inf on the first chunk -> 0
    l *= corr;
#pragma unroll
    for (int r = 0; r < 4; ++r) { o[0][r] *= corr; o[1][r] *= corr; }
    m = mn;
#pragma unroll
    for (int P = 0; P < 2; ++P) {
      f16x8 ph, pl;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float pv = __builtin_amdgcn_exp2f(x[2 * P + (i >> 2)][i & 3] - mn);
        l += pv;
        _Float16 hh, ll;
        split2h(pv, hh, ll);
        ph[i] = hh;
        pl[i] = ll;
      }
#pragma unroll
      for (int db = 0; db < 2; ++db) {
        const int vo = (db * 16 + r16) * X3_VLD + P * 32 + g * 8;
        const f16x8 vh = *(const f16x8*)(Vh + vo), vl = *(const f16x8*)(Vl + vo);
        o[db] = __builtin_amdgcn_mfma_f32_16x16x32_f16(vh, ph, o[db], 0, 0, 0);
        o[db] = __builtin_amdgcn_mfma_f32_16x16x32_f16(vh, pl, o[db], 0, 0, 0);
        o[db] = __builtin_amdgcn_mfma_f32_16x16x32_f16(vl, ph, o[db], 0, 0, 0);
      }
    }
  }
  l += __shfl_xor(l, 16, 64);
  l += __shfl_xor(l, 32, 64);
  if (!qv) return;
  // lane: query qi, head dims 16 db + 4 g + [0, 4)
  const int64_t ro = qrow * a.ldo + h * 32 + 4 * g;
#pragma unroll
  for (int db = 0; db < 2; ++db) {
    float ov[4], hv[4], lv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      ov[r] = o[db][r] / l;
      hv[r] = rh(ov[r]);
      lv[r] = ov[r] - hv[r];
    }
    *(uint2*)(oh + ro + 16 * db) = pack4h(hv);
    *(uint2*)(ol + ro + 16 * db) = pack4h(lv);
    if (ob) *(uint2*)(ob + ro + 16 * db) = pack4(ov);
  }
  if (g == 0 && lse) lse[(int64_t)h * a.M + qrow] = (m + log2f(l)) * X3_LN2;   // natural log
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
  const bool quad = P % 4 == 0 && W % 4 == 0 && ldo % 4 == 0 && aligned16(out) && aligned16(gamma) &&
                    aligned16(beta) && ((uintptr_t)video & (is_f32 ? 15 : 7)) == 0;
  if (quad) {
    hipLaunchKernelGGL(patch_ln_f32_q_kernel, dim3((unsigned)cdiv(ntok, 4)), dim3(256), 0, (hipStream_t)stream, video,
                       is_f32, is_hu, ntok, T, Hg, Wg, (int64_t)C * F * H * W, (int64_t)H * W, W, PT, P, offs, pd, eps,
                       gamma, beta, out, ldo);
    CT_CHECK_LAUNCH();
    return 0;
  }
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
  CT_REQUIRE(D / 4 <= 256 && aligned16(weight), CT_EALIGN);
  const int64_t per_block = (int64_t)(256 / (D / 4)) * PEG_NT;
  hipLaunchKernelGGL(peg_f32_kernel, dim3((unsigned)cdiv(ntok, per_block)), dim3(256), 0, (hipStream_t)stream, x,
                     ntok, D, weight, bias, T, H, W, mode, out);
  CT_CHECK_LAUNCH();
  return 0;
}

extern "C" int ctclip_l2norm_scale_fwd_f32(const float* x, int64_t ldx, int64_t rows, int32_t H, int32_t D,
                                           const float* scale, float* y, int64_t ldy, void* stream) {
  return ctclip_l2norm_scale_fwd_f32b(x, ldx, rows, H, D, scale, y, ldy, nullptr, 0, stream);
}

extern "C" int ctclip_l2norm_scale_fwd_f32b(const float* x, int64_t ldx, int64_t rows, int32_t H, int32_t D,
                                            const float* scale, float* y, int64_t ldy, void* y_bf16, int64_t ldyb,
                                            void* stream) {
  if (rows == 0) return 0;
  const bool vec = (D == 32 || D == 64) && aligned16(x) && aligned16(y) && aligned16(scale) && ldx % 4 == 0 &&
                   ldy % 4 == 0;
  if (y_bf16) CT_REQUIRE(vec && ((uintptr_t)y_bf16 & 7) == 0 && ldyb % 4 == 0, CT_EALIGN);
  if (vec) {
    const int G = D / 4;
    const unsigned nb = (unsigned)cdiv(rows * H, 256 / G);
    if (G == 8)
      hipLaunchKernelGGL(l2norm_f32_vec_kernel<8>, dim3(nb), dim3(256), 0, (hipStream_t)stream, x, ldx, rows, H, scale,
                         y, ldy, (u16*)y_bf16, ldyb);
    else
      hipLaunchKernelGGL(l2norm_f32_vec_kernel<16>, dim3(nb), dim3(256), 0, (hipStream_t)stream, x, ldx, rows, H,
                         scale, y, ldy, (u16*)y_bf16, ldyb);
    CT_CHECK_LAUNCH();
    return 0;
  }
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
  static const bool valu = [] { const char* e = getenv("CTCLIP_F32_ATTN_VALU"); return e && e[0] == '1'; }();
  const bool mfma_ok = a->D == 32 && (!a->bias_u || ((2 * a->grid_h - 1) * (2 * a->grid_w - 1) <= FA_MAXNB &&
                                                     a->L <= FA_MAXL));
  if (mfma_ok && !valu) {
    CT_REQUIRE(aligned16(a->k) && aligned16(a->v) && aligned16(a->o) && a->ldk % 4 == 0 && a->ldv % 4 == 0 &&
                   a->ldo % 4 == 0, CT_EALIGN);
    hipLaunchKernelGGL(attn_f32_mfma_kernel, grid, dim3(256), 0, (hipStream_t)stream, *a);
  } else if (a->D == 32)
    hipLaunchKernelGGL(attn_f32_kernel<32>, grid, dim3(64), 0, (hipStream_t)stream, *a);
  else if (a->D == 64)
    hipLaunchKernelGGL(attn_f32_kernel<64>, grid, dim3(64), 0, (hipStream_t)stream, *a);
  else
    return CT_ESHAPE;
  CT_CHECK_LAUNCH();
  return 0;
}

// split-fp16 x3 attention forward (precise 'split' mode, round 6): q, k, v f32 in `a` (D = 32, as
// ctclip_attn_fwd_f32's MFMA kernel); O written as an fp16 pair (oh, ol; ldo) + optional bf16 copy ob,
// optional natural-log lse [H][M].
extern "C" int ctclip_attn_fwd_x3(const ctclip_attn_args* a, void* oh, void* ol, void* ob, float* lse, void* stream) {
  CT_REQUIRE(a && a->q && a->k && a->v && oh && ol && a->L > 0 && a->nseq >= 0 && a->n_inner > 0, CT_EINVAL);
  CT_REQUIRE(a->D == 32 && !a->kmask && a->dropout_p == 0.f, CT_EINVAL);
  if (a->bias_u)
    CT_REQUIRE(a->grid_h > 0 && a->grid_w > 0 && a->grid_h * a->grid_w == a->L &&
                   (2 * a->grid_h - 1) * (2 * a->grid_w - 1) <= FA_MAXNB && a->L <= FA_MAXL,
               CT_ESHAPE);
  CT_REQUIRE(aligned16(a->q) && aligned16(a->k) && aligned16(a->v) && a->ldq % 4 == 0 && a->ldk % 4 == 0 &&
                 a->ldv % 4 == 0 && ((uintptr_t)oh & 7) == 0 && ((uintptr_t)ol & 7) == 0 &&
                 ((uintptr_t)ob & 7) == 0 && a->ldo % 4 == 0,
             CT_EALIGN);
  if (a->nseq == 0) return 0;
  dim3 grid((unsigned)cdiv(a->L, 64), (unsigned)a->H, (unsigned)a->nseq);
  hipLaunchKernelGGL(attn_x3_fwd_kernel, grid, dim3(256), 0, (hipStream_t)stream, *a, (u16*)oh, (u16*)ol, (u16*)ob,
                     lse);
  CT_CHECK_LAUNCH();
  return 0;
}
