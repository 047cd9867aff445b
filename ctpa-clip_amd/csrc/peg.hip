// PEG: depthwise 3x3x3 Conv3d with causal temporal padding, residual fused.
// ct_clip/attention.py:56-84 (PEG, causal=True via ctvit.py:183) and the residual at
// attention.py:324.  Tokens live in the canonical (b, t, h, w) row order everywhere; the conv
// runs in the reference's *view* coordinates:
//   mode 0 (spatial transformer): view == canonical.
//   mode 1 (temporal transformer): the reference holds x as '(b h w) t d' and raw-reshapes it
//     to (b, t, h, w, d) (attention.py:69-70), so view position p (within a batch) is the
//     reference's physical row p = (h*W + w)*T + t  ->  canonical row t*H*W + h*W + w.
//   Both index maps are integer-exact; tests/test_gpu_ops.py checks them against the oracle.
// out(v) = x(v) + bias + sum_{kt,kh,kw} w[c][kt][kh][kw] * x(v + (kt-2, kh-1, kw-1)), zero outside.
#include <type_traits>

#include "common.h"
#include "../../include/ctclip_hip.h"

namespace {

struct Geo {
  int T, H, W;
  int thw;
  int mode;
};

// token rows fit in 32 bits (B*T*H*W < 2^31); only the final row*D product is 64-bit
__device__ __forceinline__ int canon(const Geo& g, int b, int p) {
  if (g.mode == 0) return b * g.thw + p;
  const int hw = p / g.T, t = p - hw * g.T;
  return b * g.thw + t * (g.H * g.W) + hw;
}

// forward (transpose = 0) or input-gradient (transpose = 1) of the depthwise conv
template <int TRANSPOSE>
__global__ __launch_bounds__(256) void peg_kernel(const u16* __restrict__ xin, int64_t ntok, int D,
                                                  const float* __restrict__ w, const float* __restrict__ bias,
                                                  const float* __restrict__ res, Geo g, float* __restrict__ out,
                                                  u16* __restrict__ outb) {
  __shared__ float ws[27][64];
  __shared__ float bs[64];
  const int c0 = blockIdx.y * 64;
  for (int i = threadIdx.x; i < 27 * 64; i += 256) {
    const int c = i / 27, tap = i - c * 27;
    ws[tap][c] = (c0 + c < D) ? w[(int64_t)(c0 + c) * 27 + tap] : 0.f;
  }
  if (threadIdx.x < 64) bs[threadIdx.x] = (bias && c0 + threadIdx.x < D) ? bias[c0 + threadIdx.x] : 0.f;
  __syncthreads();
  const int ch = threadIdx.x & 7;
  const int v = blockIdx.x * 32 + (threadIdx.x >> 3);
  if (v >= ntok) return;
  const int col = c0 + ch * 8;
  if (col >= D) return;
  const int b = v / g.thw;
  const int p = v - b * g.thw;
  const int hwq = p / g.W;
  const int wq = p - hwq * g.W;
  const int tq = hwq / g.H;
  const int hq = hwq - tq * g.H;
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = TRANSPOSE ? 0.f : bs[ch * 8 + j];
#pragma unroll
  for (int kt = 0; kt < 3; ++kt) {
    const int tt = TRANSPOSE ? tq + 2 - kt : tq + kt - 2;
    if (tt < 0 || tt >= g.T) continue;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const int hh = TRANSPOSE ? hq + 1 - kh : hq + kh - 1;
      if (hh < 0 || hh >= g.H) continue;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int ww = TRANSPOSE ? wq + 1 - kw : wq + kw - 1;
        if (ww < 0 || ww >= g.W) continue;
        const int pn = (tt * g.H + hh) * g.W + ww;
        float xv[8];
        unpack8(*(const u32x4*)(xin + (int64_t)canon(g, b, pn) * D + col), xv);
        const int tap = (kt * 3 + kh) * 3 + kw;
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += ws[tap][ch * 8 + j] * xv[j];
      }
    }
  }
  const int64_t co = (int64_t)canon(g, b, p) * D + col;
  if (res) {
    const f32x4 a = *(const f32x4*)(res + co), bb = *(const f32x4*)(res + co + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) { acc[j] += a[j]; acc[4 + j] += bb[j]; }
  }
  if (out) {
    *(f32x4*)(out + co) = f32x4{acc[0], acc[1], acc[2], acc[3]};
    *(f32x4*)(out + co + 4) = f32x4{acc[4], acc[5], acc[6], acc[7]};
  }
  if (outb) *(u32x4*)(outb + co) = pack8(acc);
}

// weight / bias gradient partials: part[blk][c][28] (27 taps + bias)
// thread = (kt in 0..2, chunk in 0..7, token lane in 0..7) : 192 threads
__global__ __launch_bounds__(192) void peg_wgrad_kernel(const u16* __restrict__ dout, const u16* __restrict__ xin,
                                                        int64_t ntok, int D, Geo g, int64_t tok_per_blk,
                                                        float* __restrict__ part) {
  __shared__ float red[3][8][10][8];  // [kt][chunk][9 taps + bias][8 ch]
  const int tl = threadIdx.x & 7, ch = (threadIdx.x >> 3) & 7, kt = threadIdx.x >> 6;
  const int c0 = blockIdx.y * 64;
  const int col = c0 + ch * 8;
  float acc[9][8], accb[8];
#pragma unroll
  for (int i = 0; i < 9; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) accb[j] = 0.f;
  const int v0 = blockIdx.x * (int)tok_per_blk;
  const int v1 = min((int)ntok, v0 + (int)tok_per_blk);
  if (col < D) {
    for (int v = v0 + tl; v < v1; v += 8) {
      const int b = v / g.thw;
      const int p = v - b * g.thw;
      const int hwq = p / g.W;
      const int wq = p - hwq * g.W;
      const int tq = hwq / g.H;
      const int hq = hwq - tq * g.H;
      float dv[8];
      unpack8(*(const u32x4*)(dout + (int64_t)canon(g, b, p) * D + col), dv);
      if (kt == 0) {
#pragma unroll
        for (int j = 0; j < 8; ++j) accb[j] += dv[j];
      }
      const int tt = tq + kt - 2;
      if (tt < 0 || tt >= g.T) continue;
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        const int hh = hq + kh - 1;
        if (hh < 0 || hh >= g.H) continue;
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
          const int ww = wq + kw - 1;
          if (ww < 0 || ww >= g.W) continue;
          const int pn = (tt * g.H + hh) * g.W + ww;
          float xv[8];
          unpack8(*(const u32x4*)(xin + (int64_t)canon(g, b, pn) * D + col), xv);
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[kh * 3 + kw][j] += dv[j] * xv[j];
        }
      }
    }
  }
  // fold the 8 token lanes (lane bits 0..2) with shuffles, then one LDS slot per (kt, chunk)
#pragma unroll
  for (int i = 0; i < 9; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float v = acc[i][j];
      v += __shfl_xor(v, 1, 64);
      v += __shfl_xor(v, 2, 64);
      v += __shfl_xor(v, 4, 64);
      if (tl == 0) red[kt][ch][i][j] = v;
    }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float v = accb[j];
    v += __shfl_xor(v, 1, 64);
    v += __shfl_xor(v, 2, 64);
    v += __shfl_xor(v, 4, 64);
    if (tl == 0) red[kt][ch][9][j] = v;
  }
  __syncthreads();
  // 64 channels x 28 outputs = 1792 values; 192 threads
  for (int o = threadIdx.x; o < 64 * 28; o += 192) {
    const int c = o / 28, k = o - c * 28;
    if (c0 + c >= D) continue;
    const int chh = c >> 3, j = c & 7;
    const float s = k < 27 ? red[k / 9][chh][k % 9][j] : red[0][chh][9][j];
    part[((int64_t)blockIdx.x * D + c0 + c) * 28 + k] = s;
  }
}

// ---------------------------------------------------------------------------------------------
// Plane-streaming kernels (the fast path).  A workgroup owns HT view rows x all W columns x 64
// channels of one batch element and walks the view-time axis.  Input planes (HT+2 rows with
// the h halo, W+2 columns with zero padding, 64 channels, bf16) stream through a 4-slot LDS ring:
// each input byte is fetched from L2/HBM ~(HT+2)/HT times instead of 27, and every output is
// computed from LDS.  A thread covers SEG consecutive w positions of one 8-channel chunk and
// slides a (SEG+2)-wide window along w, so each (kt, kh) costs SEG+2 window reads + 3 weight
// reads for SEG outputs.  The ring slot written in step t is (t+lead+1)&3, never one of the
// three read in step t, so one barrier per step suffices.
// W <= 24 (one item per thread); 3 ring slots + weights = 47 KB -> 3 workgroups per CU, so the
// base grid (8 x 12 x 8 = 768 workgroups) is resident in one round
#ifndef CTCLIP_PEG_SEG
#define CTCLIP_PEG_SEG 3
#endif
// SEG w positions per conv thread; TNTH = one (row, segment, chunk) item per thread on the 24-wide
// grid; PLANE_CH = 16-B chunks a plane (HT + 2 rows x W + 2 columns x 8 chunks) may hold
constexpr int HT = 2, SEG = CTCLIP_PEG_SEG, SEGW = 6, TNTH = HT * ((24 + SEG - 1) / SEG) * 8, WNTH = 256,
              PLANE_CH = 1024, NSLOT = 3;
template <int NT> constexpr int nld() { return (PLANE_CH + NT - 1) / NT; }   // plane loads per thread

__host__ __device__ inline int plane_bytes(int W) { return (HT + 2) * (W + 2) * 128; }

// issue this thread's loads of plane tp (view coordinates) into registers.  The loads are
// unconditional (out-of-plane / padding slots re-read the tensor's first chunk) and the zero
// padding is applied in plane_store from the returned bit mask: a conditional load (value or
// zero) makes the compiler merge the two with register copies right after the load, i.e. an
// immediate s_waitcnt vmcnt(0) that serialises the prefetch with the step it should overlap.
// BF = false keeps conditional loads (zero in the register, mask all ones): the weight-gradient
// kernel, whose register budget (3 workgroups per CU) the branch-free form overflows (measured
// 107 -> 126 us there, while the conv kernels gain 174 -> 156 us)
template <int NT, bool BF = true>
__device__ __forceinline__ unsigned plane_load(const u16* __restrict__ x, const Geo& g, int D, int b, int h0, int c0,
                                               int tp, u32x4 (&reg)[nld<NT>()], int hoff = 1) {
  const int nl = (HT + 2) * (g.W + 2) * 8;
  unsigned valid = BF ? 0u : ~0u;
#pragma unroll
  for (int m = 0; m < nld<NT>(); ++m) {
    const int i = threadIdx.x + m * NT;
    const int k = i & 7, cw = (i >> 3) % (g.W + 2), hr = (i >> 3) / (g.W + 2);
    const int h = h0 - hoff + hr, w = cw - 1;
    const bool ok = i < nl && h >= 0 && h < g.H && w >= 0 && w < g.W;
    if constexpr (BF) {
      const int64_t row = ok ? (int64_t)canon(g, b, (tp * g.H + h) * g.W + w) : 0;
      reg[m] = *(const u32x4*)(x + row * D + c0 + k * 8);
      valid |= (unsigned)ok << m;
    } else {
      reg[m] = u32x4{0u, 0u, 0u, 0u};
      if (ok) reg[m] = *(const u32x4*)(x + (int64_t)canon(g, b, (tp * g.H + h) * g.W + w) * D + c0 + k * 8);
    }
  }
  return valid;
}

template <int NT>
__device__ __forceinline__ void plane_store(char* ring, int W, int tp, const u32x4 (&reg)[nld<NT>()],
                                            unsigned valid) {
  const int nl = (HT + 2) * (W + 2) * 8;
  char* dst = ring + (tp % NSLOT) * plane_bytes(W);
#pragma unroll
  for (int m = 0; m < nld<NT>(); ++m) {
    const int i = threadIdx.x + m * NT;
    if (i < nl) *(u32x4*)(dst + i * 16) = ((valid >> m) & 1) ? reg[m] : u32x4{0u, 0u, 0u, 0u};
  }
}

// forward (TR = 0) or input-gradient (TR = 1); grid (B * ceil(H/HT), D/64), TNTH threads
// GK > 0: the geometry is the compile-time cube T = H = W = GK with index map MD (the 3D-ViT's
// 24^3 token grid in both transformers), so every division of the plane / row index maps is by
// a constant (the runtime form spends most of its issue slots on integer divisions)
// MD = 2: the temporal transformer's raw-reshape view (mode 1) on a cube T = H = W, walked in
// CANONICAL order.  For T = H = W the view is a pure axis permutation of the canonical (t, h, w)
// rows -- view (t_v, h_v, w_v) = (h, w, t) (attention.py:69-70: flat f = (h W + w) T + t =
// (t_v H + h_v) W + w_v) -- so the view's conv is a canonical-space conv with the causal offsets
// {-2, -1, 0} on canonical h, {-1, 0, 1} on canonical t and w, and tap (kt, kh, kw) of the view
// applied at canonical offset (dt, dh, dw) = (kw - 1, kt - 2, kh - 1).  Walking canonical t with
// planes of canonical (h, w) rows makes every plane a contiguous run of rows (the view walk gathered
// rows 576 apart: 217 vs 159 us per forward launch, r03).  Same outputs up to f32 summation order.
template <int GK, int MD>
__device__ __forceinline__ void fix_geo(Geo& g) {
  if constexpr (GK > 0) {
    g.T = GK;
    g.H = GK;
    g.W = GK;
    g.thw = GK * GK * GK;
    g.mode = MD == 2 ? 0 : MD;    // MD 2 addresses rows canonically
  }
}

// loop index (a = walk plane, b = plane row, c = plane column) -> offsets and the tap they use; TR =
// the transposed conv (input gradient): every offset negated
template <int MD, int TR>
struct Taps {
  static constexpr int dt(int a) { return MD == 2 ? (TR ? 1 - a : a - 1) : (TR ? 2 - a : a - 2); }
  static constexpr int dh(int b) { return MD == 2 ? (TR ? 2 - b : b - 2) : (TR ? 1 - b : b - 1); }
  static constexpr int tap(int a, int b, int c) { return MD == 2 ? (b * 3 + c) * 3 + a : (a * 3 + b) * 3 + c; }
  static constexpr int hoff = MD == 2 ? (TR ? 0 : 2) : 1;   // plane row 0 = h0 - hoff
  static constexpr int lead = MD == 2 ? 1 : (TR ? 2 : 0);    // planes needed ahead of t
};

template <int TR, int GK = 0, int MD = 0>
__global__ __launch_bounds__(TNTH) void peg_tile_kernel(const u16* __restrict__ xin, int D,
                                                        const float* __restrict__ w, const float* __restrict__ bias,
                                                        const float* __restrict__ res, Geo g,
                                                        float* __restrict__ out, u16* __restrict__ outb,
                                                        float* __restrict__ stats) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  fix_geo<GK, MD>(g);
  const int nht = (g.H + HT - 1) / HT;
  const int b = blockIdx.x / nht, h0 = (blockIdx.x - b * nht) * HT, c0 = blockIdx.y * 64;
  const int pb = plane_bytes(g.W);
  char* ring = smem;
  float* ws = (float*)(smem + NSLOT * pb);   // [27][64]
  float* bs = ws + 27 * 64;
  for (int i = threadIdx.x; i < 27 * 64; i += TNTH) {
    const int c = i / 27, tap = i - c * 27;
    ws[tap * 64 + c] = w[(int64_t)(c0 + c) * 27 + tap];
  }
  if (threadIdx.x < 64) bs[threadIdx.x] = bias ? bias[c0 + threadIdx.x] : 0.f;
  using TP = Taps<MD, TR>;
  constexpr int lead = TP::lead, hoff = TP::hoff;
  u32x4 reg[nld<TNTH>()];
  unsigned rvalid = 0;
  for (int tp = 0; tp <= lead && tp < g.T; ++tp) {
    rvalid = plane_load<TNTH>(xin, g, D, b, h0, c0, tp, reg, hoff);
    plane_store<TNTH>(ring, g.W, tp, reg, rvalid);
  }
  __syncthreads();
  // one (row, w-segment, chunk) item per thread (tiled_ok: HT * ceil(W/SEG) * 8 <= TNTH)
  const int ns = (g.W + SEG - 1) / SEG;
  const int o = threadIdx.x;
  const int ch = o & 7, s = (o >> 3) % ns, r = (o >> 3) / ns;
  const int h = h0 + r, w0 = s * SEG;
  const bool active = o < HT * ns * 8 && h < g.H;
  // residual rows of this thread's outputs, prefetched one step ahead with the plane
  // (unconditional loads as in plane_load; rows without a residual read w[0..7] and are masked)
  auto res_load = [&](int t, f32x4 (&rv)[SEG][2]) {
#pragma unroll
    for (int j = 0; j < SEG; ++j) {
      const bool ok = res && active && w0 + j < g.W;
      const float* p = ok ? res + (int64_t)canon(g, b, (t * g.H + h) * g.W + w0 + j) * D + c0 + ch * 8 : w;
      rv[j][0] = *(const f32x4*)p;
      rv[j][1] = *(const f32x4*)(p + 4);
    }
  };
  const bool has_res = res != nullptr;
  f32x4 rv[SEG][2];
  res_load(0, rv);
  for (int t = 0; t < g.T; ++t) {
    const int tn = t + lead + 1;
    // always issued (the last steps re-read plane T-1, never stored) so no branch merges `reg`
    const unsigned nvalid = plane_load<TNTH>(xin, g, D, b, h0, c0, min(tn, g.T - 1), reg, hoff);
    f32x4 rn[SEG][2];
    res_load(min(t + 1, g.T - 1), rn);
    if (active) {
      float acc[SEG][8];
#pragma unroll
      for (int j = 0; j < SEG; ++j)
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[j][e] = TR ? 0.f : bs[ch * 8 + e];
      // rolled (kt, kh) loops: one (SEG+2) x 8 window live at a time (unrolled, hipcc hoists all
      // nine windows and the kernel runs at 1 wave/SIMD)
#pragma unroll 1
      for (int kt = 0; kt < 3; ++kt) {           // (a, b, c) = (kt, kh, kw) loop indices, see Taps
        const int tp = t + TP::dt(kt);
        if (tp < 0 || tp >= g.T) continue;
        const char* pl = ring + (tp % NSLOT) * pb;
#pragma unroll 1
        for (int kh = 0; kh < 3; ++kh) {
          const int lr = r + TP::dh(kh) + hoff;
          float xv[SEG + 2][8];
#pragma unroll
          for (int q = 0; q < SEG + 2; ++q) {
            // LDS column of w0 - 1 + q; columns past W + 1 only feed outputs w >= W
            const int cw = min(w0 + q, g.W + 1);
            unpack8(*(const u32x4*)(pl + ((lr * (g.W + 2) + cw) * 8 + ch) * 16), xv[q]);
          }
#pragma unroll
          for (int kw = 0; kw < 3; ++kw) {
            const float* wp = ws + TP::tap(kt, kh, kw) * 64 + ch * 8;
            const f32x4 wa = *(const f32x4*)wp, wb = *(const f32x4*)(wp + 4);
            const float wv[8] = {wa[0], wa[1], wa[2], wa[3], wb[0], wb[1], wb[2], wb[3]};
#pragma unroll
            for (int j = 0; j < SEG; ++j) {
              const int q = TR ? j + 2 - kw : j + kw;
#pragma unroll
              for (int e = 0; e < 8; ++e) acc[j][e] += wv[e] * xv[q][e];
            }
          }
        }
      }
#pragma unroll
      for (int j = 0; j < SEG; ++j) {
        const int wq = w0 + j;
        if (wq >= g.W) break;
        const int64_t orow = canon(g, b, (t * g.H + h) * g.W + wq);
        const int64_t co = orow * D + c0 + ch * 8;
        if (has_res) {
#pragma unroll
          for (int e = 0; e < 4; ++e) { acc[j][e] += rv[j][0][e]; acc[j][4 + e] += rv[j][1][e]; }
        }
        if (out) {
          *(f32x4*)(out + co) = f32x4{acc[j][0], acc[j][1], acc[j][2], acc[j][3]};
          *(f32x4*)(out + co + 4) = f32x4{acc[j][4], acc[j][5], acc[j][6], acc[j][7]};
        }
        if (outb) *(u32x4*)(outb + co) = pack8(acc[j]);
        if (!TR && stats) {
          // the output row's (mean, M2) over this workgroup's 64 channels (two-pass over the 8 lanes
          // ch = 0..7 of the token, which sit in 8 consecutive lanes), for the LayerNorm that reads
          // this output (attention.py:139-141): ctclip_ln_stats_merge combines the D / 64 groups
          float sm = 0.f;
#pragma unroll
          for (int e = 0; e < 8; ++e) sm += acc[j][e];
          sm += __shfl_xor(sm, 1, 64);
          sm += __shfl_xor(sm, 2, 64);
          sm += __shfl_xor(sm, 4, 64);
          const float mu = sm * (1.f / 64.f);
          float m2 = 0.f;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float d = acc[j][e] - mu;
            m2 = fmaf(d, d, m2);
          }
          m2 += __shfl_xor(m2, 1, 64);
          m2 += __shfl_xor(m2, 2, 64);
          m2 += __shfl_xor(m2, 4, 64);
          if (ch == 0) {
            const int64_t ntok = (int64_t)(gridDim.x / nht) * g.thw;
            *(float2*)(stats + ((int64_t)blockIdx.y * ntok + orow) * 2) = make_float2(mu, m2);
          }
        }
      }
    }
    // the slot of plane tn held plane tn - 3, read in this step: write it after a barrier
    __syncthreads();
    if (tn < g.T) plane_store<TNTH>(ring, g.W, tn, reg, nvalid);
#pragma unroll
    for (int j = 0; j < SEG; ++j) { rv[j][0] = rn[j][0]; rv[j][1] = rn[j][1]; }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------------
// Forward from the f32 residual stream (round 5, the default forward).  The bf16 kernel above
// reads the conv taps from the layer input's bf16 shadow: every PEG output then carries that
// shadow's 2^-9 rounding, ~22 % of the bf16 tower's squared pre-VQ token error
// (tools/vit_precision.py: the 'xb' site alone 4.8e-3 of the 1.0e-2 median).  Here the LDS planes
// hold the f32 tokens, 32 channels per workgroup (128 B per plane position, as the bf16 kernel's 64
// channels), 4 channels per thread, and the residual is the centre tap of the plane (no separate
// residual read: HBM reads per launch 113 + 226 MB -> 226 MB at B = 8).
// Walk: each plane is read from LDS ONCE and scattered into the three outputs it feeds.  A plane p
// along the walk axis contributes tap a (kt) to output t = p + 2 - lead - a, so three rolling
// accumulator sets (t mod 3) collect an output over three steps and output p - lead is complete
// after plane p.  Only one plane is live in LDS (plus the next one landing): a 2-slot ring, one
// barrier per step, and a 4-row tile (halo 1.5x instead of 2x) in 43.5 KB -> 3 workgroups of 256
// threads per CU, the base grid (8 x 6 x 16 = 768 workgroups) resident in one round.
// Outputs: f32, bf16 shadow, optional f16 copy (a 16-bit MFMA A operand) and optional (mean, M2)
// per 32-channel group (D / 32 groups, ctclip_ln_stats_merge).
#ifndef CTCLIP_PEGX_WAVES
#define CTCLIP_PEGX_WAVES 1   // launch-bounds occupancy floor (waves per SIMD): 1 = the compiler's choice
#endif
constexpr int XC = 32;             // channels per workgroup
constexpr int XHT = 4;             // output rows per workgroup
constexpr int XNT = 256;           // threads: XHT x ceil(W / SEG) x 8 chunks of 4 channels
constexpr int XPCH = 1280;         // 16-B chunks a plane may hold: (XHT + 2) x (W + 2) x 8
constexpr int XNLD = XPCH / XNT;   // plane loads per thread
__host__ __device__ inline int xplane_bytes(int W) { return (XHT + 2) * (W + 2) * 128; }

__device__ __forceinline__ unsigned xplane_load(const float* __restrict__ x, const Geo& g, int D, int b, int h0,
                                                int c0, int tp, u32x4 (&reg)[XNLD], int hoff) {
  const int nl = (XHT + 2) * (g.W + 2) * 8;
  unsigned valid = 0u;
#pragma unroll
  for (int m = 0; m < XNLD; ++m) {
    const int i = threadIdx.x + m * XNT;
    const int k = i & 7, cw = (i >> 3) % (g.W + 2), hr = (i >> 3) / (g.W + 2);
    const int h = h0 - hoff + hr, w = cw - 1;
    const bool ok = i < nl && h >= 0 && h < g.H && w >= 0 && w < g.W;
    const int64_t row = ok ? (int64_t)canon(g, b, (tp * g.H + h) * g.W + w) : 0;
    reg[m] = *(const u32x4*)(x + row * D + c0 + k * 4);
    valid |= (unsigned)ok << m;
  }
  return valid;
}

__device__ __forceinline__ void xplane_store(char* dst, int W, const u32x4 (&reg)[XNLD], unsigned valid) {
  const int nl = (XHT + 2) * (W + 2) * 8;
#pragma unroll
  for (int m = 0; m < XNLD; ++m) {
    const int i = threadIdx.x + m * XNT;
    if (i < nl) *(u32x4*)(dst + i * 16) = ((valid >> m) & 1) ? reg[m] : u32x4{0u, 0u, 0u, 0u};
  }
}

// TR = 1: the input gradient dx = dout + conv^T(dout) from the f32 dout (round 5; the bf16 tile kernel
// reads the conv taps from dout's bf16 copy plus the f32 residual).  The transposed conv's offsets
// are the forward's negated: with the view-space walk (MD 0 / 1) output t needs planes t .. t + 2,
// so the walk runs BACKWARD in t (virtual time t' = T - 1 - t), where the offsets are the forward's
// again and no plane is needed ahead; the canonical walk (MD 2: offsets -1 .. 1 on the walk axis)
// keeps its direction and its one plane of lead.  Columns mirror (x[w + 1 - kw] instead of
// x[w - 1 + kw]); rows use the transposed row offsets (Taps<MD, 1>).  No bias, no statistics.
template <int GK = 0, int MD = 0, int TR = 0>
__global__ __launch_bounds__(XNT, CTCLIP_PEGX_WAVES) void peg_fwd32_kernel(const float* __restrict__ xin, int D,
                                                        const float* __restrict__ w, const float* __restrict__ bias,
                                                        Geo g, float* __restrict__ out, u16* __restrict__ outb,
                                                        u16* __restrict__ outh, float* __restrict__ stats,
                                                        u16* __restrict__ outl, int* status) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  fix_geo<GK, MD>(g);
  bool bad = false;   // an fp16 output out of range (CT_STATUS_F16_RANGE)
  const int nht = (g.H + XHT - 1) / XHT;
  const int b = blockIdx.x / nht, h0 = (blockIdx.x - b * nht) * XHT, c0 = blockIdx.y * XC;
  const int pb = xplane_bytes(g.W);
  float* ws = (float*)(smem + 2 * pb);   // [27][XC]
  float* bs = ws + 27 * XC;
  for (int i = threadIdx.x; i < 27 * XC; i += XNT) {
    const int c = i / 27, tap = i - c * 27;
    ws[tap * XC + c] = w[(int64_t)(c0 + c) * 27 + tap];
  }
  if (threadIdx.x < XC) bs[threadIdx.x] = bias && !TR ? bias[c0 + threadIdx.x] : 0.f;
  using TP = Taps<MD, TR>;
  constexpr bool REV = TR && MD != 2;            // backward walk (see above)
  using TW = Taps<MD, REV ? 0 : TR>;             // walk-axis offsets in walk time
  constexpr int lead = TW::lead, hoff = TP::hoff;
  auto real_t = [&](int p) { return REV ? g.T - 1 - p : p; };   // walk time -> t
  u32x4 reg[XNLD];
  {
    const unsigned v = xplane_load(xin, g, D, b, h0, c0, real_t(0), reg, hoff);
    xplane_store(smem, g.W, reg, v);
  }
  __syncthreads();
  const int ns = (g.W + SEG - 1) / SEG;
  const int o = threadIdx.x;
  const int ch = o & 7, s = (o >> 3) % ns, r = (o >> 3) / ns;
  const int h = h0 + r, w0 = s * SEG;
  const bool active = o < XHT * ns * 8 && h < g.H;
  // three rolling accumulator sets, indexed by t mod 3 -- compile-time indices: the walk is unrolled
  // by three (step<P3> handles planes p = P3 mod 3), so no set is ever selected at run time (which
  // would put the arrays in scratch).  The residual of output t is plane t's centre row, still in LDS
  // when t completes (plane t + lead is the newest; plane t + 1 overwrites slot t & 1 only after
  // the finalize)
  float acc[3][SEG][4];
#pragma unroll
  for (int u = 0; u < 3; ++u)
#pragma unroll
    for (int j = 0; j < SEG; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[u][j][e] = bs[ch * 4 + e];
  const int nsteps = g.T + lead;
  // step p: plane p (p < T) sits in LDS slot p & 1; output p - lead completes
  auto step = [&](auto p3c, int p) {
    constexpr int P3 = decltype(p3c)::value;
    const bool have = p < g.T;
    // next plane into registers (always issued, clamped: no branch merges `reg`)
    const unsigned nvalid = xplane_load(xin, g, D, b, h0, c0, real_t(min(p + 1, g.T - 1)), reg, hoff);
    if (active && have) {
      const char* pl = smem + (p & 1) * pb;
#pragma unroll 1
      for (int kh = 0; kh < 3; ++kh) {
        const int lr = r + TP::dh(kh) + hoff;
        float xv[SEG + 2][4];
#pragma unroll
        for (int q = 0; q < SEG + 2; ++q) {
          const int cw = min(w0 + q, g.W + 1);
          const f32x4 v = *(const f32x4*)(pl + ((lr * (g.W + 2) + cw) * 8 + ch) * 16);
#pragma unroll
          for (int e = 0; e < 4; ++e) xv[q][e] = v[e];
        }
#pragma unroll
        for (int kt = 0; kt < 3; ++kt) {
          const int t = p - TW::dt(kt);          // the output (walk time) this tap of plane p feeds
          if (t < 0 || t >= g.T) continue;
          const int u = (P3 - TW::dt(kt) + 3) % 3;   // compile-time after the unroll
#pragma unroll
          for (int kw = 0; kw < 3; ++kw) {
            const f32x4 wv = *(const f32x4*)(ws + TP::tap(kt, kh, kw) * XC + ch * 4);
#pragma unroll
            for (int j = 0; j < SEG; ++j) {
              const int q = TR ? j + 2 - kw : j + kw;
#pragma unroll
              for (int e = 0; e < 4; ++e) acc[u][j][e] += wv[e] * xv[q][e];
            }
          }
        }
      }
    }
    const int tf = p - lead;   // the output completed by plane p
    if (active && tf >= 0) {
      constexpr int uf = (P3 - lead + 3) % 3;   // t mod 3 of that output
      const char* rp = smem + (tf & 1) * pb + (((r + hoff) * (g.W + 2) + w0 + 1) * 8 + ch) * 16;   // centre row
#pragma unroll
      for (int j = 0; j < SEG; ++j) {
        const int wq = w0 + j;
        const f32x4 xr = *(const f32x4*)(rp + j * 128);   // (columns past W read padding; unused)
        float v4[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v4[e] = acc[uf][j][e] + xr[e];
          acc[uf][j][e] = bs[ch * 4 + e];
        }
        if (wq < g.W) {
          const int64_t orow = canon(g, b, (real_t(tf) * g.H + h) * g.W + wq);
          const int64_t co = orow * D + c0 + ch * 4;
          *(f32x4*)(out + co) = f32x4{v4[0], v4[1], v4[2], v4[3]};
          if (outb) *(uint2*)(outb + co) = pack4(v4);
          if (outh) {
            *(uint2*)(outh + co) = make_uint2(pack2h(v4[0], v4[1]), pack2h(v4[2], v4[3]));
            bad |= !(f16_ok(v4[0]) && f16_ok(v4[1]) && f16_ok(v4[2]) && f16_ok(v4[3]));
            if (outl)   // the split-fp16 pair's lo residual (x3 GEMM operand)
              *(uint2*)(outl + co) = make_uint2(pack2h(v4[0] - rh(v4[0]), v4[1] - rh(v4[1])),
                                                pack2h(v4[2] - rh(v4[2]), v4[3] - rh(v4[3])));
          }
        }
        if (!TR && stats) {
          // the output row's (mean, M2) over this workgroup's 32 channels (two-pass over the 8 lanes
          // ch = 0..7 of the token), merged over the D / 32 groups by ctclip_ln_stats_merge
          float sm = v4[0] + v4[1] + v4[2] + v4[3];
          sm += __shfl_xor(sm, 1, 64);
          sm += __shfl_xor(sm, 2, 64);
          sm += __shfl_xor(sm, 4, 64);
          const float mu = sm * (1.f / XC);
          float m2 = 0.f;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float d = v4[e] - mu;
            m2 = fmaf(d, d, m2);
          }
          m2 += __shfl_xor(m2, 1, 64);
          m2 += __shfl_xor(m2, 2, 64);
          m2 += __shfl_xor(m2, 4, 64);
          if (ch == 0 && wq < g.W) {
            const int64_t ntok = (int64_t)(gridDim.x / nht) * g.thw;
            const int64_t orow = canon(g, b, (real_t(tf) * g.H + h) * g.W + wq);
            *(float2*)(stats + ((int64_t)blockIdx.y * ntok + orow) * 2) = make_float2(mu, m2);
          }
        }
      }
    }
    // slot (p + 1) & 1 holds plane p - 1.  lead 0: last read in step p - 1, before the barrier that
    // ended it, so one barrier per step (after the store) orders the new plane before its reads.
    // lead 1 (the temporal map's canonical walk): this step's finalize just read plane p - 1's centre
    // row (the residual of output p - 1), so the store waits for every thread's finalize first
    if constexpr (lead > 0) __syncthreads();
    if (p + 1 < g.T) xplane_store(smem + ((p + 1) & 1) * pb, g.W, reg, nvalid);
    __syncthreads();
  };
  for (int p = 0; p < nsteps; p += 3) {
    step(std::integral_constant<int, 0>{}, p);
    if (p + 1 < nsteps) step(std::integral_constant<int, 1>{}, p + 1);
    if (p + 2 < nsteps) step(std::integral_constant<int, 2>{}, p + 2);
  }
  if (!TR) status_or(status, CT_STATUS_F16_RANGE, bad);
}

// any geometry / width (D % 4 == 0): one thread per (token, 4 channels), taps from global memory
__global__ __launch_bounds__(256) void peg_fwd32_naive_kernel(const float* __restrict__ xin, int64_t ntok, int D,
                                                              const float* __restrict__ w,
                                                              const float* __restrict__ bias, Geo g,
                                                              float* __restrict__ out, u16* __restrict__ outb,
                                                              u16* __restrict__ outh, u16* __restrict__ outl,
                                                              int* status) {
  const int nc = D / 4;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= ntok * nc) return;
  const int v = (int)(i / nc), col = (int)(i - (int64_t)v * nc) * 4;
  const int b = v / g.thw, p = v - b * g.thw;
  const int hwq = p / g.W, wq = p - hwq * g.W, tq = hwq / g.H, hq = hwq - tq * g.H;
  float acc[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) acc[e] = bias ? bias[col + e] : 0.f;
  for (int kt = 0; kt < 3; ++kt) {
    const int tt = tq + kt - 2;
    if (tt < 0 || tt >= g.T) continue;
    for (int kh = 0; kh < 3; ++kh) {
      const int hh = hq + kh - 1;
      if (hh < 0 || hh >= g.H) continue;
      for (int kw = 0; kw < 3; ++kw) {
        const int ww = wq + kw - 1;
        if (ww < 0 || ww >= g.W) continue;
        const f32x4 x = *(const f32x4*)(xin + (int64_t)canon(g, b, (tt * g.H + hh) * g.W + ww) * D + col);
        const int tap = (kt * 3 + kh) * 3 + kw;
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[e] += w[(int64_t)(col + e) * 27 + tap] * x[e];
      }
    }
  }
  const int64_t co = (int64_t)canon(g, b, p) * D + col;
  const f32x4 rx = *(const f32x4*)(xin + co);
#pragma unroll
  for (int e = 0; e < 4; ++e) acc[e] += rx[e];
  *(f32x4*)(out + co) = f32x4{acc[0], acc[1], acc[2], acc[3]};
  if (outb) *(uint2*)(outb + co) = pack4(acc);
  if (outh) {
    *(uint2*)(outh + co) = make_uint2(pack2h(acc[0], acc[1]), pack2h(acc[2], acc[3]));
    if (outl)
      *(uint2*)(outl + co) = make_uint2(pack2h(acc[0] - rh(acc[0]), acc[1] - rh(acc[1])),
                                        pack2h(acc[2] - rh(acc[2]), acc[3] - rh(acc[3])));
  }
  status_or(status, CT_STATUS_F16_RANGE,
            outh && !(f16_ok(acc[0]) && f16_ok(acc[1]) && f16_ok(acc[2]) && f16_ok(acc[3])));
}

// weight/bias gradient: grid (B * ceil(H/HT), D/64), WNTH threads; thread = (row, w-segment of
// SEGW, channel pair); part[blockIdx.x][c][28] (27 taps in (kt,kh,kw) order, then bias).
// Channel pairs keep the 27 x 2 accumulators + windows under 128 VGPRs (4 waves/SIMD).
template <int GK = 0, int MD = 0>
__global__ __launch_bounds__(WNTH, 3) void peg_wgrad_tile_kernel(const u16* __restrict__ dout,
                                                              const u16* __restrict__ xin, int D, Geo g,
                                                              float* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  fix_geo<GK, MD>(g);
  const int nht = (g.H + HT - 1) / HT;
  const int b = blockIdx.x / nht, h0 = (blockIdx.x - b * nht) * HT, c0 = blockIdx.y * 64;
  const int pb = plane_bytes(g.W);
  char* ring = smem;
  const int pair = threadIdx.x & 31;
  float acc[27][2], accb[2] = {0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 27; ++i) acc[i][0] = acc[i][1] = 0.f;
  // planes two steps ahead (regA = plane t+1, regB = plane t+2), this thread's dout one step
  // ahead (one (row, segment) item per thread: wgrad_ok)
  // (planes L + 1 and L + 2 ahead, L = the forward conv's lead: 0, or 1 for the canonical walk MD 2)
  using TP = Taps<MD, 0>;
  constexpr int L = TP::lead, hoff = TP::hoff;
  u32x4 regA[nld<WNTH>()], regB[nld<WNTH>()];
  unsigned va = ~0u, vb = ~0u;
  for (int tp = 0; tp <= L && tp < g.T; ++tp) {
    va = plane_load<WNTH, false>(xin, g, D, b, h0, c0, tp, regA, hoff);
    plane_store<WNTH>(ring, g.W, tp, regA, va);
  }
  if (g.T > L + 1) va = plane_load<WNTH, false>(xin, g, D, b, h0, c0, L + 1, regA, hoff);
  const int ns = (g.W + SEGW - 1) / SEGW;
  const int items = HT * ns * 32;
  const int o = threadIdx.x;
  const int s = (o >> 5) % ns, r = (o >> 5) / ns;
  const int h = h0 + r, w0 = s * SEGW;
  const bool act = o < items && h < g.H;
  unsigned dmask = 0;
#pragma unroll
  for (int j = 0; j < SEGW; ++j) dmask |= (unsigned)(act && w0 + j < g.W) << j;
  auto dload = [&](int t, uint32_t (&u)[SEGW]) {
#pragma unroll
    for (int j = 0; j < SEGW; ++j) {
      u[j] = 0;
      if ((dmask >> j) & 1)
        u[j] = *(const uint32_t*)(dout + (int64_t)canon(g, b, (t * g.H + h) * g.W + w0 + j) * D + c0 + pair * 2);
    }
  };
  uint32_t du[SEGW], dn[SEGW];
  dload(0, du);
  __syncthreads();
  for (int t = 0; t < g.T; ++t) {
    const int tn = t + 1, tq = t + L + 1;     // tq: the plane stored at the end of this step
    if (tq + 1 < g.T) vb = plane_load<WNTH, false>(xin, g, D, b, h0, c0, tq + 1, regB, hoff);
    if (tn < g.T) dload(tn, dn);
    if (act) {
      float dv[SEGW][2];
#pragma unroll
      for (int j = 0; j < SEGW; ++j) {
        dv[j][0] = __uint_as_float(du[j] << 16);
        dv[j][1] = __uint_as_float(du[j] & 0xffff0000u);
        accb[0] += dv[j][0];
        accb[1] += dv[j][1];
      }
#pragma unroll
      for (int kt = 0; kt < 3; ++kt) {
        const int tp = t + TP::dt(kt);     // <= T: plane T is stored as zeros (the causal tail, L > 0)
        if (tp < 0) continue;
        const char* pl = ring + (tp % NSLOT) * pb;
#pragma unroll
        for (int kh = 0; kh < 3; ++kh) {
          const int lr = r + TP::dh(kh) + hoff;
          float xv[SEGW + 2][2];
#pragma unroll
          for (int q = 0; q < SEGW + 2; ++q) {
            const int cw = min(w0 + q, g.W + 1);
            const uint32_t u = *(const uint32_t*)(pl + (lr * (g.W + 2) + cw) * 128 + pair * 4);
            xv[q][0] = __uint_as_float(u << 16);
            xv[q][1] = __uint_as_float(u & 0xffff0000u);
          }
#pragma unroll
          for (int kw = 0; kw < 3; ++kw)
#pragma unroll
            for (int j = 0; j < SEGW; ++j) {
              acc[TP::tap(kt, kh, kw)][0] += dv[j][0] * xv[j + kw][0];
              acc[TP::tap(kt, kh, kw)][1] += dv[j][1] * xv[j + kw][1];
            }
        }
      }
    }
    __syncthreads();   // slot of plane tq held plane tq - 3, read in this step
    // (with L > 0 the plane past the end, tq == T, is stored as zeros: no upper-bound branch above,
    // which kept values live across it and spilled)
    if (tq < g.T || (L > 0 && tq == g.T)) plane_store<WNTH>(ring, g.W, tq, regA, tq < g.T ? va : 0u);
#pragma unroll
    for (int m = 0; m < nld<WNTH>(); ++m) regA[m] = regB[m];
    va = vb;
#pragma unroll
    for (int j = 0; j < SEGW; ++j) du[j] = dn[j];
    __syncthreads();
  }
  // fold the two (row, segment) items of a wave sharing a pair (lane bit 5), then the waves
  constexpr int NWV = WNTH / 64;
  float* red = (float*)smem;   // [NWV][64 ch][28]; the ring is dead after the last barrier
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < 28; ++i)
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      float v = i < 27 ? acc[i][e] : accb[e];
      v += __shfl_xor(v, 32, 64);
      if (lane < 32) red[(wv * 64 + pair * 2 + e) * 28 + i] = v;
    }
  __syncthreads();
  for (int i = threadIdx.x; i < 64 * 28; i += WNTH) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < NWV; ++k) s += red[k * 64 * 28 + i];
    part[((int64_t)blockIdx.x * D + c0) * 28 + i] = s;
  }
}

// one thread per (channel, tap-or-bias) output, the nblk slabs summed in order
__global__ __launch_bounds__(256) void peg_wgrad_reduce_kernel(const float* __restrict__ part, int nblk, int D,
                                                               float* __restrict__ dw, float* __restrict__ db,
                                                               int accumulate) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= D * 28) return;
  const int64_t stride = (int64_t)D * 28;
  float s = 0.f;
#pragma unroll 8
  for (int b = 0; b < nblk; ++b) s += part[b * stride + i];
  const int c = i / 28, k = i - c * 28;
  float* o = k < 27 ? (dw ? dw + c * 27 + k : nullptr) : (db ? db + c : nullptr);
  if (o) *o = accumulate ? *o + s : s;
}

bool tiled_ok(int W, int D) {
  return D % 64 == 0 && HT * ((W + SEG - 1) / SEG) * 8 <= TNTH && (HT + 2) * (W + 2) * 8 <= PLANE_CH &&
         HT * ((W + SEGW - 1) / SEGW) * 32 <= WNTH;   // wgrad: one item per thread
}

size_t tile_smem(int W) { return (size_t)NSLOT * plane_bytes(W) + (27 * 64 + 64) * 4; }
size_t wgrad_smem(int W) { return std::max<size_t>((size_t)NSLOT * plane_bytes(W), (WNTH / 64) * 64 * 28 * 4); }

bool s_tile_attr = false;
void tile_attrs() {
  if (s_tile_attr) return;
  // up to W = 30: 4 x 4 x 32 x 128 B + weights = 72 KB
  const void* ks[] = {(const void*)peg_tile_kernel<0>,         (const void*)peg_tile_kernel<1>,
                      (const void*)peg_tile_kernel<0, 24, 0>,  (const void*)peg_tile_kernel<0, 24, 1>,
                      (const void*)peg_tile_kernel<1, 24, 0>,  (const void*)peg_tile_kernel<1, 24, 1>,
                      (const void*)peg_tile_kernel<0, 24, 2>,  (const void*)peg_tile_kernel<1, 24, 2>,
                      (const void*)peg_wgrad_tile_kernel<>,    (const void*)peg_wgrad_tile_kernel<24, 0>,
                      (const void*)peg_wgrad_tile_kernel<24, 1>, (const void*)peg_wgrad_tile_kernel<24, 2>};
  for (const void* k : ks) (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024);
  s_tile_attr = true;
}

// the compile-time 24^3 instantiations (CTCLIP_PEG_FIXED=0: the runtime-geometry kernels, A/B)
bool fixed24(const Geo& g) {
  static int on = -1;
  if (on < 0) { const char* e = getenv("CTCLIP_PEG_FIXED"); on = e ? atoi(e) != 0 : 1; }
  return on && g.T == 24 && g.H == 24 && g.W == 24 && (g.mode == 0 || g.mode == 1);
}

// mode 1 on the 24^3 cube through the canonical walk (MD 2); CTCLIP_PEG_CANON1=0 or
// ctclip_peg_set_canon1(0): the view walk (A/B)
int g_canon1 = -1;
bool canon1() {
  if (g_canon1 < 0) { const char* e = getenv("CTCLIP_PEG_CANON1"); g_canon1 = e ? atoi(e) != 0 : 1; }
  return g_canon1 != 0;
}

template <int TR>
void launch_tile(dim3 grid, size_t smem, hipStream_t st, const u16* x, int D, const float* w, const float* bias,
                 const float* res, const Geo& g, float* out, u16* outb, float* stats = nullptr) {
  if (fixed24(g)) {
    if (g.mode == 0)
      hipLaunchKernelGGL((peg_tile_kernel<TR, 24, 0>), grid, dim3(TNTH), smem, st, x, D, w, bias, res, g, out, outb,
                         stats);
    else if (canon1())
      hipLaunchKernelGGL((peg_tile_kernel<TR, 24, 2>), grid, dim3(TNTH), smem, st, x, D, w, bias, res, g, out, outb,
                         stats);
    else
      hipLaunchKernelGGL((peg_tile_kernel<TR, 24, 1>), grid, dim3(TNTH), smem, st, x, D, w, bias, res, g, out, outb,
                         stats);
    return;
  }
  hipLaunchKernelGGL((peg_tile_kernel<TR>), grid, dim3(TNTH), smem, st, x, D, w, bias, res, g, out, outb, stats);
}

}  // namespace

extern "C" int ctclip_peg_set_canon1(int on) {
  const int old = canon1();
  g_canon1 = on != 0;
  return old;
}

extern "C" int ctclip_peg_wgrad_slabs(int64_t B, int32_t T, int32_t H, int32_t W, int32_t D) {
  (void)T;
  return tiled_ok(W, D) ? (int)(B * ((H + HT - 1) / HT)) : 256;
}

extern "C" int ctclip_peg_fwd(const void* x_bf16, const float* x_f32, int64_t B, int32_t T, int32_t H, int32_t W,
                              int32_t D, const float* weight, const float* bias, int32_t mode, float* out_f32,
                              void* out_bf16, void* stream) {
  return ctclip_peg_fwd_stats(x_bf16, x_f32, B, T, H, W, D, weight, bias, mode, out_f32, out_bf16, nullptr, stream);
}

extern "C" int ctclip_peg_fwd_stats(const void* x_bf16, const float* x_f32, int64_t B, int32_t T, int32_t H,
                                    int32_t W, int32_t D, const float* weight, const float* bias, int32_t mode,
                                    float* out_f32, void* out_bf16, float* stats, void* stream) {
  CT_REQUIRE(D % 8 == 0, CT_EALIGN);
  Geo g{T, H, W, T * H * W, mode};
  const int64_t ntok = B * g.thw;
  if (ntok == 0) return 0;
  if (stats) CT_REQUIRE(tiled_ok(W, D) && D % 64 == 0 && (((uintptr_t)stats) & 7) == 0, CT_EINVAL);
  if (tiled_ok(W, D)) {
    tile_attrs();
    dim3 grid(B * ((H + HT - 1) / HT), D / 64);
    launch_tile<0>(grid, tile_smem(W), (hipStream_t)stream, (const u16*)x_bf16, D, weight, bias, x_f32, g, out_f32,
                   (u16*)out_bf16, stats);
  } else {
    dim3 grid(cdiv(ntok, 32), cdiv(D, 64));
    hipLaunchKernelGGL(peg_kernel<0>, grid, dim3(256), 0, (hipStream_t)stream, (const u16*)x_bf16, ntok, D, weight,
                       bias, x_f32, g, out_f32, (u16*)out_bf16);
  }
  CT_CHECK_LAUNCH();
  return 0;
}

extern "C" int ctclip_peg_fwd_x32(const float* x_f32, int64_t B, int32_t T, int32_t H, int32_t W, int32_t D,
                                  const float* weight, const float* bias, int32_t mode, float* out_f32, void* out_bf16,
                                  void* out_f16, float* stats, void* stream) {
  return ctclip_peg_fwd_x32s(x_f32, B, T, H, W, D, weight, bias, mode, out_f32, out_bf16, out_f16, nullptr, stats,
                             nullptr, stream);
}

extern "C" int ctclip_peg_fwd_x32s(const float* x_f32, int64_t B, int32_t T, int32_t H, int32_t W, int32_t D,
                                   const float* weight, const float* bias, int32_t mode, float* out_f32, void* out_bf16,
                                   void* out_f16, void* out_f16lo, float* stats, int32_t* status, void* stream) {
  if (out_f16lo && !out_f16) return CT_EINVAL;
  CT_REQUIRE(D % 4 == 0 && x_f32 && out_f32 && aligned16(x_f32) && aligned16(out_f32), CT_EALIGN);
  Geo g{T, H, W, T * H * W, mode};
  const int64_t ntok = B * g.thw;
  if (ntok == 0) return 0;
  const bool tiled = D % XC == 0 && XHT * ((W + SEG - 1) / SEG) * 8 <= XNT && (XHT + 2) * (W + 2) * 8 <= XPCH;
  if (stats) CT_REQUIRE(tiled && (((uintptr_t)stats) & 7) == 0, CT_EINVAL);
  const hipStream_t st = (hipStream_t)stream;
  if (tiled) {
    static bool attr = false;
    const size_t smem = (size_t)2 * xplane_bytes(W) + (27 * XC + XC) * 4;
    if (!attr) {
      const void* ks[] = {(const void*)peg_fwd32_kernel<>, (const void*)peg_fwd32_kernel<24, 0>,
                          (const void*)peg_fwd32_kernel<24, 1>, (const void*)peg_fwd32_kernel<24, 2>};
      for (const void* k : ks) (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024);
      attr = true;
    }
    dim3 grid(B * ((H + XHT - 1) / XHT), D / XC);
    const auto ob = (u16*)out_bf16;
    const auto oh = (u16*)out_f16;
    const auto ol = (u16*)out_f16lo;
    int* sw = (int*)status;
    if (fixed24(g) && g.mode == 0)
      hipLaunchKernelGGL((peg_fwd32_kernel<24, 0>), grid, dim3(XNT), smem, st, x_f32, D, weight, bias, g, out_f32, ob,
                         oh, stats, ol, sw);
    else if (fixed24(g) && canon1())
      hipLaunchKernelGGL((peg_fwd32_kernel<24, 2>), grid, dim3(XNT), smem, st, x_f32, D, weight, bias, g, out_f32, ob,
                         oh, stats, ol, sw);
    else if (fixed24(g))
      hipLaunchKernelGGL((peg_fwd32_kernel<24, 1>), grid, dim3(XNT), smem, st, x_f32, D, weight, bias, g, out_f32, ob,
                         oh, stats, ol, sw);
    else
      hipLaunchKernelGGL((peg_fwd32_kernel<>), grid, dim3(XNT), smem, st, x_f32, D, weight, bias, g, out_f32, ob, oh,
                         stats, ol, sw);
  } else {
    hipLaunchKernelGGL(peg_fwd32_naive_kernel, dim3(cdiv(ntok * (D / 4), 256)), dim3(256), 0, st, x_f32, ntok, D,
                       weight, bias, g, out_f32, (u16*)out_bf16, (u16*)out_f16, (u16*)out_f16lo, (int*)status);
  }
  CT_CHECK_LAUNCH();
  return 0;
}

// dx = dout + conv^T(dout) from the f32 dout alone (the x32 kernel with TR = 1): the conv taps in
// f32, no bf16 dout read.  Fixed 24^3 grids with the tiled shape only (CT_ESHAPE otherwise: the
// caller runs ctclip_peg_bwd_data)
extern "C" int ctclip_peg_bwd_data_x32(const float* dout_f32, int64_t B, int32_t T, int32_t H, int32_t W, int32_t D,
                                       const float* weight, int32_t mode, float* dx_f32, void* dx_bf16, void* stream) {
  CT_REQUIRE(D % 4 == 0 && dout_f32 && dx_f32 && aligned16(dout_f32) && aligned16(dx_f32), CT_EALIGN);
  Geo g{T, H, W, T * H * W, mode};
  if (B * g.thw == 0) return 0;
  const bool tiled = D % XC == 0 && XHT * ((W + SEG - 1) / SEG) * 8 <= XNT && (XHT + 2) * (W + 2) * 8 <= XPCH;
  if (!tiled || !fixed24(g)) return CT_ESHAPE;
  const hipStream_t st = (hipStream_t)stream;
  static bool attr = false;
  const size_t smem = (size_t)2 * xplane_bytes(W) + (27 * XC + XC) * 4;
  if (!attr) {
    const void* ks[] = {(const void*)peg_fwd32_kernel<24, 0, 1>, (const void*)peg_fwd32_kernel<24, 1, 1>,
                        (const void*)peg_fwd32_kernel<24, 2, 1>};
    for (const void* k : ks) (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024);
    attr = true;
  }
  dim3 grid(B * ((H + XHT - 1) / XHT), D / XC);
  const auto ob = (u16*)dx_bf16;
  if (g.mode == 0)
    hipLaunchKernelGGL((peg_fwd32_kernel<24, 0, 1>), grid, dim3(XNT), smem, st, dout_f32, D, weight,
                       (const float*)nullptr, g, dx_f32, ob, (u16*)nullptr, (float*)nullptr, (u16*)nullptr,
                       (int*)nullptr);
  else if (canon1())
    hipLaunchKernelGGL((peg_fwd32_kernel<24, 2, 1>), grid, dim3(XNT), smem, st, dout_f32, D, weight,
                       (const float*)nullptr, g, dx_f32, ob, (u16*)nullptr, (float*)nullptr, (u16*)nullptr,
                       (int*)nullptr);
  else
    hipLaunchKernelGGL((peg_fwd32_kernel<24, 1, 1>), grid, dim3(XNT), smem, st, dout_f32, D, weight,
                       (const float*)nullptr, g, dx_f32, ob, (u16*)nullptr, (float*)nullptr, (u16*)nullptr,
                       (int*)nullptr);
  CT_CHECK_LAUNCH();
  return 0;
}

// dx = dout (residual path) + conv^T(dout)
extern "C" int ctclip_peg_bwd_data(const void* dout_bf16, const float* dout_f32, int64_t B, int32_t T, int32_t H,
                                   int32_t W, int32_t D, const float* weight, int32_t mode, float* dx_f32,
                                   void* dx_bf16, void* stream) {
  CT_REQUIRE(D % 8 == 0, CT_EALIGN);
  Geo g{T, H, W, T * H * W, mode};
  const int64_t ntok = B * g.thw;
  if (ntok == 0) return 0;
  if (tiled_ok(W, D)) {
    tile_attrs();
    dim3 grid(B * ((H + HT - 1) / HT), D / 64);
    launch_tile<1>(grid, tile_smem(W), (hipStream_t)stream, (const u16*)dout_bf16, D, weight, (const float*)nullptr,
                   dout_f32, g, dx_f32, (u16*)dx_bf16);
  } else {
    dim3 grid(cdiv(ntok, 32), cdiv(D, 64));
    hipLaunchKernelGGL(peg_kernel<1>, grid, dim3(256), 0, (hipStream_t)stream, (const u16*)dout_bf16, ntok, D,
                       weight, (const float*)nullptr, dout_f32, g, dx_f32, (u16*)dx_bf16);
  }
  CT_CHECK_LAUNCH();
  return 0;
}

extern "C" int ctclip_peg_wgrad_reduce(const float* part, int32_t nblk, int32_t D, float* dweight, float* dbias,
                                       int32_t accumulate, void* stream) {
  CT_REQUIRE(part && nblk > 0 && D > 0, CT_EINVAL);
  hipLaunchKernelGGL(peg_wgrad_reduce_kernel, dim3(cdiv((int64_t)D * 28, 256)), dim3(256), 0, (hipStream_t)stream, part,
                     nblk, D, dweight, dbias, accumulate);
  CT_CHECK_LAUNCH();
  return 0;
}

// part: [nblk][D][28] f32 partials (27 taps in (kt,kh,kw) order, then bias)
extern "C" int ctclip_peg_bwd_weight(const void* dout_bf16, const void* x_bf16, int64_t B, int32_t T, int32_t H,
                                     int32_t W, int32_t D, int32_t mode, float* part, int32_t nblk, void* stream) {
  CT_REQUIRE(D % 8 == 0, CT_EALIGN);
  CT_REQUIRE(nblk == ctclip_peg_wgrad_slabs(B, T, H, W, D), CT_ESHAPE);
  Geo g{T, H, W, T * H * W, mode};
  const int64_t ntok = B * g.thw;
  if (tiled_ok(W, D)) {
    tile_attrs();
    dim3 grid(nblk, D / 64);
    const hipStream_t st = (hipStream_t)stream;
    if (fixed24(g) && g.mode == 0)
      hipLaunchKernelGGL((peg_wgrad_tile_kernel<24, 0>), grid, dim3(WNTH), wgrad_smem(W), st, (const u16*)dout_bf16,
                         (const u16*)x_bf16, D, g, part);
    else if (fixed24(g) && canon1())
      hipLaunchKernelGGL((peg_wgrad_tile_kernel<24, 2>), grid, dim3(WNTH), wgrad_smem(W), st, (const u16*)dout_bf16,
                         (const u16*)x_bf16, D, g, part);
    else if (fixed24(g))
      hipLaunchKernelGGL((peg_wgrad_tile_kernel<24, 1>), grid, dim3(WNTH), wgrad_smem(W), st, (const u16*)dout_bf16,
                         (const u16*)x_bf16, D, g, part);
    else
      hipLaunchKernelGGL((peg_wgrad_tile_kernel<>), grid, dim3(WNTH), wgrad_smem(W), st, (const u16*)dout_bf16,
                         (const u16*)x_bf16, D, g, part);
  } else {
    const int64_t per = (ntok + nblk - 1) / nblk;
    dim3 grid(nblk, cdiv(D, 64));
    hipLaunchKernelGGL(peg_wgrad_kernel, grid, dim3(192), 0, (hipStream_t)stream, (const u16*)dout_bf16,
                       (const u16*)x_bf16, ntok, D, g, per, part);
  }
  CT_CHECK_LAUNCH();
  return 0;
}
