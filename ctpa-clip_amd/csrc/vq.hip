// Cosine-similarity vector quantiser (vector_quantize_pytorch==1.1.2, used at
// ct_clip/ctvit.py:187,421-427) and the image pooling of CTCLIP.forward (ct_clip.py:724,740).
//
// The distance matmul l2norm(x) . codebook^T runs as a bf16 MFMA GEMM whose epilogue keeps,
// per (row, 64-code group), the bf16 argmax and the group's second-best bf16 score (gemm.hip
// act=3 with C2).  vq_select then re-scores in f32, against the f32 codebook and the f32
// tokens, every code whose bf16 score can be within `margin` of the best: each group winner
// within the margin, and ALL codes of a group whose second-best is within it too.  Every
// bf16 score is within 2^-7 of the f32 cosine (bf16 x, its l2norm and the codebook each round
// at 2^-9 relative; Cauchy-Schwarz on unit vectors), so the true f32 winner's bf16 score is
// >= best - 2^-6 and margin 2e-2 > 2^-6 makes the result the exact f32 argmax (first index on
// f32 ties), independent of the bf16 rounding.  The default path (round 6) feeds the GEMM fp16
// operands instead (vq_l2norm_h16 + the codebook's fp16 high half): 2^-11 roundings, every
// score within 2^-9 of the f32 cosine, margin 4e-3 > 2^-8, fewer full groups to re-score.
// Every candidate is re-scored with one summation order (slice_partial + butterfly), so the candidate set --
// which depends on the GEMM's operand rounding -- cannot change the f32 winner.
#include "common.h"
#include "../../include/ctclip_hip.h"

// diagnostic build only (timing the full-group re-score; wrong indices): treat every group as single
#ifndef CTCLIP_VQ_DIAG_NOFULL
#define CTCLIP_VQ_DIAG_NOFULL 0
#endif

namespace {

constexpr int VQ_SB = 4;   // single-code candidates re-scored together
constexpr int VQ_CT = 2;   // candidate words of up to 2 x 64 groups (C <= 8192) held in registers
static_assert(VQ_CT == 2, "vq_select picks the preloaded word with a select");
constexpr int VQ_XR = 8;   // the token in registers for D <= 512

// Scoring a candidate code (x_n . cb_row in f32).  The fast sum: lane l sums its slice
// k in {4l .. 4l+3} + 256 j (j ascending, one fused multiply-add per term), then the 64 slice
// partials are added as the xor butterfly of warp_sum (lane l + lane l^32, then ^16, ...) -- the
// same bits whether a code is scored alone or in a full group (score_group).  The deciding sum
// (score_seq): k = 0 .. D-1 in order, one lane.  vq_select returns the argmax under score_seq
// (lowest index on ties); score_seq runs only for the codes whose fast score is within `win` of
// the fast best, win = twice the two sums' worst-case difference, so the rows that need it
// (a near-tie, ~1 %) are the only ones that pay for a D-long dependent chain.  Either way the
// answer cannot depend on which codes became candidates (the low-precision GEMM's rounding).
__device__ __forceinline__ float slice_partial(const float* xs, const float* __restrict__ cr, int D, int lane) {
  float d = 0.f;
  for (int k = lane * 4; k < D; k += 256) {
    const f32x4 w = *(const f32x4*)(cr + k);
    const f32x4 xv = *(const f32x4*)(xs + k);
    d = fmaf(xv[0], w[0], d);
    d = fmaf(xv[1], w[1], d);
    d = fmaf(xv[2], w[2], d);
    d = fmaf(xv[3], w[3], d);
  }
  return d;
}

// all 64 codes of group g at once: every lane forms its slice partial of each code, then a
// reduce-scatter butterfly (63 shuffles instead of 64 warp sums) leaves code g*64 + lane's score --
// the same additions, operand for operand, as warp_sum(slice_partial(code)) -- in lane `lane`
__device__ __forceinline__ float score_group(const float* xs, const float* __restrict__ cb, int g, int C, int D,
                                             int lane) {
  float v[64];
#pragma unroll
  for (int c = 0; c < 64; ++c) v[c] = 0.f;
  for (int k = lane * 4; k < D; k += 256) {
    const f32x4 xv = *(const f32x4*)(xs + k);
#pragma unroll
    for (int c = 0; c < 64; ++c) {
      const int ci = min(g * 64 + c, C - 1);   // past the codebook: a valid row, result discarded
      const f32x4 w = *(const f32x4*)(cb + (int64_t)ci * D + k);
      v[c] = fmaf(xv[0], w[0], v[c]);
      v[c] = fmaf(xv[1], w[1], v[c]);
      v[c] = fmaf(xv[2], w[2], v[c]);
      v[c] = fmaf(xv[3], w[3], v[c]);
    }
  }
#pragma unroll
  for (int h = 32; h >= 1; h >>= 1) {   // lane bit h <-> code bit h
    const bool up = lane & h;
#pragma unroll
    for (int i = 0; i < h; ++i) {
      const float send = up ? v[i] : v[i + h];
      const float keep = up ? v[i + h] : v[i];
      v[i] = keep + __shfl_xor(send, h, 64);
    }
  }
  return v[0];
}

__device__ __forceinline__ float score_seq(const float* xs, const float* __restrict__ cr, int D) {
  float d = 0.f;
  for (int k = 0; k < D; k += 4) {
    const f32x4 w = *(const f32x4*)(cr + k);
    const f32x4 xv = *(const f32x4*)(xs + k);
    d = fmaf(xv[0], w[0], d);
    d = fmaf(xv[1], w[1], d);
    d = fmaf(xv[2], w[2], d);
    d = fmaf(xv[3], w[3], d);
  }
  return d;
}

// fold the wave's (d, i) into (bv, bi): max score, ties to the lowest index (order independent)
__device__ __forceinline__ void wave_argmax(float dv, int di, float& bv, int& bi) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const float ov = __shfl_xor(dv, o, 64);
    const int oi = __shfl_xor(di, o, 64);
    if (ov > dv || (ov == dv && oi < di)) { dv = ov; di = oi; }
  }
  if (dv > bv || (dv == bv && di < bi)) { bv = dv; bi = di; }
}

// one wave per row; the row's f32 l2norm lives in a wave-private LDS strip (D floats) so the
// full-group re-score can run one code per lane
__global__ __launch_bounds__(256) void vq_select_kernel(const float2* __restrict__ cand,
                                                        const float* __restrict__ cand2, int ntiles,
                                                        const float* __restrict__ x, int64_t rows, int D,
                                                        const float* __restrict__ cb, int C, float margin,
                                                        int32_t* __restrict__ idx_out, float* __restrict__ xn_out,
                                                        int* status) {
  extern __shared__ float xs_all[];
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  float* xs = xs_all + (threadIdx.x >> 6) * D;
  const float* xr = x + row * D;
  // the row's candidate words first (up to VQ_CT x 64 groups, held in registers), so their loads are
  // in flight beside the token's
  const bool pre = ntiles <= 64 * VQ_CT;   // wave-uniform
  float2 cpre[VQ_CT];
  float c2pre[VQ_CT];
#pragma unroll
  for (int j = 0; j < VQ_CT; ++j) {
    const int t = j * 64 + lane;
    const bool in = pre && t < ntiles;
    cpre[j] = in ? cand[row * ntiles + t] : make_float2(-INFINITY, 0.f);
    c2pre[j] = in && cand2 ? cand2[row * ntiles + t] : -INFINITY;
  }
  // f32 l2norm of x (F.normalize, eps 1e-12); D <= 64 VQ_XR: the token held in registers
  float ss = 0.f;
  float xreg[VQ_XR];
  const bool xin = D <= 64 * VQ_XR;   // wave-uniform
  if (xin) {
#pragma unroll
    for (int j = 0; j < VQ_XR; ++j) {
      const int c = lane + 64 * j;
      xreg[j] = c < D ? xr[c] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < VQ_XR; ++j) ss += xreg[j] * xreg[j];   // (past D: + 0, exactly)
  } else {
    for (int c = lane; c < D; c += 64) ss += xr[c] * xr[c];
  }
  ss = warp_sum(ss);
  const float inv = 1.f / fmaxf(sqrtf(ss), 1e-12f);
  if (xin) {
#pragma unroll
    for (int j = 0; j < VQ_XR; ++j) {
      const int c = lane + 64 * j;
      if (c < D) {
        const float v = xreg[j] * inv;
        xs[c] = v;
        if (xn_out) xn_out[row * D + c] = v;
      }
    }
  } else {
    for (int c = lane; c < D; c += 64) {
      const float v = xr[c] * inv;
      xs[c] = v;
      if (xn_out) xn_out[row * D + c] = v;
    }
  }
  // best 16-bit score over groups
  float best = -INFINITY;
  if (pre) {
#pragma unroll
    for (int j = 0; j < VQ_CT; ++j) best = fmaxf(best, cpre[j].x);
  } else {
    for (int t = lane; t < ntiles; t += 64) best = fmaxf(best, cand[row * ntiles + t].x);
  }
  best = warp_max(best);
  const float thr = best - margin;
  // every candidate code: onfull(score, code) per lane for the 64 codes of a full group (code >= C
  // past the codebook's end: skip), onsingle(score, code) wave-uniform for a single code
  auto walk = [&](auto&& onfull, auto&& onsingle) {
    auto chunk = [&](int t0, float2 c, float c2) {
      const int t = t0 + lane;
      const bool take = t < ntiles && c.x >= thr;
      const bool full = !CTCLIP_VQ_DIAG_NOFULL && take && cand2 && c2 >= thr;
      unsigned long long gmask = __ballot(full);
      unsigned long long smask = __ballot(take) & ~gmask;
      while (gmask) {
        const int src = __ffsll((long long)gmask) - 1;
        gmask &= gmask - 1;
        // several codes of this group are within the margin: score all of them, one per lane
        onfull(score_group(xs, cb, t0 + src, C, D, lane), (t0 + src) * 64 + lane);
      }
      while (smask) {   // single-code candidates, VQ_SB at a time (their loads interleaved)
        int ci[VQ_SB];
#pragma unroll
        for (int q = 0; q < VQ_SB; ++q) {
          ci[q] = -1;
          if (smask) {   // wave-uniform
            const int src = __ffsll((long long)smask) - 1;
            smask &= smask - 1;
            ci[q] = __float_as_int(__shfl(c.y, src, 64));
          }
        }
        float d[VQ_SB];
#pragma unroll
        for (int q = 0; q < VQ_SB; ++q)
          d[q] = ci[q] >= 0 ? slice_partial(xs, cb + (int64_t)ci[q] * D, D, lane) : 0.f;
#pragma unroll
        for (int q = 0; q < VQ_SB; ++q)
          if (ci[q] >= 0) onsingle(warp_sum(d[q]), ci[q]);
      }
    };
#pragma unroll 1
    for (int t0 = 0; t0 < ntiles; t0 += 64) {
      const int t = t0 + lane;
      float2 c;
      float c2;
      if (pre) {   // (VQ_CT == 2: a select, not a dynamically indexed register array)
        c = t0 == 0 ? cpre[0] : cpre[1];
        c2 = t0 == 0 ? c2pre[0] : c2pre[1];
      } else {
        c = t < ntiles ? cand[row * ntiles + t] : make_float2(-INFINITY, 0.f);
        c2 = t < ntiles && cand2 ? cand2[row * ntiles + t] : -INFINITY;
      }
      chunk(t0, c, c2);
    }
  };
  // pass 1: the fast scores' best (ties to the lowest code) and runner-up, per lane then per wave
  float b1v = -INFINITY, b2v = -INFINITY;
  int b1i = 0x7fffffff;
  auto top2 = [&](float v, int i) {
    if (v > b1v || (v == b1v && i < b1i)) {
      b2v = b1v;
      b1v = v;
      b1i = i;
    } else if (v > b2v) {
      b2v = v;
    }
  };
  walk([&](float v, int i) { if (i < C) top2(v, i); }, top2);
  float bv = -INFINITY;
  int bi = 0x7fffffff;
  wave_argmax(b1v, b1i, bv, bi);
  const float sec = warp_max(b1v == bv && b1i == bi ? b2v : b1v);
  // |fast - seq| <= (D + D/64 + 6) 2^-24 ||cb row|| per code (unit x); win: twice that, for rows of
  // norm <= 4 (the cosine codebook's are unit)
  const float win = 8.f * (float)(D + D / 64 + 8) * 5.9604645e-8f;
  if (sec >= bv - win) {   // wave-uniform: a near-tie -> pass 2, the deciding sum
    const float lo = bv - win;
    float sv = -INFINITY;
    int si = 0x7fffffff;
    walk(
        [&](float v, int i) {
          if (i < C && v >= lo) {
            const float q = score_seq(xs, cb + (int64_t)i * D, D);
            if (q > sv || (q == sv && i < si)) { sv = q; si = i; }
          }
        },
        [&](float v, int i) {
          if (v >= lo) {
            const float q = score_seq(xs, cb + (int64_t)i * D, D);
            if (q > sv || (q == sv && i < si)) { sv = q; si = i; }
          }
        });
    bv = -INFINITY;
    bi = 0x7fffffff;
    wave_argmax(sv, si, bv, bi);
  }
  // a row without any finite score (NaN / inf tokens) keeps bi = INT_MAX: clamp it into the
  // codebook so no consumer (pool, gather, EMA statistics) reads outside it, and zero its
  // normalised row so the EMA statistics take no direction from it (a NaN row would otherwise
  // reach vq_ema_accum's float -> int64 conversion and corrupt code 0's running mean for good;
  // the non-finite loss of such a step is what surfaces the problem)
  const bool bad = (unsigned)bi >= (unsigned)C;   // wave-uniform
  if (lane == 0) idx_out[row] = bad ? 0 : bi;
  if (bad && xn_out)
    for (int c = lane; c < D; c += 64) xn_out[row * D + c] = 0.f;
  // ... and it flags the step (CT_STATUS_VQ_NONFINITE): the trainer skips the step's Adam on every
  // rank and raises, and the guarded EMA finalize drops the step's codebook update
  status_or(status, CT_STATUS_VQ_NONFINITE, bad);
}

// pooled[b][hw][d] = (1/T) sum_t cb[idx[b][t*HW + hw]][d]
__global__ __launch_bounds__(256) void vq_pool_kernel(const int32_t* __restrict__ idx, const float* __restrict__ cb,
                                                      int64_t B, int T, int HW, int D, float* __restrict__ out,
                                                      u16* __restrict__ outb) {
  const int nch = D / 4;
  const int64_t total = B * HW * nch;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % nch);
    const int64_t bh = i / nch;
    const int hw = (int)(bh % HW);
    const int64_t b = bh / HW;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int t = 0; t < T; ++t) {
      const int ci = idx[b * (int64_t)T * HW + (int64_t)t * HW + hw];
      acc += *(const f32x4*)(cb + (int64_t)ci * D + c * 4);
    }
    acc *= (1.f / (float)T);
    if (out) *(f32x4*)(out + bh * D + c * 4) = acc;
    if (outb) {
      uint2 pk;
      pk.x = pack2(acc[0], acc[1]);
      pk.y = pack2(acc[2], acc[3]);
      *(uint2*)(outb + bh * D + c * 4) = pk;
    }
  }
}

// out[r][:] = cb[idx[r]][:]
__global__ __launch_bounds__(256) void vq_gather_kernel(const int32_t* __restrict__ idx, const float* __restrict__ cb,
                                                        int64_t rows, int D, float* __restrict__ out) {
  const int nch = D / 4;
  const int64_t total = rows * nch;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / nch;
    const int c = (int)(i - r * nch);
    *(f32x4*)(out + r * D + c * 4) = *(const f32x4*)(cb + (int64_t)idx[r] * D + c * 4);
  }
}

// EMA statistics: bins[c] += count (f32 adds of 1: exact below 2^24), esum[c][:] += xn rows in
// signed 2^-40 fixed point (int64 adds): integer addition is associative, so the sums are
// bit-identical whatever order the atomics land in, on one GPU and through the SUM all-reduce
// across ranks (dist_sync.sum_codebook_stats).  xn rows are unit vectors: |sum| < 2^23 rows.
constexpr float VQ_FX = 0x1p40f;
constexpr int VQ_EMA_RUN = 16;   // consecutive rows per wave
// a wave walks VQ_EMA_RUN consecutive rows, summing runs of equal codes in registers (neighbouring
// tokens often share a code; an untrained codebook sends most tokens to a few) and adding each
// run once; lane owns columns lane + 64 j, D <= 1024
__global__ __launch_bounds__(256) void vq_ema_accum_kernel(const int32_t* __restrict__ idx,
                                                           const float* __restrict__ xn, int64_t rows, int D,
                                                           float* __restrict__ bins,
                                                           unsigned long long* __restrict__ esum) {
  const int lane = threadIdx.x & 63;
  const int64_t r0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * VQ_EMA_RUN;
  const int64_t r1 = r0 + VQ_EMA_RUN < rows ? r0 + VQ_EMA_RUN : rows;
  long long acc[16];
  int cur = -1, cnt = 0;
  auto flush = [&]() {
    if (lane == 0) atomicAdd(&bins[cur], (float)cnt);
#pragma unroll
    for (int j = 0; j < 16; ++j)
      if (lane + 64 * j < D) atomicAdd(&esum[(int64_t)cur * D + lane + 64 * j], (unsigned long long)acc[j]);
  };
  for (int64_t row = r0; row < r1; ++row) {
    const int ci = idx[row];
    if (ci != cur) {
      if (cur >= 0) flush();
      cur = ci;
      cnt = 0;
#pragma unroll
      for (int j = 0; j < 16; ++j) acc[j] = 0;
    }
    ++cnt;
#pragma unroll
    for (int j = 0; j < 16; ++j)
      if (lane + 64 * j < D) acc[j] += (long long)rintf(xn[row * D + lane + 64 * j] * VQ_FX);
  }
  if (cur >= 0) flush();
}

// Code-sorted EMA statistics (round 5; same sums as vq_ema_accum_kernel, bit for bit).  The
// token-order kernel above flushes a run whenever the code changes; with a trained codebook
// neighbouring tokens rarely share one, so it issues ~rows x D int64 atomics (56.6 M at B = 8:
// ~1 ms on the auxiliary stream, beside the next step's HBM-bound patch LayerNorm).  Here the rows
// are first bucketed by code (a counting sort: rank within the code by an int32 atomic, one
// workgroup's exclusive scan, a scatter), then each wave walks VQ_EMA_CH consecutive positions of
// the sorted order, where a code's rows are contiguous, so it flushes once per (code, chunk):
// ~(C + rows / VQ_EMA_CH) x D atomics.  Integer addition is associative, so neither the rank order
// nor the chunking changes any sum.  work (int32): cnt [C] (zero on entry, left zero), off [C],
// rank [rows], perm [rows].
constexpr int VQ_EMA_CH = 32;   // sorted positions per wave
__global__ __launch_bounds__(256) void vq_rank_kernel(const int32_t* __restrict__ idx, int64_t rows, int C,
                                                      int32_t* __restrict__ cnt, int32_t* __restrict__ rank) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < rows; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = min(max(idx[i], 0), C - 1);
    rank[i] = atomicAdd(&cnt[c], 1);
  }
}

// one workgroup of 1024 threads: off = exclusive prefix sum of cnt; bins += cnt (exact f32
// integers, as the token-order kernel's f32 adds of run lengths); cnt zeroed for the next call
__global__ __launch_bounds__(1024) void vq_code_scan_kernel(int32_t* __restrict__ cnt, int32_t* __restrict__ off, int C,
                                                            float* __restrict__ bins) {
  __shared__ int wsum[16];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int per = (C + 1023) / 1024, c0 = min(C, t * per), c1 = min(C, c0 + per);
  int s = 0;
  for (int c = c0; c < c1; ++c) s += cnt[c];
  int incl = s;   // inclusive scan over the wave
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int v = __shfl_up(incl, o, 64);
    if (lane >= o) incl += v;
  }
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  int base = 0;
  for (int k = 0; k < w; ++k) base += wsum[k];
  int run = base + incl - s;
  for (int c = c0; c < c1; ++c) {
    const int n = cnt[c];
    off[c] = run;
    run += n;
    if (n) bins[c] += (float)n;
    cnt[c] = 0;
  }
}

__global__ __launch_bounds__(256) void vq_scatter_kernel(const int32_t* __restrict__ idx, int64_t rows, int C,
                                                         const int32_t* __restrict__ off,
                                                         const int32_t* __restrict__ rank, int32_t* __restrict__ perm) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < rows; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = min(max(idx[i], 0), C - 1);
    perm[off[c] + rank[i]] = (int32_t)i;
  }
}

// lane owns columns lane + 64 j (D <= 1024); the next row's data is loaded before this row's adds
__global__ __launch_bounds__(256) void vq_ema_sorted_kernel(const int32_t* __restrict__ idx,
                                                            const int32_t* __restrict__ perm,
                                                            const float* __restrict__ xn, int64_t rows, int D, int C,
                                                            unsigned long long* __restrict__ esum) {
  const int lane = threadIdx.x & 63;
  const int64_t j0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * VQ_EMA_CH;
  if (j0 >= rows) return;
  const int64_t j1 = j0 + VQ_EMA_CH < rows ? j0 + VQ_EMA_CH : rows;
  const int nj = (D + 63) >> 6;
  long long acc[16];
  float nx[16];
  int cur = -1;
  auto load = [&](int64_t j, float (&v)[16], int& code) {
    const int r = perm[j];
    code = min(max(idx[r], 0), C - 1);
#pragma unroll
    for (int k = 0; k < 16; ++k)
      if (k < nj && lane + 64 * k < D) v[k] = xn[(int64_t)r * D + lane + 64 * k];
  };
  auto flush = [&]() {
#pragma unroll
    for (int k = 0; k < 16; ++k)
      if (k < nj && lane + 64 * k < D) atomicAdd(&esum[(int64_t)cur * D + lane + 64 * k], (unsigned long long)acc[k]);
  };
  int code;
  load(j0, nx, code);
  for (int64_t j = j0; j < j1; ++j) {
    float v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = nx[k];
    const int c = code;
    if (j + 1 < j1) load(j + 1, nx, code);
    if (c != cur) {
      if (cur >= 0) flush();
      cur = c;
#pragma unroll
      for (int k = 0; k < 16; ++k) acc[k] = 0;
    }
#pragma unroll
    for (int k = 0; k < 16; ++k)
      if (k < nj && lane + 64 * k < D) acc[k] += (long long)rintf(v[k] * VQ_FX);
  }
  if (cur >= 0) flush();
}

// cluster_size = cs*decay + bins*(1-decay);  en = l2norm(esum / max(bins,1)); zero bins keep the
// old code;  embed = embed*decay + en*(1-decay);  also refresh the bf16 working codebook.
// RESET: the statistics are zeroed behind their reads (bins / esum are then ready for the next
// step's accumulation: persistent buffers instead of two fill launches per step)
template <bool RESET = false>
__global__ __launch_bounds__(64) void vq_ema_finalize_kernel(float* __restrict__ bins,
                                                             long long* __restrict__ esum, int C, int D,
                                                             float decay, float* __restrict__ embed,
                                                             float* __restrict__ cluster, u16* __restrict__ embed_bf16,
                                                             const float* __restrict__ guard) {
  const int c = blockIdx.x;
  const int lane = threadIdx.x;
  const float nb = bins[c];
  if (guard && *guard != 0.f) {
    // a flagged step (the summed step status words ride the statistics' all-reduce in the slot
    // after the bins, so every rank takes this branch together): its codebook update is dropped --
    // embed / cluster_size untouched -- and only the statistics are cleared for the next step
    if (RESET) {
      if (lane == 0) bins[c] = 0.f;
      for (int k = lane; k < D; k += 64) esum[(int64_t)c * D + k] = 0;
    }
    return;
  }
  if (lane == 0) cluster[c] = cluster[c] * decay + nb * (1.f - decay);
  if (RESET && lane == 0) bins[c] = 0.f;   // one wave: every lane read it above
  float* e = embed + (int64_t)c * D;
  if (nb == 0.f) {
    if (embed_bf16)
      for (int k = lane; k < D; k += 64) embed_bf16[(int64_t)c * D + k] = f2bf(e[k]);
    return;
  }
  long long* s = esum + (int64_t)c * D;
  constexpr double FX_INV = 0x1p-40;
  float ss = 0.f;
  for (int k = lane; k < D; k += 64) { const float v = (float)((double)s[k] * FX_INV) / nb; ss += v * v; }
  ss = warp_sum(ss);
  const float inv = 1.f / fmaxf(sqrtf(ss), 1e-12f);
  for (int k = lane; k < D; k += 64) {
    const float en = (float)((double)s[k] * FX_INV) / nb * inv;
    if (RESET) s[k] = 0;                   // this lane's own element, read above
    const float v = e[k] * decay + en * (1.f - decay);
    e[k] = v;
    if (embed_bf16) embed_bf16[(int64_t)c * D + k] = f2bf(v);
  }
}

// STE + mean-over-t backward: dx[b][t][hw][:] = dpooled[b][hw][:] / T
__global__ __launch_bounds__(256) void vq_pool_bwd_kernel(const float* __restrict__ dp, int64_t B, int T, int HW,
                                                          int D, float* __restrict__ dx, u16* __restrict__ dxb) {
  const int nch = D / 4;
  const int64_t total = B * (int64_t)T * HW * nch;
  const float invT = 1.f / (float)T;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % nch);
    const int64_t row = i / nch;
    const int hw = (int)(row % HW);
    const int64_t b = row / ((int64_t)T * HW);
    const f32x4 v = *(const f32x4*)(dp + (b * HW + hw) * D + c * 4) * invT;
    if (dx) *(f32x4*)(dx + row * D + c * 4) = v;
    if (dxb) {
      uint2 pk;
      pk.x = pack2(v[0], v[1]);
      pk.y = pack2(v[2], v[3]);
      *(uint2*)(dxb + row * D + c * 4) = pk;
    }
  }
}

inline int gridn(int64_t n) { return (int)std::min<int64_t>(8192, std::max<int64_t>(1, (n + 255) / 256)); }

// fp16 l2norm of the f32 tokens (round 6): the A operand of the fp16 VQ distance GEMM, one wave per
// row, 16-B loads; y = fp16(x / max(||x||, 1e-12)) (F.normalize).  With the fp16 codebook image
// every score is within ~2^-10 of the f32 cosine (one 2^-11 rounding per unit-norm operand), so
// vq_select's re-score margin drops from 2e-2 (bf16: three 2^-9 roundings) to 4e-3
__global__ __launch_bounds__(256) void vq_l2norm_h16_kernel(const float* __restrict__ x, int64_t ldx, int64_t rows,
                                                            int D, u16* __restrict__ y, int64_t ldy) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;   // (wave-uniform)
  const float* xr = x + row * ldx;
  if (D <= 512) {   // wave-uniform: the row in registers (two 16-B words per lane), read once
    const int c0 = lane * 4, c1 = c0 + 256;
    const f32x4 z = {0.f, 0.f, 0.f, 0.f};
    const f32x4 a = c0 < D ? *(const f32x4*)(xr + c0) : z, b = c1 < D ? *(const f32x4*)(xr + c1) : z;
    float s = 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e) s = fmaf(a[e], a[e], s);
#pragma unroll
    for (int e = 0; e < 4; ++e) s = fmaf(b[e], b[e], s);
    s = warp_sum(s);
    const float r = 1.f / fmaxf(sqrtf(s), 1e-12f);   // (the GEMM operand: x r rounds to the same fp16 as
                                                      // x / n but at the last f32 ulp; vq_select re-scores)
    if (c0 < D) {
      const float o[4] = {a[0] * r, a[1] * r, a[2] * r, a[3] * r};
      *(uint2*)(y + row * ldy + c0) = pack4h(o);
    }
    if (c1 < D) {
      const float o[4] = {b[0] * r, b[1] * r, b[2] * r, b[3] * r};
      *(uint2*)(y + row * ldy + c1) = pack4h(o);
    }
    return;
  }
  float s = 0.f;
  for (int c = lane * 4; c < D; c += 256) {
    const f32x4 v = *(const f32x4*)(xr + c);
#pragma unroll
    for (int e = 0; e < 4; ++e) s = fmaf(v[e], v[e], s);
  }
  s = warp_sum(s);
  const float n = fmaxf(sqrtf(s), 1e-12f);
  for (int c = lane * 4; c < D; c += 256) {
    const f32x4 v = *(const f32x4*)(xr + c);
    const float o[4] = {v[0] / n, v[1] / n, v[2] / n, v[3] / n};
    *(uint2*)(y + row * ldy + c) = pack4h(o);
  }
}

}  // namespace

extern "C" int ctclip_vq_l2norm_h16(const float* x, int64_t ldx, int64_t rows, int32_t D, void* y, int64_t ldy,
                                    void* stream) {
  if (rows == 0) return 0;
  CT_REQUIRE(D % 4 == 0 && ldx % 4 == 0 && ldy % 4 == 0 && aligned16(x) && ((uintptr_t)y & 7) == 0, CT_EALIGN);
  hipLaunchKernelGGL(vq_l2norm_h16_kernel, dim3((unsigned)cdiv(rows, 4)), dim3(256), 0, (hipStream_t)stream, x, ldx,
                     rows, D, (u16*)y, ldy);
  CT_CHECK_LAUNCH();
  return 0;
}

extern "C" int ctclip_vq_select(const float* cand, const float* cand2, int32_t ntiles, const float* x, int64_t rows,
                                int32_t D, const float* codebook, int32_t C, float margin, int32_t* idx,
                                float* xn_out, void* stream) {
  if (rows == 0) return 0;
  CT_REQUIRE(D % 4 == 0 && D <= 4096 && aligned16(codebook) && ntiles == (C + 63) / 64, CT_EINVAL);
  return ctclip_vq_select_s(cand, cand2, ntiles, x, rows, D, codebook, C, margin, idx, xn_out, nullptr, stream);
}

extern "C" int ctclip_vq_select_s(const float* cand, const float* cand2, int32_t ntiles, const float* x, int64_t rows,
                                  int32_t D, const float* codebook, int32_t C, float margin, int32_t* idx,
                                  float* xn_out, int32_t* status, void* stream) {
  if (rows == 0) return 0;
  CT_REQUIRE(D % 4 == 0 && D <= 4096 && aligned16(codebook) && ntiles == (C + 63) / 64, CT_EINVAL);
  hipLaunchKernelGGL(vq_select_kernel, dim3(cdiv(rows, 4)), dim3(256), 4 * D * sizeof(float), (hipStream_t)stream,
                     (const float2*)cand, cand2, ntiles, x, rows, D, codebook, C, margin, idx, xn_out, (int*)status);
  CT_CHECK_LAUNCH();
  return 0;
}

extern "C" int ctclip_vq_pool(const int32_t* idx, const float* codebook, int64_t B, int32_t T, int32_t HW, int32_t D,
                              float* out, void* out_bf16, void* stream) {
  CT_REQUIRE(D % 4 == 0, CT_EALIGN);
  hipLaunchKernelGGL(vq_pool_kernel, dim3(gridn(B * HW * D / 4)), dim3(256), 0, (hipStream_t)stream, idx, codebook, B,
                     T, HW, D, out, (u16*)out_bf16);
  CT_CHECK_LAUNCH();
  return 0;
}

extern "C" int ctclip_vq_gather(const int32_t* idx, const float* codebook, int64_t rows, int32_t D, float* out,
                                void* stream) {
  CT_REQUIRE(D % 4 == 0, CT_EALIGN);
  hipLaunchKernelGGL(vq_gather_kernel, dim3(gridn(rows * D / 4)), dim3(256), 0, (hipStream_t)stream, idx, codebook,
                     rows, D, out);
  CT_CHECK_LAUNCH();
  return 0;
}

extern "C" int ctclip_vq_ema_accum(const int32_t* idx, const float* xn, int64_t rows, int32_t D, float* bins,
                                   int64_t* esum, void* stream) {
  if (rows == 0) return 0;
  CT_REQUIRE(D <= 1024, CT_EINVAL);
  const int blocks = cdiv(rows, 4 * VQ_EMA_RUN);
  hipLaunchKernelGGL(vq_ema_accum_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, idx, xn, rows, D, bins,
                     (unsigned long long*)esum);
  CT_CHECK_LAUNCH();
  return 0;
}

// the same statistics through the code-sorted kernels (work: int32 [2 C + 2 rows], the first C
// entries zero on entry and left zero)
extern "C" int ctclip_vq_ema_accum_sorted(const int32_t* idx, const float* xn, int64_t rows, int32_t D, int32_t C,
                                          float* bins, int64_t* esum, int32_t* work, void* stream) {
  if (rows == 0) return 0;
  CT_REQUIRE(D <= 1024 && C > 0 && rows < (int64_t)1 << 31, CT_EINVAL);
  hipStream_t st = (hipStream_t)stream;
  int32_t *cnt = work, *off = work + C, *rank = work + 2 * (int64_t)C, *perm = rank + rows;
  const int g = (int)std::min<int64_t>(cdiv(rows, 256), 2048);
  hipLaunchKernelGGL(vq_rank_kernel, dim3(g), dim3(256), 0, st, idx, rows, C, cnt, rank);
  CT_CHECK_LAUNCH();
  hipLaunchKernelGGL(vq_code_scan_kernel, dim3(1), dim3(1024), 0, st, cnt, off, C, bins);
  CT_CHECK_LAUNCH();
  hipLaunchKernelGGL(vq_scatter_kernel, dim3(g), dim3(256), 0, st, idx, rows, C, off, rank, perm);
  CT_CHECK_LAUNCH();
  hipLaunchKernelGGL(vq_ema_sorted_kernel, dim3(cdiv(rows, 4 * VQ_EMA_CH)), dim3(256), 0, st, idx, perm, xn, rows, D,
                     C, (unsigned long long*)esum);
  CT_CHECK_LAUNCH();
  return 0;
}

extern "C" int ctclip_vq_ema_finalize(const float* bins, const int64_t* esum, int32_t C, int32_t D, float decay,
                                      float* embed, float* cluster_size, void* embed_bf16, void* stream) {
  hipLaunchKernelGGL(vq_ema_finalize_kernel<false>, dim3(C), dim3(64), 0, (hipStream_t)stream, (float*)bins,
                     (long long*)esum, C, D, decay, embed, cluster_size, (u16*)embed_bf16, (const float*)nullptr);
  CT_CHECK_LAUNCH();
  return 0;
}

extern "C" int ctclip_vq_ema_finalize_reset(float* bins, int64_t* esum, int32_t C, int32_t D, float decay,
                                            float* embed, float* cluster_size, void* embed_bf16, void* stream) {
  return ctclip_vq_ema_finalize_guard(bins, esum, C, D, decay, embed, cluster_size, embed_bf16, nullptr, stream);
}

extern "C" int ctclip_vq_ema_finalize_guard(float* bins, int64_t* esum, int32_t C, int32_t D, float decay,
                                            float* embed, float* cluster_size, void* embed_bf16, const float* guard,
                                            void* stream) {
  hipLaunchKernelGGL(vq_ema_finalize_kernel<true>, dim3(C), dim3(64), 0, (hipStream_t)stream, bins,
                     (long long*)esum, C, D, decay, embed, cluster_size, (u16*)embed_bf16, guard);
  CT_CHECK_LAUNCH();
  return 0;
}

extern "C" int ctclip_vq_pool_bwd(const float* dpooled, int64_t B, int32_t T, int32_t HW, int32_t D, float* dx,
                                  void* dx_bf16, void* stream) {
  CT_REQUIRE(D % 4 == 0, CT_EALIGN);
  hipLaunchKernelGGL(vq_pool_bwd_kernel, dim3(gridn(B * T * HW * D / 4)), dim3(256), 0, (hipStream_t)stream, dpooled,
                     B, T, HW, D, dx, (u16*)dx_bf16);
  CT_CHECK_LAUNCH();
  return 0;
}
