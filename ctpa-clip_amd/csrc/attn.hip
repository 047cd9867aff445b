// Fused multi-head attention (forward + backward) for gfx950, head dim 32 or 64.
//
// Replaces the core of Attention.forward (ct_clip/attention.py:156-180): sim = scale * q.k^T
// (+ continuous position bias, attention.py:160-162) -> softmax -> attn @ v; and BERT's
// self-attention (scale 1/sqrt(64), additive key mask).  q and k arrive already
// l2-normalised and multiplied by q_scale / k_scale (norm.hip), so `scale` = 8 for CTViT.
//
// Sequences are gathered straight from the canonical token layout:
//   row(s, i) = (s / n_inner) * s_outer + (s % n_inner) * s_inner + i * s_pos
// (spatial: s = b*T + t, 576 rows per frame; temporal: s = b*H*W + hw, stride H*W; BERT: s = b).
//
// Layout trick: scores are computed transposed, S^T = K.Q^T with v_mfma_f32_16x16x32_bf16,
// so each lane owns ONE query column and its probabilities feed the P.V MFMA as the B operand
// with a permuted key order; V (and K in the backward) are read from their row-major LDS
// image with ds_read_b64_tr_b16 in that same permuted order.  Online softmax keeps the
// running max/sum per lane, in the log2 domain (log2(e) folded into the score scale and the
// bias table, so every probability is one v_exp_f32).
//
// The kernels are VALU-bound (head dim 32: 2 MFMAs of S per 32 keys against 8 softmax elements
// per lane), so per-element work is kept to table reads:
//   * CPB bias: bin(q, k) = (hq-hk+Hg-1)(2Wg-1) + (wq-wk+Wg-1) = C(q) - kb[k] with the position
//     table kb[i] = (i / Wg)(2Wg-1) + i % Wg in LDS; the deduplicated bias u[h][bin] (2,209
//     entries at 24x24, pre-scaled by log2 e) is read from LDS by that index;
//   * key validity (padding past L, BERT key mask) is an additive 0 / -inf row in LDS;
//   * query validity in the backward rides on lse = +inf for padded queries.
// The bias gradient is binned with the same index arithmetic (frame-inner kernel below).
#include "common.h"
#include "../../include/ctclip_hip.h"

namespace {

constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;

struct AP {
  const u16* q; int64_t ldq;
  const u16* k; int64_t ldk;
  const u16* v; int64_t ldv;
  const u16* o; int64_t ldo;      // forward output (read in backward for delta)
  u16* out; int64_t ldout;        // forward: O
  u16* out16;                     // forward, optional: an fp16 copy of O (ldout), the fp16 to_out GEMM's A
  const u16* dout; int64_t lddo;  // backward: dO
  u16* dq; int64_t lddq;
  u16* dk; int64_t lddk;
  u16* dv; int64_t lddv;
  float* lse;                     // [H][M]
  float* delta;                   // [H][M]
  const float* bias_u;            // [H][nbins] or null
  float* dbias_u;                 // [H][nbins] (accumulated with atomics) or null
  float* dbias_ws;                // spatial dQ kernel: [workgroups per head][H][nbins] partial bins, or null
  const int32_t* kmask;           // [nseq][L] 1 = keep, or null
  float scale;
  int L, H, nseq;
  int64_t M;
  int Hg, Wg, nbins;
  int n_inner;
  int64_t s_outer, s_inner, s_pos;
  int pp;                         // (seq, head) pairs per workgroup
  // attention-probability dropout (BertSelfAttention.dropout, non-bias kernels only):
  // keep(s, h, q, k) = hash(seed, index) >= thresh, kept probabilities scaled by 1 / (1 - p)
  float drop_p, drop_scale;
  unsigned thresh;
  uint64_t seed;
  float lazy;                     // forward: lazy-rescale threshold (log2 units), <= 0 = every chunk
};

constexpr int NW = 8;             // waves per workgroup
constexpr int NT = NW * 64;
// staging loads in flight per thread (stage2): fwd / dK-dV kernels, and the frame-inner dQ +
// bias-gradient kernel (194 VGPRs already).  Measured at the base spatial shape: spatial backward
// 1,074 -> 984 us; 3 / 6 / 9 / 12 in flight within 1 %.
constexpr int SU = 6;
constexpr int SUB = 3;

__device__ __forceinline__ int64_t seq_row(const AP& p, int s, int i) {
  return (int64_t)(s / p.n_inner) * p.s_outer + (int64_t)(s % p.n_inner) * p.s_inner + (int64_t)i * p.s_pos;
}

// dropout multiplier of P[q][k] for (seq s, head h): 0 or 1 / (1 - p), a pure function of
// (seed, s, h, q, k) so the backward kernels regenerate the forward's mask (splitmix64 finaliser)
__device__ __forceinline__ float drop_keep(const AP& p, int s, int h, int q, int k) {
  uint64_t x = p.seed ^ ((((uint64_t)(s * p.H + h) * p.L + q) * p.L + k) * 0x9E3779B97F4A7C15ull);
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return (unsigned)x >= p.thresh ? p.drop_scale : 0.f;
}

// bias table constants: bin(q, k) = kb[q] + boff - kb[k]
__device__ __forceinline__ int kb_of(const AP& p, int i) { return (i / p.Wg) * (2 * p.Wg - 1) + i % p.Wg; }
__device__ __forceinline__ int boff(const AP& p) { return (p.Hg - 1) * (2 * p.Wg - 1) + p.Wg - 1; }
// the same position in two VALU ops instead of an LDS table read inside the chunk loops (whose
// result the bias read's address waits on: a two-deep LDS chain per chunk becomes one):
// kb(i) = (i / Wg)(2 Wg - 1) + i % Wg = i + (i / Wg)(Wg - 1), with i / Wg = umulhi(i, mg),
// mg = floor((2^32 - 1) / Wg) + 1 (= ceil(2^32 / Wg), exact division for i < 2^29 / Wg * Wg)
struct KbFast {
  unsigned mg;
  int wg1;
};
__device__ __forceinline__ KbFast kb_fast_init(const AP& p) {
  return p.Wg > 0 ? KbFast{0xFFFFFFFFu / (unsigned)p.Wg + 1u, p.Wg - 1} : KbFast{0u, 0};
}
__device__ __forceinline__ int kb_fast(const KbFast& f, int i) {
  return i + (int)__umulhi((unsigned)i, f.mg) * f.wg1;
}

template <int D>
struct Img {
  static constexpr int RS = D * 2 + 16;  // padded row stride (bytes)
};

// stage rows [0, Lp) of one head's [L][D] slice into a padded LDS image (zero rows >= L)
template <int D>
__device__ __forceinline__ void stage(char* img, const u16* base, int64_t ld, const AP& p, int s, int h, int Lp,
                                      int tid, int nth) {
  constexpr int CH = D / 8;
  for (int idx = tid; idx < Lp * CH; idx += nth) {
    const int r = idx / CH, c = idx - r * CH;
    u32x4 v = make_uint4(0, 0, 0, 0);
    if (r < p.L) v = *(const u32x4*)(base + seq_row(p, s, r) * ld + h * D + c * 8);
    *(u32x4*)(img + r * Img<D>::RS + c * 16) = v;
  }
}

// stage two images (e.g. K and V) of one (seq, head) pair with U loads in flight per thread
// before their LDS writes: the staging then pays ceil(chunks / (U * nth)) memory latencies
// instead of one per 16-B chunk per thread
template <int D, int U>
__device__ __forceinline__ void stage2(char* imgA, const u16* a, int64_t lda, char* imgB, const u16* b, int64_t ldb,
                                       const AP& p, int s, int h, int Lp, int tid, int nth) {
  constexpr int CH = D / 8;
  const int n1 = Lp * CH, n = 2 * n1;
  for (int i0 = tid; i0 < n; i0 += U * nth) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int idx = i0 + u * nth, isb = idx >= n1, id = isb ? idx - n1 : idx;
      const int r = id / CH, c = id - r * CH;
      v[u] = make_uint4(0, 0, 0, 0);
      if (idx < n && r < p.L) {
        const int64_t row = seq_row(p, s, r);
        v[u] = isb ? *(const u32x4*)(b + row * ldb + h * D + c * 8) : *(const u32x4*)(a + row * lda + h * D + c * 8);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int idx = i0 + u * nth, isb = idx >= n1, id = isb ? idx - n1 : idx;
      const int r = id / CH, c = id - r * CH;
      if (idx < n) *(u32x4*)((isb ? imgB : imgA) + r * Img<D>::RS + c * 16) = v[u];
    }
  }
}

// A/B fragment from a row-major image: lane gets [r0 + (lane&15)][kk*32 + 8*(lane>>4) + 0..7]
template <int D>
__device__ __forceinline__ bf16x8 rowfrag(const char* img, int r0, int kk, int lane) {
  return *(const bf16x8*)(img + (r0 + (lane & 15)) * Img<D>::RS + ((kk * 4 + (lane >> 4)) << 4));
}

// transposed fragment: lane gets column c0 + (lane&15) of rows
//   r0 + 4g + 0..3 (elements 0..3) and r0 + 16 + 4g + 0..3 (elements 4..7),  g = lane>>4
template <int D>
__device__ __forceinline__ bf16x8 trfrag(const char* img, int r0, int c0, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, pp = i & 3;
  const char* a1 = img + (r0 + 4 * g + q) * Img<D>::RS + (c0 + 4 * pp) * 2;
  const char* a2 = a1 + 16 * Img<D>::RS;
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, a1));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, a2));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// Swizzled 64-B-row images (head dim 32): the 16-B chunk of row r sits at chunk ^ kv_swz(r), which
// keeps the ds_read_b128 row fragments and the ds_read_b64_tr_b16 transposed ones conflict-free
// under gfx950's lane groups (searched); the padded 80-B rows above conflict (r02 / r03 PMC:
// 23-35 % of LDS-active cycles).
__device__ __forceinline__ int kv_swz(int row) { return (row >> 1) & 3; }
__device__ __forceinline__ bf16x8 rowfrag_sw(const char* img, int r0, int lane) {
  const int row = r0 + (lane & 15);
  return *(const bf16x8*)(img + row * 64 + (((lane >> 4) ^ kv_swz(row)) << 4));
}
__device__ __forceinline__ bf16x8 trfrag_sw(const char* img, int r0, int c0, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, pp = i & 3;
  const int row = r0 + 4 * g + q, colb = 2 * c0 + 8 * pp;
  const char* a1 = img + row * 64 + (((colb >> 4) ^ kv_swz(row)) << 4) + (colb & 15);
  const char* a2 = a1 + 16 * 64;   // row + 16: same swizzle
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, a1));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, a2));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// stage2 into swizzled 64-B-row images (head dim 32)
template <int U>
__device__ __forceinline__ void stage2_sw(char* imgA, const u16* a, int64_t lda, char* imgB, const u16* b, int64_t ldb,
                                          const AP& p, int s, int h, int Lp, int tid, int nth) {
  constexpr int D = 32, CH = 4;
  const int n1 = Lp * CH, n = 2 * n1;
  for (int i0 = tid; i0 < n; i0 += U * nth) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int idx = i0 + u * nth, isb = idx >= n1, id = isb ? idx - n1 : idx;
      const int r = id / CH, c = id - r * CH;
      v[u] = make_uint4(0, 0, 0, 0);
      if (idx < n && r < p.L) {
        const int64_t row = seq_row(p, s, r);
        v[u] = isb ? *(const u32x4*)(b + row * ldb + h * D + c * 8) : *(const u32x4*)(a + row * lda + h * D + c * 8);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int idx = i0 + u * nth, isb = idx >= n1, id = isb ? idx - n1 : idx;
      const int r = id / CH, c = id - r * CH;
      if (idx < n) *(u32x4*)((isb ? imgB : imgA) + r * 64 + ((c ^ kv_swz(r)) << 4)) = v[u];
    }
  }
}

__device__ __forceinline__ bf16x8 pack_perm(const f32x4& a, const f32x4& b) {
  bf16x8 r;
  r[0] = (bf16)a[0]; r[1] = (bf16)a[1]; r[2] = (bf16)a[2]; r[3] = (bf16)a[3];
  r[4] = (bf16)b[0]; r[5] = (bf16)b[1]; r[6] = (bf16)b[2]; r[7] = (bf16)b[3];
  return r;
}

__device__ __forceinline__ bf16x8 gload8(const u16* p) { return __builtin_bit_cast(bf16x8, *(const u32x4*)p); }
__device__ __forceinline__ bf16x8 zero8() { return __builtin_bit_cast(bf16x8, make_uint4(0, 0, 0, 0)); }
__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }

// shared LDS tables of a workgroup (after the K/V or Q/dO images):
//   ub[nbins]  bias table * log2 e        (BIAS)
//   kb[Lp]     position table             (BIAS)
//   madd[pp][Lp] additive key validity     (0 / -inf: padding past L, key mask)
// REV (the C-init forward below): the table reversed and in units of the raw score, ub[i] =
// bias[nbins - 1 - i] / scale, so 4 keys of one grid row read 4 ascending entries
template <bool BIAS, int NTH = NT, bool REV = false>
__device__ __forceinline__ void load_tables(const AP& p, char* tab, int Lp, int tid, int h, float*& ub, int*& kb,
                                            float*& madd) {
  char* t = tab;
  if (BIAS) {
    ub = (float*)t;
    t += ((p.nbins + 3) & ~3) * 4;   // keep kb / madd 16-B aligned for the vector reads
    kb = (int*)t;
    t += Lp * 4;
    if constexpr (REV) {
      // (the RUN shapes have no padded / masked keys: no validity table; the position table, read
      // once per query block, from kb_fast instead of two integer divisions per entry)
      const float isc = 1.f / p.scale;   // exact for the power-of-two scale 8
      for (int i = tid; i < p.nbins; i += NTH) ub[i] = p.bias_u[(int64_t)h * p.nbins + p.nbins - 1 - i] * isc;
      const KbFast f = kb_fast_init(p);
      for (int i = tid; i < Lp; i += NTH) kb[i] = kb_fast(f, i);
      madd = (float*)t;
      return;
    } else {
      for (int i = tid; i < p.nbins; i += NTH) ub[i] = p.bias_u[(int64_t)h * p.nbins + i] * LOG2E;
    }
    for (int i = tid; i < Lp; i += NTH) kb[i] = i < p.L ? kb_of(p, i) : 0;
  }
  madd = (float*)t;
  for (int pl = 0; pl < p.pp; ++pl) {
    const int pair = blockIdx.x * p.pp + pl;
    const int s = pair / p.H;
    for (int i = tid; i < Lp; i += NTH) {
      bool v = i < p.L && pair < p.nseq * p.H;
      if (v && p.kmask) v = p.kmask[(int64_t)s * p.L + i] != 0;
      madd[pl * Lp + i] = v ? 0.f : -INFINITY;
    }
  }
}

// ------------------------------------------------------------------------------------ forward
// W waves per workgroup: 12 for the spatial (BIAS) shapes, whose 36 query blocks then split
// evenly (3 per wave) at 12 waves per CU; 8 otherwise.
// RUN (bias shapes with Wg % 4 == 0 and L % 32 == 0): the 4 keys a lane scores per MFMA block
// are consecutive in one grid row, so their bins are cq - kb[k0] - 0..3 -- one table read and one
// address for all four bias reads (fixed offsets) -- and there are no padded keys to mask.
// QB query blocks per wave are processed TOGETHER (same key chunk loop): their score / softmax /
// PV chains are independent, so they interleave and hide each other's MFMA -> VALU -> LDS
// latencies (the kernel ran at ~3 waves per SIMD with one dependent chain each), and the K / V
// fragments of a key chunk are read from LDS once for all QB blocks.  Per-query arithmetic is
// unchanged (bit-identical to QB = 1).
// SMAX (RUN shapes): the softmax max is a per-query STATIC bound instead of the online running
// max -- |q.k| <= ||q|| max_k ||k|| (Cauchy-Schwarz), so x <= Mq = scale ||q|| max||k|| + max bias
// (log2 units) -- which removes the per-chunk cross-lane max, the rescale of the running sum and
// of the output, and keeps every probability <= 1.  Used for a query group only while the bound's
// span (2 scale ||q|| max||k|| + bias range) stays <= 64, so no probability can underflow more
// than exp2(-64) below the row's largest; otherwise that group runs the online-max code.  Same
// softmax in exact arithmetic, f32-level differences in rounding.
// A/B build switch (tools/attn_lazy_ab.py): 1 = the swizzled 64-B-row K / V images for head dim 32.
// Measured 1.2 % SLOWER in this VALU-bound kernel (profiles/r04h_attn_lazy_ab.log: 252.4 vs 249.5 us),
// so the padded 80-B rows stay the default
#ifndef CTCLIP_ATTN_FWD_SWZ
#define CTCLIP_ATTN_FWD_SWZ 0
#endif
// CINIT (RUN shapes, round 6): the score chain with the least vector work per score -- the bias
// enters as the MFMA's C operand (read from the reversed, 1/scale table straight into the
// accumulator), so score -> probability is one v_fma (scale log2 e, minus the running max) and one
// v_exp; the row sums come from one more MFMA per key chunk (an all-ones A operand against the
// bf16 probabilities, i.e. the sum of exactly the P the PV product uses) instead of a v_add per
// score; the lazy-rescale logic is unchanged.  Per score: fma + exp + 1/4 max3 + 1/2 cvt_pk
// against fma + max + sub + exp + add + 1/2 cvt_pk.
template <int D, bool BIAS, int W = (BIAS ? 12 : NW), bool RUN = false, int QB = 1, bool SMAX = false,
          bool CINIT = false>
__global__ __launch_bounds__(W * 64) void attn_fwd_kernel(AP p) {
  static_assert(!CINIT || (RUN && !SMAX && BIAS), "CINIT: the RUN shapes' online-max forward");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // head dim 32: swizzled 64-B-row K / V images (kv_swz); 64: the padded rows
  constexpr bool SWZ = D == 32 && CTCLIP_ATTN_FWD_SWZ;
  constexpr int KK = D / 32, DB = D / 16, RS = SWZ ? 64 : Img<D>::RS, NTH = W * 64;
  const int L = p.L, Lp = (L + 31) & ~31;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wpp = W / p.pp;                          // waves per pair
  const int pair_local = w / wpp, wi = w - pair_local * wpp;
  const int pair_bytes = 2 * Lp * RS;
  for (int pl = 0; pl < p.pp; ++pl) {
    const int pair = blockIdx.x * p.pp + pl;
    if (pair >= p.nseq * p.H) break;
    const int s = pair / p.H, h = pair - s * p.H;
    if constexpr (SWZ)
      stage2_sw<SU>(smem + pl * pair_bytes, p.k, p.ldk, smem + pl * pair_bytes + Lp * RS, p.v, p.ldv, p, s, h, Lp,
                    tid, NTH);
    else
      stage2<D, SU>(smem + pl * pair_bytes, p.k, p.ldk, smem + pl * pair_bytes + Lp * RS, p.v, p.ldv, p, s, h, Lp,
                    tid, NTH);
  }
  auto kfrag = [&](const char* img, int r0, int kk) {
    if constexpr (SWZ) return rowfrag_sw(img, r0, lane);
    else return rowfrag<D>(img, r0, kk, lane);
  };
  auto vfrag = [&](const char* img, int r0, int c0) {
    if constexpr (SWZ) return trfrag_sw(img, r0, c0, lane);
    else return trfrag<D>(img, r0, c0, lane);
  };
  float* ub = nullptr;
  int* kb = nullptr;
  float* madd = nullptr;
  load_tables<BIAS, NTH, CINIT>(p, smem + p.pp * pair_bytes, Lp, tid, blockIdx.x % p.H, ub, kb,
                                madd);  // pp == 1 with BIAS
  __syncthreads();
  const int pair = blockIdx.x * p.pp + pair_local;
  if (pair >= p.nseq * p.H) return;
  const int s = pair / p.H, h = pair - s * p.H;
  const char* Kimg = smem + pair_local * pair_bytes;
  const char* Vimg = Kimg + Lp * RS;
  const float* mrow = madd + pair_local * Lp;
  const int g = lane >> 4, li = lane & 15;
  const int nqb = (L + 15) >> 4;
  const float sc2 = p.scale * LOG2E;
  const KbFast kbf = kb_fast_init(p);
  (void)kbf;
  float kmax2 = 0.f, bhi = 0.f, blo = 0.f;
  if constexpr (SMAX) {
    // max_k ||k||^2 of this pair's keys and the bias table's range (log2 units): one block reduction
    float k2 = 0.f, bh = -INFINITY, bl = INFINITY;
    for (int r = tid; r < L; r += NTH) {
      float s2 = 0.f;
#pragma unroll
      for (int c = 0; c < D / 8; ++c) {
        float x[8];
        unpack8(*(const u32x4*)(Kimg + r * RS + c * 16), x);
#pragma unroll
        for (int j = 0; j < 8; ++j) s2 = fmaf(x[j], x[j], s2);
      }
      k2 = fmaxf(k2, s2);
    }
    for (int i = tid; i < p.nbins; i += NTH) { bh = fmaxf(bh, ub[i]); bl = fminf(bl, ub[i]); }
#pragma unroll
    for (int o_ = 1; o_ < 64; o_ <<= 1) {
      k2 = fmaxf(k2, __shfl_xor(k2, o_, 64));
      bh = fmaxf(bh, __shfl_xor(bh, o_, 64));
      bl = fminf(bl, __shfl_xor(bl, o_, 64));
    }
    float* red = madd + p.pp * Lp;      // 3 * W floats past the tables (host: + 256 B)
    if (lane == 0) { red[w] = k2; red[W + w] = bh; red[2 * W + w] = bl; }
    __syncthreads();
    kmax2 = red[0]; bhi = red[W]; blo = red[2 * W];
#pragma unroll
    for (int i = 1; i < W; ++i) { kmax2 = fmaxf(kmax2, red[i]); bhi = fmaxf(bhi, red[W + i]); blo = fminf(blo, red[2 * W + i]); }
  }
  for (int qb0 = wi; qb0 < nqb; qb0 += QB * wpp) {
    int q[QB], cq[QB];
    bool qv[QB];
    int64_t qrow[QB];
    bf16x8 qf[QB][KK];
    float m[QB], lsum[QB];
    f32x4 o[QB][DB];
#pragma unroll
    for (int u = 0; u < QB; ++u) {
      q[u] = (qb0 + u * wpp) * 16 + li;           // blocks qb0, qb0 + wpp, ... (an idle block has q >= L)
      qv[u] = q[u] < L;
      qrow[u] = qv[u] ? seq_row(p, s, q[u]) : 0;
#pragma unroll
      for (int kk = 0; kk < KK; ++kk)
        qf[u][kk] = qv[u] ? gload8(p.q + qrow[u] * p.ldq + h * D + kk * 32 + 8 * g) : zero8();
      cq[u] = BIAS ? kb[min(q[u], L - 1)] + boff(p) : 0;   // padded queries: any in-range bin
      m[u] = -INFINITY;
      lsum[u] = 0.f;
#pragma unroll
      for (int d = 0; d < DB; ++d) o[u][d] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    bool use_static = false;
    if constexpr (SMAX) {
      bool ok = true;
#pragma unroll
      for (int u = 0; u < QB; ++u) {
        float q2 = 0.f;
#pragma unroll
        for (int kk = 0; kk < KK; ++kk)
#pragma unroll
          for (int j = 0; j < 8; ++j) q2 = fmaf((float)qf[u][kk][j], (float)qf[u][kk][j], q2);
        q2 += __shfl_xor(q2, 16, 64);
        q2 += __shfl_xor(q2, 32, 64);
        const float xb = sc2 * sqrtf(q2 * kmax2);
        m[u] = xb + bhi;                           // the static bound Mq (log2 units)
        ok = ok && 2.f * xb + (bhi - blo) <= 64.f;
      }
      use_static = __all(ok);
    }
    if (use_static) {
      if constexpr (SMAX) {
        for (int kc = 0; kc < Lp; kc += 32) {
          bf16x8 kf[2][KK];
#pragma unroll
          for (int bi = 0; bi < 2; ++bi)
#pragma unroll
            for (int kk = 0; kk < KK; ++kk) kf[bi][kk] = kfrag(Kimg, kc + 16 * bi, kk);
          bf16x8 pb[QB];
#pragma unroll
          for (int u = 0; u < QB; ++u) {
            f32x4 sa[2];
#pragma unroll
            for (int bi = 0; bi < 2; ++bi) {
              sa[bi] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
              for (int kk = 0; kk < KK; ++kk)
                sa[bi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[bi][kk], qf[u][kk], sa[bi], 0, 0, 0);
            }
#pragma unroll
            for (int bi = 0; bi < 2; ++bi) {
              const float* up = ub + (cq[u] - kb[kc + 16 * bi + 4 * g] - 3);   // up[3 - r] = ub[bin(q, k0 + r)]
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const float e = fexp2(fmaf(sa[bi][r], sc2, up[3 - r]) - m[u]);
                sa[bi][r] = e;
                lsum[u] += e;
              }
            }
            pb[u] = pack_perm(sa[0], sa[1]);
          }
#pragma unroll
          for (int d = 0; d < DB; ++d) {
            const bf16x8 vf = vfrag(Vimg, kc, d * 16);
#pragma unroll
            for (int u = 0; u < QB; ++u) o[u][d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pb[u], o[u][d], 0, 0, 0);
          }
        }
      }
    } else if constexpr (CINIT) {
      const bf16x8 ones = __builtin_bit_cast(bf16x8, make_uint4(0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u));
      f32x4 osum[QB];
      int cqr[QB];
      // per block: nm = -m (log2 units, 0 before the first rescale) -- the exponent argument
      // x = sc2 * score + nm is formed FIRST (one fma per score), and the chunk max / lazy test run
      // on x: x is an ordinary VALU result, so the max needs no canonicalising v_max per MFMA output
      // (and no inline asm, whose MFMA read hazards the compiler does not see); the first chunk
      // always rescales
      float nm[QB];
#pragma unroll
      for (int u = 0; u < QB; ++u) {
        m[u] = -INFINITY;
        nm[u] = 0.f;
        osum[u] = f32x4{0.f, 0.f, 0.f, 0.f};
        cqr[u] = p.nbins - 1 - cq[u];          // reversed-table index of key 0's bin offset
      }
      for (int kc = 0; kc < Lp; kc += 32) {
        bf16x8 kf[2][KK];
#pragma unroll
        for (int bi = 0; bi < 2; ++bi)
#pragma unroll
          for (int kk = 0; kk < KK; ++kk) kf[bi][kk] = kfrag(Kimg, kc + 16 * bi, kk);
        int kx[2];
#pragma unroll
        for (int bi = 0; bi < 2; ++bi) kx[bi] = kb_fast(kbf, kc + 16 * bi + 4 * g);
        f32x4 sa[QB][2];
#pragma unroll
        for (int u = 0; u < QB; ++u)
#pragma unroll
          for (int bi = 0; bi < 2; ++bi) {
            const float* up = ub + (kx[bi] + cqr[u]);   // up[r] = bias(q, k0 + r) / scale
            sa[u][bi] = f32x4{up[0], up[1], up[2], up[3]};
#pragma unroll
            for (int kk = 0; kk < KK; ++kk)
              sa[u][bi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[bi][kk], qf[u][kk], sa[u][bi], 0, 0, 0);
          }
        float cmax[QB];      // chunk max of x, relative to the running max
        bool need = p.lazy <= 0.f || kc == 0;
#pragma unroll
        for (int u = 0; u < QB; ++u) {
#pragma unroll
          for (int bi = 0; bi < 2; ++bi)
#pragma unroll
            for (int r = 0; r < 4; ++r) sa[u][bi][r] = fmaf(sa[u][bi][r], sc2, nm[u]);
          cmax[u] = fmaxf(fmaxf(fmaxf(sa[u][0][0], sa[u][0][1]), fmaxf(sa[u][0][2], sa[u][0][3])),
                          fmaxf(fmaxf(sa[u][1][0], sa[u][1][1]), fmaxf(sa[u][1][2], sa[u][1][3])));
          need = need || cmax[u] > p.lazy;
        }
        if (__builtin_amdgcn_readfirstlane((int)__any(need)) != 0) {
#pragma unroll
          for (int u = 0; u < QB; ++u) {
            float c = fmaxf(cmax[u], __shfl_xor(cmax[u], 16, 64));
            c = fmaxf(c, __shfl_xor(c, 32, 64));
            // the shift d moves the running max to the query's full max (first chunk: the chunk max
            // itself; later: only upwards)
            const bool first = m[u] == -INFINITY;
            const float d = first ? c : fmaxf(c, 0.f);
            const float alpha = first ? 1.f : fexp2(-d);     // (o, osum are still zero on the first)
            nm[u] -= d;
            m[u] = -nm[u];
#pragma unroll
            for (int bi = 0; bi < 2; ++bi)
#pragma unroll
              for (int r = 0; r < 4; ++r) sa[u][bi][r] -= d;
#pragma unroll
            for (int dd = 0; dd < DB; ++dd) o[u][dd] *= alpha;
            osum[u] *= alpha;
          }
        }
        bf16x8 pb[QB];
#pragma unroll
        for (int u = 0; u < QB; ++u) {
#pragma unroll
          for (int bi = 0; bi < 2; ++bi)
#pragma unroll
            for (int r = 0; r < 4; ++r) sa[u][bi][r] = fexp2(sa[u][bi][r]);
          pb[u] = pack_perm(sa[u][0], sa[u][1]);
        }
#pragma unroll
        for (int d = 0; d < DB; ++d) {
          const bf16x8 vf = vfrag(Vimg, kc, d * 16);
#pragma unroll
          for (int u = 0; u < QB; ++u) o[u][d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pb[u], o[u][d], 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < QB; ++u) osum[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, pb[u], osum[u], 0, 0, 0);
      }
      // every row of the all-ones product is the query's full sum: no cross-lane reduction below
#pragma unroll
      for (int u = 0; u < QB; ++u) lsum[u] = osum[u][0];
    } else {
#pragma unroll
    for (int u = 0; u < QB; ++u) m[u] = -INFINITY;
    for (int kc = 0; kc < Lp; kc += 32) {
      bf16x8 kf[2][KK];
#pragma unroll
      for (int bi = 0; bi < 2; ++bi)
#pragma unroll
        for (int kk = 0; kk < KK; ++kk) kf[bi][kk] = kfrag(Kimg, kc + 16 * bi, kk);
      f32x4 sa[QB][2];
#pragma unroll
      for (int u = 0; u < QB; ++u)
#pragma unroll
        for (int bi = 0; bi < 2; ++bi) {
          sa[u][bi] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int kk = 0; kk < KK; ++kk)
            sa[u][bi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[bi][kk], qf[u][kk], sa[u][bi], 0, 0, 0);
        }
      bf16x8 pb[QB];
      float alpha[QB];
      bool rescale[QB];
#pragma unroll
      for (int u = 0; u < QB; ++u) {
        float cmax = -INFINITY;
#pragma unroll
        for (int bi = 0; bi < 2; ++bi) {
          const int k0 = kc + 16 * bi + 4 * g;
          if constexpr (RUN) {
            const float* up = ub + (cq[u] - kb_fast(kbf, k0) - 3);   // up[3 - r] = ub[bin(q, k0 + r)]
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float x = sa[u][bi][r] * sc2 + up[3 - r];
              sa[u][bi][r] = x;
              cmax = fmaxf(cmax, x);
            }
            continue;
          }
          const f32x4 ma = *(const f32x4*)(mrow + k0);
          int4 kbv;
          if (BIAS) kbv = *(const int4*)(kb + k0);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float x = sa[u][bi][r] * sc2 + ma[r];
            if (BIAS) x += ub[cq[u] - kbv[r]];
            sa[u][bi][r] = x;
            cmax = fmaxf(cmax, x);
          }
        }
        // lazy rescale (p.lazy > 0, CTCLIP_ATTN_LAZY, default 16): the running max only moves when
        // some lane's chunk max exceeds it by more than p.lazy (log2 units), so after the first
        // chunks the wave skips the alpha exp2, the lsum and the o rescale; probabilities stay <= 2^p.lazy (f32 sums,
        // bf16 P operands: no range issue), and lse = m + log2(lsum) is exact either way.
        // The test needs no cross-lane max: m[u] is equal on the 4 lanes of a query, so some
        // lane's PARTIAL max exceeds m + lazy iff the query's full chunk max does.  The two
        // lane ^ 16 / ^ 32 exchanges (LDS permutes on the chunk's critical path) run only on the
        // chunks that rescale; the rescaled max is the same full max as before (bit-identical).
        // m[u] == -inf (every key so far masked, e.g. a left-padded BERT mask): rescale, so the
        // exp2 below never sees -inf - -inf
        // (read back through an SGPR: the flag is wave-uniform, and as a VGPR condition hipcc
        // if-converts the branches below into per-element selects)
        rescale[u] = __builtin_amdgcn_readfirstlane(
            (int)(p.lazy <= 0.f || __any(cmax > m[u] + p.lazy || m[u] == -INFINITY)));
        float msafe;
        if (rescale[u]) {
          cmax = fmaxf(cmax, __shfl_xor(cmax, 16, 64));
          cmax = fmaxf(cmax, __shfl_xor(cmax, 32, 64));
          const float mnew = fmaxf(m[u], cmax);
          msafe = mnew == -INFINITY ? 0.f : mnew;
          alpha[u] = fexp2(m[u] - msafe);
          m[u] = mnew;
        } else {
          msafe = m[u];        // finite: m == -inf always takes the rescale branch
          alpha[u] = 1.f;
        }
        float psum = 0.f;
#pragma unroll
        for (int bi = 0; bi < 2; ++bi)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float e = fexp2(sa[u][bi][r] - msafe);
            sa[u][bi][r] = e;
            psum += e;
          }
        lsum[u] = rescale[u] ? lsum[u] * alpha[u] + psum : lsum[u] + psum;
        if constexpr (!BIAS) {
          if (p.drop_p > 0.f) {
#pragma unroll
            for (int bi = 0; bi < 2; ++bi)
#pragma unroll
              for (int r = 0; r < 4; ++r) sa[u][bi][r] *= drop_keep(p, s, h, q[u], kc + 16 * bi + 4 * g + r);
          }
        }
        pb[u] = pack_perm(sa[u][0], sa[u][1]);
      }
      // rescale the running outputs only on chunks where some query block moved its max (wave-
      // uniform; alpha = 1 for the others): the steady-state chunk skips the multiplies
      int anyr = 0;
#pragma unroll
      for (int u = 0; u < QB; ++u) anyr |= (int)rescale[u];
      if (__builtin_amdgcn_readfirstlane(anyr)) {
#pragma unroll
        for (int d = 0; d < DB; ++d)
#pragma unroll
          for (int u = 0; u < QB; ++u) o[u][d] *= alpha[u];
      }
#pragma unroll
      for (int d = 0; d < DB; ++d) {
        const bf16x8 vf = vfrag(Vimg, kc, d * 16);
#pragma unroll
        for (int u = 0; u < QB; ++u) o[u][d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pb[u], o[u][d], 0, 0, 0);
      }
    }
    }
#pragma unroll
    for (int u = 0; u < QB; ++u) {
      float ls = lsum[u];
      if constexpr (!CINIT) {
        ls += __shfl_xor(ls, 16, 64);
        ls += __shfl_xor(ls, 32, 64);
      }
      const float inv = ls > 0.f ? 1.f / ls : 0.f;
      if (qv[u]) {
#pragma unroll
        for (int d = 0; d < DB; ++d) {
          const float o4[4] = {o[u][d][0] * inv, o[u][d][1] * inv, o[u][d][2] * inv, o[u][d][3] * inv};
          const int64_t off = qrow[u] * p.ldout + h * D + d * 16 + 4 * g;
          if (p.out) *(uint2*)(p.out + off) = pack4(o4);   // (bf16 O optional: eval forward, round 6)
          if (p.out16) *(uint2*)(p.out16 + off) = pack4h(o4);
        }
        // natural-log LSE: ln(sum exp(x)) = (m2 + log2(lsum)) * ln 2
        if (g == 0 && p.lse) p.lse[(int64_t)h * p.M + qrow[u]] = ls > 0.f ? (m[u] + __log2f(ls)) * LN2 : INFINITY;
      }
    }
  }
}

// ------------------------------------------------------------------------------- backward dQ
// also writes delta = rowsum(dO * O); with BIAS, bins the bias gradient (LDS atomics; the
// spatial shapes use the frame-inner kernel below instead)
template <int D, bool BIAS>
__global__ __launch_bounds__(NT) void attn_bwd_dq_kernel(AP p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int KK = D / 32, DB = D / 16, RS = Img<D>::RS;
  const int L = p.L, Lp = (L + 31) & ~31;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wpp = NW / p.pp;
  const int pair_local = w / wpp, wi = w - pair_local * wpp;
  const int pair_bytes = 2 * Lp * RS;
  for (int pl = 0; pl < p.pp; ++pl) {
    const int pair = blockIdx.x * p.pp + pl;
    if (pair >= p.nseq * p.H) break;
    const int s = pair / p.H, h = pair - s * p.H;
    stage<D>(smem + pl * pair_bytes, p.k, p.ldk, p, s, h, Lp, tid, NT);
    stage<D>(smem + pl * pair_bytes + Lp * RS, p.v, p.ldv, p, s, h, Lp, tid, NT);
  }
  float* ub = nullptr;
  int* kb = nullptr;
  float* madd = nullptr;
  load_tables<BIAS>(p, smem + p.pp * pair_bytes, Lp, tid, blockIdx.x % p.H, ub, kb, madd);
  float* bins = madd + p.pp * Lp;
  if (BIAS)
    for (int i = tid; i < p.nbins; i += NT) bins[i] = 0.f;
  __syncthreads();
  const int pair = blockIdx.x * p.pp + pair_local;
  const bool active = pair < p.nseq * p.H;
  const int s = active ? pair / p.H : 0, h = active ? pair - s * p.H : 0;
  const char* Kimg = smem + pair_local * pair_bytes;
  const char* Vimg = Kimg + Lp * RS;
  const float* mrow = madd + pair_local * Lp;
  const int g = lane >> 4, li = lane & 15;
  const int nqb = active ? (L + 15) >> 4 : 0;
  const float sc2 = p.scale * LOG2E;
  for (int qb = wi; qb < nqb; qb += wpp) {
    const int q = qb * 16 + li;
    const bool qv = q < L;
    const int64_t qrow = qv ? seq_row(p, s, q) : 0;
    bf16x8 qf[KK], df[KK];
    float dl = 0.f;
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      if (qv) {
        qf[kk] = gload8(p.q + qrow * p.ldq + h * D + kk * 32 + 8 * g);
        df[kk] = gload8(p.dout + qrow * p.lddo + h * D + kk * 32 + 8 * g);
        const bf16x8 of = gload8(p.o + qrow * p.ldo + h * D + kk * 32 + 8 * g);
#pragma unroll
        for (int j = 0; j < 8; ++j) dl += (float)df[kk][j] * (float)of[j];
      } else {
        qf[kk] = zero8();
        df[kk] = zero8();
      }
    }
    dl += __shfl_xor(dl, 16, 64);
    dl += __shfl_xor(dl, 32, 64);
    const float lse2 = qv ? p.lse[(int64_t)h * p.M + qrow] * LOG2E : INFINITY;
    if (qv && g == 0) p.delta[(int64_t)h * p.M + qrow] = dl;
    const int cq = BIAS ? kb[min(q, L - 1)] + boff(p) : 0;
    f32x4 dq[DB];
#pragma unroll
    for (int d = 0; d < DB; ++d) dq[d] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int kc = 0; kc < Lp; kc += 32) {
      f32x4 sa[2], da[2];
#pragma unroll
      for (int bi = 0; bi < 2; ++bi) {
        sa[bi] = f32x4{0.f, 0.f, 0.f, 0.f};
        da[bi] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < KK; ++kk) {
          sa[bi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rowfrag<D>(Kimg, kc + 16 * bi, kk, lane), qf[kk], sa[bi], 0, 0, 0);
          da[bi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rowfrag<D>(Vimg, kc + 16 * bi, kk, lane), df[kk], da[bi], 0, 0, 0);
        }
      }
#pragma unroll
      for (int bi = 0; bi < 2; ++bi) {
        const int k0 = kc + 16 * bi + 4 * g;
        const f32x4 ma = *(const f32x4*)(mrow + k0);
        int4 kbv;
        if (BIAS) kbv = *(const int4*)(kb + k0);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float x = sa[bi][r] * sc2 + ma[r];
          if (BIAS) x += ub[cq - kbv[r]];
          float dp = da[bi][r];
          if constexpr (!BIAS) {
            if (p.drop_p > 0.f) dp *= drop_keep(p, s, h, q, k0 + r);
          }
          const float ds = fexp2(x - lse2) * (dp - dl);   // 0 for masked keys / padded queries
          if (BIAS && p.dbias_u && qv) atomicAdd(&bins[cq - kbv[r]], ds);
          sa[bi][r] = ds * p.scale;
        }
      }
      const bf16x8 dsb = pack_perm(sa[0], sa[1]);
#pragma unroll
      for (int d = 0; d < DB; ++d)
        dq[d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(trfrag<D>(Kimg, kc, d * 16, lane), dsb, dq[d], 0, 0, 0);
    }
    if (qv) {
#pragma unroll
      for (int d = 0; d < DB; ++d) {
        uint2 pk;
        pk.x = pack2(dq[d][0], dq[d][1]);
        pk.y = pack2(dq[d][2], dq[d][3]);
        *(uint2*)(p.dq + qrow * p.lddq + h * D + d * 16 + 4 * g) = pk;
      }
    }
  }
  if (BIAS && p.dbias_u) {
    __syncthreads();
    const int hh = blockIdx.x % p.H;
    for (int i = tid; i < p.nbins; i += NT) {
      const float v = bins[i];
      if (v != 0.f) atomicAdd(&p.dbias_u[(int64_t)hh * p.nbins + i], v);
    }
  }
}

// ----------------------------------------------------------------------------- backward dK dV
// lane owns a key; elements run over queries.  Padded queries carry lse = +inf (probability 0);
// a masked / padded key adds -inf through kadd.
// W waves per workgroup as in attn_fwd_kernel (12 for the spatial shapes: 3 key blocks per wave)
template <int D, bool BIAS, int W = (BIAS ? 12 : NW), bool RUN = false>
__global__ __launch_bounds__(W * 64) void attn_bwd_dkv_kernel(AP p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int KK = D / 32, DB = D / 16, RS = Img<D>::RS, NTH = W * 64;
  const int L = p.L, Lp = (L + 31) & ~31;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wpp = W / p.pp;
  const int pair_local = w / wpp, wi = w - pair_local * wpp;
  const int pair_bytes = 2 * Lp * RS + 2 * Lp * 4;
  for (int pl = 0; pl < p.pp; ++pl) {
    const int pair = blockIdx.x * p.pp + pl;
    if (pair >= p.nseq * p.H) break;
    const int s = pair / p.H, h = pair - s * p.H;
    char* base = smem + pl * pair_bytes;
    stage2<D, SU>(base, p.q, p.ldq, base + Lp * RS, p.dout, p.lddo, p, s, h, Lp, tid, NTH);
    float* ls = (float*)(base + 2 * Lp * RS);
    float* dls = ls + Lp;
    for (int i = tid; i < Lp; i += NTH) {
      const bool v = i < L;
      const int64_t r = v ? seq_row(p, s, i) : 0;
      ls[i] = v ? p.lse[(int64_t)h * p.M + r] * LOG2E : INFINITY;
      dls[i] = v ? p.delta[(int64_t)h * p.M + r] : 0.f;
    }
  }
  float* ub = nullptr;
  int* kb = nullptr;
  float* madd = nullptr;
  load_tables<BIAS, NTH>(p, smem + p.pp * pair_bytes, Lp, tid, blockIdx.x % p.H, ub, kb, madd);
  __syncthreads();
  const int pair = blockIdx.x * p.pp + pair_local;
  if (pair >= p.nseq * p.H) return;
  const int s = pair / p.H, h = pair - s * p.H;
  const char* Qimg = smem + pair_local * pair_bytes;
  const char* Dimg = Qimg + Lp * RS;
  const float* ls = (const float*)(Qimg + 2 * Lp * RS);
  const float* dls = ls + Lp;
  const int g = lane >> 4, li = lane & 15;
  const int nkb = (L + 15) >> 4;
  const float sc2 = p.scale * LOG2E;
  for (int kbk = wi; kbk < nkb; kbk += wpp) {
    const int key = kbk * 16 + li;
    const bool kin = key < L;
    const float kadd = madd[pair_local * Lp + key];
    const int64_t krow = kin ? seq_row(p, s, key) : 0;
    bf16x8 kf[KK], vf[KK];
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      kf[kk] = kin ? gload8(p.k + krow * p.ldk + h * D + kk * 32 + 8 * g) : zero8();
      vf[kk] = kin ? gload8(p.v + krow * p.ldv + h * D + kk * 32 + 8 * g) : zero8();
    }
    // bin(q, key) = kb[q] - ck
    const int ck = BIAS && kin ? kb[key] - boff(p) : 0;
    f32x4 dk[DB], dv[DB];
#pragma unroll
    for (int d = 0; d < DB; ++d) { dk[d] = f32x4{0.f, 0.f, 0.f, 0.f}; dv[d] = f32x4{0.f, 0.f, 0.f, 0.f}; }
    for (int qc = 0; qc < Lp; qc += 32) {
      f32x4 sa[2], da[2];
#pragma unroll
      for (int bi = 0; bi < 2; ++bi) {
        sa[bi] = f32x4{0.f, 0.f, 0.f, 0.f};
        da[bi] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < KK; ++kk) {
          sa[bi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rowfrag<D>(Qimg, qc + 16 * bi, kk, lane), kf[kk], sa[bi], 0, 0, 0);
          da[bi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rowfrag<D>(Dimg, qc + 16 * bi, kk, lane), vf[kk], da[bi], 0, 0, 0);
        }
      }
      // element (bi, r): query = qc + 16bi + 4g + r, key = this lane's key
#pragma unroll
      for (int bi = 0; bi < 2; ++bi) {
        const int q0 = qc + 16 * bi + 4 * g;
        const f32x4 lv = *(const f32x4*)(ls + q0);
        const f32x4 dlv = *(const f32x4*)(dls + q0);
        int4 qbv;
        const float* up = nullptr;
        if constexpr (RUN) up = ub + (kb[q0] - ck);   // up[r] = ub[bin(q0 + r, key)]
        else if (BIAS) qbv = *(const int4*)(kb + q0);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float x;
          if constexpr (RUN) x = sa[bi][r] * sc2 + up[r];
          else x = sa[bi][r] * sc2 + kadd;
          if (BIAS && !RUN) x += ub[qbv[r] - ck];
          const float pr = fexp2(x - lv[r]);
          float keep = 1.f;
          if constexpr (!BIAS) {
            if (p.drop_p > 0.f) keep = drop_keep(p, s, h, q0 + r, key);
          }
          const float ds = pr * (da[bi][r] * keep - dlv[r]);
          sa[bi][r] = pr * keep;
          da[bi][r] = ds * p.scale;
        }
      }
      const bf16x8 pa = pack_perm(sa[0], sa[1]);
      const bf16x8 dsa = pack_perm(da[0], da[1]);
#pragma unroll
      for (int d = 0; d < DB; ++d) {
        dv[d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, trfrag<D>(Dimg, qc, d * 16, lane), dv[d], 0, 0, 0);
        dk[d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(dsa, trfrag<D>(Qimg, qc, d * 16, lane), dk[d], 0, 0, 0);
      }
    }
    // C[key][d]: rows = keys kbk*16 + 4g + r, col = d*16 + li
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int kr = kbk * 16 + 4 * g + r;
      if (kr >= L) continue;
      const int64_t row = seq_row(p, s, kr);
#pragma unroll
      for (int d = 0; d < DB; ++d) {
        p.dk[row * p.lddk + h * D + d * 16 + li] = f2bf(dk[d][r]);
        p.dv[row * p.lddv + h * D + d * 16 + li] = f2bf(dv[d][r]);
      }
    }
  }
}

// ------------------------------------------------------------ backward dQ, biased (spatial) case
// The continuous-position bias is shared by every frame, so its gradient is a sum over all
// B*T frames of dS.  This kernel puts the FRAME loop innermost: a workgroup owns (head h,
// 64 queries, a chunk of frames); its 8 waves = 4 query sub-blocks x 2 key halves keep the
// frame-summed dS of their (16 queries x L/2 keys) tile in registers, and bin it to the
// (2gh-1)(2gw-1) offsets once at the end (LDS atomics, then one global atomic per bin).
// dQ of each frame is complete inside the workgroup (the two key halves meet in LDS).
template <int MAXCH, bool RUN = false>   // max 32-key chunks per key half; RUN as attn_fwd_kernel
__global__ __launch_bounds__(NT) void attn_bwd_dq_bias_kernel(AP p, int nfc) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int D = 32, RS = Img<D>::RS, DB = 2;
  const int L = p.L, Lp = (L + 31) & ~31, nc = Lp / 32, nc0 = (nc + 1) / 2;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int h = blockIdx.x, qg = blockIdx.y, fc = blockIdx.z;
  const int qsub = w & 3, khalf = w >> 2;
  const int c_begin = khalf ? nc0 : 0, c_end = khalf ? nc : nc0;
  char* Kimg = smem;
  char* Vimg = smem + Lp * RS;
  float* ub = (float*)(smem + 2 * Lp * RS);
  const int nb4 = (p.nbins + 3) & ~3;
  float* bins = ub + nb4;
  int* kb = (int*)(bins + nb4);
  float* madd = (float*)(kb + Lp);
  float* xch = madd + Lp;   // [4 waves][64 lanes][8] dq exchange
  for (int i = tid; i < p.nbins; i += NT) { ub[i] = p.bias_u[(int64_t)h * p.nbins + i] * LOG2E; bins[i] = 0.f; }
  for (int i = tid; i < Lp; i += NT) {
    kb[i] = i < L ? kb_of(p, i) : 0;
    madd[i] = i < L ? 0.f : -INFINITY;
  }
  const int g = lane >> 4, li = lane & 15;
  const int q = qg * 64 + qsub * 16 + li;
  const bool qv = q < L;
  const float sc2 = p.scale * LOG2E;
  f32x4 acc[MAXCH][2];
#pragma unroll
  for (int c = 0; c < MAXCH; ++c) { acc[c][0] = f32x4{0.f, 0.f, 0.f, 0.f}; acc[c][1] = f32x4{0.f, 0.f, 0.f, 0.f}; }
  const int f0 = (int)((int64_t)p.nseq * fc / nfc), f1 = (int)((int64_t)p.nseq * (fc + 1) / nfc);
  __syncthreads();
  const int cq = kb[min(q, L - 1)] + boff(p);
  for (int s = f0; s < f1; ++s) {
    __syncthreads();   // previous frame's LDS reads done
    stage2<D, SUB>(Kimg, p.k, p.ldk, Vimg, p.v, p.ldv, p, s, h, Lp, tid, NT);
    const int64_t qrow = qv ? seq_row(p, s, q) : 0;
    bf16x8 qf, df;
    float dl = 0.f;
    if (qv) {
      qf = gload8(p.q + qrow * p.ldq + h * D + 8 * g);
      df = gload8(p.dout + qrow * p.lddo + h * D + 8 * g);
      const bf16x8 of = gload8(p.o + qrow * p.ldo + h * D + 8 * g);
#pragma unroll
      for (int j = 0; j < 8; ++j) dl += (float)df[j] * (float)of[j];
    } else {
      qf = zero8();
      df = zero8();
    }
    dl += __shfl_xor(dl, 16, 64);
    dl += __shfl_xor(dl, 32, 64);
    const float lse2 = qv ? p.lse[(int64_t)h * p.M + qrow] * LOG2E : INFINITY;
    if (qv && g == 0 && khalf == 0) p.delta[(int64_t)h * p.M + qrow] = dl;
    __syncthreads();
    f32x4 dq[DB];
#pragma unroll
    for (int d = 0; d < DB; ++d) dq[d] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ci = 0; ci < MAXCH; ++ci) {
      const int c = c_begin + ci;
      if (c < c_end) {
        const int kc = c * 32;
        f32x4 sa[2], da[2];
#pragma unroll
        for (int bi = 0; bi < 2; ++bi) {
          sa[bi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rowfrag<D>(Kimg, kc + 16 * bi, 0, lane), qf,
                                                           f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
          da[bi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rowfrag<D>(Vimg, kc + 16 * bi, 0, lane), df,
                                                           f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        }
#pragma unroll
        for (int bi = 0; bi < 2; ++bi) {
          const int k0 = kc + 16 * bi + 4 * g;
          int4 kbv;
          f32x4 ma;
          const float* up = nullptr;
          if constexpr (RUN) {
            up = ub + (cq - kb[k0] - 3);   // up[3 - r] = ub[bin(q, k0 + r)]
          } else {
            kbv = *(const int4*)(kb + k0);
            ma = *(const f32x4*)(madd + k0);
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float x = RUN ? sa[bi][r] * sc2 + up[3 - r] : sa[bi][r] * sc2 + ma[r] + ub[cq - kbv[r]];
            const float ds = fexp2(x - lse2) * (da[bi][r] - dl);
            acc[ci][bi][r] += ds;
            sa[bi][r] = ds * p.scale;
          }
        }
        const bf16x8 dsb = pack_perm(sa[0], sa[1]);
#pragma unroll
        for (int d = 0; d < DB; ++d)
          dq[d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(trfrag<D>(Kimg, kc, d * 16, lane), dsb, dq[d], 0, 0, 0);
      }
    }
    // combine the two key halves of this frame's dQ
    if (khalf == 1) {
#pragma unroll
      for (int d = 0; d < DB; ++d)
#pragma unroll
        for (int r = 0; r < 4; ++r) xch[(qsub * 64 + lane) * 8 + d * 4 + r] = dq[d][r];
    }
    __syncthreads();
    if (khalf == 0 && qv) {
#pragma unroll
      for (int d = 0; d < DB; ++d) {
        f32x4 v = dq[d];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += xch[(qsub * 64 + lane) * 8 + d * 4 + r];
        uint2 pk;
        pk.x = pack2(v[0], v[1]);
        pk.y = pack2(v[2], v[3]);
        *(uint2*)(p.dq + qrow * p.lddq + h * D + d * 16 + 4 * g) = pk;
      }
    }
  }
  // bin the frame-summed dS once, without LDS float atomics (bit-reproducible): the 8 waves'
  // (16 queries x key half) tiles go to LDS one at a time, over the K / V images (free now:
  // 16 x 32 nc0 floats <= 2 Lp RS bytes), and each thread sums whole bins along their diagonals,
  // bin (dh, dw) += sum over the tile's queries q of dS[q][q - (dh, dw)], in a fixed order
  // (key half, query sub-block, query)
  {
    float* S = (float*)smem;
    const int LH = nc0 * 32;
    const int Wg = p.Wg, Hg = p.Hg, W2 = 2 * Wg - 1;
    for (int part = 0; part < 8; ++part) {
      const int ph = part >> 2, pq = part & 3;
      __syncthreads();   // every wave past its last K / V read (part 0) / the previous tile's sums
      if (khalf == ph && qsub == pq) {
#pragma unroll
        for (int ci = 0; ci < MAXCH; ++ci) {
          const int c = c_begin + ci;
          if (c < c_end) {
#pragma unroll
            for (int bi = 0; bi < 2; ++bi)
#pragma unroll
              for (int r = 0; r < 4; ++r) S[li * LH + (c - c_begin) * 32 + 16 * bi + 4 * g + r] = acc[ci][bi][r];
          }
        }
      }
      __syncthreads();
      const int k0 = ph * LH, k1 = min(L, k0 + LH);
      const int q0 = qg * 64 + pq * 16;
      for (int b = tid; b < p.nbins; b += NT) {
        const int dh = b / W2 - (Hg - 1), dw = b % W2 - (Wg - 1);
        float sum = 0.f;
        for (int j = 0; j < 16 && q0 + j < L; ++j) {
          const int qi = q0 + j, kh = qi / Wg - dh, kw = qi % Wg - dw;
          if (kh >= 0 && kh < Hg && kw >= 0 && kw < Wg) {
            const int key = kh * Wg + kw;
            if (key >= k0 && key < k1) sum += S[j * LH + key - k0];
          }
        }
        bins[b] += sum;
      }
    }
  }
  __syncthreads();
  for (int i = tid; i < p.nbins; i += NT) {
    const float v = bins[i];
    if (p.dbias_ws) p.dbias_ws[((int64_t)(qg * nfc + fc) * p.H + h) * p.nbins + i] = v;
    else if (v != 0.f) atomicAdd(&p.dbias_u[(int64_t)h * p.nbins + i], v);
  }
}

// ------------------------------------------ backward dQ, biased, base spatial shape (L = LF = 576)
// attn_bwd_dq_bias_kernel specialised to a full 24 x 24 grid (r02), same grid, LDS tables,
// bias-gradient binning and results (up to the summation order of the dQ parts):
//  * the NEXT frame's K / V land in a second LDS buffer by LDS-DMA (global_load_lds, 9 x 1 KB per
//    wave) while this frame computes: one counted wait + one barrier per frame, no staging
//    registers (the generic kernel waits on every frame's staging: 67 % of its wave cycles
//    parked in s_waitcnt / s_barrier, r02 PMC).  The images are unpadded 64-B rows with the 16-B
//    chunk XOR (row >> 1) & 3 (conflict-free for the ds_read_b128 row fragments and the
//    ds_read_b64_tr_b16 transposed ones: searched over the gfx950 lane groups);
//  * 8 waves = 4 query sub-blocks x 2 key halves of NC / 2 = 9 chunks, as the generic kernel, but
//    straight-line chunk code (254 VGPRs, no spills; 12 waves x 3 parts spill at the 168 cap);
//  * the dQ exchange of the key parts reuses the finished frame's buffer; the bias bins reuse
//    buffer 0 after the last frame.
// KP = 3 (12 waves, 6 chunks per key part, 48 accumulator registers instead of 72): 168 VGPRs +
// 140 B of scratch per lane whose per-frame reloads wait behind the LDS-DMA queue -- 887 vs 697 us
// per spatial backward (profiles/r05e_attn_kp_ab.log), so 8 waves stay
constexpr int DQD_W = 8, DQD_NT = DQD_W * 64, DQD_KP = 2;
// the spatial backward kernels fold each query's lse and delta into the score / dP MFMAs'
// accumulator inputs (one VALU subtraction per score and per dP less; round 5), 0 = subtract them
// per element (A/B build switch)
#ifndef CTCLIP_ATTN_CFOLD
#define CTCLIP_ATTN_CFOLD 1
#endif
// the same in the dQ kernel: its two constant accumulator inputs hold 8 more VGPRs across the frame
// loop at a 256-VGPR budget (scratch 40 -> 128 B per lane), so off
#ifndef CTCLIP_ATTN_CFOLD_DQ
#define CTCLIP_ATTN_CFOLD_DQ 0
#endif
// key positions of the bias reads: 1 = kb_fast (VALU), 0 = the LDS table (A/B build switch).
// Measured (profiles/r05d_attn_ab.log): the table, 699-705 us per spatial backward vs 718 for
// kb_fast, whose per-chunk VALU spills 40 -> 56 B per lane at this kernel's 256-VGPR budget
#ifndef CTCLIP_ATTN_DQ_KBFAST
#define CTCLIP_ATTN_DQ_KBFAST 0
#endif
// bias-gradient binning of the dQ kernel: 1 = diagonal sums over an LDS image of the block's
// frame-summed dS (no LDS float atomics); 0 = LDS atomics per (query, key) (A/B build switch).
// Measured (profiles/r02ba_attn_bin_ab.log): spatial backward 837 -> 807 us per layer; without
// any binning it would be 692 us -- the remainder is the 1,008 workgroups x 2,209 global atomics
#ifndef CTCLIP_ATTN_DIAG_BIN
#define CTCLIP_ATTN_DIAG_BIN 1
#endif
// round 6: the score MFMA's accumulator input is the CPB bias itself (the forward's C-init chain:
// reversed 1/scale table, one fma with the query's -lse per score instead of fma + sub)
#ifndef CTCLIP_ATTN_DQ_CINIT
#define CTCLIP_ATTN_DQ_CINIT 1
#endif
template <int LF, int KP = DQD_KP>
__global__ __launch_bounds__(4 * KP * 64) void attn_bwd_dq_bias_dma_kernel(AP p, int nfc) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int D = 32, DB = 2, L = LF, NC = L / 32, NCP = NC / KP, NW = 4 * KP, NTH = NW * 64;
  constexpr int IMG = L * 64, BUF = 2 * IMG, NG = BUF / 1024 / NW;   // glds per wave per frame
  static_assert(L % 64 == 0 && NC % KP == 0 && (BUF / 1024) % NW == 0 && (IMG / 1024) % NG == 0 &&
                (KP - 1) * 4 * 64 * 8 * 4 <= BUF, "full-shape specialisation");
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int h = blockIdx.x, qg = blockIdx.y, fc = blockIdx.z;
  const int qsub = w & 3, kpart = w >> 2;
  const int c_begin = kpart * NCP;
  float* ub = (float*)(smem + 2 * BUF);
  const int nb4 = (p.nbins + 3) & ~3;
  int* kb = (int*)(ub + nb4);
#if CTCLIP_ATTN_DQ_CINIT
  {
    const float isc = 1.f / p.scale;   // the forward's table (load_tables REV), bit for bit
    for (int i = tid; i < p.nbins; i += NTH) ub[i] = p.bias_u[(int64_t)h * p.nbins + p.nbins - 1 - i] * isc;
  }
#else
  for (int i = tid; i < p.nbins; i += NTH) ub[i] = p.bias_u[(int64_t)h * p.nbins + i] * LOG2E;
#endif
  for (int i = tid; i < L; i += NTH) kb[i] = kb_of(p, i);
  const int g = lane >> 4, li = lane & 15;
  const int q = qg * 64 + qsub * 16 + li;   // < L: L % 64 == 0
  const float sc2 = p.scale * LOG2E;
  f32x4 acc[NCP][2];
#pragma unroll
  for (int c = 0; c < NCP; ++c) { acc[c][0] = f32x4{0.f, 0.f, 0.f, 0.f}; acc[c][1] = f32x4{0.f, 0.f, 0.f, 0.f}; }
  const int f0 = (int)((int64_t)p.nseq * fc / nfc), f1 = (int)((int64_t)p.nseq * (fc + 1) / nfc);
  // LDS-DMA map: instruction j of wave w fills bytes [(w NG + j) KB, +1 KB) of a buffer, lane l the
  // 16 B at + 16 l: image (K below IMG, V above; wave-uniform), row, swizzled chunk
  auto stage_frame = [&](int s, int b) {
    const int64_t fb = (int64_t)s * p.s_outer;   // spatial: row(s, i) = s * s_outer + i (host-checked)
#pragma unroll
    for (int j = 0; j < NG; ++j) {
      const int pos = (w * NG + j) * 1024 + lane * 16;
      const bool isv = pos >= IMG;
      const int pi = isv ? pos - IMG : pos, row = pi >> 6, ch = ((pi >> 4) & 3) ^ kv_swz(row);
      const u16* src = isv ? p.v + (fb + row) * p.ldv : p.k + (fb + row) * p.ldk;
      glds16_asm(src + h * D + ch * 8, smem + b * BUF + (w * NG + j) * 1024);   // (common.h)
    }
  };
  // per-query operands of one frame (registers, loaded one frame ahead)
  bf16x8 qf = zero8(), df = zero8(), of = zero8();
  float lse2 = 0.f;
  auto load_q = [&](int s) {
    const int64_t qrow = (int64_t)s * p.s_outer + q;
    qf = gload8(p.q + qrow * p.ldq + h * D + 8 * g);
    df = gload8(p.dout + qrow * p.lddo + h * D + 8 * g);
    of = gload8(p.o + qrow * p.ldo + h * D + 8 * g);
    lse2 = p.lse[(int64_t)h * p.M + qrow];   // scaled after the frame's wait: a use here would
  };                                          // make the compiler drain the DMA queue (vmcnt(0))
  if (f0 < f1) {
    load_q(f0);
    stage_frame(f0, 0);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();   // tables (frame f0's DMA may still be in flight)
  __builtin_amdgcn_sched_barrier(0);
  const int cq = kb[q] + boff(p);
  [[maybe_unused]] const int cqr = p.nbins - 1 - cq;   // (C-init: reversed-table index of key 0)
  [[maybe_unused]] const KbFast kbf = kb_fast_init(p);
  for (int s = f0; s < f1; ++s) {
    const int b = (s - f0) & 1;
    const char* Kimg = smem + b * BUF;
    const char* Vimg = Kimg + IMG;
    // frame s landed (this wave's DMA), published by the barrier; the other buffer's last readers
    // (frame s - 1) all passed the previous frame's exchange barriers
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    // consume this frame's per-query registers BEFORE the next frame's loads are issued: hipcc
    // waits vmcnt(0) at the first use of an ordinary load result while LDS-DMA is outstanding
    bf16x8 qc = qf, dc = df;
    float l2 = lse2 * LOG2E;
    float dl = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) dl += (float)df[j] * (float)of[j];
    dl += __shfl_xor(dl, 16, 64);
    dl += __shfl_xor(dl, 32, 64);
    {
      typedef unsigned int v4u __attribute__((ext_vector_type(4)));
      v4u qv = __builtin_bit_cast(v4u, qc), dv = __builtin_bit_cast(v4u, dc);
      asm volatile("" : "+v"(qv), "+v"(dv), "+v"(l2), "+v"(dl));
      qc = __builtin_bit_cast(bf16x8, qv);
      dc = __builtin_bit_cast(bf16x8, dv);
    }
    const int64_t qrow = (int64_t)s * p.s_outer + q;
    if (g == 0 && kpart == 0) p.delta[(int64_t)h * p.M + qrow] = dl;
#if CTCLIP_ATTN_CFOLD_DQ
    // the query's lse and delta ride in the score / dP MFMAs' accumulator inputs (S^T layout: all 4
    // registers of a lane are its query): x - l2 = sc2 (q.k - lse / scale) + bias, dP - delta
    const float cl = -lse2 / p.scale;
    const f32x4 cS = f32x4{cl, cl, cl, cl}, cD = f32x4{-dl, -dl, -dl, -dl};
#else
    const f32x4 cS = f32x4{0.f, 0.f, 0.f, 0.f}, cD = cS;
#endif
    __builtin_amdgcn_sched_barrier(0);
    if (s + 1 < f1) {
      load_q(s + 1);
      stage_frame(s + 1, b ^ 1);
    }
    __builtin_amdgcn_sched_barrier(0);
    f32x4 dq[DB];
#pragma unroll
    for (int d = 0; d < DB; ++d) dq[d] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ci = 0; ci < NCP; ++ci) {
      const int kc = (c_begin + ci) * 32;
      f32x4 sa[2], da[2];
#if CTCLIP_ATTN_DQ_CINIT
      (void)cS;
      const float nl2 = -l2;
#pragma unroll
      for (int bi = 0; bi < 2; ++bi) {
        const float* up = ub + (kb[kc + 16 * bi + 4 * g] + cqr);   // up[r] = bias(q, k0 + r) / scale
        sa[bi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rowfrag_sw(Kimg, kc + 16 * bi, lane), qc,
                                                         f32x4{up[0], up[1], up[2], up[3]}, 0, 0, 0);
        da[bi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rowfrag_sw(Vimg, kc + 16 * bi, lane), dc, cD, 0, 0, 0);
      }
#pragma unroll
      for (int bi = 0; bi < 2; ++bi)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
#if CTCLIP_ATTN_CFOLD_DQ
          const float ds = fexp2(fmaf(sa[bi][r], sc2, nl2)) * da[bi][r];
#else
          const float ds = fexp2(fmaf(sa[bi][r], sc2, nl2)) * (da[bi][r] - dl);
#endif
          acc[ci][bi][r] += ds;
          sa[bi][r] = ds;
        }
#else
#pragma unroll
      for (int bi = 0; bi < 2; ++bi) {
        sa[bi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rowfrag_sw(Kimg, kc + 16 * bi, lane), qc, cS, 0, 0, 0);
        da[bi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rowfrag_sw(Vimg, kc + 16 * bi, lane), dc, cD, 0, 0, 0);
      }
#pragma unroll
      for (int bi = 0; bi < 2; ++bi) {
        int k0 = kc + 16 * bi + 4 * g;
#if CTCLIP_ATTN_DQ_KBFAST
        asm volatile("" : "+v"(k0));   // computed here, per chunk: hoisted out of the frame loop the
                                       // 18 positions spill
        // up[3 - r] = ub[bin(q, k0 + r)] (RUN); the key's position by VALU, not a table read the
        // bias read's address would wait on (a two-deep LDS chain per chunk)
        const float* up = ub + (cq - kb_fast(kbf, k0) - 3);
#else
        const float* up = ub + (cq - kb[k0] - 3);   // up[3 - r] = ub[bin(q, k0 + r)] (RUN)
#endif
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float x = sa[bi][r] * sc2 + up[3 - r];
#if CTCLIP_ATTN_CFOLD_DQ
          const float ds = fexp2(x) * da[bi][r];
#else
          const float ds = fexp2(x - l2) * (da[bi][r] - dl);
#endif
          acc[ci][bi][r] += ds;
          sa[bi][r] = ds;   // the score scale is applied once per dQ output below (exact for 8)
        }
      }
#endif
      const bf16x8 dsb = pack_perm(sa[0], sa[1]);
#pragma unroll
      for (int d = 0; d < DB; ++d)
        dq[d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(trfrag_sw(Kimg, kc, d * 16, lane), dsb, dq[d], 0, 0, 0);
    }
#pragma unroll
    for (int d = 0; d < DB; ++d) dq[d] *= p.scale;
    // combine the key parts of this frame's dQ through the finished buffer (after every wave's
    // last K / V read of it); part 0 sums and stores
    float* xch = (float*)(smem + b * BUF);   // [KP - 1][4 sub-blocks][64 lanes][8]
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (kpart > 0) {
#pragma unroll
      for (int d = 0; d < DB; ++d)
#pragma unroll
        for (int r = 0; r < 4; ++r) xch[(((kpart - 1) * 4 + qsub) * 64 + lane) * 8 + d * 4 + r] = dq[d][r];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (kpart == 0) {
#pragma unroll
      for (int d = 0; d < DB; ++d) {
        f32x4 v = dq[d];
#pragma unroll
        for (int pp = 0; pp < KP - 1; ++pp)
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] += xch[((pp * 4 + qsub) * 64 + lane) * 8 + d * 4 + r];
        uint2 pk;
        pk.x = pack2(v[0], v[1]);
        pk.y = pack2(v[2], v[3]);
        *(uint2*)(p.dq + qrow * p.lddq + h * D + d * 16 + 4 * g) = pk;
      }
    }
  }
  // bin the frame-summed dS once (bins in buffer 0: every wave is past its last read of it)
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();
#if CTCLIP_ATTN_DIAG_BIN
  // without LDS float atomics: the block's 64 x L frame-summed dS go to LDS (both K / V buffers,
  // free now: 64 x 576 x 4 B = 147,456 B = 2 BUF), then each thread sums whole bins along their
  // diagonals, bin (dh, dw) = sum over the 64 queries q of dS[q][q - (dh, dw)], in a fixed order
  {
    // rows padded to LP = L + 3 floats: the 16 query rows of a half-wave's stores land in distinct
    // banks (an L-float stride put all 16 in one); the image may run over the bias / position
    // tables after the frame buffers, which nothing reads any more
    constexpr int LP = L + 3;
    static_assert(64 * LP * 4 <= 2 * BUF + 4 * (2209 + 3) + 4 * L, "dS block fits the buffers and tables");
    float* S = (float*)smem;
    const int ql = qsub * 16 + li;
#pragma unroll
    for (int ci = 0; ci < NCP; ++ci)
#pragma unroll
      for (int bi = 0; bi < 2; ++bi)
#pragma unroll
        for (int r = 0; r < 4; ++r) S[ql * LP + (c_begin + ci) * 32 + 16 * bi + 4 * g + r] = acc[ci][bi][r];
    __syncthreads();
    const int Wg = p.Wg, Hg = p.Hg, W2 = 2 * Wg - 1, q0 = qg * 64;
    const int r_lo = q0 / Wg, r_hi = (q0 + 63) / Wg;
    for (int b = tid; b < p.nbins; b += NTH) {
      const int dh = b / W2 - (Hg - 1), dw = b % W2 - (Wg - 1);
      float sum = 0.f;
      // bin (dh, dw) = sum over the block's queries q = (qh, qw) of dS[q][(qh - dh, qw - dw)]: per
      // grid row of the block, the queries with an in-grid key are one qw run, and their entries
      // one diagonal of the image (stride LP + 1); q ascends as in the per-query walk it replaces
      // (same sum, same order: only the 3 / 4 of (query, bin) pairs without a key are skipped)
      for (int r = r_lo; r <= r_hi; ++r) {
        const int kh = r - dh;
        if (kh < 0 || kh >= Hg) continue;
        const int lo = max(max(q0 - r * Wg, 0), dw), hi = min(min(q0 + 63 - r * Wg, Wg - 1), Wg - 1 + dw);
        const float* sp = S + (r * Wg - q0) * LP + kh * Wg - dw;
        for (int qw = lo; qw <= hi; ++qw) sum += sp[qw * (LP + 1)];
      }
      if (p.dbias_ws) p.dbias_ws[((int64_t)(qg * nfc + fc) * p.H + h) * p.nbins + b] = sum;
      else if (sum != 0.f) atomicAdd(&p.dbias_u[(int64_t)h * p.nbins + b], sum);
    }
  }
#else
  float* bins = (float*)smem;
  for (int i = tid; i < p.nbins; i += NTH) bins[i] = 0.f;
  __syncthreads();
#ifndef CTCLIP_ATTN_NO_BIN   // diagnostic build only: skip the binning (wrong bias gradient) to time it
#pragma unroll
  for (int ci = 0; ci < NCP; ++ci)
#pragma unroll
    for (int bi = 0; bi < 2; ++bi)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = (c_begin + ci) * 32 + 16 * bi + 4 * g + r;
        atomicAdd(&bins[cq - kb[key]], acc[ci][bi][r]);
      }
#else
  if (acc[0][0][0] == 12345.f) bins[0] = 1.f;   // keep acc live
#endif
  __syncthreads();
  for (int i = tid; i < p.nbins; i += NTH) {
    const float v = bins[i];
    if (v != 0.f) atomicAdd(&p.dbias_u[(int64_t)h * p.nbins + i], v);
  }
#endif
}

// --------------------------------------------- backward dK dV, biased, base spatial shape (L = LF)
// attn_bwd_dkv_kernel<32, true, 12, true> made persistent over frames (r02): 32 workgroups per
// head walk frames s = blockIdx.x / H, + gridDim.x / H, ... with their head's bias table loaded
// once, and the NEXT frame's Q / dO rows (6 x 16 B per thread) and lse / delta are loaded into
// registers while this frame computes, then written to the LDS images behind one barrier (the
// per-pair kernel pays every (frame, head) pair's staging latency with nothing to overlap it:
// 1 workgroup per CU).  Each wave's K / V fragments of its next key block are loaded one block
// ahead.  The Q / dO images are unpadded 64-B rows with the dQ kernel's chunk swizzle (the
// padded 80-B rows conflict under gfx950's ds_read_b128 lane groups: 35 % of the per-pair
// kernel's LDS cycles, r02 PMC).  Same arithmetic and results as the per-pair kernel.
constexpr int DKP_W = 12, DKP_NT = DKP_W * 64;
template <int LF>
__global__ __launch_bounds__(DKP_NT) void attn_bwd_dkv_persist_kernel(AP p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int D = 32, DB = 2, RS = 64, W = DKP_W, NTH = DKP_NT, L = LF, CH = D / 8;
  constexpr int NLD = 2 * L * CH / NTH, RPU = NTH / CH, NKB = L / 16;
  static_assert((2 * L * CH) % NTH == 0 && L % 32 == 0 && L % 16 == 0 && (W * 64 / CH) % 16 == 0, "shape");
  const int tid = threadIdx.x, lane = tid & 63, wi = tid >> 6;
  const int h = blockIdx.x % p.H, wg = blockIdx.x / p.H, nwg = gridDim.x / p.H;
  char* Qimg = smem;
  char* Dimg = smem + L * RS;
  float* ls = (float*)(smem + 2 * L * RS);
  float* dls = ls + L;
  float* ub = dls + L;
  const int nb4 = (p.nbins + 3) & ~3;
  int* kb = (int*)(ub + nb4);
  for (int i = tid; i < p.nbins; i += NTH) ub[i] = p.bias_u[(int64_t)h * p.nbins + i] * LOG2E;
  for (int i = tid; i < L; i += NTH) kb[i] = kb_of(p, i);
  const int g = lane >> 4, li = lane & 15;
  const float sc2 = p.scale * LOG2E;
  const KbFast kbf = kb_fast_init(p);
  // staging map: chunk u of a thread is row R = tid / CH + RPU u of the stacked [Q; dO] image
  // (dO when R >= L: wave-uniform as 64 / CH rows per wave divide L), 16-B column tid % CH
  const int r0 = tid / CH, c0 = tid % CH;
  const int64_t offq = (int64_t)r0 * p.ldq + h * D + c0 * 8, offd = (int64_t)r0 * p.lddo + h * D + c0 * 8;
  u32x4 st[NLD];
  float lsv = 0.f, dlv = 0.f;   // this thread's lse / delta row (tid < L)
#define CT_DKV_LOAD(S_)                                                                          \
  do {                                                                                           \
    const int64_t fb_ = (int64_t)(S_) * p.s_outer;   /* row(s, i) = s * s_outer + i (host-checked) */ \
    _Pragma("unroll") for (int u = 0; u < NLD; ++u) {                                            \
      const bool isq = u * RPU + (wi * 64) / CH < L;                                             \
      const u16* src_ = isq ? p.q + (fb_ + u * RPU) * p.ldq + offq : p.dout + (fb_ + u * RPU - L) * p.lddo + offd; \
      st[u] = *(const u32x4*)src_;                                                               \
    }                                                                                            \
    if (tid < L) {                                                                               \
      lsv = p.lse[(int64_t)h * p.M + fb_ + tid];                                                 \
      dlv = p.delta[(int64_t)h * p.M + fb_ + tid];                                               \
    }                                                                                            \
  } while (0)
  int s = wg;
  if (s < p.nseq) CT_DKV_LOAD(s);
  for (; s < p.nseq; s += nwg) {
    __syncthreads();   // previous frame's LDS reads done (and, first time, the tables written)
#pragma unroll
    for (int u = 0; u < NLD; ++u) {
      const bool isq = u * RPU + (wi * 64) / CH < L;
      char* dst = isq ? Qimg + (u * RPU) * RS : Dimg + (u * RPU - L) * RS;
      *(u32x4*)(dst + r0 * RS + ((c0 ^ kv_swz(u * RPU + r0)) << 4)) = st[u];   // R = u RPU + r0, same swizzle for the dO part (L % 8 == 0)
    }
    if (tid < L) {
      ls[tid] = lsv * LOG2E;
      dls[tid] = dlv;
    }
    __syncthreads();
    if (s + nwg < p.nseq) CT_DKV_LOAD(s + nwg);   // in flight under this frame's key blocks
    const int64_t fb = (int64_t)s * p.s_outer;
    // K / V fragments one key block ahead
    bf16x8 kf = zero8(), vf = zero8();
    {
      const int64_t krow = fb + wi * 16 + li;
      kf = gload8(p.k + krow * p.ldk + h * D + 8 * g);
      vf = gload8(p.v + krow * p.ldv + h * D + 8 * g);
    }
    for (int kbk = wi; kbk < NKB; kbk += W) {
      const bf16x8 kc = kf, vc = vf;
      if (kbk + W < NKB) {
        const int64_t krow = fb + (kbk + W) * 16 + li;
        kf = gload8(p.k + krow * p.ldk + h * D + 8 * g);
        vf = gload8(p.v + krow * p.ldv + h * D + 8 * g);
      }
      const int key = kbk * 16 + li;
      const int ck = kb[key] - boff(p);   // bin(q, key) = kb[q] - ck
      f32x4 dk[DB], dv[DB];
#pragma unroll
      for (int d = 0; d < DB; ++d) { dk[d] = f32x4{0.f, 0.f, 0.f, 0.f}; dv[d] = f32x4{0.f, 0.f, 0.f, 0.f}; }
      for (int qc = 0; qc < L; qc += 32) {
        f32x4 sa[2], da[2];
#pragma unroll
        for (int bi = 0; bi < 2; ++bi) {
          sa[bi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rowfrag_sw(Qimg, qc + 16 * bi, lane), kc,
                                                           f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
          da[bi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rowfrag_sw(Dimg, qc + 16 * bi, lane), vc,
                                                           f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        }
#pragma unroll
        for (int bi = 0; bi < 2; ++bi) {
          const int q0 = qc + 16 * bi + 4 * g;
          const f32x4 lv = *(const f32x4*)(ls + q0);
          const f32x4 dlq = *(const f32x4*)(dls + q0);
          const float* up = ub + (kb_fast(kbf, q0) - ck);   // up[r] = ub[bin(q0 + r, key)]
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float x = sa[bi][r] * sc2 + up[r];
            const float pr = fexp2(x - lv[r]);
            const float ds = pr * (da[bi][r] - dlq[r]);
            sa[bi][r] = pr;
            da[bi][r] = ds;   // the score scale is applied once per dK output below (exact for 8)
          }
        }
        const bf16x8 pa = pack_perm(sa[0], sa[1]);
        const bf16x8 dsa = pack_perm(da[0], da[1]);
#pragma unroll
        for (int d = 0; d < DB; ++d) {
          dv[d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, trfrag_sw(Dimg, qc, d * 16, lane), dv[d], 0, 0, 0);
          dk[d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(dsa, trfrag_sw(Qimg, qc, d * 16, lane), dk[d], 0, 0, 0);
        }
      }
#pragma unroll
      for (int d = 0; d < DB; ++d) dk[d] *= p.scale;
      // C[key][d]: rows = keys kbk*16 + 4g + r, col = d*16 + li
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = fb + kbk * 16 + 4 * g + r;
#pragma unroll
        for (int d = 0; d < DB; ++d) {
          p.dk[row * p.lddk + h * D + d * 16 + li] = f2bf(dk[d][r]);
          p.dv[row * p.lddv + h * D + d * 16 + li] = f2bf(dv[d][r]);
        }
      }
    }
  }
}
#undef CT_DKV_LOAD

// --------------------------- backward dK dV, biased, base spatial shape, LDS-DMA staged (round 5)
// attn_bwd_dkv_persist_kernel with the next frame's Q / dO images landing in a second LDS buffer by
// LDS-DMA (6 x 1 KB per wave, the dQ kernel's swizzled 64-B rows) instead of through 6 x 16 B of
// staging registers per thread: at the 168-VGPR cap of 12 waves those registers went to scratch
// right after their loads (112 B per lane), so every frame's staging latency was paid in full.
// The frame's lse / delta still come through registers (2 floats per thread) into one LDS copy,
// written between two barriers.  The K / V fragments of a wave's next key block -- the next
// frame's first one during its last block -- are loaded one block ahead; their first use also
// drains the DMA queue (hipcc cannot see it), which gives the next frame's images one key block
// (of three) to land.  Same arithmetic and results as the persist kernel.
// LDS: 2 x (Q + dO) 147,456 + lse / delta 4,608 + bias 8,848 + positions 2,304 = 163,216 B.
constexpr int DKD_W = 12, DKD_NT = DKD_W * 64;
template <int LF>
__global__ __launch_bounds__(DKD_NT) void attn_bwd_dkv_dma_kernel(AP p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int D = 32, DB = 2, W = DKD_W, NTH = DKD_NT, L = LF, NKB = L / 16;
  constexpr int IMG = L * 64, BUF = 2 * IMG, NG = BUF / 1024 / W;   // 1-KB DMA rows per wave per frame
  static_assert(L % 32 == 0 && BUF % (1024 * W) == 0 && IMG % (1024 * NG) == 0 && NKB >= W, "full shape");
  const int tid = threadIdx.x, lane = tid & 63, wi = tid >> 6;
  const int h = blockIdx.x % p.H, wg = blockIdx.x / p.H, nwg = gridDim.x / p.H;
  float* ls = (float*)(smem + 2 * BUF);
  float* dls = ls + L;
  float* ub = dls + L;
  const int nb4 = (p.nbins + 3) & ~3;
  int* kb = (int*)(ub + nb4);
  for (int i = tid; i < p.nbins; i += NTH) ub[i] = p.bias_u[(int64_t)h * p.nbins + i] * LOG2E;
  for (int i = tid; i < L; i += NTH) kb[i] = kb_of(p, i);
  const int g = lane >> 4, li = lane & 15;
  const float sc2 = p.scale * LOG2E;
  const KbFast kbf = kb_fast_init(p);
  // DMA map: instruction j of wave wi fills bytes [(wi NG + j) KB, +1 KB) of a buffer (Q image below
  // IMG, dO above: wave-uniform), lane l the 16 B at + 16 l: row, swizzled chunk
  auto stage_frame = [&](int s, int b) {
    const int64_t fb = (int64_t)s * p.s_outer;   // spatial: row(s, i) = s * s_outer + i (host-checked)
#pragma unroll
    for (int j = 0; j < NG; ++j) {
      const int pos = (wi * NG + j) * 1024 + lane * 16;
      const bool isd = pos >= IMG;
      const int pi = isd ? pos - IMG : pos, row = pi >> 6, ch = ((pi >> 4) & 3) ^ kv_swz(row);
      const u16* src = isd ? p.dout + (fb + row) * p.lddo : p.q + (fb + row) * p.ldq;
      glds16_asm(src + h * D + ch * 8, smem + b * BUF + (wi * NG + j) * 1024);
    }
  };
  float lsv = 0.f, dlv = 0.f;   // this thread's lse / delta row of the next frame (tid < L)
  bf16x8 kf = zero8(), vf = zero8();
  auto load_kv = [&](int s, int kbk) {
    const int64_t krow = (int64_t)s * p.s_outer + kbk * 16 + li;
    kf = gload8(p.k + krow * p.ldk + h * D + 8 * g);
    vf = gload8(p.v + krow * p.ldv + h * D + 8 * g);
  };
  int s = wg;
  if (s < p.nseq) {
    stage_frame(s, 0);
    if (tid < L) {
      lsv = p.lse[(int64_t)h * p.M + (int64_t)s * p.s_outer + tid];
      dlv = p.delta[(int64_t)h * p.M + (int64_t)s * p.s_outer + tid];
    }
    load_kv(s, wi);
  }
  for (int it = 0; s < p.nseq; s += nwg, ++it) {
    const int b = it & 1;
    // this wave's DMA of frame s (and its lse / delta / first K V registers) landed; after the
    // barrier every wave's has, and every wave is past frame s - nwg (lse / delta copy and the
    // other buffer free)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid < L) {
#if CTCLIP_ATTN_CFOLD
      ls[tid] = -lsv / p.scale;   // the score MFMA's accumulator input: sc2 (q.k - lse / scale) = x - lse
      dls[tid] = -dlv;            // the dP MFMA's: dP - delta
#else
      ls[tid] = lsv * LOG2E;
      dls[tid] = dlv;
#endif
    }
    __syncthreads();
    const int sn = s + nwg;
    if (sn < p.nseq) {
      stage_frame(sn, b ^ 1);
      if (tid < L) {
        lsv = p.lse[(int64_t)h * p.M + (int64_t)sn * p.s_outer + tid];
        dlv = p.delta[(int64_t)h * p.M + (int64_t)sn * p.s_outer + tid];
      }
    }
    const char* Qimg = smem + b * BUF;
    const char* Dimg = Qimg + IMG;
    const int64_t fb = (int64_t)s * p.s_outer;
    for (int kbk = wi; kbk < NKB; kbk += W) {
      const bf16x8 kc = kf, vc = vf;
      if (kbk + W < NKB) load_kv(s, kbk + W);
      else if (sn < p.nseq) load_kv(sn, wi);
      const int key = kbk * 16 + li;
      const int ck = kb[key] - boff(p);   // bin(q, key) = kb[q] - ck
      f32x4 dk[DB], dv[DB];
#pragma unroll
      for (int d = 0; d < DB; ++d) { dk[d] = f32x4{0.f, 0.f, 0.f, 0.f}; dv[d] = f32x4{0.f, 0.f, 0.f, 0.f}; }
      for (int qc = 0; qc < L; qc += 32) {
        f32x4 sa[2], da[2];
#pragma unroll
        for (int bi = 0; bi < 2; ++bi) {
#if CTCLIP_ATTN_CFOLD
          // C[q][key], register r = query q0 + r: its -lse / scale and -delta as the accumulator inputs
          const int q0 = qc + 16 * bi + 4 * g;
          const f32x4 cS = *(const f32x4*)(ls + q0), cD = *(const f32x4*)(dls + q0);
#else
          const f32x4 cS = f32x4{0.f, 0.f, 0.f, 0.f}, cD = cS;
#endif
          sa[bi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rowfrag_sw(Qimg, qc + 16 * bi, lane), kc, cS, 0, 0, 0);
          da[bi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rowfrag_sw(Dimg, qc + 16 * bi, lane), vc, cD, 0, 0, 0);
        }
#pragma unroll
        for (int bi = 0; bi < 2; ++bi) {
          const int q0 = qc + 16 * bi + 4 * g;
#if !CTCLIP_ATTN_CFOLD
          const f32x4 lv = *(const f32x4*)(ls + q0);
          const f32x4 dlq = *(const f32x4*)(dls + q0);
#endif
          const float* up = ub + (kb_fast(kbf, q0) - ck);   // up[r] = ub[bin(q0 + r, key)]
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float x = sa[bi][r] * sc2 + up[r];
#if CTCLIP_ATTN_CFOLD
            const float pr = fexp2(x);
            const float ds = pr * da[bi][r];
#else
            const float pr = fexp2(x - lv[r]);
            const float ds = pr * (da[bi][r] - dlq[r]);
#endif
            sa[bi][r] = pr;
            da[bi][r] = ds;   // the score scale is applied once per dK output below (exact for 8)
          }
        }
        const bf16x8 pa = pack_perm(sa[0], sa[1]);
        const bf16x8 dsa = pack_perm(da[0], da[1]);
#pragma unroll
        for (int d = 0; d < DB; ++d) {
          dv[d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, trfrag_sw(Dimg, qc, d * 16, lane), dv[d], 0, 0, 0);
          dk[d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(dsa, trfrag_sw(Qimg, qc, d * 16, lane), dk[d], 0, 0, 0);
        }
      }
#pragma unroll
      for (int d = 0; d < DB; ++d) dk[d] *= p.scale;
      // C[key][d]: rows = keys kbk*16 + 4g + r, col = d*16 + li
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = fb + kbk * 16 + 4 * g + r;
#pragma unroll
        for (int d = 0; d < DB; ++d) {
          p.dk[row * p.lddk + h * D + d * 16 + li] = f2bf(dk[d][r]);
          p.dv[row * p.lddv + h * D + d * 16 + li] = f2bf(dv[d][r]);
        }
      }
    }
  }
}

bool s_attr = false;

template <int D, bool BIAS>
void set_attrs_b() {
  (void)hipFuncSetAttribute((const void*)attn_fwd_kernel<D, BIAS>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024);
  (void)hipFuncSetAttribute((const void*)attn_bwd_dq_kernel<D, BIAS>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024);
  (void)hipFuncSetAttribute((const void*)attn_bwd_dkv_kernel<D, BIAS>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024);
}

void set_attrs() {
  set_attrs_b<32, false>();
  set_attrs_b<32, true>();
  set_attrs_b<64, false>();
  set_attrs_b<64, true>();
  (void)hipFuncSetAttribute((const void*)attn_bwd_dq_bias_kernel<9>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024);
  (void)hipFuncSetAttribute((const void*)attn_bwd_dq_bias_kernel<9, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024);
  (void)hipFuncSetAttribute((const void*)attn_bwd_dq_bias_dma_kernel<576>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  (void)hipFuncSetAttribute((const void*)attn_bwd_dkv_persist_kernel<576>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  (void)hipFuncSetAttribute((const void*)attn_bwd_dkv_dma_kernel<576>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  (void)hipFuncSetAttribute((const void*)attn_fwd_kernel<32, true, 12, true>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  (void)hipFuncSetAttribute((const void*)attn_fwd_kernel<32, true, 12, true, 2>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  (void)hipFuncSetAttribute((const void*)attn_fwd_kernel<32, true, 12, true, 3>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  (void)hipFuncSetAttribute((const void*)attn_fwd_kernel<32, true, 12, true, 3, true>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  (void)hipFuncSetAttribute((const void*)attn_fwd_kernel<32, true, 12, true, 3, false, true>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  (void)hipFuncSetAttribute((const void*)attn_bwd_dkv_kernel<32, true, 12, true>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
}

// bias shapes whose 4-key / 4-query MFMA groups never straddle a grid row and have no padding
bool run_ok(const AP& p) { return p.bias_u && p.Wg % 4 == 0 && p.L % 32 == 0; }

int fill(AP& p, const ctclip_attn_args* a) {
  if (a->D != 32 && a->D != 64) return CT_ESHAPE;
  if (a->L <= 0 || a->L > 1024) return CT_ESHAPE;
  p.q = (const u16*)a->q; p.ldq = a->ldq;
  p.k = (const u16*)a->k; p.ldk = a->ldk;
  p.v = (const u16*)a->v; p.ldv = a->ldv;
  p.o = (const u16*)a->o; p.ldo = a->ldo;
  p.out = (u16*)a->o; p.ldout = a->ldo;
  p.out16 = (u16*)a->o16;
  p.dout = (const u16*)a->dout; p.lddo = a->lddo;
  p.dq = (u16*)a->dq; p.lddq = a->lddq;
  p.dk = (u16*)a->dk; p.lddk = a->lddk;
  p.dv = (u16*)a->dv; p.lddv = a->lddv;
  p.lse = a->lse; p.delta = a->delta;
  p.bias_u = a->bias_u; p.dbias_u = a->dbias_u;
  p.dbias_ws = a->dbias_ws;
  p.kmask = a->kmask;
  p.scale = a->scale;
  p.drop_p = a->dropout_p;
  if (!(p.drop_p >= 0.f && p.drop_p < 1.f)) return CT_EINVAL;
  if (p.drop_p > 0.f && a->bias_u) return CT_EINVAL;            // BERT path only
  p.drop_scale = p.drop_p > 0.f ? 1.f / (1.f - p.drop_p) : 1.f;
  p.thresh = (unsigned)std::min(4294967295.0, (double)p.drop_p * 4294967296.0);
  p.seed = a->dropout_seed;
  static const float lazy = [] { const char* e = getenv("CTCLIP_ATTN_LAZY"); return e ? (float)atof(e) : 16.f; }();
  p.lazy = lazy;
  p.L = a->L; p.H = a->H; p.nseq = a->nseq; p.M = a->M;
  p.Hg = a->grid_h; p.Wg = a->grid_w;
  p.nbins = (2 * a->grid_h - 1) * (2 * a->grid_w - 1);
  p.n_inner = a->n_inner > 0 ? a->n_inner : 1;
  p.s_outer = a->s_outer; p.s_inner = a->s_inner; p.s_pos = a->s_pos;
  if (p.bias_u && (a->grid_w <= 0 || a->grid_h * a->grid_w != a->L)) return CT_ESHAPE;
  // every kernel moves 8 head-dim elements per lane access (16 B): rows 16-B aligned
  auto a16 = [](const void* x, int64_t ld) { return ((uintptr_t)x & 15) == 0 && ld % 8 == 0; };
  if (!(a16(a->q, a->ldq) && a16(a->k, a->ldk) && a16(a->v, a->ldv) && a16(a->o, a->ldo) && a16(a->o16, a->ldo) &&
        a16(a->dout, a->lddo) && a16(a->dq, a->lddq) && a16(a->dk, a->lddk) && a16(a->dv, a->lddv)))
    return CT_EALIGN;
  // pairs per workgroup: enough (seq, head) pairs that every wave has query blocks
  const int nqb = (a->L + 15) / 16;
  int pp = NW / std::max(1, std::min(NW, nqb));
  while (NW % pp) --pp;
  if (p.bias_u) pp = 1;
  p.pp = pp;
  return 0;
}

// LDS bytes of the tables after the images: [BIAS: ub + kb] + madd[pp][Lp] (+ bins for dq)
size_t table_bytes(const AP& p, int Lp, bool bins) {
  size_t b = (size_t)p.pp * Lp * 4;
  const size_t nb4 = (size_t)((p.nbins + 3) & ~3);
  if (p.bias_u) b += nb4 * 4 + (size_t)Lp * 4 + (bins ? nb4 * 4 : 0);
  return b;
}

int g_fwd_qb = -1;
// static-bound softmax in the QB = 3 forward (CTCLIP_ATTN_FWD_SMAX=1): measured SLOWER at the base
// shape, 254 vs 235 us per layer (profiles/r03d_attnsmax_ab.log) -- its per-workgroup prologue (the
// key norms and bias-table range over 576 rows + 2,209 bins, a block reduction and a barrier for
// each of 1,536 workgroups) costs more than the per-chunk max / rescale it removes -- so off
int g_fwd_smax = -1;
// the C-init score chain (attn_fwd_kernel CINIT; CTCLIP_ATTN_FWD_CINIT=0 restores the round-5 kernel)
int g_fwd_cinit = -1;

template <int D>
void launch_fwd(const AP& p, dim3 grid, size_t lds, hipStream_t st) {
  if constexpr (D == 32) {
    if (run_ok(p)) {
      // query blocks processed together per wave (1 = the r02 kernel): CTCLIP_ATTN_FWD_QB or
      // ctclip_attn_set_fwd_qb (A/B, bit-identical results)
      if (g_fwd_qb < 0) { const char* e = getenv("CTCLIP_ATTN_FWD_QB"); g_fwd_qb = e ? atoi(e) : 3; }
      const int qb = g_fwd_qb;
      if (g_fwd_smax < 0) { const char* e = getenv("CTCLIP_ATTN_FWD_SMAX"); g_fwd_smax = e ? atoi(e) != 0 : 0; }
      if (g_fwd_cinit < 0) { const char* e = getenv("CTCLIP_ATTN_FWD_CINIT"); g_fwd_cinit = e ? atoi(e) != 0 : 1; }
      if (qb == 3 && g_fwd_smax)
        hipLaunchKernelGGL((attn_fwd_kernel<D, true, 12, true, 3, true>), grid, dim3(12 * 64), lds, st, p);
      else if (qb == 3 && g_fwd_cinit)
        hipLaunchKernelGGL((attn_fwd_kernel<D, true, 12, true, 3, false, true>), grid, dim3(12 * 64), lds, st, p);
      else if (qb == 3) hipLaunchKernelGGL((attn_fwd_kernel<D, true, 12, true, 3>), grid, dim3(12 * 64), lds, st, p);
      else if (qb == 2) hipLaunchKernelGGL((attn_fwd_kernel<D, true, 12, true, 2>), grid, dim3(12 * 64), lds, st, p);
      else hipLaunchKernelGGL((attn_fwd_kernel<D, true, 12, true>), grid, dim3(12 * 64), lds, st, p);
      return;
    }
  }
  if (p.bias_u) hipLaunchKernelGGL((attn_fwd_kernel<D, true>), grid, dim3(12 * 64), lds, st, p);
  else hipLaunchKernelGGL((attn_fwd_kernel<D, false>), grid, dim3(NT), lds, st, p);
}

template <int D>
void launch_dq(const AP& p, dim3 grid, size_t lds, hipStream_t st) {
  if (p.bias_u) hipLaunchKernelGGL((attn_bwd_dq_kernel<D, true>), grid, dim3(NT), lds, st, p);
  else hipLaunchKernelGGL((attn_bwd_dq_kernel<D, false>), grid, dim3(NT), lds, st, p);
}

template <int D>
void launch_dkv(const AP& p, dim3 grid, size_t lds, hipStream_t st) {
  if constexpr (D == 32) {
    static int persist = -1;   // CTCLIP_ATTN_DKV_PERSIST=0: the per-pair kernel (A/B)
    if (persist < 0) { const char* e = getenv("CTCLIP_ATTN_DKV_PERSIST"); persist = e ? atoi(e) != 0 : 1; }
    if (persist && run_ok(p) && p.L == 576 && p.s_pos == 1 && p.n_inner == 1 && p.pp == 1 && !p.kmask &&
        p.nseq >= 2 && 256 % p.H == 0) {
      const int per_head = std::min(p.nseq, 256 / p.H);
      // LDS-DMA staged variant (CTCLIP_ATTN_DKV_DMA=0: the register-staged persist kernel; A/B)
      static int dma = -1;
      if (dma < 0) { const char* e = getenv("CTCLIP_ATTN_DKV_DMA"); dma = e ? atoi(e) != 0 : 1; }
      const size_t lds_d = (size_t)4 * 576 * 64 + 2 * 576 * 4 + (size_t)((p.nbins + 3) & ~3) * 4 + 576 * 4;
      if (dma && lds_d <= 160 * 1024) {
        hipLaunchKernelGGL((attn_bwd_dkv_dma_kernel<576>), dim3(per_head * p.H), dim3(DKD_NT), lds_d, st, p);
        return;
      }
      const size_t lds_p = (size_t)2 * 576 * 64 + 2 * 576 * 4 + (size_t)((p.nbins + 3) & ~3) * 4 + 576 * 4;
      if (lds_p <= 160 * 1024) {
        hipLaunchKernelGGL((attn_bwd_dkv_persist_kernel<576>), dim3(per_head * p.H), dim3(DKP_NT), lds_p, st, p);
        return;
      }
    }
    if (run_ok(p)) {
      hipLaunchKernelGGL((attn_bwd_dkv_kernel<D, true, 12, true>), grid, dim3(12 * 64), lds, st, p);
      return;
    }
  }
  if (p.bias_u) hipLaunchKernelGGL((attn_bwd_dkv_kernel<D, true>), grid, dim3(12 * 64), lds, st, p);
  else hipLaunchKernelGGL((attn_bwd_dkv_kernel<D, false>), grid, dim3(NT), lds, st, p);
}


// ---------------------------------------------------------------------------------------------
// Short sequences (L <= 32, head dim 32, no bias / key mask): the temporal transformer's
// attention (24 frames per (b, h, w) sequence).  One WAVE per (sequence, head) holds the whole
// problem: Q, K, V (and dO, O) of the pair are read once as MFMA row fragments (32 rows,
// zero past L) and every product is a single 32-deep MFMA block set -- no online softmax, no key
// loop.  The backward is fused (dQ, dK, dV in one pass, no delta pre-pass): it computes the
// scores twice, in S^T layout (lane = query: P^T, dP^T, dS^T feed dQ^T = K^T dS^T) and in S
// layout (lane = key: P, dP, dS feed dV^T = dO^T P and dK^T = Q^T dS), so every MFMA operand is
// a row fragment (loaded straight from HBM in MFMA operand layout) or a ds_read_b64_tr_b16 column
// fragment of a wave-private LDS image, and the accumulators are consumed where they lie.  Four
// waves (four heads of one sequence) per workgroup.
constexpr int SW = 4;                          // waves per workgroup
constexpr int SIMG = 32 * Img<32>::RS;         // one 32 x 32 bf16 image (2,560 B)

__device__ __forceinline__ void wave_lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

// A lane's two token rows 16u + (lane & 15) of sequence s: every load and store of the pair (Q, K,
// V, dO, O, lse; O, dQ, dK, dV) touches only these.  The sequence base is wave-uniform (s derives
// from a readfirstlane'd wave index, so its division and products run on the scalar unit); the
// per-tensor offsets are 32 x 32 -> 64-bit products (small_ok: M and every ld < 2^31).  Written
// per call, seq_row's division by n_inner and its int64 products had made both kernels VALU-issue
// bound (895 / 1,564 VALU instructions per wave, 13 / 21 of them integer divisions).
struct SmallRows {
  unsigned row[2];
  bool ok[2];
};
__device__ __forceinline__ SmallRows small_rows(const AP& p, int s, int lane) {
  const unsigned base = (unsigned)seq_row(p, s, 0);
  const unsigned sp = (unsigned)p.s_pos;
  SmallRows R;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int r = 16 * u + (lane & 15);
    R.ok[u] = r < p.L;
    R.row[u] = base + (unsigned)r * sp;
  }
  return R;
}
__device__ __forceinline__ uint64_t roff(unsigned row, int64_t ld) { return (uint64_t)row * (unsigned)ld; }

// row fragments of rows 16u + (lane & 15), d chunk lane >> 4 (zero past L): exactly the MFMA
// operand layout of rowfrag(), read straight from HBM (16 B per lane per block)
__device__ __forceinline__ void load_rows(bf16x8 (&f)[2], const u16* x, int64_t ld, const SmallRows& R, int h,
                                          int lane) {
#pragma unroll
  for (int u = 0; u < 2; ++u) f[u] = R.ok[u] ? gload8(x + roff(R.row[u], ld) + h * 32 + 8 * (lane >> 4)) : zero8();
}

// the same fragments into a wave-private image for the trfrag column reads, its d columns
// interleaved in 4-element chunks: image columns 0-15 hold d = 8c + 0..3 and columns 16-31
// d = 8c + 4..7 (c = 0..3).  An MFMA pair over the two column blocks (rows 4g + r of each) then
// leaves lane group g holding d = 8g .. 8g + 7 of its token row, stored as ONE 16-B piece per lane:
// 64 contiguous bytes per row per instruction instead of two 32-B halves in two instructions (the
// partial-line stores had bound the kernels: the forward's fp16 copy of O alone cost 44 -> 87 us).
__device__ __forceinline__ void put_rows(char* img, const bf16x8 (&f)[2], int lane) {
  const int g = lane >> 4;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    char* row = img + (16 * u + (lane & 15)) * Img<32>::RS;
    const u32x4 v = __builtin_bit_cast(u32x4, f[u]);
    *(uint2*)(row + 8 * g) = make_uint2(v.x, v.y);           // d 8g .. 8g + 3   -> column 4g
    *(uint2*)(row + 32 + 8 * g) = make_uint2(v.z, v.w);      // d 8g + 4 .. + 7 -> column 16 + 4g
  }
}
__device__ __forceinline__ void cat8(float (&o)[8], const f32x4& a, const f32x4& b, float sc) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    o[r] = a[r] * sc;
    o[4 + r] = b[r] * sc;
  }
}

// COOP (H % SW == 0: a workgroup's four waves are four adjacent heads of ONE sequence): O and its
// fp16 copy are staged in LDS tiles [32 rows][4 heads x 64 B] (over the V images) and stored by the
// whole workgroup, 256 contiguous bytes of a token row per 16 lanes (two full 128-B lines), instead
// of each wave storing 64-B halves of 16 rows per instruction.
constexpr int SRS = 4 * 64 + 16;               // staging row stride (four heads + 16-B pad)
constexpr size_t small_fwd_lds(bool coop) { return coop ? 2 * 32 * SRS : SW * SIMG; }

__device__ __forceinline__ void coop_store_rows(u16* dst, int64_t ld, const char* tile, const AP& p, int s, int h0) {
  const unsigned base = (unsigned)seq_row(p, s, 0), sp = (unsigned)p.s_pos;
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    const int idx = pass * SW * 64 + threadIdx.x, row = idx >> 4, c = idx & 15;
    if (row < p.L)
      *(u32x4*)(dst + roff(base + (unsigned)row * sp, ld) + h0 * 32 + c * 8) = *(const u32x4*)(tile + row * SRS + c * 16);
  }
}

template <bool COOP>
__global__ __launch_bounds__(SW * 64) void attn_small_fwd_kernel(AP p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int pair = blockIdx.x * SW + w;
  if (pair >= p.nseq * p.H) return;            // wave-uniform (never taken when COOP: no partial workgroups)
  const int s = pair / p.H, h = pair - s * p.H;
  char* Vi = smem + w * SIMG;
  const SmallRows R = small_rows(p, s, lane);
  bf16x8 qr[2], kr[2], vr[2];
  load_rows(qr, p.q, p.ldq, R, h, lane);
  load_rows(kr, p.k, p.ldk, R, h, lane);
  load_rows(vr, p.v, p.ldv, R, h, lane);
  put_rows(Vi, vr, lane);
  const int g = lane >> 4;                      // (query 16qb + (lane & 15): the lane's row qb)
  const float c2 = p.scale * LOG2E;
  const f32x4 z4 = f32x4{0.f, 0.f, 0.f, 0.f};
  // S^T blocks (key block kb, query block qb): lane column = query 16qb + i, rows = keys 16kb + 4g + r
  f32x4 st[2][2];
#pragma unroll
  for (int qb = 0; qb < 2; ++qb)
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) st[kb][qb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kr[kb], qr[qb], z4, 0, 0, 0);
  wave_lds_sync();
  // V^T column fragments (image column block db: d = 8 (i / 4) + 4 db + i % 4), keys 4g + 0..3 and
  // 16 + 4g + 0..3
  const bf16x8 vt[2] = {trfrag<32>(Vi, 0, 0, lane), trfrag<32>(Vi, 0, 16, lane)};
  u32x4 ob[2], hb[2];
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    float m = -INFINITY;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float x = (16 * kb + 4 * g + r < p.L) ? st[kb][qb][r] * c2 : -INFINITY;
        st[kb][qb][r] = x;
        m = fmaxf(m, x);
      }
    m = fmaxf(m, __shfl_xor(m, 16, 64));
    m = fmaxf(m, __shfl_xor(m, 32, 64));
    float l = 0.f;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float e = fexp2(st[kb][qb][r] - m);
        st[kb][qb][r] = e;
        l += e;
      }
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
    const bf16x8 pf = pack_perm(st[0][qb], st[1][qb]);       // P^T: keys in the trfrag order
    const float inv = 1.f / l;
    // O^T blocks: lane column = query 16 qb + i (the lane's row qb), rows d = 8g + 4db + r
    const f32x4 o0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vt[0], pf, z4, 0, 0, 0);
    const f32x4 o1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vt[1], pf, z4, 0, 0, 0);
    float o8[8];
    cat8(o8, o0, o1, inv);
    if constexpr (COOP) {
      ob[qb] = pack8(o8);
      if (p.out16) hb[qb] = pack8h(o8);
    } else if (R.ok[qb]) {
      const uint64_t off = roff(R.row[qb], p.ldout) + h * 32 + 8 * g;
      if (p.out) *(u32x4*)(p.out + off) = pack8(o8);
      if (p.out16) *(u32x4*)(p.out16 + off) = pack8h(o8);
    }
    if (g == 0 && R.ok[qb] && p.lse) p.lse[(int64_t)h * p.M + R.row[qb]] = (m + __log2f(l)) * LN2;
  }
  if constexpr (COOP) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();                            // every wave is past its V^T reads (the tiles overlay them)
    char* t0 = smem;
    char* t1 = smem + 32 * SRS;
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
      const int row = 16 * qb + (lane & 15);
      *(u32x4*)(t0 + row * SRS + w * 64 + g * 16) = ob[qb];
      if (p.out16) *(u32x4*)(t1 + row * SRS + w * 64 + g * 16) = hb[qb];
    }
    __syncthreads();
    if (p.out) coop_store_rows(p.out, p.ldout, t0, p, s, h - w);
    if (p.out16) coop_store_rows(p.out16, p.ldout, t1, p, s, h - w);
  }
}

// per-wave staging areas -> workgroup stores: 16 threads per token row, head c / 4 from wave c / 4's
// area at byte offset off0 (rows of Img<32>::RS bytes, 16-B chunk c % 4)
__device__ __forceinline__ void coop_store_areas(u16* dst, int64_t ld, const char* smem, int wstride, int off0,
                                                 const AP& p, int s, int h0) {
  const unsigned base = (unsigned)seq_row(p, s, 0), sp = (unsigned)p.s_pos;
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    const int idx = pass * SW * 64 + threadIdx.x, row = idx >> 4, c = idx & 15;
    if (row < p.L)
      *(u32x4*)(dst + roff(base + (unsigned)row * sp, ld) + h0 * 32 + c * 8) =
          *(const u32x4*)(smem + (c >> 2) * wstride + off0 + row * Img<32>::RS + (c & 3) * 16);
  }
}

template <bool COOP>   // as attn_small_fwd_kernel: each wave stages dQ / dK / dV in its own K / Q / dO
                       // image once it has read it, and the workgroup stores whole token rows
__global__ __launch_bounds__(SW * 64) __attribute__((amdgpu_waves_per_eu(5, 8))) void attn_small_bwd_kernel(AP p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int pair = blockIdx.x * SW + w;
  if (pair >= p.nseq * p.H) return;
  const int s = pair / p.H, h = pair - s * p.H;
  const SmallRows R = small_rows(p, s, lane);
  char* Qi = smem + w * (3 * SIMG + 256);
  char* Ki = Qi + SIMG;
  char* Di = Ki + SIMG;                         // dO
  float* lse2 = (float*)(Di + SIMG);            // [32] lse * log2 e (+inf past L)
  float* dlt = lse2 + 32;                       // [32] delta = rowsum(dO * O)
  const int i = lane & 15, g = lane >> 4;
  bf16x8 qr[2], kr[2], vr[2], dr[2], orr[2];
  load_rows(qr, p.q, p.ldq, R, h, lane);
  load_rows(kr, p.k, p.ldk, R, h, lane);
  load_rows(vr, p.v, p.ldv, R, h, lane);
  load_rows(dr, p.dout, p.lddo, R, h, lane);
  load_rows(orr, p.o, p.ldo, R, h, lane);
  float lq[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) lq[u] = R.ok[u] ? p.lse[(int64_t)h * p.M + R.row[u]] * LOG2E : INFINITY;
  put_rows(Qi, qr, lane);
  put_rows(Ki, kr, lane);
  put_rows(Di, dr, lane);
  // delta per query row 16u + i: partial dot of this lane's 8 d, summed over the 4 chunks g
  float dq[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    float dd = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) dd += (float)orr[u][e] * (float)dr[u][e];
    dd += __shfl_xor(dd, 16, 64);
    dd += __shfl_xor(dd, 32, 64);
    dq[u] = dd;
    if (g == 0) {
      dlt[16 * u + i] = dd;
      lse2[16 * u + i] = lq[u];
    }
  }
  const float c2 = p.scale * LOG2E;
  const f32x4 z4 = f32x4{0.f, 0.f, 0.f, 0.f};
  // ---- S^T layout (lane = query): dQ^T[d][q] = scale * sum_k K^T[d][k] dS^T[k][q]
  bf16x8 dsf[2];
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    f32x4 ds[2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      const f32x4 sv = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kr[kb], qr[qb], z4, 0, 0, 0);
      const f32x4 dp = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vr[kb], dr[qb], z4, 0, 0, 0);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const bool kv = 16 * kb + 4 * g + r < p.L;
        const float pr = kv ? fexp2(sv[r] * c2 - lq[qb]) : 0.f;   // 0 for padded queries (lq = +inf)
        ds[kb][r] = pr * (dp[r] - dq[qb]);
      }
    }
    dsf[qb] = pack_perm(ds[0], ds[1]);
  }
  wave_lds_sync();
  const bf16x8 kt0 = trfrag<32>(Ki, 0, 0, lane), kt1 = trfrag<32>(Ki, 0, 16, lane);
  // COOP: the dO^T and Q^T column fragments (the same for both key blocks) read up front, so all
  // three images are free for staging
  bf16x8 dt[2], qt[2];
  if constexpr (COOP) {
    dt[0] = trfrag<32>(Di, 0, 0, lane); dt[1] = trfrag<32>(Di, 0, 16, lane);
    qt[0] = trfrag<32>(Qi, 0, 0, lane); qt[1] = trfrag<32>(Qi, 0, 16, lane);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    // dQ^T blocks, rows d = 8g + 4db + r (interleaved images), column = query 16 qb + i
    const f32x4 a0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kt0, dsf[qb], z4, 0, 0, 0);
    const f32x4 a1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kt1, dsf[qb], z4, 0, 0, 0);
    float d8[8];
    cat8(d8, a0, a1, p.scale);
    if constexpr (COOP) *(u32x4*)(Ki + (16 * qb + (lane & 15)) * Img<32>::RS + g * 16) = pack8(d8);
    else if (R.ok[qb]) *(u32x4*)(p.dq + roff(R.row[qb], p.lddq) + h * 32 + 8 * g) = pack8(d8);
  }
  // ---- S layout (lane = key): dV^T = dO^T P, dK^T = scale * Q^T dS
#pragma unroll
  for (int kb = 0; kb < 2; ++kb) {
    const bool kv = R.ok[kb];                   // key 16 kb + i: the lane's row kb
    f32x4 pm[2], ds[2];
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
      const f32x4 sv = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qr[qb], kr[kb], z4, 0, 0, 0);
      const f32x4 dp = __builtin_amdgcn_mfma_f32_16x16x32_bf16(dr[qb], vr[kb], z4, 0, 0, 0);
      const f32x4 l4 = *(const f32x4*)(lse2 + 16 * qb + 4 * g);
      const f32x4 d4 = *(const f32x4*)(dlt + 16 * qb + 4 * g);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float pr = kv ? fexp2(sv[r] * c2 - l4[r]) : 0.f;
        pm[qb][r] = pr;
        ds[qb][r] = pr * (dp[r] - d4[r]);
      }
    }
    const bf16x8 pf = pack_perm(pm[0], pm[1]), dsk = pack_perm(ds[0], ds[1]);
    f32x4 dv[2], dk[2];
#pragma unroll
    for (int db = 0; db < 2; ++db) {
      const bf16x8 a_dv = COOP ? dt[db] : trfrag<32>(Di, 0, 16 * db, lane);
      const bf16x8 a_dk = COOP ? qt[db] : trfrag<32>(Qi, 0, 16 * db, lane);
      dv[db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a_dv, pf, z4, 0, 0, 0);
      dk[db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a_dk, dsk, z4, 0, 0, 0);
    }
    float v8[8], k8[8];   // rows d = 8g + 4db + r (interleaved images)
    cat8(v8, dv[0], dv[1], 1.f);
    cat8(k8, dk[0], dk[1], p.scale);
    if constexpr (COOP) {
      const int o = (16 * kb + (lane & 15)) * Img<32>::RS + g * 16;
      *(u32x4*)(Di + o) = pack8(v8);
      *(u32x4*)(Qi + o) = pack8(k8);
    } else if (kv) {
      *(u32x4*)(p.dv + roff(R.row[kb], p.lddv) + h * 32 + 8 * g) = pack8(v8);
      *(u32x4*)(p.dk + roff(R.row[kb], p.lddk) + h * 32 + 8 * g) = pack8(k8);
    }
  }
  if constexpr (COOP) {
    __syncthreads();                            // every wave's staging written
    constexpr int WS = 3 * SIMG + 256;
    coop_store_areas(p.dq, p.lddq, smem, WS, SIMG, p, s, h - w);        // K image: dQ
    coop_store_areas(p.dk, p.lddk, smem, WS, 0, p, s, h - w);           // Q image: dK
    coop_store_areas(p.dv, p.lddv, smem, WS, 2 * SIMG, p, s, h - w);    // dO image: dV
  }
}

// (32-bit token rows and 32 x 32-bit offset products in the small kernels: SmallRows / roff)
bool small_ok(const AP& p, int D) {
  const int64_t lim = (int64_t)1 << 31;
  const bool fits = p.M < lim && p.ldq < lim && p.ldk < lim && p.ldv < lim && p.ldo < lim && p.ldout < lim &&
                    p.lddo < lim && p.lddq < lim && p.lddk < lim && p.lddv < lim;
  return D == 32 && p.L <= 32 && !p.bias_u && !p.kmask && p.drop_p == 0.f && fits;
}

}  // namespace

extern "C" int ctclip_attn_fwd(const ctclip_attn_args* a, void* stream) {
  AP p;
  int rc = fill(p, a);
  if (rc) return rc;
  if (!s_attr) { set_attrs(); s_attr = true; }
  const int Lp = (p.L + 31) & ~31;
  const int pairs = p.nseq * p.H;
  if (small_ok(p, a->D)) {
    static const int coop_env = [] { const char* e = getenv("CTCLIP_ATTN_SMALL_COOP"); return e ? atoi(e) : 1; }();
    if (coop_env && p.H % SW == 0)   // CTCLIP_ATTN_SMALL_COOP=0: per-wave stores (A/B)
      hipLaunchKernelGGL(attn_small_fwd_kernel<true>, dim3(cdiv(pairs, SW)), dim3(SW * 64), small_fwd_lds(true),
                         (hipStream_t)stream, p);
    else
      hipLaunchKernelGGL(attn_small_fwd_kernel<false>, dim3(cdiv(pairs, SW)), dim3(SW * 64), small_fwd_lds(false),
                         (hipStream_t)stream, p);
    CT_CHECK_LAUNCH();
    return 0;
  }
  const size_t RSb = a->D * 2 + 16;
  const size_t lds = (size_t)p.pp * 2 * Lp * RSb + table_bytes(p, Lp, false) + 256;   // + block-reduce scratch
  if (lds > 160 * 1024) return CT_ESHAPE;
  dim3 grid(cdiv(pairs, p.pp));
  if (a->D == 32) launch_fwd<32>(p, grid, lds, (hipStream_t)stream);
  else launch_fwd<64>(p, grid, lds, (hipStream_t)stream);
  CT_CHECK_LAUNCH();
  return 0;
}

// launch plan of the frame-inner dQ + bias-gradient kernels (shared with the workspace query)
struct DqPlan {
  int nqg = 0, nfc = 0;
  bool dma = false;
  size_t lds = 0, lds_dma = 0;
};
bool dq_plan(const AP& p, int D, DqPlan& pl) {
  const int Lp = (p.L + 31) & ~31, nc = Lp / 32;
  if (!(D == 32 && p.bias_u && p.dbias_u && !p.kmask && (nc + 1) / 2 <= 9)) return false;
  const size_t RSb = D * 2 + 16;
  pl.nqg = cdiv(p.L, 64);
  // frame chunks: at least two workgroups per CU, then (up to twice that) the count whose last
  // dispatch round is fullest -- 72 x 14 = 1,008 workgroups = 3.94 rounds of 256 at the base
  // shape (measured: nfc 8 / 14 / 28 -> spatial backward 1,109 / 1,074 / 1,242 us)
  const int per = p.H * pl.nqg;
  const int lo = std::max(1, std::min(p.nseq, (2 * 256 + per - 1) / per));
  pl.nfc = lo;
  double best = 0.0;
  for (int f = lo; f <= std::min(p.nseq, 2 * lo); ++f) {
    const long wgs = (long)per * f, rounds = (wgs + 255) / 256;
    const double eff = (double)wgs / (double)(rounds * 256);
    if (eff > best + 1e-3) { best = eff; pl.nfc = f; }
  }
  pl.lds = (size_t)2 * Lp * RSb + 2 * (size_t)((p.nbins + 3) & ~3) * 4 + 2 * (size_t)Lp * 4 + 4 * 64 * 8 * 4;
  static int dma_ok = -1;   // CTCLIP_ATTN_DQ_DMA=0: the generic kernel (A/B)
  if (dma_ok < 0) { const char* e = getenv("CTCLIP_ATTN_DQ_DMA"); dma_ok = e ? atoi(e) != 0 : 1; }
  pl.lds_dma = (size_t)2 * 2 * 576 * 64 + (size_t)((p.nbins + 3) & ~3) * 4 + 576 * 4;
  pl.dma = dma_ok && run_ok(p) && p.L == 576 && p.s_pos == 1 && p.n_inner == 1 && p.nbins * 4 <= 2 * 576 * 64 &&
           pl.lds_dma <= 160 * 1024;
  return true;
}

// floats of the optional bias-gradient workspace (ctclip_attn_args.dbias_ws) for this shape;
// 0 when the shape bins with atomics (no frame-inner dQ kernel / not the LDS-DMA one)
extern "C" int ctclip_attn_bwd_ws_floats(const ctclip_attn_args* a) {
  AP p;
  if (fill(p, a)) return 0;
  DqPlan pl;
  if (!dq_plan(p, a->D, pl) || (pl.dma && !CTCLIP_ATTN_DIAG_BIN) || (p.H * p.nbins) % 4) return 0;
  return pl.nqg * pl.nfc * p.H * p.nbins;
}

extern "C" int ctclip_attn_bwd(const ctclip_attn_args* a, void* stream) {
  AP p;
  int rc = fill(p, a);
  if (rc) return rc;
  if (!s_attr) { set_attrs(); s_attr = true; }
  const int Lp = (p.L + 31) & ~31;
  const int pairs = p.nseq * p.H;
  const size_t RSb = a->D * 2 + 16;
  const size_t lds1 = (size_t)p.pp * 2 * Lp * RSb + table_bytes(p, Lp, true);
  const size_t lds2 = (size_t)p.pp * (2 * Lp * RSb + 2 * Lp * 4) + table_bytes(p, Lp, false);
  if (lds1 > 160 * 1024 || lds2 > 160 * 1024) return CT_ESHAPE;
  dim3 grid(cdiv(pairs, p.pp));
  hipStream_t st = (hipStream_t)stream;
  if (small_ok(p, a->D)) {
    static const int coop_env = [] { const char* e = getenv("CTCLIP_ATTN_SMALL_COOP"); return e ? atoi(e) : 1; }();
    const size_t lds = (size_t)SW * (3 * SIMG + 256);
    if (coop_env && p.H % SW == 0)
      hipLaunchKernelGGL(attn_small_bwd_kernel<true>, dim3(cdiv(pairs, SW)), dim3(SW * 64), lds, st, p);
    else
      hipLaunchKernelGGL(attn_small_bwd_kernel<false>, dim3(cdiv(pairs, SW)), dim3(SW * 64), lds, st, p);
    CT_CHECK_LAUNCH();
    return 0;
  }
  DqPlan pl;
  if (dq_plan(p, a->D, pl)) {
    // frame-inner dQ + bias-gradient kernel (see attn_bwd_dq_bias_kernel)
    const int nqg = pl.nqg, nfc = pl.nfc;
    if (pl.lds > 160 * 1024) return CT_ESHAPE;
    const bool slab = (CTCLIP_ATTN_DIAG_BIN || !pl.dma) && p.dbias_ws && (p.H * p.nbins) % 4 == 0 &&
                      a->dbias_ws_floats >= (int64_t)nqg * nfc * p.H * p.nbins;
    if (!slab) p.dbias_ws = nullptr;
    if (pl.dma)
      hipLaunchKernelGGL((attn_bwd_dq_bias_dma_kernel<576>), dim3(p.H, nqg, nfc), dim3(DQD_NT), pl.lds_dma, st, p, nfc);
    else if (run_ok(p)) hipLaunchKernelGGL((attn_bwd_dq_bias_kernel<9, true>), dim3(p.H, nqg, nfc), dim3(NT), pl.lds, st, p, nfc);
    else hipLaunchKernelGGL((attn_bwd_dq_bias_kernel<9>), dim3(p.H, nqg, nfc), dim3(NT), pl.lds, st, p, nfc);
    CT_CHECK_LAUNCH();
    if (slab) {   // deterministic sum of the workgroups' partial bins into dbias_u
      // [H][nbins] summed as one row of H * nbins floats (nbins = 2,209 is odd; the product is not)
      const int64_t n = (int64_t)p.H * p.nbins;
      const int r = ctclip_reduce_slabs(p.dbias_ws, (int64_t)nqg * nfc, 1, n, n, p.dbias_u, n, 1, 1, stream);
      if (r) return r;
    }
    launch_dkv<32>(p, grid, lds2, st);
    CT_CHECK_LAUNCH();
    return 0;
  }
  if (a->D == 32) {
    launch_dq<32>(p, grid, lds1, st);
    launch_dkv<32>(p, grid, lds2, st);
  } else {
    launch_dq<64>(p, grid, lds1, st);
    launch_dkv<64>(p, grid, lds2, st);
  }
  CT_CHECK_LAUNCH();
  return 0;
}

// diagnostic: query blocks per wave of the spatial forward kernel (1, 2 or 3; results are
// bit-identical); returns the previous setting
extern "C" int ctclip_attn_set_fwd_smax(int on) {
  if (g_fwd_smax < 0) { const char* e = getenv("CTCLIP_ATTN_FWD_SMAX"); g_fwd_smax = e ? atoi(e) != 0 : 0; }
  const int old = g_fwd_smax;
  g_fwd_smax = on != 0;
  return old;
}

extern "C" int ctclip_attn_set_fwd_cinit(int on) {
  if (g_fwd_cinit < 0) { const char* e = getenv("CTCLIP_ATTN_FWD_CINIT"); g_fwd_cinit = e ? atoi(e) != 0 : 1; }
  const int old = g_fwd_cinit;
  g_fwd_cinit = on != 0;
  return old;
}

extern "C" int ctclip_attn_set_fwd_qb(int qb) {
  if (g_fwd_qb < 0) { const char* e = getenv("CTCLIP_ATTN_FWD_QB"); g_fwd_qb = e ? atoi(e) : 3; }
  const int old = g_fwd_qb;
  if (qb >= 1 && qb <= 3) g_fwd_qb = qb;
  return old;
}
