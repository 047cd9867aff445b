// Large-tile bf16 MFMA GEMM for gfx950: 256x256x64 block tile, 8 waves (2 x 4), each wave a
// 128x64 tile of 8x4 v_mfma_f32_16x16x32_bf16 (128 accumulator VGPRs).  Operands stream
// HBM -> LDS with global_load_lds_dwordx4 (no register staging) into a 2-stage LDS ring
// (2 x 64 KB); the next K-step's loads are in flight under the current step's MFMAs, one
// vmcnt(0) + barrier per step.  LDS images are lane-linear (the glds contract) with the XOR
// swizzle applied on the GLOBAL source address and undone on the fragment read:
//   K-contiguous operand  [256 rows][64 k], 128-B rows: 16-B chunk ^= (row >> 1) & 7
//     -> the 16 rows of a ds_read_b128 lane group hit 16 distinct 16-B bank slots;
//   MN-contiguous operand [64 k][256], 512-B rows: 32-B block ^= (k & 3) | ((k >> 3) & 1) << 2
//     -> ds_read_b64_tr_b16 (hardware transpose) lane halves are conflict-free.
// Epilogue: each wave stages its own 64-row halves through a private LDS region and writes
// 16-B row chunks with the same fused ops as gemm.hip (bias, residual, GELU, GEGLU in
// 32-column pairs, argmax, split-K slabs).  Requires K % 64 == 0 (checked by the caller).
#include "common.h"
#include <string.h>
#include "../../include/ctclip_hip.h"

namespace g256 {

// Two shapes of one kernel template, WR = wave rows of 128:
//   WR = 2: 256 x 256 tile, 8 waves, 4-slot ring (128 KB LDS, 1 workgroup per CU);
//   WR = 1: 128 x 256 tile, 4 waves, 3-slot ring (72 KB LDS, 2 workgroups per CU), so one
//           workgroup's epilogue stores drain while the other one's MFMAs run.
constexpr int BN = 256, BK = 32;
constexpr int EP_LD = 68;                    // f32 staging row stride (64 cols + pad)
template <int WR> struct Cfg {
  static constexpr int BM = 128 * WR, NTH = 256 * WR;
  static constexpr int ABYTES = BM * BK * 2, BBYTES = BN * BK * 2, STAGE = ABYTES + BBYTES;
  static constexpr int NSTAGE = WR == 2 ? 4 : 3;
  static constexpr int SMEM = NSTAGE * STAGE;
  static constexpr int GA = ABYTES / 16 / NTH, GB = BBYTES / 16 / NTH, G = GA + GB;   // glds per thread per tile
};

struct P {
  int64_t M, N, K;
  const u16* A; int64_t lda;
  const u16* B; int64_t ldb;
  void* C; int64_t ldc; int c_f32;
  u16* C2; int64_t ldc2;
  const float* bias;
  const void* R; int64_t ldr; int r_f32;
  float alpha; int act; int accumulate; int split_k;
  int64_t sA, sB, sC, sC2, sR;
  int n2;        // act 5: columns of C2 (the per-head l2norm of C)
  int64_t kper;
  int debug;     // diagnostic knob (CTCLIP_G256_DEBUG): 1 = skip the epilogue, 2 = skip the main loop
  int group_gx;  // grouped (8-row) tile walk when the N tile count >= this (CTCLIP_GEMM_GROUP_GX, default 8)
  int group_gm;  // rows per group of that walk (CTCLIP_GEMM_GROUP_GM; 0 = 8)
  int stagger;   // start delay (s_sleep units of 64 cycles) for the second co-resident workgroup
  int gz;        // batch * split_k (8-phase tile count = ceil(N/256) * ceil(M/256) * gz)
  int persist;   // 8-phase: persistent workgroups (one per CU) walking the tile sequence
  int pre1;      // 8-phase TR: the next tile's whole K-step 1 staged before the epilogue (CTCLIP_GEMM_PRE1)
  // LayerNorm epilogues (EP -6 forward, -7 backward; ctclip_gemm_ln)
  const float* ln_gamma; const float* ln_beta; float ln_eps;
  u16* ln_y; int64_t ln_ldy;         // -6: LN output (bf16)
  float* ln_mean; float* ln_rstd;    // -6: written; -7: read
  const u16* ln_x; int64_t ln_ldx;   // -7: the LN input (bf16)
  float* ln_pg; float* ln_pb;        // -7: [M / 128][N] column partials (dgamma, dbeta)
  unsigned long long* xchg;          // [2 tiles][M][2] {epoch, value} granules
  unsigned epoch;
  int* status;
  unsigned spin_limit;               // polls before giving up on the partner (status = 1)
  int ln_debug;                      // test knob: tile 1 of row block 0 never publishes
  int epi_lds;                       // transposed bf16 / GEGLU epilogues: lane-contiguous stores via LDS
  // EP 8 (ctclip_gemm_qkv_lnfold): columns < nfold carry the LayerNorm fold
  //   C = rstd[row] * (acc - mean[row] * fold_cs[col])   (ln_mean / ln_rstd read)
  const float* fold_cs;
  int nfold;
  // fp16 (round 5): h16 = FF1's h is fp16 -- written by the GEGLU epilogue of the fp16 kernel (EP 2,
  // H16), read by the GEGLU backward (EP 4); ln_y16 = optional fp16 copy of the -6 LayerNorm output
  int h16;
  u16* ln_y16;
  // split-fp16 "x3" GEMM (round 6, ctclip_gemm_args.A_lo / B_lo): A = Ah + Al, B = Bh + Bl as fp16
  // image pairs; every 64-deep K-step runs three products Ah Bh, Ah Bl, Al Bh into the one f32
  // accumulator (Al Bl, ~2^-22 relative, is dropped), so the GEMM sees ~22-bit operands at 3x the
  // fp16 MFMA work (the X3 kernels: tile_at's K-step count triples).  The x3 GEGLU
  // epilogue writes h (fp16, C), g = gelu(gate) x from the unrounded f32 h as an fp16 pair (C2 hi,
  // C3 lo, the FF2 GEMM's A operand) and as bf16 (C4, the FF2 weight gradient's operand).
  const u16* alo;
  const u16* blo;
  u16* C3; int64_t ldc3;
  u16* C4; int64_t ldc4;
  int x3;
  int c_col0;    // EP 6 / 8: first C column stored (ctclip_gemm_qkv_lnfold2; 0 = all)
};

__device__ __forceinline__ int mn_swz(int k) { return (k & 3) | (((k >> 3) & 1) << 2); }

typedef __attribute__((address_space(1))) void gvoid;
typedef __attribute__((address_space(3))) void lvoid;

// K-contiguous image [256 rows][32 k], 64-B rows: 16-B chunk ^= (row >> 2) & 2 makes every
// ds_read_b128 lane group of a fragment read (row = lane & 15, chunk = lane >> 4) hit 16
// distinct 16-B bank slots (searched exhaustively over the four gfx950 lane groups)
__device__ __forceinline__ int kc_swz(int row) { return (row >> 2) & 2; }

// issue this thread's NJ glds for one ROWS x 32 operand tile (ROWS * 4 16-B chunks)
template <bool KC, int ROWS, int NJ>
__device__ __forceinline__ void stage_tile(char* lds, const u16* base, int64_t ld, int64_t rows, int64_t row0,
                                           int64_t k0, int w, int lane) {
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = (w * NJ + j) * 64 + lane;   // 16-B chunk index in the tile image
    const u16* src;
    if constexpr (KC) {
      const int row = c >> 2, pc = c & 3, lc = pc ^ kc_swz(row);
      const int64_t gr = min(row0 + row, rows - 1);
      src = base + gr * ld + k0 + lc * 8;
    } else {
      constexpr int CPR = ROWS / 8;             // chunks per k-row
      const int kk = c / CPR, pc = c % CPR, pb = pc >> 1, half = pc & 1;
      const int lb = pb ^ mn_swz(kk);
      const int64_t gm = min(row0 + (int64_t)(lb * 2 + half) * 8, rows - 8);
      src = base + (k0 + kk) * ld + gm;
    }
    __builtin_amdgcn_global_load_lds((gvoid*)src, (lvoid*)(lds + (w * NJ + j) * 1024), 16, 0, 0);
  }
}

template <bool KC, int ROWS>
__device__ __forceinline__ bf16x8 frag(const char* tile, int r0, int lane) {
  if constexpr (KC) {
    const int row = r0 + (lane & 15);
    const int lc = lane >> 4;
    return *(const bf16x8*)(tile + row * 64 + ((lc ^ kc_swz(row)) << 4));
  } else {
    const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const int m = r0 + 4 * p;
    const int k1 = 8 * g + q, k2 = k1 + 4;
    const int cb = m >> 4, within = (m & 15) * 2;
    const int o1 = k1 * (ROWS * 2) + ((cb ^ mn_swz(k1)) << 5) + within;
    const int o2 = k2 * (ROWS * 2) + ((cb ^ mn_swz(k2)) << 5) + within;
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, tile + o1));
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, tile + o2));
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
  }
}

__device__ __forceinline__ void xcd_remap(int& tx, int& ty) {
  const int gx = gridDim.x, nwg = gridDim.x * gridDim.y;
  const int orig = blockIdx.y * gx + blockIdx.x;
  int id = orig;
  if (nwg >= 16) {
    const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
    id = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  }
  ty = id / gx;
  tx = id - ty * gx;
}

// Shared epilogue: wave (wr, wc) owns output rows m0 + wr*128 + [0,128), cols n0 + wc*64 + [0,64);
// acc[i][j] is the 16x16 block (i, j) of that region in the MFMA 16x16 C layout.  Stages each
// 32-row quarter through a wave-private LDS region (8.7 KB per wave) and writes 16-B row chunks.
// LM (compile time, one kernel instantiation each so only that path's registers are allocated):
// -1 = general (bias / residual / GELU / f32 or bf16 / accumulate / shadow; GEGLU), -3 = argmax,
// -5 = split-K slabs
template <int LM = -1>
__device__ __forceinline__ void epilogue(const P& p, f32x4 (&acc)[8][4], char* smem, int w, int wr, int wc, int lane,
                                         int64_t m0, int64_t n0, int split, int bidx) {
  float* cs = (float*)(smem + w * (32 * EP_LD * 4));   // 8.7 KB per wave, 8 waves = 70 KB
  const int64_t wrow0 = m0 + wr * 128, wcol0 = n0 + wc * 64;
  const bool slab = LM == -5 || (LM == -1 && p.split_k > 1);
#pragma unroll
  for (int quarter = 0; quarter < 4; ++quarter) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          cs[(i * 16 + (lane >> 4) * 4 + r) * EP_LD + j * 16 + (lane & 15)] = acc[quarter * 2 + i][j][r];
    // wave-private region: no block barrier needed, only LDS write->read ordering in the wave
    __builtin_amdgcn_s_waitcnt(0xC07F);
    const int64_t rbase = wrow0 + quarter * 32;
    if (LM == -3 || (LM == -1 && p.act == 3)) {   // (LM -2 never takes the argmax / GEGLU paths)
      // argmax over this wave's 64 columns: 2 lanes per row (32 columns each), (value, index)
      // per (row, 64-col group), first-max tie-break
      // (+ the group's second-best score into the optional f32 C2, see gemm.hip)
      const int row = lane >> 1, hc = lane & 1;
      const int64_t gm = rbase + row;
      float best = -INFINITY, second = -INFINITY;
      int bi = 0x7fffffff;
      const int ncol = (int)max((int64_t)0, min((int64_t)64, p.N - wcol0));
      for (int c = hc * 32; c < hc * 32 + 32; ++c) {
        const float v = cs[row * EP_LD + c];
        if (c < ncol) {
          if (v > best) { second = best; best = v; bi = c; }
          else if (v > second) second = v;
        }
      }
      const float ob = __shfl_xor(best, 1, 64);
      const float os = __shfl_xor(second, 1, 64);
      const int oi = __shfl_xor(bi, 1, 64);
      if (ob > best || (ob == best && oi < bi)) { second = fmaxf(best, os); best = ob; bi = oi; }
      else second = fmaxf(second, ob);
      if (hc == 0 && gm < p.M && ncol > 0) {
        float2* out = (float2*)p.C + bidx * p.sC;
        out[gm * p.ldc + (wcol0 >> 6)] = make_float2(best, __int_as_float((int)(wcol0 + bi)));
        if (p.C2) ((float*)p.C2)[bidx * p.sC2 + gm * p.ldc2 + (wcol0 >> 6)] = second;
      }
    } else if (LM == -1 && p.act == 2) {
      // GEGLU pairs of 32 columns: [x | gate] -> 32 outputs; h (C) keeps both halves
      for (int it = 0; it < 4; ++it) {
        const int c = lane + 64 * it;          // 256 chunks of 8 = 32 rows x 8
        const int row = c >> 3, cc = (c & 7) * 8;
        const int64_t gm = rbase + row, gn = wcol0 + cc;
        if (gm >= p.M || gn >= p.N) continue;
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = cs[row * EP_LD + cc + j] * p.alpha;
        *(u32x4*)((u16*)p.C + bidx * p.sC + gm * p.ldc + gn) = pack8(v);
      }
      for (int it = 0; it < 2; ++it) {
        const int c = lane + 64 * it;          // 128 chunks = 32 rows x 4
        const int row = c >> 2, cc = (c & 3) * 8;
        const int64_t gm = rbase + row;
        if (gm >= p.M || wcol0 >= p.N) continue;
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float xb = bf2f(f2bf(cs[row * EP_LD + cc + j] * p.alpha));
          const float gb = bf2f(f2bf(cs[row * EP_LD + 32 + cc + j] * p.alpha));
          v[j] = gelu_erf(gb) * xb;
        }
        *(u32x4*)(p.C2 + bidx * p.sC2 + gm * p.ldc2 + (wcol0 >> 1) + cc) = pack8(v);
      }
    } else {
      // Every load this quarter's stores depend on (the residual, else the accumulate target)
      // is issued first.  With the previous quarter's stores still pending, the compiler can
      // only wait for a load with vmcnt(0) (read and write events retire out of order), so a
      // load interleaved with the stores costs a full store round trip each: 4+ per quarter
      // before (r02 ISA), one now.  The column gn = wcol0 + (lane & 7) * 8 is the same in all
      // four row chunks, so the bias is loaded once.
      const int64_t gn = wcol0 + (lane & 7) * 8;
      const int cc = (lane & 7) * 8;
      const bool pre_acc = LM == -1 && !p.R && p.accumulate;
      if constexpr (LM == -2 || LM == -8) {
        // residual mode: C (f32) = alpha acc + bias + R (f32), bf16 shadow into C2 when given
        // unconditional loads (rows / columns clamped into the matrix, results of clamped
        // chunks unused): a load under a branch must complete before its phi copy, which put a
        // vmcnt(0) behind every pair
        // LM -8 (ctclip_gemm_lnfold_bwd): also - c1[row] - beta[row] * X[row][col] (X bf16 in
        // ln_x, c1 / beta in ln_mean / ln_rstd): the folded LayerNorm backward
        f32x4 ra[4], rb[4];
        const int64_t gnc = min(gn, p.N - 8);
#pragma unroll
        for (int it = 0; it < 4; ++it) {
          const int64_t gm = min(rbase + ((lane + 64 * it) >> 3), p.M - 1);
          const float* Rp = (const float*)p.R + bidx * p.sR + gm * p.ldr + gnc;
          ra[it] = *(const f32x4*)Rp;
          rb[it] = *(const f32x4*)(Rp + 4);
        }
        if constexpr (LM == -8) {
#pragma unroll
          for (int it = 0; it < 4; ++it) {
            const int64_t gm = min(rbase + ((lane + 64 * it) >> 3), p.M - 1);
            float xv[8];
            unpack8(*(const u32x4*)(p.ln_x + gm * p.ln_ldx + gnc), xv);
            const float c1 = p.ln_mean[gm], be = p.ln_rstd[gm];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              ra[it][j] -= fmaf(be, xv[j], c1);
              rb[it][j] -= fmaf(be, xv[4 + j], c1);
            }
          }
        }
        f32x4 b0 = f32x4{0.f, 0.f, 0.f, 0.f}, b1 = b0;
        if (p.bias) {
          b0 = *(const f32x4*)(p.bias + gnc);
          b1 = *(const f32x4*)(p.bias + gnc + 4);
        }
        // wave-uniform: the wave's 32 x 64 quarter lies inside the matrix (every tile of the
        // 3D-ViT's residual GEMMs), so the stores run without per-lane branches -- a divergent
        // branch around each store group made the compiler drain vmcnt at every block boundary
        const bool full = rbase + 32 <= p.M && wcol0 + 64 <= p.N;
        auto row_out = [&](int it) {
          const int row = (lane + 64 * it) >> 3;
          const int64_t gm = rbase + row;
          const f32x4 lo = *(const f32x4*)(cs + row * EP_LD + cc);
          const f32x4 hi = *(const f32x4*)(cs + row * EP_LD + cc + 4);
          float v[8];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            v[j] = lo[j] * p.alpha + b0[j] + ra[it][j];
            v[4 + j] = hi[j] * p.alpha + b1[j] + rb[it][j];
          }
          float* Cf = (float*)p.C + bidx * p.sC + gm * p.ldc + gn;
          *(f32x4*)Cf = f32x4{v[0], v[1], v[2], v[3]};
          *(f32x4*)(Cf + 4) = f32x4{v[4], v[5], v[6], v[7]};
          if (p.C2) *(u32x4*)(p.C2 + bidx * p.sC2 + gm * p.ldc2 + gn) = pack8(v);
        };
        if (full) {
          // phase by phase (all LDS reads, all math, all stores), so the four chunks' store
          // operands occupy distinct registers and no store waits for an earlier one to drain
          f32x4 lo[4], hi[4];
#pragma unroll
          for (int it = 0; it < 4; ++it) {
            const int row = (lane + 64 * it) >> 3;
            lo[it] = *(const f32x4*)(cs + row * EP_LD + cc);
            hi[it] = *(const f32x4*)(cs + row * EP_LD + cc + 4);
          }
#pragma unroll
          for (int it = 0; it < 4; ++it)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              lo[it][j] = lo[it][j] * p.alpha + b0[j] + ra[it][j];
              hi[it][j] = hi[it][j] * p.alpha + b1[j] + rb[it][j];
            }
#pragma unroll
          for (int it = 0; it < 4; ++it) {
            float* Cf = (float*)p.C + bidx * p.sC + (rbase + ((lane + 64 * it) >> 3)) * p.ldc + gn;
            *(f32x4*)Cf = lo[it];
            *(f32x4*)(Cf + 4) = hi[it];
          }
          if (p.C2) {
#pragma unroll
            for (int it = 0; it < 4; ++it) {
              const float v[8] = {lo[it][0], lo[it][1], lo[it][2], lo[it][3], hi[it][0], hi[it][1], hi[it][2], hi[it][3]};
              *(u32x4*)(p.C2 + bidx * p.sC2 + (rbase + ((lane + 64 * it) >> 3)) * p.ldc2 + gn) = pack8(v);
            }
          }
        } else {
#pragma unroll
          for (int it = 0; it < 4; ++it)
            if (rbase + ((lane + 64 * it) >> 3) < p.M && gn < p.N) row_out(it);
        }
      } else {
      f32x4 ra[4], rb[4];
#pragma unroll
      for (int it = 0; it < 4; ++it) {
        const int row = (lane + 64 * it) >> 3;
        const int64_t gm = rbase + row;
        ra[it] = rb[it] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (slab || gm >= p.M || gn >= p.N) continue;
        if (LM == -1 && p.R) {
          if (p.r_f32) {
            const float* Rp = (const float*)p.R + bidx * p.sR + gm * p.ldr + gn;
            ra[it] = *(const f32x4*)Rp;
            rb[it] = *(const f32x4*)(Rp + 4);
          } else {
            ra[it] = __builtin_bit_cast(f32x4, *(const u32x4*)((const u16*)p.R + bidx * p.sR + gm * p.ldr + gn));
          }
        } else if (pre_acc) {
          if (p.c_f32) {
            const float* Cf = (const float*)p.C + bidx * p.sC + gm * p.ldc + gn;
            ra[it] = *(const f32x4*)Cf;
            rb[it] = *(const f32x4*)(Cf + 4);
          } else {
            ra[it] = __builtin_bit_cast(f32x4, *(const u32x4*)((const u16*)p.C + bidx * p.sC + gm * p.ldc + gn));
          }
        }
      }
      f32x4 b0 = f32x4{0.f, 0.f, 0.f, 0.f}, b1 = b0;
      if (p.bias && !slab && gn < p.N) {
        b0 = *(const f32x4*)(p.bias + gn);
        b1 = *(const f32x4*)(p.bias + gn + 4);
      }
#pragma unroll
      for (int it = 0; it < 4; ++it) {
        const int row = (lane + 64 * it) >> 3;
        const int64_t gm = rbase + row;
        if (gm >= p.M || gn >= p.N) continue;
        float v[8];
        const f32x4 lo = *(const f32x4*)(cs + row * EP_LD + cc);
        const f32x4 hi = *(const f32x4*)(cs + row * EP_LD + cc + 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) { v[j] = lo[j] * p.alpha; v[4 + j] = hi[j] * p.alpha; }
        if (slab) {
          float* Cf = (float*)p.C + (int64_t)split * p.M * p.ldc + bidx * p.sC + gm * p.ldc + gn;
          *(f32x4*)Cf = f32x4{v[0], v[1], v[2], v[3]};
          *(f32x4*)(Cf + 4) = f32x4{v[4], v[5], v[6], v[7]};
          continue;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) { v[j] += b0[j]; v[4 + j] += b1[j]; }
        if (p.R) {
          if (p.r_f32) {
#pragma unroll
            for (int j = 0; j < 4; ++j) { v[j] += ra[it][j]; v[4 + j] += rb[it][j]; }
          } else {
            float rr[8];
            unpack8(__builtin_bit_cast(u32x4, ra[it]), rr);
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] += rr[j];
          }
        }
        if (p.act == 1) {
          if (p.C2) *(u32x4*)(p.C2 + bidx * p.sC2 + gm * p.ldc2 + gn) = pack8(v);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = gelu_erf(v[j]);
        }
        if (p.c_f32) {
          float* Cf = (float*)p.C + bidx * p.sC + gm * p.ldc + gn;
          if (p.accumulate) {
            const f32x4 a = pre_acc ? ra[it] : *(const f32x4*)Cf;
            const f32x4 b = pre_acc ? rb[it] : *(const f32x4*)(Cf + 4);
#pragma unroll
            for (int j = 0; j < 4; ++j) { v[j] += a[j]; v[4 + j] += b[j]; }
          }
          *(f32x4*)Cf = f32x4{v[0], v[1], v[2], v[3]};
          *(f32x4*)(Cf + 4) = f32x4{v[4], v[5], v[6], v[7]};
        } else {
          u16* Cb = (u16*)p.C + bidx * p.sC + gm * p.ldc + gn;
          if (p.accumulate) {
            float rr[8];
            unpack8(pre_acc ? __builtin_bit_cast(u32x4, ra[it]) : *(const u32x4*)Cb, rr);
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] += rr[j];
          }
          *(u32x4*)Cb = pack8(v);
        }
        if (p.C2 && p.act == 0) *(u32x4*)(p.C2 + bidx * p.sC2 + gm * p.ldc2 + gn) = pack8(v);
      }
      }
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);   // reads of this half done before it is overwritten
  }
}

template <int WR, bool AK, bool BKC>
__global__ __launch_bounds__(Cfg<WR>::NTH, 2 / WR) void gemm256_kernel(P p) {
  using C = Cfg<WR>;
  constexpr int NSTAGE = C::NSTAGE, STAGE = C::STAGE, G = C::G;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, wr = w >> 2, wc = w & 3;
  int tx, ty;
  xcd_remap(tx, ty);
  const int split = blockIdx.z % p.split_k, bidx = blockIdx.z / p.split_k;
  const int64_t m0 = (int64_t)ty * C::BM, n0 = (int64_t)tx * BN;
  const int64_t kbeg = split * p.kper;
  const int64_t kend = min(p.K, kbeg + p.kper);
  const u16* A = p.A + bidx * p.sA;
  const u16* B = p.B + bidx * p.sB;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // NSTAGE-slot ring of 32-deep K tiles: tile kt lives in slot kt % NSTAGE; NSTAGE - 1 tiles
  // are in flight while one is computed.  Each tile is G glds per thread; the wait before step
  // kt leaves the younger tiles' loads outstanding (counted vmcnt, never 0 in steady state) and
  // a raw s_barrier publishes the landed tile (a __syncthreads fence would drain every glds).
  // The slot refilled at step kt held tile kt - 1, which every wave finished before the barrier.
  const int nk = (kend > kbeg && !(p.debug & 2)) ? (int)((kend - kbeg) / BK) : 0;
  // the first dispatch round holds two workgroups per CU (WR = 1); delaying the second one
  // offsets their store-heavy epilogues against each other's MFMA main loops
  if (p.stagger > 0) {
    const int lin = (blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
    const int ncu = 256;
    if (lin >= ncu && lin < 2 * ncu)
      for (int s = 0; s < p.stagger; s += 64) __builtin_amdgcn_s_sleep(64);
  }
  auto stage = [&](int t) {
    char* st = smem + (t % NSTAGE) * STAGE;
    const int64_t k1 = kbeg + (int64_t)t * BK;
    stage_tile<AK, C::BM, C::GA>(st, A, p.lda, p.M, m0, k1, w, lane);
    stage_tile<BKC, BN, C::GB>(st + C::ABYTES, B, p.ldb, p.N, n0, k1, w, lane);
  };
  for (int t = 0; t < NSTAGE - 1 && t < nk; ++t) stage(t);
  for (int kt = 0; kt < nk; ++kt) {
    if constexpr (NSTAGE == 4) {
      if (kt + 2 < nk) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * G) : "memory");
      else if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (kt + NSTAGE - 1 < nk) stage(kt + NSTAGE - 1);
    const char* As = smem + (kt % NSTAGE) * STAGE;
    const char* Bs = As + C::ABYTES;
    bf16x8 bfr[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) bfr[j] = frag<BKC, BN>(Bs, wc * 64 + j * 16, lane);
    bf16x8 af[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) af[i] = frag<AK, C::BM>(As, wr * 128 + i * 16, lane);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  }
  __syncthreads();   // every wave's last fragment reads done before the epilogue reuses LDS
  if (p.debug & 1) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(acc[i][j]));
    return;
  }

  epilogue(p, acc, smem, w, wr, wc, lane, m0, n0, split, bidx);
}


// ============================================================================================
// 8-phase 256 x 256 x 64 kernel (1 workgroup per CU, 8 waves as 2 (M) x 4 (N), wave tile
// 128 x 64 = four 64 x 32 quadrants).  Each K-tile is computed in 4 PHASES, one quadrant per
// phase (16 MFMAs per wave); a phase is [load segment: fragment ds_reads + one half-tile of
// glds] s_barrier [compute segment: 16 MFMAs] s_barrier.  Waves 4-7 run one barrier behind
// waves 0-3, so on every SIMD one wave's MFMA segment overlaps its partner's load segment.
//
// LDS: two 64 KB buffers (even / odd K-tiles), each = four 16 KB half-tiles A0 A1 B0 B1.
// A half h holds the block rows {h*64 + [0,64)} u {128 + h*64 + [0,64)} (quadrant row h of
// both wave rows); B half h the block cols {wc*64 + h*32 + [0,32)} for wc = 0..3.  Quadrant
// order per tile: (m0,n0) reads A0+B0, (m0,n1) reads B1, (m1,n1) reads A1, (m1,n0) reads none
// (B0 frags kept in registers), so each half's last read is at a known phase.
// Restage schedule (phase p of the 8-phase iteration i, tiles 2i in E, 2i+1 in O):
//   p0 B1->O(2i+1)  p1 A1->O(2i+1)  p2 A0->E(2i+2)  p3 B0->E(2i+2) + wait O complete
//   p4 B1->E(2i+2)  p5 A1->E(2i+2)  p6 A0->O(2i+3)  p7 B0->O(2i+3) + wait E complete
// Every restage is >= 2 phases after the last read of that half (WAR safe under the one-
// barrier stagger); every wait retires a buffer one phase before its first read (RAW), with
// two younger half-tiles (4 glds) left in flight: s_waitcnt vmcnt(4), never 0 in the loop.
// ============================================================================================
namespace p8 {
constexpr int BM = 256, BNN = 256, BKK = 64, NTH = 512;
constexpr int HALF = 128 * 64 * 2;   // 16 KB
constexpr int TILEB = 4 * HALF;      // 64 KB per buffer
// LDS: two 64 KB buffers (E, O)
constexpr int SMEM_P = TILEB + 8 * 32 * EP_LD * 4;   // persistent: E + (O + staging overhang) = 132 KB
enum { A0 = 0, A1 = 1, B0 = 2, B1 = 3 };

__device__ __forceinline__ int kswz(int row) { return (row >> 1) & 7; }

// block-local row of half-local row j: A halves interleave 64-row groups, B halves 32-col groups
template <bool ISA>
__device__ __forceinline__ int half_row(int j, int h) {
  if constexpr (ISA) return (j >> 6) * 128 + h * 64 + (j & 63);
  else return (j >> 5) * 64 + h * 32 + (j & 31);
}

// this thread's 2 glds of one 128-row x 64-k half-tile
template <bool KC, bool ISA>
__device__ __forceinline__ void stage_half(char* dst, const u16* base, int64_t ld, int64_t rows, int64_t row0,
                                           int64_t k0, int h, int w, int lane) {
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int c = (w * 2 + j) * 64 + lane;
    const u16* src;
    if constexpr (KC) {
      const int r = c >> 3, pc = c & 7, lc = pc ^ kswz(r);
      const int64_t gr = min(row0 + half_row<ISA>(r, h), rows - 1);
      src = base + gr * ld + k0 + lc * 8;
    } else {
      const int kk = c >> 4, pc = c & 15, pb = pc >> 1, hf = pc & 1;
      const int lb = pb ^ mn_swz(kk);
      const int64_t gm = min(row0 + half_row<ISA>(lb * 16 + hf * 8, h), rows - 8);
      src = base + (k0 + kk) * ld + gm;
    }
    __builtin_amdgcn_global_load_lds((gvoid*)src, (lvoid*)(dst + (w * 2 + j) * 1024), 16, 0, 0);
  }
}

// A-operand-layout fragment (16 rows x 32 k) of half-local rows r0 + blk*16 + [0,16), k-substep s.
// K-contiguous image [128 rows][64 k]: ds_read_b128 at row r, 16-B chunk (s*4 + lane/16) ^ kswz(r);
// the swizzle depends only on lane bits, so blocks are plain immediate offsets (blk * 2 KB).
// MN-contiguous image [64 k][128 rows] via ds_read_b64_tr_b16: the per-lane byte offset of block 0
// is mn_base(); block blk flips bits 5-6 (32-B block index ^ blk, legal because r0 / 16 has its
// low bits clear), the k-substep adds 8 KB and the second k-quad adds 1 KB.
template <bool KC>
__device__ __forceinline__ int frag_base(int r0, int lane) {
  if constexpr (KC) {
    const int r = r0 + (lane & 15);
    return r * 128 + (((lane >> 4) ^ kswz(r)) << 4);
  } else {
    const int g = lane >> 4, i = lane & 15, q = i >> 2, pp = i & 3;
    const int k1 = 8 * g + q;
    return k1 * 256 + (((r0 >> 4) ^ mn_swz(k1)) << 5) + pp * 8;
  }
}
// ds_read_b64_tr_b16 at LDS byte address a + off through inline asm (off folds to one immediate
// once the phase loops are unrolled).  hipcc (ROCm 7.2) puts s_waitcnt vmcnt(0) in front of every
// ds_read_tr INTRINSIC while any global_load_lds is outstanding (it cannot prove they do not
// alias): 60-140 per MN-operand kernel, each draining the glds ring.  The asm form escapes that
// check and the compiler's lgkmcnt tracking: every fragment is consumed after compute_phase()'s
// explicit s_waitcnt lgkmcnt(0).
__device__ __forceinline__ s16x4 tr_asm(unsigned a, int off) {
  s16x4 r;
  switch (off) {
#define CT_TR(o) \
  case o: asm volatile("ds_read_b64_tr_b16 %0, %1 offset:" #o : "=v"(r) : "v"(a)); break;
    CT_TR(0) CT_TR(1024) CT_TR(8192) CT_TR(9216) CT_TR(16384) CT_TR(17408) CT_TR(24576) CT_TR(25600)
    CT_TR(32768) CT_TR(33792) CT_TR(40960) CT_TR(41984) CT_TR(49152) CT_TR(50176) CT_TR(57344) CT_TR(58368)
#undef CT_TR
    default: asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(a + off)); break;
  }
  return r;
}

// buf: base of the 64 KB buffer; which: half-tile index (A0 A1 B0 B1)
template <bool KC>
__device__ __forceinline__ bf16x8 hfrag(const char* buf, int which, int base, int blk, int s) {
  if constexpr (KC) {
    // chunk s*4 + c ^ sw = (c ^ sw) ^ (s*4): the k-substep flips bit 6 of the byte offset
    return *(const bf16x8*)(buf + which * HALF + ((base + blk * 2048) ^ (s << 6)));
  } else {
    const unsigned a = (unsigned)(size_t)LDS_PTR(char, buf) + (unsigned)(base ^ (blk << 5));
    const int off = which * HALF + s * 8192;
    s16x4 lo = tr_asm(a, off);
    s16x4 hi = tr_asm(a, off + 1024);
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
  }
}

__device__ __forceinline__ void bar() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

}  // namespace p8

// Epilogue for the TRANSPOSED accumulator layout of gemm8p (MFMA operands swapped, so block
// (i, j) holds D^T): lane l owns output row m = l & 15 of 16-row block i and the 4 consecutive
// columns 16 j + 4 g + [0, 4) (g = l >> 4).  No LDS staging: f32 outputs are 16-B stores per
// block; bf16 outputs pair blocks (j, j+1) with v_permlane16_swap so every lane stores 16
// contiguous bytes (lanes g = 0,1,2,3 -> columns 16j, 16j+16, 16j+8, 16j+24 of the pair).
__device__ __forceinline__ uint2 pk4(const float* v) { return make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3])); }

// one permlane16 pair: lanes g=0..3 end with 16 contiguous bytes at column offset pair_coff(g)
__device__ __forceinline__ u32x4 pair_swap(const float* x4, const float* y4) {
  const uint2 x = pk4(x4), y = pk4(y4);
  const auto r0 = __builtin_amdgcn_permlane16_swap(x.x, y.x, false, false);
  const auto r1 = __builtin_amdgcn_permlane16_swap(x.y, y.y, false, false);
  return make_uint4(r0[0], r1[0], r0[1], r1[1]);
}
__device__ __forceinline__ int pair_coff(int g) { return ((g & 1) ? 16 : 0) + ((g & 2) ? 8 : 0); }
// the same pairing for fp16 values
__device__ __forceinline__ u32x4 pair_swap_h(const float* x4, const float* y4) {
  const uint2 x = pack4h(x4), y = pack4h(y4);
  const auto r0 = __builtin_amdgcn_permlane16_swap(x.x, y.x, false, false);
  const auto r1 = __builtin_amdgcn_permlane16_swap(x.y, y.y, false, false);
  return make_uint4(r0[0], r1[0], r0[1], r1[1]);
}

// value of lane ^ 16 / lane ^ 32 through v_permlane16_swap / v_permlane32_swap (VALU) instead of
// ds_bpermute (the LDS crossbar, ~100+ cycles each in the argmax / l2norm epilogues).  Swapping x
// with itself leaves (even rows / low half in [0], odd rows / high half in [1]) exchanged copies.
__device__ __forceinline__ unsigned xor16_u(unsigned x, int lane) {
  const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
  return (lane & 16) ? r[0] : r[1];
}
__device__ __forceinline__ unsigned xor32_u(unsigned x, int lane) {
  const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
  return (lane & 32) ? r[0] : r[1];
}
template <int O> __device__ __forceinline__ float xorf(float x, int lane) {
  return __uint_as_float(O == 16 ? xor16_u(__float_as_uint(x), lane) : xor32_u(__float_as_uint(x), lane));
}
template <int O> __device__ __forceinline__ int xori(int x, int lane) {
  return (int)(O == 16 ? xor16_u((unsigned)x, lane) : xor32_u((unsigned)x, lane));
}

// 16-B epilogue store; CTCLIP_EPI_SC1 (A/B build): write-through sc1, which drops the line from
// the XCD's L2 instead of keeping it (MI355X_MICROARCH.md, store flavours), so the output stream
// does not evict the operand panels that the XCD's other tiles re-read
__device__ __forceinline__ void st16(void* p, u32x4 d) {
#ifdef CTCLIP_EPI_SC1
  typedef unsigned int v4u __attribute__((ext_vector_type(4)));
  const v4u dv = {d.x, d.y, d.z, d.w};
  asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(dv) : "memory");
#else
  *(u32x4*)p = d;
#endif
}

// 16-B store that drops its line from the XCD's L2 (sc1; MI355X_MICROARCH.md, store flavours)
__device__ __forceinline__ void st16_sc1(void* p, u32x4 d) {
  typedef unsigned int v4u __attribute__((ext_vector_type(4)));
  const v4u dv = {d.x, d.y, d.z, d.w};
  asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(dv) : "memory");
}

// store one row's 4 j-blocks x 4 cols as bf16; rowp = row base at the wave's first column c0
__device__ __forceinline__ void store_row_bf16(u16* rowp, const float (&v)[4][4], int g, bool ok, int64_t c0,
                                               int64_t N, bool sc1 = false) {
#pragma unroll
  for (int jp = 0; jp < 2; ++jp) {
    const u32x4 d = pair_swap(v[2 * jp], v[2 * jp + 1]);
    const int coff = 32 * jp + pair_coff(g);
    if (ok && c0 + coff < N) {
      if (sc1) st16_sc1(rowp + coff, d);
      else st16(rowp + coff, d);
    }
  }
}

// store one row's 4 j-blocks x 4 cols as fp16 (FF1's h in the fp16 GEMM)
__device__ __forceinline__ void store_row_f16(u16* rowp, const float (&v)[4][4], int g, bool ok, int64_t c0,
                                              int64_t N) {
#pragma unroll
  for (int jp = 0; jp < 2; ++jp) {
    const u32x4 d = pair_swap_h(v[2 * jp], v[2 * jp + 1]);
    const int coff = 32 * jp + pair_coff(g);
    if (ok && c0 + coff < N) st16(rowp + coff, d);
  }
}

// The same 16-row block of 64 bf16 columns (rows gm0 .. gm0 + 15, C at (gm0, c0)) through the
// wave's LDS scratch: a lane of the transposed layout holds one row (lane & 15), so its 16-B stores
// are 16 rows x 64 B per instruction with consecutive lanes on different rows -- the per-CU store
// path drains that at ~16 B/cycle, against ~57 B/cycle when consecutive lanes write consecutive
// 16 B of a row (tools/store_probe.hip, profiles/r04c_store_probe.log).  Rows are staged at a
// 144-B pitch (16 distinct bank quads for the b128 writes) and read back row-major, 8 lanes per
// 128-B row.  Wave-private scratch: LDS order within the wave is program order, no barrier.
constexpr int SCR_H = 144, SCR_G = 80, SCR_GOFF = 16 * SCR_H;   // h block 2304 B + g block 1280 B
__device__ __forceinline__ void store_blk_bf16_lds(char* scr, u16* C, int64_t ldc, int64_t gm0, int64_t M, int64_t c0,
                                                   int64_t N, const float (&v)[4][4], int g, int m, int lane,
                                                   bool sc1) {
#pragma unroll
  for (int jp = 0; jp < 2; ++jp)
    *(u32x4*)(scr + m * SCR_H + (32 * jp + pair_coff(g)) * 2) = pair_swap(v[2 * jp], v[2 * jp + 1]);
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int r = 8 * h + (lane >> 3), c = (lane & 7) * 8;
    const u32x4 d = *(const u32x4*)(scr + r * SCR_H + c * 2);
    if (gm0 + r < M && c0 + c < N) {
      if (sc1) st16_sc1(C + r * ldc + c, d);
      else st16(C + r * ldc + c, d);
    }
  }
}

// MODE (compile time, so each variant's row loop stays small enough to unroll fully and the
// accumulator never leaves registers): 0 = general (bias / residual / GELU / f32 or bf16 /
// accumulate / shadow), 2 = GEGLU, 3 = argmax, 4 = GEGLU backward, 5 = split-K slab.
#ifndef CTCLIP_GEMM_PERMLANE
#define CTCLIP_GEMM_PERMLANE 0
#endif
// A/B build switch of the xor16 / xor32 exchanges: permlane swaps measured 2 % slower than
// ds_bpermute on the VQ argmax GEMM (1.193 vs 1.171-1.176 ms, profiles/r02aw_*), so off
constexpr bool GEMM_PERMLANE = CTCLIP_GEMM_PERMLANE;

template <int MODE, bool LDS = false, bool H16 = false, bool X3 = false>
__device__ __forceinline__ void epilogue_t(const P& p, f32x4 (&acc)[8][4], int wr, int wc, int lane, int64_t m0,
                                           int64_t n0, int split, int bidx, char* scr) {
  const int m = lane & 15, g = lane >> 4;
  const int64_t wrow0 = m0 + wr * 128, wcol0 = n0 + wc * 64;
  const int64_t cl = wcol0 + 4 * g;          // this lane's column in block j: cl + 16 j
  float bias[4][4];
  // EP 8: this wave's columns are LayerNorm-folded (wave-uniform); bias[][] then holds fold_cs
  const bool fold = MODE == 8 && wcol0 < p.nfold;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    f32x4 b = f32x4{0.f, 0.f, 0.f, 0.f};
    if (MODE == 8) {
      if (fold) b = *(const f32x4*)(p.fold_cs + cl + 16 * j);
    } else if (p.bias && p.split_k <= 1 && p.act != 3 && p.act != 5 && cl + 16 * j < p.N) b = *(const f32x4*)(p.bias + cl + 16 * j);
#pragma unroll
    for (int r = 0; r < 4; ++r) bias[j][r] = b[r];
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int64_t gm = wrow0 + i * 16 + m;
    const bool rok = gm < p.M;
    float v[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) v[j][r] = acc[i][j][r] * p.alpha;
    if constexpr (MODE == 3) {
      // argmax over the wave's 64 columns of row gm (first-max tie-break): 16 values per lane,
      // then across the 4 lanes g = 0..3 that hold the same row
      // branch-free (selects): the if / else form compiled to exec-mask branches per element and
      // made this epilogue as long as the tile's whole main loop (r02 stamps: 31.5 k cycles).  A
      // lane scans its columns in increasing order, so the in-lane tie-break (first max) is a
      // strict >; columns past N read as -inf and never win (bi stays 0x7fffffff when all are)
      // (best, second) as max / med3: second = med3(best, second, x) is the old best when x wins,
      // x when it lands between, else unchanged -- the select chain's values with 2 VALU instead of
      // 4; the column guard only on a wave whose 64 columns cross N (wave-uniform)
      float best = -INFINITY, second = -INFINITY;
      int bi = 0x7fffffff;
      const bool cfull = wcol0 + 64 <= p.N;
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int c = 16 * j + 4 * g + r;
          const float x = cfull || wcol0 + c < p.N ? v[j][r] : -INFINITY;
          bi = x > best ? c : bi;
          second = __builtin_amdgcn_fmed3f(best, second, x);
          best = fmaxf(best, x);
        }
      auto merge = [&](float ob, float os, int oi) {
        const bool take = ob > best || (ob == best && oi < bi);
        second = take ? fmaxf(best, os) : fmaxf(second, ob);
        bi = take ? oi : bi;
        best = take ? ob : best;
      };
      if (GEMM_PERMLANE) {
        { const float ob = xorf<16>(best, lane), os = xorf<16>(second, lane); merge(ob, os, xori<16>(bi, lane)); }
        { const float ob = xorf<32>(best, lane), os = xorf<32>(second, lane); merge(ob, os, xori<32>(bi, lane)); }
      } else {
#pragma unroll
        for (int o = 16; o <= 32; o <<= 1)
          merge(__shfl_xor(best, o, 64), __shfl_xor(second, o, 64), __shfl_xor(bi, o, 64));
      }
      if (g == 0 && rok && wcol0 < p.N) {
        float2* out = (float2*)p.C + bidx * p.sC;
        out[gm * p.ldc + (wcol0 >> 6)] = make_float2(best, __int_as_float((int)(wcol0 + bi)));
        if (p.C2) ((float*)p.C2)[bidx * p.sC2 + gm * p.ldc2 + (wcol0 >> 6)] = second;
      }
      continue;
    }
    if constexpr (MODE == 8) {
      // LayerNorm folded into the projection (ctclip_gemm_qkv_lnfold): LN(x) W^T =
      // rstd (x (gamma o W)^T - mean (W gamma)), gamma o W pre-packed, W gamma = fold_cs
      if (fold) {
        const int64_t gr = rok ? gm : p.M - 1;
        const float mu = p.ln_mean[gr], rs = p.ln_rstd[gr];
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) v[j][r] = rs * (v[j][r] - mu * bias[j][r]);
      }
    }
    if constexpr (MODE == 6 || MODE == 8) {
      // C = bf16 result; C2 = its l2norm over each 32-column head (the wave's 64 columns are two
      // heads) times the head-dim scale p.bias[c % 32], bit-identical to ctclip_l2norm_scale_fwd
      // (EP 8: p.bias holds two 32-scales, the folded columns' then the rest's):
      // the permlane16 pair swap leaves each lane 8 consecutive columns (a chunk: offset
      // pair_coff(g)), summed in that kernel's order, then combined chunk 0+1, 2+3 (lanes g ^ 2)
      // and the two pairs (g ^ 1), as its xor-1 / xor-2 shuffles over the 4 lanes of a head
      float qb[4][4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) qb[j][r] = bf2f(f2bf(v[j][r]));
      // (EP 8: columns below c_col0 -- q, k in the eval forward, round 6 -- only feed the l2norm)
      store_row_bf16((u16*)p.C + bidx * p.sC + gm * p.ldc + wcol0, v, g, rok && wcol0 >= p.c_col0, wcol0, p.N);
      if (wcol0 < p.n2) {
        const int d0 = pair_coff(g);
        const float* sp = p.bias + d0 + (MODE == 8 && !fold ? 32 : 0);   // EP 8: the second scale set
        const f32x4 s0v = *(const f32x4*)sp, s1v = *(const f32x4*)(sp + 4);
#pragma unroll
        for (int jp = 0; jp < 2; ++jp) {
          float c8[8];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(qb[2 * jp][k]),
                                                            __float_as_uint(qb[2 * jp + 1][k]), false, false);
            c8[k] = __uint_as_float(r[0]);
            c8[4 + k] = __uint_as_float(r[1]);
          }
          float ss = 0.f;
#pragma unroll
          for (int e = 0; e < 8; ++e) ss += c8[e] * c8[e];
          if (GEMM_PERMLANE) {
            ss += xorf<32>(ss, lane);
            ss += xorf<16>(ss, lane);
          } else {
            ss += __shfl_xor(ss, 32, 64);
            ss += __shfl_xor(ss, 16, 64);
          }
          const float inv = 1.f / fmaxf(sqrtf(ss), 1e-12f);
          float o8[8];
#pragma unroll
          for (int e = 0; e < 4; ++e) { o8[e] = c8[e] * inv * s0v[e]; o8[4 + e] = c8[4 + e] * inv * s1v[e]; }
          const int64_t c0 = wcol0 + 32 * jp + d0;
          if (rok && c0 < p.n2) st16(p.C2 + bidx * p.sC2 + gm * p.ldc2 + c0, pack8(o8));
        }
      }
      continue;
    }
    if constexpr (MODE == 5) {
      float* Cf = (float*)p.C + (int64_t)split * p.M * p.ldc + bidx * p.sC + gm * p.ldc + cl;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (rok && cl + 16 * j < p.N) *(f32x4*)(Cf + 16 * j) = f32x4{v[j][0], v[j][1], v[j][2], v[j][3]};
      continue;
    }
    if constexpr (MODE == 2) {
      // GEGLU in 32-column pairs: blocks 0,1 = x, blocks 2,3 = gate; h keeps both halves
      if constexpr (LDS) {
        const int64_t gm0 = wrow0 + i * 16;
        store_blk_bf16_lds(scr, (u16*)p.C + bidx * p.sC + gm0 * p.ldc + wcol0, p.ldc, gm0, p.M, wcol0, p.N, v, g, m,
                           lane, p.epi_lds == 2);
        float gg[2][4];
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) gg[j][r] = gelu_erf(bf2f(f2bf(v[j + 2][r]))) * bf2f(f2bf(v[j][r]));
        *(u32x4*)(scr + SCR_GOFF + m * SCR_G + pair_coff(g) * 2) = pair_swap(gg[0], gg[1]);
        const int r = lane >> 2, c = (lane & 3) * 8;
        const u32x4 d = *(const u32x4*)(scr + SCR_GOFF + r * SCR_G + c * 2);
        if (gm0 + r < p.M && wcol0 < p.N) {
          if (p.epi_lds == 2) st16_sc1(p.C2 + bidx * p.sC2 + (gm0 + r) * p.ldc2 + (wcol0 >> 1) + c, d);
          else st16(p.C2 + bidx * p.sC2 + (gm0 + r) * p.ldc2 + (wcol0 >> 1) + c, d);
        }
        continue;
      }
      if constexpr (X3) {
        // split-fp16 kernel: h stored as fp16 (the GEGLU backward's operand), g from the unrounded
        // f32 h (the x3 forward carries ~22-bit values end to end), stored as its fp16 pair
        // (hi, lo = fp16(g - hi): FF2's A operand) and as bf16 (FF2's weight-gradient operand)
        // (h in the derivative form of the fp16 kernel below)
        float gg[2][4], gh[2][4], gl[2][4], hv[4][4];
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float ge, dge;
            gelu_erf_and_grad(v[j + 2][r], ge, dge);
            hv[j][r] = ge;
            hv[j + 2][r] = v[j][r] * dge;
            gg[j][r] = ge * v[j][r];
            gh[j][r] = rh(gg[j][r]);
            gl[j][r] = gg[j][r] - gh[j][r];
          }
        store_row_f16((u16*)p.C + bidx * p.sC + gm * p.ldc + wcol0, hv, g, rok, wcol0, p.N);
        // (cross-lane swaps outside the store guard: every lane takes part)
        const u32x4 dh = pair_swap_h(gh[0], gh[1]), dl = pair_swap_h(gl[0], gl[1]), db = pair_swap(gg[0], gg[1]);
        if (rok && wcol0 < p.N) {
          const int64_t gc = (wcol0 >> 1) + pair_coff(g);
          st16(p.C2 + bidx * p.sC2 + gm * p.ldc2 + gc, dh);
          st16(p.C3 + gm * p.ldc3 + gc, dl);
          if (p.C4) st16(p.C4 + gm * p.ldc4 + gc, db);
        }
        continue;
      }
      // fp16 kernel (round 6): h is stored in its DERIVATIVE form, the two factors the GEGLU backward
      // multiplies dg by -- [gelu(gate) | x gelu'(gate)] in place of [x | gate] (same bytes), so the
      // backward epilogue is two multiplies per element instead of an erf + exp per element; g and
      // the factors from the fp16-rounded x / gate (the round-5 forward arithmetic: g bit for bit as
      // before, the factors its exact derivative).  bf16 kernel: h = [x | gate] in bf16, g from the
      // bf16-rounded h (the backward recomputes gelu from the stored h).
      // (h may be discarded, C = NULL: the eval forward needs only g, round 6)
      float gg[2][4];
      if constexpr (H16) {
        float hv[4][4];
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float xb = rh(v[j][r]);
            float ge, dge;
            gelu_erf_and_grad(rh(v[j + 2][r]), ge, dge);
            hv[j][r] = ge;
            hv[j + 2][r] = xb * dge;
            gg[j][r] = ge * xb;
          }
        store_row_f16((u16*)p.C + bidx * p.sC + gm * p.ldc + wcol0, hv, g, rok && p.C, wcol0, p.N);
      } else {
        store_row_bf16((u16*)p.C + bidx * p.sC + gm * p.ldc + wcol0, v, g, rok, wcol0, p.N, p.epi_lds == 3);
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) gg[j][r] = gelu_erf(bf2f(f2bf(v[j + 2][r]))) * bf2f(f2bf(v[j][r]));
      }
      const u32x4 d = pair_swap(gg[0], gg[1]);
      if (rok && wcol0 < p.N) {
        if (p.epi_lds == 3) st16_sc1(p.C2 + bidx * p.sC2 + gm * p.ldc2 + (wcol0 >> 1) + pair_coff(g), d);
        else st16(p.C2 + bidx * p.sC2 + gm * p.ldc2 + (wcol0 >> 1) + pair_coff(g), d);
      }
      continue;
    }
    if constexpr (MODE != 0) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) v[j][r] += bias[j][r];
    if (p.R) {
      if (p.r_f32) {
        const float* Rp = (const float*)p.R + bidx * p.sR + gm * p.ldr + cl;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (rok && cl + 16 * j < p.N) {
            const f32x4 a = *(const f32x4*)(Rp + 16 * j);
#pragma unroll
            for (int r = 0; r < 4; ++r) v[j][r] += a[r];
          }
      } else {
        const u16* Rp = (const u16*)p.R + bidx * p.sR + gm * p.ldr + cl;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (rok && cl + 16 * j < p.N) {
            float rr[4];
            unpack4(*(const uint2*)(Rp + 16 * j), rr);
#pragma unroll
            for (int r = 0; r < 4; ++r) v[j][r] += rr[r];
          }
      }
    }
    if (p.act == 1) {
      if (p.C2) store_row_bf16(p.C2 + bidx * p.sC2 + gm * p.ldc2 + wcol0, v, g, rok, wcol0, p.N);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) v[j][r] = gelu_erf(v[j][r]);
    }
    if (p.c_f32) {
      float* Cf = (float*)p.C + bidx * p.sC + gm * p.ldc + cl;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (rok && cl + 16 * j < p.N) {
          if (p.accumulate) {
            const f32x4 a = *(const f32x4*)(Cf + 16 * j);
#pragma unroll
            for (int r = 0; r < 4; ++r) v[j][r] += a[r];
          }
          *(f32x4*)(Cf + 16 * j) = f32x4{v[j][0], v[j][1], v[j][2], v[j][3]};
        }
    } else {
      u16* Cb = (u16*)p.C + bidx * p.sC + gm * p.ldc + wcol0;
      if (p.accumulate) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (rok && cl + 16 * j < p.N) {
            float rr[4];
            unpack4(*(const uint2*)(Cb + 16 * j + 4 * g), rr);
#pragma unroll
            for (int r = 0; r < 4; ++r) v[j][r] += rr[r];
          }
      }
      if constexpr (LDS) {
        const int64_t gm0 = wrow0 + i * 16;
        store_blk_bf16_lds(scr, (u16*)p.C + bidx * p.sC + gm0 * p.ldc + wcol0, p.ldc, gm0, p.M, wcol0, p.N, v, g, m,
                           lane, p.epi_lds == 2);
      } else {
        store_row_bf16(Cb, v, g, rok, wcol0, p.N, p.epi_lds == 3);
      }
    }
    if (p.C2 && p.act == 0) {
      if constexpr (LDS) {
        const int64_t gm0 = wrow0 + i * 16;
        store_blk_bf16_lds(scr, p.C2 + bidx * p.sC2 + gm0 * p.ldc2 + wcol0, p.ldc2, gm0, p.M, wcol0, p.N, v, g, m,
                           lane, p.epi_lds == 2);
      } else {
        store_row_bf16(p.C2 + bidx * p.sC2 + gm * p.ldc2 + wcol0, v, g, rok, wcol0, p.N, p.epi_lds == 3);
      }
    }
  }
}

// GEGLU backward fused into dg = dy . W2 (TR layout): the accumulator is dg over g-space
// columns; block pair (0,1) is 32-group t0 = wcol0 / 32, pair (2,3) group t0 + 1.  dg is
// rounded to bf16 (as the stand-alone geglu_bwd reads it) and permlane-paired so every lane
// owns 8 consecutive g-columns: one 16-B load of h's x part, one of its gate part, one 16-B
// store each of dh.  The next row block's h loads are issued before this block's math.
#ifndef GEGLU_BWD_LA
#define GEGLU_BWD_LA 1
#endif
__device__ __forceinline__ void epilogue_geglu_bwd(const P& p, f32x4 (&acc)[8][4], int wr, int wc, int lane,
                                                   int64_t m0, int64_t n0, int bidx) {
  const int m = lane & 15, g = lane >> 4;
  const int64_t wrow0 = m0 + wr * 128, wcol0 = n0 + wc * 64, t0 = wcol0 >> 5;
  const int co = pair_coff(g);
  const u16* hb = (const u16*)p.R + bidx * p.sR;
  u16* db = (u16*)p.C + bidx * p.sC;
  constexpr int LA = GEGLU_BWD_LA;   // row blocks of h loads in flight ahead of the math
  u32x4 hx[LA + 1][2], hg[LA + 1][2];
  auto load = [&](int i, int b) {
    const int64_t gm = wrow0 + i * 16 + m;
#pragma unroll
    for (int jp = 0; jp < 2; ++jp) {
      const int64_t t = t0 + jp;
      if (gm < p.M && t * 32 < p.N) {
        const u16* hp = hb + gm * p.ldr + t * 64 + co;
        hx[b][jp] = *(const u32x4*)hp;
        hg[b][jp] = *(const u32x4*)(hp + 32);
      } else {
        hx[b][jp] = make_uint4(0, 0, 0, 0);
        hg[b][jp] = make_uint4(0, 0, 0, 0);
      }
    }
  };
#pragma unroll
  for (int i = 0; i < LA; ++i) load(i, i);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int b = i % (LA + 1);
    if (i + LA < 8) load(i + LA, (i + LA) % (LA + 1));
    const int64_t gm = wrow0 + i * 16 + m;
#pragma unroll
    for (int jp = 0; jp < 2; ++jp) {
      float v0[4], v1[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) { v0[r] = acc[i][2 * jp][r] * p.alpha; v1[r] = acc[i][2 * jp + 1][r] * p.alpha; }
      float d[8], x[8], gt[8], ox[8], og[8];
      unpack8(pair_swap(v0, v1), d);
      if (p.h16) {   // h from the fp16 forward (wave-uniform): the derivative form, two multiplies
        unpack8h(hx[b][jp], x);    // gelu(gate)
        unpack8h(hg[b][jp], gt);   // x gelu'(gate)
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          ox[k] = d[k] * x[k];
          og[k] = d[k] * gt[k];
        }
      } else {
        unpack8(hx[b][jp], x);
        unpack8(hg[b][jp], gt);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          float ge, dge;
          gelu_erf_and_grad(gt[k], ge, dge);
          ox[k] = d[k] * ge;
          og[k] = d[k] * x[k] * dge;
        }
      }
      const int64_t t = t0 + jp;
      if (gm < p.M && t * 32 < p.N) {
        u16* dp = db + gm * p.ldc + t * 64 + co;
        st16(dp, pack8(ox));
        st16(dp + 32, pack8(og));
      }
    }
  }
}

// ============================================================================================
// LayerNorm fused into the epilogue of an N = 512 GEMM (ctclip_gemm_ln; the 3D-ViT's d = 512
// rows).  A row's 512 columns are two 256-column tiles.  In the persistent walk tile_at hands the
// row block's tiles 2k, 2k + 1 to workgroups w, w ^ 8 of the SAME round whenever ntiles % 16 == 0
// and the grid is min(ntiles, 256) (the host checks both), so the pair is co-scheduled and each
// waits only on the other.  Each tile reduces its 256 columns per row (a wave: 8 lanes x 8 values
// through xor shuffles, then the 4 column waves through LDS), publishes the two per-row values as
// 8-byte {epoch, value} granules (relaxed agent-scope atomic stores, sc1: the data is the flag,
// MI355X_MICROARCH.md § visibility, R2) and polls the partner's with relaxed agent-scope loads
// (sc1, bypassing L1; bounded: a timeout sets *status and continues).  Both tiles combine the two
// halves with symmetric formulas, so the two halves of a row see bit-identical statistics.
//   MODE 6 (forward): v = alpha acc + bias + R -> C (f32) and C2 (bf16); per-row (mean, M2) merged
//     pairwise at equal counts (Chan et al.), y = (v - mean) rstd gamma + beta -> ln_y (bf16);
//     tile 0 writes mean / rstd.  Replaces residual GEMM + ln_fwd_kernel.
//   MODE 7 (backward): dy = bf16(alpha acc) (what the unfused GEMM stored), xh = (x - mean) rstd,
//     g = dy gamma; the row sums of g and g xh are exchanged; C = rstd (g - mean(g) - xh mean(g xh))
//     + R, C2 = bf16(C); per 128-row block the column sums of dy xh / dy -> ln_pg / ln_pb.  Replaces
//     the GEMM + ln_bwd_kernel pair (same arithmetic, the sums in another order).
// LDS: the staging area of the general epilogue (buffer O and beyond) plus 10 KB of statistics.
// ============================================================================================
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) int gi32;
constexpr int LN_ST = p8::SMEM_P;                // [2 wr][128 rows][4 wc] float2 per-wave row values
constexpr int LN_FIN = LN_ST + 2 * 128 * 4 * 8;  // [256 rows] float2 (mean, rstd) / (mean g, mean g xh)
constexpr int SMEM_LN = LN_FIN + 256 * 8;
constexpr unsigned LN_SPIN_LIMIT = 1u << 21;     // default: ~0.1 s of polling before giving up

// merge two equal-count (mean, M2) partials; symmetric in its arguments, so the lanes / tiles of
// a pair that merge (a, b) and (b, a) agree bit for bit
__device__ __forceinline__ void chan(float& m, float& M2, float mb, float M2b, float half_n) {
  const float d = m - mb;
  M2 = (M2 + M2b) + d * d * half_n;
  m = 0.5f * (m + mb);
}

template <int MODE>
__device__ __forceinline__ void epilogue_ln(const P& p, f32x4 (&acc)[8][4], char* smem, int w, int wr, int wc,
                                            int lane, int64_t m0, int64_t n0) {
  float* cs = (float*)(smem + p8::TILEB + w * (32 * EP_LD * 4));
  float2* st = (float2*)(smem + LN_ST);
  float2* fin = (float2*)(smem + LN_FIN);
  const int tx = (int)(n0 >> 8);
  const int64_t wrow0 = m0 + wr * 128, wcol0 = n0 + wc * 64;
  const int cc = (lane & 7) * 8, rl = lane >> 3;
  const int64_t gn = wcol0 + cc;
  float gam[8], bet[8];
  {
    const f32x4 a = *(const f32x4*)(p.ln_gamma + gn), b = *(const f32x4*)(p.ln_gamma + gn + 4);
    f32x4 c = f32x4{0.f, 0.f, 0.f, 0.f}, d = c;
    if (MODE == 6 && p.ln_beta) { c = *(const f32x4*)(p.ln_beta + gn); d = *(const f32x4*)(p.ln_beta + gn + 4); }
#pragma unroll
    for (int j = 0; j < 4; ++j) { gam[j] = a[j]; gam[4 + j] = b[j]; bet[j] = c[j]; bet[4 + j] = d[j]; }
  }
  f32x4 b0 = f32x4{0.f, 0.f, 0.f, 0.f}, b1 = b0;
  if (MODE == 6 && p.bias) { b0 = *(const f32x4*)(p.bias + gn); b1 = *(const f32x4*)(p.bias + gn + 4); }
  float keep[4][4][8];        // MODE 6: v per quarter / row chunk
  float pg[8], pb[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { pg[j] = 0.f; pb[j] = 0.f; }

#pragma unroll
  for (int quarter = 0; quarter < 4; ++quarter) {
    __builtin_amdgcn_sched_barrier(0);   // no hoisting of a later quarter's loads over this one
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          cs[(i * 16 + (lane >> 4) * 4 + r) * EP_LD + j * 16 + (lane & 15)] = acc[quarter * 2 + i][j][r];
    __builtin_amdgcn_s_waitcnt(0xC07F);
    const int64_t rbase = wrow0 + quarter * 32;
    if constexpr (MODE == 6) {
      f32x4 ra[4], rb[4];
#pragma unroll
      for (int it = 0; it < 4; ++it) {
        const float* Rp = (const float*)p.R + (rbase + it * 8 + rl) * p.ldr + gn;
        ra[it] = *(const f32x4*)Rp;
        rb[it] = *(const f32x4*)(Rp + 4);
      }
#pragma unroll
      for (int it = 0; it < 4; ++it) {
        const f32x4 lo = *(const f32x4*)(cs + (it * 8 + rl) * EP_LD + cc);
        const f32x4 hi = *(const f32x4*)(cs + (it * 8 + rl) * EP_LD + cc + 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          keep[quarter][it][j] = lo[j] * p.alpha + b0[j] + ra[it][j];
          keep[quarter][it][4 + j] = hi[j] * p.alpha + b1[j] + rb[it][j];
        }
      }
#pragma unroll
      for (int it = 0; it < 4; ++it) {
        const float* v = keep[quarter][it];
        float* Cf = (float*)p.C + (rbase + it * 8 + rl) * p.ldc + gn;
        *(f32x4*)Cf = f32x4{v[0], v[1], v[2], v[3]};
        *(f32x4*)(Cf + 4) = f32x4{v[4], v[5], v[6], v[7]};
      }
      if (p.C2) {
#pragma unroll
        for (int it = 0; it < 4; ++it) *(u32x4*)(p.C2 + (rbase + it * 8 + rl) * p.ldc2 + gn) = pack8(keep[quarter][it]);
      }
#pragma unroll
      for (int it = 0; it < 4; ++it) {
        const float* v = keep[quarter][it];
        float m = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) m += v[j];
        m *= 0.125f;
        float M2 = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) { const float d = v[j] - m; M2 += d * d; }
#pragma unroll
        for (int o = 1; o <= 4; o <<= 1) chan(m, M2, __shfl_xor(m, o, 64), __shfl_xor(M2, o, 64), 4.f * o);
        if ((lane & 7) == 0) st[(wr * 128 + quarter * 32 + it * 8 + rl) * 4 + wc] = make_float2(m, M2);
      }
    } else {
      float mu[4], rs[4];
      u32x4 kx[4];
#pragma unroll
      for (int it = 0; it < 4; ++it) {
        const int64_t row = rbase + it * 8 + rl;
        kx[it] = *(const u32x4*)(p.ln_x + row * p.ln_ldx + gn);
        mu[it] = p.ln_mean[row];
        rs[it] = p.ln_rstd[row];
      }
#pragma unroll
      for (int it = 0; it < 4; ++it) {
        const f32x4 lo = *(const f32x4*)(cs + (it * 8 + rl) * EP_LD + cc);
        const f32x4 hi = *(const f32x4*)(cs + (it * 8 + rl) * EP_LD + cc + 4);
        float d[8];
#pragma unroll
        for (int j = 0; j < 4; ++j) { d[j] = lo[j] * p.alpha; d[4 + j] = hi[j] * p.alpha; }
        const u32x4 kd = pack8(d);
        // dy parks in C2 (the bf16 dx output, same shape): re-read by this lane in the final pass
        // and overwritten there (registers cannot hold it across the exchange without spilling)
        *(u32x4*)(p.C2 + (rbase + it * 8 + rl) * p.ldc2 + gn) = kd;
        float dy[8], xv[8];
        unpack8(kd, dy);
        unpack8(kx[it], xv);
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float xh = (xv[j] - mu[it]) * rs[it];
          const float g = dy[j] * gam[j];
          s1 += g;
          s2 += g * xh;
        }
#pragma unroll
        for (int o = 1; o <= 4; o <<= 1) { s1 += __shfl_xor(s1, o, 64); s2 += __shfl_xor(s2, o, 64); }
        if ((lane & 7) == 0) st[(wr * 128 + quarter * 32 + it * 8 + rl) * 4 + wc] = make_float2(s1, s2);
      }
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);   // staging reads done before the next quarter overwrites
  }
  __syncthreads();
  if (wc == 0) {
    // this tile's per-row values (rows lane, lane + 64 of the wave row) -> granules; the partner's
    gu64* X = (gu64*)p.xchg;
    const unsigned long long tag = (unsigned long long)p.epoch << 32;
    float a0[2], a1[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int r = lane + 64 * h;
      const float2 s0 = st[(wr * 128 + r) * 4 + 0], s1 = st[(wr * 128 + r) * 4 + 1];
      const float2 s2 = st[(wr * 128 + r) * 4 + 2], s3 = st[(wr * 128 + r) * 4 + 3];
      if constexpr (MODE == 6) {
        float m = s0.x, M2 = s0.y, mm = s2.x, MM = s2.y;
        chan(m, M2, s1.x, s1.y, 32.f);
        chan(mm, MM, s3.x, s3.y, 32.f);
        chan(m, M2, mm, MM, 64.f);
        a0[h] = m;
        a1[h] = M2;
      } else {
        a0[h] = (s0.x + s1.x) + (s2.x + s3.x);
        a1[h] = (s0.y + s1.y) + (s2.y + s3.y);
      }
      gu64* g = X + ((int64_t)tx * p.M + wrow0 + r) * 2;
      if (!(p.ln_debug && tx == 1 && m0 == 0)) {   // (test knob: a partner that never publishes)
        __hip_atomic_store(g, tag | __float_as_uint(a0[h]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(g + 1, tag | __float_as_uint(a1[h]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    const gu64* Y = X + (int64_t)(1 - tx) * p.M * 2;
    unsigned long long q[2][2];
    for (unsigned spins = 0;; ++spins) {
      bool ok = true;
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          q[h][k] = __hip_atomic_load(Y + (wrow0 + lane + 64 * h) * 2 + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ok = ok && (unsigned)(q[h][k] >> 32) == p.epoch;
        }
      if (__all(ok)) break;
      if (spins >= p.spin_limit) {
        if (lane == 0 && p.status) __hip_atomic_store((gi32*)p.status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int r = lane + 64 * h;
      const float o0 = __uint_as_float((unsigned)q[h][0]), o1 = __uint_as_float((unsigned)q[h][1]);
      float2 f;
      if constexpr (MODE == 6) {
        float m = a0[h], M2 = a1[h];
        chan(m, M2, o0, o1, 128.f);
        const float rstd = rsqrtf(M2 * (1.f / 512.f) + p.ln_eps);
        f = make_float2(m, rstd);
        if (tx == 0) {
          p.ln_mean[wrow0 + r] = m;
          p.ln_rstd[wrow0 + r] = rstd;
        }
      } else {
        f = make_float2((a0[h] + o0) * (1.f / 512.f), (a1[h] + o1) * (1.f / 512.f));
      }
      fin[wr * 128 + r] = f;
    }
  }
  __syncthreads();
  const u16* lx = p.ln_x;
  u16* lc2 = p.C2;
  const float* lmean = p.ln_mean;
  const float* lrstd = p.ln_rstd;
  // opaque copy of this lane's row / column origin: no first-pass row address is reused (kept live)
  int64_t frow0 = wrow0 + rl, fcol = gn;
  asm volatile("" : "+v"(frow0), "+v"(fcol));
#pragma unroll
  for (int quarter = 0; quarter < 4; ++quarter) {
    __builtin_amdgcn_sched_barrier(0);
    const int64_t rbase = frow0 - rl + quarter * 32;
    if constexpr (MODE == 6) {
#pragma unroll
      for (int it = 0; it < 4; ++it) {
        const float2 f = fin[wr * 128 + quarter * 32 + it * 8 + rl];
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = (keep[quarter][it][j] - f.x) * f.y * gam[j] + bet[j];
        if (p.ln_y) *(u32x4*)(p.ln_y + (rbase + it * 8 + rl) * p.ln_ldy + gn) = pack8(o);
        if (p.ln_y16) *(u32x4*)(p.ln_y16 + (rbase + it * 8 + rl) * p.ln_ldy + gn) = pack8h(o);
      }
    } else {
      // 32-bit element offsets (the host checks M * ld < 2^31); two row chunks per step (the
      // loads of four in flight at once pushed the kernel past 256 VGPRs into spills)
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        __builtin_amdgcn_sched_barrier(0);
        f32x4 ra[2], rb[2];
        float mu[2], rs[2];
        u32x4 kx[2], kd[2];
        const int r0 = (int)frow0 + quarter * 32 + half * 16, c0 = (int)fcol;
#pragma unroll
        for (int it = 0; it < 2; ++it) {
          const int row = r0 + it * 8;
          kx[it] = *(const u32x4*)(lx + (row * (int)p.ln_ldx + c0));
          kd[it] = *(const u32x4*)(lc2 + (row * (int)p.ldc2 + c0));
          const float* Rp = (const float*)p.R + (row * (int)p.ldr + c0);   // mode 2 requires R
          ra[it] = *(const f32x4*)Rp;
          rb[it] = *(const f32x4*)(Rp + 4);
          mu[it] = lmean[row];
          rs[it] = lrstd[row];
        }
#pragma unroll
        for (int it = 0; it < 2; ++it) {
          const int row = r0 + it * 8;
          const float2 f = fin[wr * 128 + quarter * 32 + half * 16 + it * 8 + rl];
          float dy[8], xv[8], o[8];
          unpack8(kd[it], dy);
          unpack8(kx[it], xv);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float xh = (xv[j] - mu[it]) * rs[it];
            pg[j] += dy[j] * xh;
            pb[j] += dy[j];
            o[j] = rs[it] * (dy[j] * gam[j] - f.x - xh * f.y) + (j < 4 ? ra[it][j] : rb[it][j - 4]);
          }
          float* Cf = (float*)p.C + (row * (int)p.ldc + c0);
          *(f32x4*)Cf = f32x4{o[0], o[1], o[2], o[3]};
          *(f32x4*)(Cf + 4) = f32x4{o[4], o[5], o[6], o[7]};
          *(u32x4*)(lc2 + (row * (int)p.ldc2 + c0)) = pack8(o);
        }
      }
    }
  }
  if constexpr (MODE == 7) {
    // column partials of this wave's 128 rows (lanes of equal lane & 7 hold the same columns),
    // one slab row per 128-row block
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int o = 8; o <= 32; o <<= 1) { pg[j] += __shfl_xor(pg[j], o, 64); pb[j] += __shfl_xor(pb[j], o, 64); }
    if (rl == 0) {
      const int64_t slab = ((m0 >> 7) + wr) * p.N + gn;
      *(f32x4*)(p.ln_pg + slab) = f32x4{pg[0], pg[1], pg[2], pg[3]};
      *(f32x4*)(p.ln_pg + slab + 4) = f32x4{pg[4], pg[5], pg[6], pg[7]};
      if (p.ln_pb) {
        *(f32x4*)(p.ln_pb + slab) = f32x4{pb[0], pb[1], pb[2], pb[3]};
        *(f32x4*)(p.ln_pb + slab + 4) = f32x4{pb[4], pb[5], pb[6], pb[7]};
      }
    }
  }
}

// TR = true: MFMA operands swapped (transposed accumulator) + the LDS-free epilogue_t, used for
// bf16 outputs; TR = false: the LDS-staged row-chunk epilogue, used for f32 / residual / argmax
// outputs (measured faster there: full-row f32 chunks, one argmax pass per staged quarter).
//
// Persistent over tiles (p.persist): the grid is at most one workgroup per CU and each walks the
// XCD-remapped tile sequence wg, wg + grid, ...  After a tile's last MFMA the workgroup issues
// the NEXT tile's prologue loads (TR: tile 0 + tile 1's A0/B0, as the cold prologue; non-TR:
// tile 0 into buffer E, the epilogue staging lives in buffer O and beyond) and only then runs
// this tile's epilogue, so the load latency and the store drain overlap instead of adding up.
struct Tile {
  int64_t m0, n0, kbeg;
  int nk, split, bidx;
};

template <bool X3 = false>
__device__ __forceinline__ Tile tile_at(const P& p, int lin, int gx, int gy, int ntiles) {
  // XCD-aware remap of the linear tile index (round-robin dispatch: lin & 7 = XCD), so each
  // XCD walks a contiguous range of tiles (x fastest, then y, then batch / split)
  int id = lin;
  if (ntiles >= 16) {
    const int xcd = lin & 7, q = ntiles >> 3, r = ntiles & 7;
    id = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (lin >> 3);
  }
  const int gxy = gx * gy, z = id / gxy, rem = id - z * gxy;
  int ty, tx;
  if (gx >= p.group_gx) {
    // wide N (the VQ distance GEMM: 32 codebook tiles = 8 MB): groups of 8 tile rows walked
    // column by column, so an XCD's ~32 concurrent tiles touch 8 A panels + 4 B panels (3 MB,
    // L2-resident) instead of 1 A panel + the whole codebook streamed through its 4 MB L2
    const int GM = p.group_gm > 0 ? p.group_gm : 8;
    const int grp = rem / (GM * gx), y0 = grp * GM, gsz = min(gy - y0, GM), r = rem - grp * GM * gx;
    ty = y0 + r % gsz;
    tx = r / gsz;
  } else {
    ty = rem / gx;
    tx = rem - ty * gx;
  }
  Tile t;
  t.split = z % p.split_k;
  t.bidx = z / p.split_k;
  t.m0 = (int64_t)ty * p8::BM;
  t.n0 = (int64_t)tx * p8::BNN;
  t.kbeg = t.split * p.kper;
  const int64_t kend = min(p.K, t.kbeg + p.kper);
  t.nk = (kend > t.kbeg && !(p.debug & 2)) ? (int)((kend - t.kbeg) / p8::BKK) * (X3 ? 3 : 1) : 0;
  return t;
}

#ifdef CTCLIP_GEMM_STAMPS
// diagnostic build only (tools/gemm_stamps.py): per (workgroup, tile) s_memtime stamps of thread 0
// (0 tile start, 1 after the first K-tile, 2 after the second, 3 after the last MFMA + barrier,
// 4 after the epilogue's stores are issued) and the tile start in s_memrealtime (5, chip-wide)
__device__ unsigned long long g_stamps[256][32][6];
#define STAMP(k, v)                                                                        \
  do {                                                                                     \
    const unsigned long long t_ = (v);                                                     \
    if (threadIdx.x == 0 && tcount < 32) g_stamps[blockIdx.x][tcount][k] = t_;             \
  } while (0)
#else
#define STAMP(k, v) do { } while (0)
#endif

template <bool AK, bool BKC, int EP, bool H16 = false, bool X3 = false>
__global__ __launch_bounds__(512, 1) void gemm8p_kernel(P p) {
  using namespace p8;
  constexpr bool TR = EP >= 0;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, wr = w >> 2, wc = w & 3;
  const int gx = (int)((p.N + BNN - 1) / BNN), gy = (int)((p.M + BM - 1) / BM);
  const int ntiles = gx * gy * p.gz;
  int lin = p.persist ? (int)blockIdx.x : (int)((blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x);
  const int lstride = p.persist ? (int)gridDim.x : ntiles;
  if (lin >= ntiles) return;
  Tile T = tile_at<X3>(p, lin, gx, gy, ntiles);
  // desynchronise the CUs: half of the first dispatch round (every other workgroup within each
  // XCD) starts p.stagger x ~2k cycles late, so later rounds' store-heavy epilogues on those CUs
  // fall under the other half's MFMA main loops instead of all CUs storing at once
  // (stagger >= 1000: four groups delayed 0, 1, 2, 3 x (stagger - 1000) units -- A/B sweeps)
  if (p.stagger > 0 && lin < 256) {
    const int ng = p.stagger >= 1000 ? 4 : 2, u = p.stagger % 1000, grp = (lin >> 3) & (ng - 1);
    for (int s = 0; s < grp * u; ++s) __builtin_amdgcn_s_sleep(32);
  }

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // TR epilogue scratch (p.epi_lds): 4 KB per wave in buffer O's A1 / B1 halves, which nothing
  // loads while the epilogue runs (the next tile's prologue fills E and O's A0 / B0)
  const int wu = __builtin_amdgcn_readfirstlane(w);   // wave-uniform: the scratch base stays scalar
  char* scr = smem + TILEB + (wu < 4 ? A1 : B1) * HALF + (wu & 3) * 4096;

  auto stage_of = [&](const Tile& tl, int which, int t) {
    if (t >= tl.nk) return;
    char* dst = smem + (t & 1) * TILEB + which * HALF;
    int tk = t;
    const u16* Ab = p.A;
    const u16* Bb = p.B;
    if constexpr (X3) {
      // step t = 3 k + s (k-step major, so the second read of Ah_k hits the L2 line the first
      // brought in): s = 0 Ah Bh, 1 Ah Bl, 2 Al Bh (t / 3 as a multiply-shift, exact for t < 2^15)
      tk = (t * 21846) >> 16;
      const int sub = t - 3 * tk;
      if (sub == 2) Ab = p.alo;
      if (sub == 1) Bb = p.blo;
    }
    const int64_t k0 = tl.kbeg + (int64_t)tk * BKK;
    if (which < 2) stage_half<AK, true>(dst, Ab + tl.bidx * p.sA, p.lda, p.M, tl.m0, k0, which, w, lane);
    else stage_half<BKC, false>(dst, Bb + tl.bidx * p.sB, p.ldb, p.N, tl.n0, k0, which - 2, w, lane);
  };
  auto stage = [&](int which, int t) { stage_of(T, which, t); };

  bf16x8 a[4][2], b0[2][2], b1[2][2];

  const int abase = frag_base<AK>(wr * 64, lane), bbase = frag_base<BKC>(wc * 32, lane);
  // load segment of quadrant q of the tile in buffer `buf`
  auto load_frags = [&](int buf, int q) {
    const char* base = smem + buf * TILEB;
    if (q == 0 || q == 2) {
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int ii = 0; ii < 4; ++ii) a[ii][s] = hfrag<AK>(base, q == 0 ? A0 : A1, abase, ii, s);
    }
    if (q == 0) {
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) b0[jj][s] = hfrag<BKC>(base, B0, bbase, jj, s);
    }
    if (q == 1) {
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) b1[jj][s] = hfrag<BKC>(base, B1, bbase, jj, s);
    }
  };
  // compute segment: quadrant q = (mi, ni) in order (0,0) (0,1) (1,1) (1,0)
  auto mma = [&](int q) {
    const int mi = (q == 0 || q == 1) ? 0 : 1;
    const int ni = (q == 1 || q == 2) ? 1 : 0;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int ii = 0; ii < 4; ++ii)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
          const bf16x8 bb = ni ? b1[jj][s] : b0[jj][s];
          acc[mi * 4 + ii][ni * 2 + jj] = TR ? mfma16<H16>(bb, a[ii][s], acc[mi * 4 + ii][ni * 2 + jj])
                                             : mfma16<H16>(a[ii][s], bb, acc[mi * 4 + ii][ni * 2 + jj]);
        }
    __builtin_amdgcn_s_setprio(0);
  };
  auto wait_ahead = [&](bool younger_issued) {
    if (younger_issued) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };
  auto compute_phase = [&]() {
    bar();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };

  // cold prologue: tile 0 complete in E, tile 1's A0/B0 halves in flight
  stage(A0, 0); stage(A1, 0); stage(B0, 0); stage(B1, 0);
  stage(A0, 1); stage(B0, 1);
  wait_ahead(T.nk > 1);

  int tcount = 0;
  (void)tcount;
  // TR epilogues without the LDS relay (EP 10 / 12 use O's A1 / B1 halves as scratch) leave buffer O
  // idle, so with p.pre1 the next tile's K-step 1 is staged whole before the epilogue: its A1 / B1
  // halves get the epilogue's duration to land instead of the three MFMA phases of K-step 0 (the
  // first two K-steps of a tile ran at ~3x the steady-state time, r02 stamps).  Older loads only
  // complete earlier, so the vmcnt(4) waits of the loop stay exact.
  // Enabled for the VQ argmax GEMM (EP 3), the GEGLU backward (EP 4) and the NN dX GEMMs (EP 0 with
  // an N-contiguous B): 1.098 -> 1.013, 0.446 -> 0.436 and 0.313 -> 0.304 ms against the previous
  // build (profiles/r04r_gemm_pre1_ab.log).  Most of the VQ gain is the compiled code rather than
  // the prefetch (spills 18 -> 14; with p.pre1 = 0 the same build runs 1.02 ms, r04s_gemm_pre1_ab.log);
  // end to end within noise (r04s_pre1_ab_bench.log).  Skipping the re-issue costs the NT plain /
  // GEGLU / l2norm kernels 4-18 spilled VGPRs (FF1 +3 %, Q / KV +7 %), and re-issuing instead
  // gains nothing, so those keep the in-loop staging.
  constexpr bool PRE_OK = TR && (EP == 3 || EP == 4 || (EP == 0 && !BKC));
  bool pre = false;
  while (true) {
    const int nk = T.nk;
    STAMP(0, __builtin_amdgcn_s_memtime());
    STAMP(5, __builtin_amdgcn_s_memrealtime());
    bar();
    if (wr == 1) bar();   // the stagger: waves 4-7 run one barrier behind
    for (int i = 0; 2 * i < nk; ++i) {
      if (i == 1) STAMP(2, __builtin_amdgcn_s_memtime());
      const int te = 2 * i, to = 2 * i + 1;
      // K-step 1's second halves already staged before the epilogue: not re-issued here (step index
      // nk = no load, the bound check stage_of makes anyway)
      const int t1 = (PRE_OK && i == 0 && pre) ? nk : to;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        load_frags(0, q);
        if (q == 0) stage(B1, t1);
        if (q == 1) stage(A1, t1);
        if (q == 2) stage(A0, te + 2);
        if (q == 3) { stage(B0, te + 2); if (to < nk) wait_ahead(te + 2 < nk); }
        compute_phase();
        mma(q);
        bar();
      }
      if (to < nk) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          load_frags(1, q);
          if (q == 0) stage(B1, te + 2);
          if (q == 1) stage(A1, te + 2);
          if (q == 2) stage(A0, to + 2);
          if (q == 3) { stage(B0, to + 2); if (te + 2 < nk) wait_ahead(to + 2 < nk); }
          compute_phase();
          mma(q);
          bar();
        }
      }
    }
    if (wr == 0) bar();   // balance the stagger barrier
    __syncthreads();      // every wave's last fragment reads done before LDS is refilled / reused
    STAMP(3, __builtin_amdgcn_s_memtime());
    lin += lstride;
    const bool more = lin < ntiles;
    if (more) {
      const Tile nx = tile_at<X3>(p, lin, gx, gy, ntiles);
      stage_of(nx, A0, 0); stage_of(nx, A1, 0); stage_of(nx, B0, 0); stage_of(nx, B1, 0);
      if constexpr (TR) { stage_of(nx, A0, 1); stage_of(nx, B0, 1); }
      if constexpr (PRE_OK) {
        if (p.pre1) { stage_of(nx, B1, 1); stage_of(nx, A1, 1); }
      }
    }
    pre = PRE_OK && more && p.pre1;
    if (p.debug & 1) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(acc[i][j]));
    } else if constexpr (EP == 2 || EP == 12) {
      epilogue_t<2, EP == 12, H16, X3>(p, acc, wr, wc, lane, T.m0, T.n0, T.split, T.bidx, scr);
    } else if constexpr (EP == 4) {
      epilogue_geglu_bwd(p, acc, wr, wc, lane, T.m0, T.n0, T.bidx);
    } else if constexpr (EP == 0 || EP == 10) {
      epilogue_t<0, EP == 10>(p, acc, wr, wc, lane, T.m0, T.n0, T.split, T.bidx, scr);
    } else if constexpr (EP == 3) {
      epilogue_t<3>(p, acc, wr, wc, lane, T.m0, T.n0, T.split, T.bidx, scr);
    } else if constexpr (EP == 6) {
      epilogue_t<6>(p, acc, wr, wc, lane, T.m0, T.n0, T.split, T.bidx, scr);
    } else if constexpr (EP == 8) {
      epilogue_t<8>(p, acc, wr, wc, lane, T.m0, T.n0, T.split, T.bidx, scr);
    } else if constexpr (EP == -8) {
      epilogue<-8>(p, acc, smem + TILEB, w, wr, wc, lane, T.m0, T.n0, T.split, T.bidx);
    } else if constexpr (EP == -6 || EP == -7) {
      epilogue_ln<EP == -6 ? 6 : 7>(p, acc, smem, w, wr, wc, lane, T.m0, T.n0);
    } else {
      // staging in buffer O and beyond (the next tile's tile 0 is landing in E)
      epilogue<EP == -2 || EP == -3 || EP == -5 ? EP : -1>(p, acc, smem + TILEB, w, wr, wc, lane, T.m0, T.n0, T.split, T.bidx);
    }
    STAMP(4, __builtin_amdgcn_s_memtime());
    ++tcount;
    if (!more) break;
    T = tile_at<X3>(p, lin, gx, gy, ntiles);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (!TR) {
      __syncthreads();    // every wave's staging reads of O done before tile 1 lands there
      stage(A0, 1); stage(B0, 1);
    }
    wait_ahead(T.nk > 1);
  }
}

// persistent grid cap (workgroups; default 256 = one per CU): lets two GEMMs on two streams share
// the chip (ctclip_gemm_set_grid_cap)
static int g_grid_cap = 0;

template <bool AK, bool BKC, int EP, bool H16 = false, bool X3 = false>
int launch8(const P& p, int batch, hipStream_t st) {
  constexpr int smem = EP == -6 || EP == -7 ? SMEM_LN : p8::SMEM_P;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm8p_kernel<AK, BKC, EP, H16, X3>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    attr = true;
  }
  const int64_t ntiles = cdiv(p.N, p8::BNN) * cdiv(p.M, p8::BM) * (int64_t)p.gz;
  static bool cap_env = false;   // CTCLIP_GEMM_GRID_CAP (A/B): persistent grid below one per CU
  if (!cap_env) {
    const char* e = getenv("CTCLIP_GEMM_GRID_CAP");
    if (e && g_grid_cap == 0) g_grid_cap = atoi(e);
    cap_env = true;
  }
  static int pre1 = -1;   // CTCLIP_GEMM_PRE1=0: K-step 1's A1 / B1 halves staged inside the loop (A/B)
  if (pre1 < 0) { const char* e = getenv("CTCLIP_GEMM_PRE1"); pre1 = e ? atoi(e) != 0 : 1; }
  if (p.persist) {
    const int64_t cap = g_grid_cap > 0 && g_grid_cap < 256 ? g_grid_cap : 256;
    dim3 grid((unsigned)(ntiles < cap ? ntiles : cap));
    P q = p;
    q.pre1 = pre1;
    hipLaunchKernelGGL((gemm8p_kernel<AK, BKC, EP, H16, X3>), grid, dim3(p8::NTH), smem, st, q);
  } else {
    dim3 grid(cdiv(p.N, p8::BNN), cdiv(p.M, p8::BM), batch * p.split_k);
    hipLaunchKernelGGL((gemm8p_kernel<AK, BKC, EP, H16, X3>), grid, dim3(p8::NTH), smem, st, p);
  }
  CT_CHECK_LAUNCH();
  return 0;
}

template <int WR, bool AK, bool BKC>
int launch(const P& p, int batch, hipStream_t st) {
  using C = Cfg<WR>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm256_kernel<WR, AK, BKC>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              C::SMEM);
    attr = true;
  }
  dim3 grid(cdiv(p.N, BN), cdiv(p.M, C::BM), batch * p.split_k);
  hipLaunchKernelGGL((gemm256_kernel<WR, AK, BKC>), grid, dim3(C::NTH), C::SMEM, st, p);
  CT_CHECK_LAUNCH();
  return 0;
}

template <int WR>
int launch_any(const P& p, bool ak, bool bk, int batch, hipStream_t st) {
  if (ak && bk) return launch<WR, true, true>(p, batch, st);
  if (ak) return launch<WR, true, false>(p, batch, st);
  if (bk) return launch<WR, false, true>(p, batch, st);
  return launch<WR, false, false>(p, batch, st);
}

// kernel variant: 8 = 8-phase 256 x 256 x 64 (default), 1 = 128 x 256 x 32 (2 WG/CU),
// 2 = 256 x 256 x 32 4-slot ring.  CTCLIP_GEMM_VARIANT or ctclip_gemm_set_variant() select it.
static int g_variant = -1;
static int g_stagger8 = -1;   // 8-phase start stagger (units of s_sleep(32)); -1 = default
static int g_persist = -1;    // 8-phase persistent tile loop (CTCLIP_GEMM_PERSIST, default on)
static int g_epi_lds = -1;    // transposed bf16 / GEGLU epilogues through LDS (CTCLIP_EPI_LDS)
int variant() {
  if (g_variant < 0) {
    const char* e = getenv("CTCLIP_GEMM_VARIANT");
    g_variant = e ? atoi(e) : 8;
    if (g_variant != 1 && g_variant != 2) g_variant = 8;
  }
  return g_variant;
}
int tile_rows() { return variant() == 2 ? 2 : 1; }

// epilogue kind, one kernel instantiation each (so the accumulator registers never share a
// kernel with another epilogue's live ranges): -1 = LDS-staged rows (f32 / residual / argmax /
// split-K slabs), 0 = transposed bf16, 2 = transposed GEGLU, 4 = transposed GEGLU backward,
// 10 / 12 = 0 / 2 with their bf16 stores re-laid through LDS (store_blk_bf16_lds)
template <bool AK, bool BKC>
int launch8_ep(const P& p, int batch, hipStream_t st) {
  if (p.act == 4) return launch8<AK, BKC, 4>(p, batch, st);
  if (p.act == 5) return launch8<AK, BKC, 6>(p, batch, st);
  // CTCLIP_GEMM_TR_F32=1 (A/B): f32 / residual outputs through the transposed (LDS-free) epilogue too
  static int tr_f32 = -1;
  if (tr_f32 < 0) { const char* e = getenv("CTCLIP_GEMM_TR_F32"); tr_f32 = e ? atoi(e) != 0 : 0; }
  const bool tr = (tr_f32 || (!p.c_f32 && !p.R)) && p.split_k <= 1 && p.act != 3;
  if (!tr) {
    // the argmax through the transposed (LDS-free) epilogue: VQ distance GEMM 1.73 -> 1.56 ms (r02);
    // CTCLIP_GEMM_ARGMAX_TR=0: the LDS-staged one (A/B)
    static int am_tr = -1;
    if (am_tr < 0) { const char* e = getenv("CTCLIP_GEMM_ARGMAX_TR"); am_tr = e ? atoi(e) != 0 : 1; }
    if (p.act == 3 && am_tr && p.split_k <= 1) return launch8<AK, BKC, 3>(p, batch, st);
    if (p.act == 3) return launch8<AK, BKC, -3>(p, batch, st);
    if (p.split_k > 1) return launch8<AK, BKC, -5>(p, batch, st);   // slabs: alpha only
    if (p.R && p.r_f32 && p.c_f32 && p.act == 0 && !p.accumulate) return launch8<AK, BKC, -2>(p, batch, st);
    return launch8<AK, BKC, -1>(p, batch, st);
  }
  // 10 / 12: the same epilogues with lane-contiguous stores through LDS (p.epi_lds)
  const bool relay = p.epi_lds == 1 || p.epi_lds == 2;   // 3: direct stores with sc1 (EP 0 / 2)
  if (p.act == 2) return relay ? launch8<AK, BKC, 12>(p, batch, st) : launch8<AK, BKC, 2>(p, batch, st);
  return relay ? launch8<AK, BKC, 10>(p, batch, st) : launch8<AK, BKC, 0>(p, batch, st);
}

// fp16 operands (the 3D-ViT forward: K-contiguous A and B only): the forward epilogues -- GEGLU (h in
// fp16), plain 16-bit / l2norm-free outputs, the LDS-staged f32 / bias / residual rows
int launch8_h16(const P& p, int batch, hipStream_t st) {
  if (p.split_k > 1 || p.act == 4 || p.act == 5 || p.act == 6) return CT_EINVAL;
  // the VQ distance GEMM on fp16 operands (round 6): the argmax epilogue works on the f32 sums
  if (p.act == 3) return p.x3 ? CT_EINVAL : launch8<true, true, 3, true>(p, batch, st);
  if (p.x3) {
    // split-fp16 operands: the GEGLU pair epilogue, f32 rows (bias / f32 residual / bf16 copy)
    if (p.act == 2) return launch8<true, true, 2, true, true>(p, batch, st);
    if (!p.c_f32 || p.act != 0) return CT_EINVAL;
    if (p.R && p.r_f32 && !p.accumulate) return launch8<true, true, -2, true, true>(p, batch, st);
    if (p.R) return CT_EINVAL;
    return launch8<true, true, -1, true, true>(p, batch, st);
  }
  const bool tr = !p.c_f32 && !p.R;
  if (p.act == 2) return launch8<true, true, 2, true>(p, batch, st);
  if (tr) return launch8<true, true, 0, true>(p, batch, st);
  if (p.R && p.r_f32 && p.c_f32 && p.act == 0 && !p.accumulate) return launch8<true, true, -2, true>(p, batch, st);
  return launch8<true, true, -1, true>(p, batch, st);
}

template <bool AK>
int launch8_any(const P& p, bool bk, int batch, hipStream_t st) {
  return bk ? launch8_ep<AK, true>(p, batch, st) : launch8_ep<AK, false>(p, batch, st);
}

}  // namespace g256

// called from ctclip_gemm (gemm.hip) after argument validation
int ctclip_gemm256(const ctclip_gemm_args* a, int split, int batch, void* stream) {
  using namespace g256;
  P p{};
  memset(&p, 0, sizeof(p));
  p.M = a->M; p.N = a->N; p.K = a->K;
  p.A = (const u16*)a->A; p.lda = a->lda;
  p.B = (const u16*)a->B; p.ldb = a->ldb;
  p.C = a->C; p.ldc = a->ldc; p.c_f32 = a->c_f32;
  p.C2 = (u16*)a->C2; p.ldc2 = a->ldc2;
  p.bias = a->bias;
  p.R = a->R; p.ldr = a->ldr; p.r_f32 = a->r_f32;
  p.alpha = a->alpha; p.act = a->act; p.accumulate = a->accumulate; p.split_k = split;
  p.sA = a->sA; p.sB = a->sB; p.sC = a->sC; p.sC2 = a->sC2; p.sR = a->sR;
  p.n2 = a->n2;
  p.fold_cs = nullptr;
  p.nfold = 0;
  p.h16 = a->ab_f16 || a->r_f16;
  p.ln_y16 = nullptr;
  p.x3 = a->A_lo != nullptr;
  p.alo = (const u16*)a->A_lo;
  p.blo = (const u16*)a->B_lo;
  p.C3 = (u16*)a->C3; p.ldc3 = a->ldc3;
  p.C4 = (u16*)a->C4; p.ldc4 = a->ldc4;
  const int kstep = (variant() == 8 || a->act == 4 || a->act == 5) ? p8::BKK : BK;
  p.kper = (a->K / kstep + split - 1) / split * kstep;
  static int dbg = -1, stag = 0;
  if (dbg < 0) {
    const char* e = getenv("CTCLIP_G256_DEBUG");
    dbg = e ? atoi(e) : 0;
    const char* s = getenv("CTCLIP_G256_STAGGER");
    stag = s ? atoi(s) : 0;
  }
  p.debug = dbg;
  if (g_persist < 0) {
    const char* e = getenv("CTCLIP_GEMM_PERSIST");
    g_persist = e ? (atoi(e) != 0) : 1;
  }
  p.gz = batch * split;
  p.persist = g_persist;
  if (g_epi_lds < 0) {
    const char* e = getenv("CTCLIP_EPI_LDS");
    g_epi_lds = e ? std::min(3, std::max(0, atoi(e))) : 0;
  }
  p.epi_lds = g_epi_lds;
  // 8-phase default: stagger only the GEGLU GEMM, whose epilogue (h + g stores + erf) is long
  // enough that desynchronised CUs pay off (r01 sweep: 0.52 -> 0.48 ms at B = 8; neutral to
  // slightly negative on the plain / residual epilogues)
  static int ggx = -1;
  if (ggx < 0) { const char* e = getenv("CTCLIP_GEMM_GROUP_GX"); ggx = e ? atoi(e) : 8; }   // r02: FF1 (11 tiles) -2%, VQ (32) -17%; N <= 6 tiles: neutral to +4% (not grouped)
  p.group_gx = ggx;
  static int ggm = -1;
  if (ggm < 0) { const char* e = getenv("CTCLIP_GEMM_GROUP_GM"); ggm = e ? atoi(e) : 8; }
  p.group_gm = ggm;
  // (round 4 sweep, profiles/r04a_stagger.log, interleaved rounds: no start stagger is best for the
  // GEGLU GEMM now -- 0.4229 vs 0.4289 ms at the old default 4; the GEGLU backward gains ~1.5 % at 8)
  p.stagger = variant() == 8 ? (g_stagger8 >= 0 ? g_stagger8 : (a->act == 4 ? 8 : 0)) : (tile_rows() == 1 ? stag : 0);
  hipStream_t st = (hipStream_t)stream;
  if (a->ab_f16) {
    if (!a->a_kcontig || !a->b_kcontig) return CT_EINVAL;
    p.stagger = 0;
    return launch8_h16(p, batch, st);
  }
  if (variant() == 8 || a->act == 4 || a->act == 5)
    return a->a_kcontig ? launch8_any<true>(p, a->b_kcontig, batch, st) : launch8_any<false>(p, a->b_kcontig, batch, st);
  if (tile_rows() == 2) return launch_any<2>(p, a->a_kcontig, a->b_kcontig, batch, st);
  return launch_any<1>(p, a->a_kcontig, a->b_kcontig, batch, st);
}

// LayerNorm-fused N = 512 GEMM (include/ctclip_hip.h).  The pair exchange needs the persistent
// 8-phase walk on its full grid with ntiles % 16 == 0 (tile_at pairs tiles 2k, 2k + 1 on
// workgroups w, w ^ 8 of one round); anything else is refused (CT_EINVAL) and the caller runs the
// GEMM and the LayerNorm kernel separately.
extern "C" int ctclip_gemm_ln(const ctclip_gemm_args* a, const ctclip_ln_epilogue* ln, void* stream) {
  using namespace g256;
  if (!a || !ln || (ln->mode != 1 && ln->mode != 2)) return CT_EINVAL;
  if (a->M == 0) return 0;
  CT_REQUIRE(a->N == 512 && a->M > 0 && a->M % 2048 == 0 && a->K > 0 && a->K % 64 == 0, CT_ESHAPE);
  CT_REQUIRE(a->split_k <= 1 && a->batch <= 1 && a->act == 0 && !a->accumulate && a->c_f32 && !a->B2, CT_EINVAL);
  CT_REQUIRE(variant() == 8 && g_persist != 0 && g_grid_cap == 0, CT_EINVAL);
  CT_REQUIRE(aligned16(a->A) && aligned16(a->B) && aligned16(a->C) && a->lda % 8 == 0 && a->ldb % 8 == 0 &&
                 a->ldc % 8 == 0, CT_EALIGN);
  if (a->C2) CT_REQUIRE(aligned16(a->C2) && a->ldc2 % 8 == 0, CT_EALIGN);
  if (a->R) CT_REQUIRE(a->r_f32 && aligned16(a->R) && a->ldr % 8 == 0, CT_EINVAL);
  if (a->bias) CT_REQUIRE(ln->mode == 1 && aligned16(a->bias), CT_EINVAL);
  CT_REQUIRE(ln->gamma && aligned16(ln->gamma) && ln->mean && ln->rstd && ln->xchg && ln->epoch != 0 &&
                 (((uintptr_t)ln->xchg) & 7) == 0, CT_EINVAL);
  {
    const int64_t ldmax = std::max(std::max(a->ldc, a->ldc2), std::max(a->ldr, ln->ldx));
    CT_REQUIRE(a->M * ldmax < ((int64_t)1 << 31), CT_ESHAPE);   // 32-bit element offsets (mode 2)
  }
  if (ln->mode == 1) {
    // Y (bf16) may be NULL when the fp16 copy Y16 is given: the eval forward (round 6)
    CT_REQUIRE(a->R && (ln->Y || ln->Y16) && aligned16(ln->Y) && aligned16(ln->Y16) && ln->ldy % 8 == 0, CT_EINVAL);
    if (ln->beta) CT_REQUIRE(aligned16(ln->beta), CT_EALIGN);
  } else {
    CT_REQUIRE(ln->X && aligned16(ln->X) && ln->ldx % 8 == 0 && ln->part_gamma && !ln->beta && a->C2 && a->R,
               CT_EINVAL);
  }
  P p{};
  memset(&p, 0, sizeof(p));
  p.M = a->M; p.N = a->N; p.K = a->K;
  p.A = (const u16*)a->A; p.lda = a->lda;
  p.B = (const u16*)a->B; p.ldb = a->ldb;
  p.C = a->C; p.ldc = a->ldc; p.c_f32 = 1;
  p.C2 = (u16*)a->C2; p.ldc2 = a->ldc2;
  p.bias = a->bias;
  p.R = a->R; p.ldr = a->ldr; p.r_f32 = 1;
  p.alpha = a->alpha; p.act = 0; p.accumulate = 0; p.split_k = 1;
  p.kper = a->K;
  p.debug = 0;
  p.group_gx = 1 << 30;   // plain row-major tile order: the pairing above relies on it
  p.stagger = 0;
  p.gz = 1;
  p.persist = 1;
  p.ln_gamma = ln->gamma; p.ln_beta = ln->beta; p.ln_eps = ln->eps;
  p.ln_y = (u16*)ln->Y; p.ln_ldy = ln->ldy;
  p.ln_mean = ln->mean; p.ln_rstd = ln->rstd;
  p.ln_x = (const u16*)ln->X; p.ln_ldx = ln->ldx;
  p.ln_pg = ln->part_gamma; p.ln_pb = ln->part_beta;
  p.xchg = (unsigned long long*)ln->xchg;
  p.epoch = ln->epoch;
  p.status = ln->status;
  p.spin_limit = ln->spin_limit ? ln->spin_limit : LN_SPIN_LIMIT;
  p.ln_debug = ln->debug;
  p.ln_y16 = ln->mode == 1 ? (u16*)ln->Y16 : nullptr;
  hipStream_t st = (hipStream_t)stream;
  if (!a->a_kcontig) return CT_EINVAL;
  if (a->ab_f16) {   // fp16 operands: the forward form only, B K-contiguous
    if (ln->mode != 1 || !a->b_kcontig) return CT_EINVAL;
    return launch8<true, true, -6, true>(p, 1, st);
  }
  if (ln->mode == 1) return a->b_kcontig ? launch8<true, true, -6>(p, 1, st) : launch8<true, false, -6>(p, 1, st);
  return a->b_kcontig ? launch8<true, true, -7>(p, 1, st) : launch8<true, false, -7>(p, 1, st);
}

// Q | K | V projection of one transformer layer as ONE GEMM over the raw residual rows, with the
// attention's LayerNorm folded into the Q columns (include/ctclip_hip.h).  Q uses LN(x) and K / V
// use x (ct_clip/attention.py:139-141,152-154), so with B = [gamma o Wq ; Wkv] (bf16, K-contiguous)
// the Q columns are LN(x) Wq^T = rstd (x (gamma o Wq)^T - mean (Wq gamma)) and the LayerNorm
// output never exists; both l2norms ride in the epilogue as in act 5.
extern "C" int ctclip_gemm_qkv_lnfold(const ctclip_gemm_args* a, const float* mean, const float* rstd,
                                      const float* fold_cs, int32_t nfold, void* stream) {
  return ctclip_gemm_qkv_lnfold2(a, mean, rstd, fold_cs, nfold, 0, stream);
}

extern "C" int ctclip_gemm_qkv_lnfold2(const ctclip_gemm_args* a, const float* mean, const float* rstd,
                                       const float* fold_cs, int32_t nfold, int32_t c_col0, void* stream) {
  using namespace g256;
  if (c_col0 < 0 || c_col0 % 64) return CT_EINVAL;
  if (!a || !mean || !rstd || !fold_cs) return CT_EINVAL;
  if (a->M == 0) return 0;
  CT_REQUIRE(a->M > 0 && a->N % 256 == 0 && a->K > 0 && a->K % 64 == 0, CT_ESHAPE);
  CT_REQUIRE(nfold > 0 && nfold % 256 == 0 && nfold < a->N && a->n2 > nfold && a->n2 % 64 == 0 && a->n2 <= a->N,
             CT_EINVAL);
  CT_REQUIRE(a->a_kcontig && a->b_kcontig && !a->c_f32 && a->C2 && a->bias && !a->R && !a->B2 && a->act == 5 &&
                 a->split_k <= 1 && a->batch <= 1 && !a->accumulate,
             CT_EINVAL);
  CT_REQUIRE(variant() == 8, CT_EINVAL);
  CT_REQUIRE(aligned16(a->A) && aligned16(a->B) && aligned16(a->C) && aligned16(a->C2) && aligned16(a->bias) &&
                 aligned16(fold_cs) && a->lda % 8 == 0 && a->ldb % 8 == 0 && a->ldc % 8 == 0 && a->ldc2 % 8 == 0,
             CT_EALIGN);
  P p{};
  memset(&p, 0, sizeof(p));
  p.M = a->M; p.N = a->N; p.K = a->K;
  p.A = (const u16*)a->A; p.lda = a->lda;
  p.B = (const u16*)a->B; p.ldb = a->ldb;
  p.C = a->C; p.ldc = a->ldc; p.c_f32 = 0;
  p.C2 = (u16*)a->C2; p.ldc2 = a->ldc2;
  p.bias = a->bias;
  p.alpha = a->alpha; p.act = 5; p.split_k = 1;
  p.n2 = a->n2;
  p.kper = a->K;
  p.gz = 1;
  if (g_persist < 0) {
    const char* e = getenv("CTCLIP_GEMM_PERSIST");
    g_persist = e ? (atoi(e) != 0) : 1;
  }
  p.persist = g_persist;
  p.group_gx = 8;
  p.ln_mean = (float*)mean;
  p.ln_rstd = (float*)rstd;
  p.fold_cs = fold_cs;
  p.nfold = nfold;
  p.c_col0 = c_col0;
  if (a->ab_f16) return launch8<true, true, 8, true>(p, 1, (hipStream_t)stream);
  return launch8<true, true, 8>(p, 1, (hipStream_t)stream);
}

// Backward of the folded LayerNorm + Q | K | V projections (include/ctclip_hip.h): with A = [dq o rstd |
// dk | dv] and B = [gamma o Wq ; Wkv] (the forward's packed operand, row-major [K][N]),
//   C = A B + R - c1[m] - beta[m] X[m][n] = LN'(dq Wq) + dkv Wkv + R
// (c1, beta from ctclip_l2norm_scale_bwd_fold, X the LayerNorm's bf16 input).  Replaces the dX GEMM
// of the Q projection, the LayerNorm backward and the K / V dX GEMM with its residual.
extern "C" int ctclip_gemm_lnfold_bwd(const ctclip_gemm_args* a, const void* X, int64_t ldx, const float* c1,
                                      const float* beta, void* stream) {
  using namespace g256;
  if (!a || !X || !c1 || !beta) return CT_EINVAL;
  if (a->M == 0) return 0;
  CT_REQUIRE(a->M > 0 && a->N > 0 && a->N % 8 == 0 && a->K > 0 && a->K % 64 == 0, CT_ESHAPE);
  CT_REQUIRE(a->a_kcontig && a->c_f32 && a->R && a->r_f32 && !a->bias && !a->B2 && a->act == 0 && a->split_k <= 1 &&
                 a->batch <= 1 && !a->accumulate,
             CT_EINVAL);
  CT_REQUIRE(variant() == 8, CT_EINVAL);
  CT_REQUIRE(aligned16(a->A) && aligned16(a->B) && aligned16(a->C) && aligned16(a->R) && aligned16(X) &&
                 a->lda % 8 == 0 && a->ldb % 8 == 0 && a->ldc % 8 == 0 && a->ldr % 8 == 0 && ldx % 8 == 0,
             CT_EALIGN);
  if (a->C2) CT_REQUIRE(aligned16(a->C2) && a->ldc2 % 8 == 0, CT_EALIGN);
  P p{};
  memset(&p, 0, sizeof(p));
  p.M = a->M; p.N = a->N; p.K = a->K;
  p.A = (const u16*)a->A; p.lda = a->lda;
  p.B = (const u16*)a->B; p.ldb = a->ldb;
  p.C = a->C; p.ldc = a->ldc; p.c_f32 = 1;
  p.C2 = (u16*)a->C2; p.ldc2 = a->ldc2;
  p.R = a->R; p.ldr = a->ldr; p.r_f32 = 1;
  p.alpha = a->alpha; p.split_k = 1;
  p.kper = a->K;
  p.gz = 1;
  if (g_persist < 0) {
    const char* e = getenv("CTCLIP_GEMM_PERSIST");
    g_persist = e ? (atoi(e) != 0) : 1;
  }
  p.persist = g_persist;
  p.group_gx = 8;
  p.ln_x = (const u16*)X;
  p.ln_ldx = ldx;
  p.ln_mean = (float*)c1;
  p.ln_rstd = (float*)beta;
  hipStream_t st = (hipStream_t)stream;
  return a->b_kcontig ? launch8<true, true, -8>(p, 1, st) : launch8<true, false, -8>(p, 1, st);
}

// A/B switch: the transposed bf16 / GEGLU epilogues' stores through the wave's LDS scratch
// (lane-contiguous 16-B stores); returns the previous value
extern "C" int ctclip_gemm_set_epi_lds(int v) {
  const int old = g256::g_epi_lds;
  g256::g_epi_lds = v >= 0 && v <= 3 ? v : 0;
  return old;
}

// diagnostic: 8-phase kernel start stagger (see gemm8p_kernel); returns the previous value
extern "C" int ctclip_gemm_set_stagger(int v) {
  const int old = g256::g_stagger8;
  g256::g_stagger8 = v;
  return old;
}

// 8-phase persistent grid cap for the launches that follow (0 = one workgroup per CU); returns the
// previous value.  Used to split the chip between two concurrent GEMMs on two streams.
extern "C" int ctclip_gemm_set_grid_cap(int v) {
  const int old = g256::g_grid_cap;
  g256::g_grid_cap = v > 0 ? v : 0;
  return old;
}

// diagnostic: 8-phase persistent tile loop on / off; returns the previous value
extern "C" int ctclip_gemm_set_persist(int v) {
  const int old = g256::g_persist;
  g256::g_persist = v != 0;
  return old;
}

// diagnostic: select the large-tile kernel variant at run time (returns the previous one)
extern "C" int ctclip_gemm_set_variant(int v) {
  const int old = g256::variant();
  if (v == 1 || v == 2 || v == 8) g256::g_variant = v;
  return old;
}

#ifdef CTCLIP_GEMM_STAMPS
// diagnostic: copy the stamp buffer (256 x 32 x 6 u64) to host memory (and clear it)
extern "C" int ctclip_gemm_stamps(void* host, int clear) {
  hipError_t e = hipMemcpyFromSymbol(host, HIP_SYMBOL(g256::g_stamps), sizeof(g256::g_stamps), 0, hipMemcpyDeviceToHost);
  if (e == hipSuccess && clear) {
    static unsigned long long zero[256 * 32 * 6];
    e = hipMemcpyToSymbol(HIP_SYMBOL(g256::g_stamps), zero, sizeof(zero), 0, hipMemcpyHostToDevice);
  }
  return (int)e;
}
#endif
