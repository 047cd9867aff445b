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
  int64_t kper;
  int debug;     // diagnostic knob (CTCLIP_G256_DEBUG): 1 = skip the epilogue, 2 = skip the main loop
  int stagger;   // start delay (s_sleep units of 64 cycles) for the second co-resident workgroup
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

  // ---------------- epilogue: per-wave private staging, four 32-row quarters
  float* cs = (float*)(smem + w * (32 * EP_LD * 4));   // 8.7 KB per wave, 8 waves = 70 KB
  const int64_t wrow0 = m0 + wr * 128, wcol0 = n0 + wc * 64;
  const bool slab = p.split_k > 1;
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
    if (p.act == 3) {
      // argmax over this wave's 64 columns: 2 lanes per row (32 columns each), (value, index)
      // per (row, 64-col group), first-max tie-break
      const int row = lane >> 1, hc = lane & 1;
      const int64_t gm = rbase + row;
      float best = -INFINITY;
      int bi = 0x7fffffff;
      const int ncol = (int)max((int64_t)0, min((int64_t)64, p.N - wcol0));
      for (int c = hc * 32; c < hc * 32 + 32; ++c) {
        const float v = cs[row * EP_LD + c];
        if (c < ncol && v > best) { best = v; bi = c; }
      }
      const float ob = __shfl_xor(best, 1, 64);
      const int oi = __shfl_xor(bi, 1, 64);
      if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
      if (hc == 0 && gm < p.M && ncol > 0) {
        float2* out = (float2*)p.C + bidx * p.sC;
        out[gm * p.ldc + (wcol0 >> 6)] = make_float2(best, __int_as_float((int)(wcol0 + bi)));
      }
    } else if (p.act == 2) {
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
      for (int it = 0; it < 4; ++it) {
        const int c = lane + 64 * it;
        const int row = c >> 3, cc = (c & 7) * 8;
        const int64_t gm = rbase + row, gn = wcol0 + cc;
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
        if (p.bias) {
          const f32x4 b0 = *(const f32x4*)(p.bias + gn), b1 = *(const f32x4*)(p.bias + gn + 4);
#pragma unroll
          for (int j = 0; j < 4; ++j) { v[j] += b0[j]; v[4 + j] += b1[j]; }
        }
        if (p.R) {
          if (p.r_f32) {
            const float* Rp = (const float*)p.R + bidx * p.sR + gm * p.ldr + gn;
            const f32x4 a = *(const f32x4*)Rp, b = *(const f32x4*)(Rp + 4);
#pragma unroll
            for (int j = 0; j < 4; ++j) { v[j] += a[j]; v[4 + j] += b[j]; }
          } else {
            float rr[8];
            unpack8(*(const u32x4*)((const u16*)p.R + bidx * p.sR + gm * p.ldr + gn), rr);
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
            const f32x4 a = *(const f32x4*)Cf, b = *(const f32x4*)(Cf + 4);
#pragma unroll
            for (int j = 0; j < 4; ++j) { v[j] += a[j]; v[4 + j] += b[j]; }
          }
          *(f32x4*)Cf = f32x4{v[0], v[1], v[2], v[3]};
          *(f32x4*)(Cf + 4) = f32x4{v[4], v[5], v[6], v[7]};
        } else {
          u16* Cb = (u16*)p.C + bidx * p.sC + gm * p.ldc + gn;
          if (p.accumulate) {
            float rr[8];
            unpack8(*(const u32x4*)Cb, rr);
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] += rr[j];
          }
          *(u32x4*)Cb = pack8(v);
        }
        if (p.C2 && p.act == 0) *(u32x4*)(p.C2 + bidx * p.sC2 + gm * p.ldc2 + gn) = pack8(v);
      }
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);   // reads of this half done before it is overwritten
  }
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

// tile shape: CTCLIP_G256_WR=2 forces the 256 x 256 form, =1 the 128 x 256 form
int tile_rows() {
  static int wr = -1;
  if (wr < 0) {
    const char* e = getenv("CTCLIP_G256_WR");
    wr = (e && atoi(e) == 2) ? 2 : 1;
  }
  return wr;
}

}  // namespace g256

// called from ctclip_gemm (gemm.hip) after argument validation
int ctclip_gemm256(const ctclip_gemm_args* a, int split, int batch, void* stream) {
  using namespace g256;
  P p;
  p.M = a->M; p.N = a->N; p.K = a->K;
  p.A = (const u16*)a->A; p.lda = a->lda;
  p.B = (const u16*)a->B; p.ldb = a->ldb;
  p.C = a->C; p.ldc = a->ldc; p.c_f32 = a->c_f32;
  p.C2 = (u16*)a->C2; p.ldc2 = a->ldc2;
  p.bias = a->bias;
  p.R = a->R; p.ldr = a->ldr; p.r_f32 = a->r_f32;
  p.alpha = a->alpha; p.act = a->act; p.accumulate = a->accumulate; p.split_k = split;
  p.sA = a->sA; p.sB = a->sB; p.sC = a->sC; p.sC2 = a->sC2; p.sR = a->sR;
  int64_t kper = (a->K / BK + split - 1) / split * BK;
  p.kper = kper;
  static int dbg = -1, stag = 0;
  if (dbg < 0) {
    const char* e = getenv("CTCLIP_G256_DEBUG");
    dbg = e ? atoi(e) : 0;
    const char* s = getenv("CTCLIP_G256_STAGGER");
    stag = s ? atoi(s) : 0;
  }
  p.debug = dbg;
  p.stagger = tile_rows() == 1 ? stag : 0;
  hipStream_t st = (hipStream_t)stream;
  if (tile_rows() == 2) return launch_any<2>(p, a->a_kcontig, a->b_kcontig, batch, st);
  return launch_any<1>(p, a->a_kcontig, a->b_kcontig, batch, st);
}
