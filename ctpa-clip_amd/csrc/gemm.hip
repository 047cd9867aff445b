// bf16 MFMA GEMM for gfx950 with fused epilogues.
//
// Tile 128x128x64, 256 threads = 4 waves (2x2), each wave a 64x64 block of 4x4
// v_mfma_f32_16x16x32_bf16.  Operands are register-staged into a double-buffered LDS
// image (one barrier per K-step, next tile's global loads in flight under the MFMAs).
//   K-contiguous operand tile: [128 rows][64 k] bf16, row stride 144 B (padding kills
//     the ds_read_b128 row-group conflicts), fragments by ds_read_b128.
//   MN-contiguous operand tile: [64 k][128] bf16, 256-B rows, 32-B chunks XOR-swizzled by
//     (k&3)|((k>>3)&1)<<2 so ds_read_b64_tr_b16 (hardware transpose) is conflict-free;
//     this lets dX = dY.W and dW = dY^T.X run without materialising transposes.
// Epilogue stages the f32 accumulator tile through LDS and writes 16-B row chunks with
// bias / residual / GELU / GEGLU / argmax fused.  blockIdx is remapped XCD-aware (T1).
#include <algorithm>
#include "common.h"
#include "../../include/ctclip_hip.h"

int ctclip_gemm256(const ctclip_gemm_args* a, int split, int batch, void* stream);  // gemm256.hip

namespace {

constexpr int BM = 128, BN = 128, BKT = 64, NTH = 256;
constexpr int KROW = BKT * 2 + 16;           // 144-byte rows for K-contiguous tiles
constexpr int TILE_BYTES = 128 * KROW;       // 18432 >= 64*256 for MN tiles
constexpr int SMEM_BYTES = 4 * TILE_BYTES;   // 2 buffers x (A, B) = 73728
constexpr int CS_LD = 132;                   // f32 epilogue staging row stride

struct P {
  int64_t M, N, K;
  const u16* A; int64_t lda;
  const u16* B; int64_t ldb;
  const u16* B2;                 // optional second B (the bf16 "lo" residual of an f32 weight)
  void* C; int64_t ldc; int c_f32;
  u16* C2; int64_t ldc2;
  const float* bias;
  const void* R; int64_t ldr; int r_f32;
  float alpha; int act; int accumulate; int split_k;
  int64_t sA, sB, sC, sC2, sR;
  int64_t kper;
  int r_f16;                     // act 4: R (h) is fp16
};

__device__ __forceinline__ int mn_swz(int k) { return (k & 3) | (((k >> 3) & 1) << 2); }

template <bool KC>
__device__ __forceinline__ void gload(u32x4 (&r)[4], const u16* __restrict__ base, int64_t ld,
                                      int64_t rows, int64_t kend, int64_t row0, int64_t k0) {
  const int t = threadIdx.x;
  if constexpr (KC) {
    const int kc = t & 7;
    const int64_t gk = k0 + kc * 8;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t gr = row0 + (t >> 3) + 32 * i;
      if (gr < rows && gk < kend) r[i] = *(const u32x4*)(base + gr * ld + gk);
      else r[i] = make_uint4(0, 0, 0, 0);
    }
  } else {
    const int mc = t & 15;
    const int64_t gm = row0 + mc * 8;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t gk = k0 + (t >> 4) + 16 * i;
      if (gk < kend && gm < rows) r[i] = *(const u32x4*)(base + gk * ld + gm);
      else r[i] = make_uint4(0, 0, 0, 0);
    }
  }
}

template <bool KC>
__device__ __forceinline__ void swrite(char* tile, const u32x4 (&r)[4]) {
  const int t = threadIdx.x;
  if constexpr (KC) {
    const int kc = t & 7;
#pragma unroll
    for (int i = 0; i < 4; ++i) *(u32x4*)(tile + ((t >> 3) + 32 * i) * KROW + kc * 16) = r[i];
  } else {
    const int mc = t & 15, c32 = mc >> 1, half = mc & 1;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int kk = (t >> 4) + 16 * i;
      *(u32x4*)(tile + kk * 256 + ((((c32 ^ mn_swz(kk)) << 1) | half) << 4)) = r[i];
    }
  }
}

template <bool KC>
__device__ __forceinline__ bf16x8 frag(const char* tile, int r0, int s, int lane) {
  if constexpr (KC) {
    const int row = r0 + (lane & 15);
    return *(const bf16x8*)(tile + row * KROW + ((s * 4 + (lane >> 4)) << 4));
  } else {
    const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const int m = r0 + 4 * p;
    const int k1 = s * 32 + 8 * g + q, k2 = k1 + 4;
    const int c32 = m >> 4, within = (m & 15) * 2;
    const int o1 = k1 * 256 + ((c32 ^ mn_swz(k1)) << 5) + within;
    const int o2 = k2 * 256 + ((c32 ^ mn_swz(k2)) << 5) + within;
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

template <bool AK, bool BK, bool H16 = false>
__global__ __launch_bounds__(NTH, 2) void gemm_kernel(P p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, wr = w >> 1, wc = w & 1;
  int tx, ty;
  xcd_remap(tx, ty);
  const int split = blockIdx.z % p.split_k, bidx = blockIdx.z / p.split_k;
  const int64_t m0 = (int64_t)ty * BM, n0 = (int64_t)tx * BN;
  const int64_t kbeg = split * p.kper;
  const int64_t kend = min(p.K, kbeg + p.kper);
  const u16* A = p.A + bidx * p.sA;
  const u16* B = p.B + bidx * p.sB;
#define AS(i) (smem + (i) * TILE_BYTES)
#define BS(i) (smem + (2 + (i)) * TILE_BYTES)

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  u32x4 ra[4], rb[4];
  // with B2 the K range is walked twice into the same accumulators: A.B^T then A.B2^T
  // (hi / lo split weights: W = hi + lo to ~16 mantissa bits, two MFMA passes, one f32 sum)
  const int nk1 = kend > kbeg ? (int)((kend - kbeg + BKT - 1) / BKT) : 0;
  const int nk = p.B2 ? 2 * nk1 : nk1;
  const u16* B2 = p.B2 ? p.B2 + bidx * p.sB : nullptr;
  if (nk > 0) {
    gload<AK>(ra, A, p.lda, p.M, kend, m0, kbeg);
    gload<BK>(rb, B, p.ldb, p.N, kend, n0, kbeg);
    swrite<AK>(AS(0), ra);
    swrite<BK>(BS(0), rb);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {
      const int kn = kt + 1 < nk1 ? kt + 1 : kt + 1 - nk1;
      gload<AK>(ra, A, p.lda, p.M, kend, m0, kbeg + (int64_t)kn * BKT);
      gload<BK>(rb, kt + 1 < nk1 ? B : B2, p.ldb, p.N, kend, n0, kbeg + (int64_t)kn * BKT);
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = frag<AK>(AS(cur), wr * 64 + i * 16, s, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = frag<BK>(BS(cur), wc * 64 + j * 16, s, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = mfma16<H16>(af[i], bfr[j], acc[i][j]);
    }
    if (kt + 1 < nk) {
      swrite<AK>(AS(cur ^ 1), ra);
      swrite<BK>(BS(cur ^ 1), rb);
    }
    __syncthreads();
  }

  // ---- epilogue: stage f32 tile in LDS
  float* cs = (float*)smem;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        cs[(wr * 64 + i * 16 + (lane >> 4) * 4 + r) * CS_LD + wc * 64 + j * 16 + (lane & 15)] = acc[i][j][r];
  __syncthreads();

  const int t = threadIdx.x;
  if (p.act == 3) {
    // argmax over this tile's columns per row: write (value, index) pairs per (row, tile)
    // C = float2 [M][ntiles]; columns >= N excluded.
    // one (value, index) per (row, 64-column group), first-max tie-break (torch.argmax semantics)
    // optional C2 (f32 [M][ldc2]): the group's second-best score, so the f32 re-score knows
    // when a non-winner of the group can still be the f32 argmax (vq.hip)
    const int row = t >> 1, half = t & 1;
    const int ncol = (int)min((int64_t)BN, p.N - n0);
    float best = -INFINITY, second = -INFINITY;
    int bi = 0x7fffffff;
    for (int c = half * 64; c < half * 64 + 64; ++c) {
      const float v = cs[row * CS_LD + c];
      if (c < ncol) {
        if (v > best) { second = best; best = v; bi = c; }
        else if (v > second) second = v;
      }
    }
    const int64_t gm = m0 + row;
    if (gm < p.M && half * 64 < ncol) {
      float2* out = (float2*)p.C + bidx * p.sC;
      out[gm * p.ldc + tx * 2 + half] = make_float2(best, __int_as_float((int)(n0 + bi)));
      if (p.C2) ((float*)p.C2)[bidx * p.sC2 + gm * p.ldc2 + tx * 2 + half] = second;
    }
    return;
  }
  const bool slab = p.split_k > 1;
  if (p.act == 4) {
    // GEGLU backward fused into dg = dy . W2 (see gemm256.hip): 8 g-columns per thread
    for (int it = 0; it < (BM * BN / 8) / NTH; ++it) {
      const int c = t + NTH * it;
      const int row = c >> 4, cc = (c & 15) * 8;
      const int64_t gm = m0 + row, gn = n0 + cc;
      if (gm >= p.M || gn >= p.N) continue;
      const int64_t tg = gn >> 5, cw = gn & 31;
      const u16* hr = (const u16*)p.R + bidx * p.sR + gm * p.ldr + tg * 64 + cw;
      u16* dr = (u16*)p.C + bidx * p.sC + gm * p.ldc + tg * 64 + cw;
      float x[8], gt[8], ox[8], og[8];
      if (p.r_f16) {   // fp16 h: the derivative form [gelu(gate) | x gelu'(gate)] (gemm256.hip EP 2)
        unpack8h(*(const u32x4*)hr, x);
        unpack8h(*(const u32x4*)(hr + 32), gt);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float d = bf2f(f2bf(cs[row * CS_LD + cc + j] * p.alpha));
          ox[j] = d * x[j];
          og[j] = d * gt[j];
        }
      } else {
        unpack8(*(const u32x4*)hr, x);
        unpack8(*(const u32x4*)(hr + 32), gt);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float d = bf2f(f2bf(cs[row * CS_LD + cc + j] * p.alpha));
          float ge, dge;
          gelu_erf_and_grad(gt[j], ge, dge);
          ox[j] = d * ge;
          og[j] = d * x[j] * dge;
        }
      }
      *(u32x4*)dr = pack8(ox);
      *(u32x4*)(dr + 32) = pack8(og);
    }
    return;
  }
  for (int it = 0; it < (BM * BN / 8) / NTH; ++it) {
    const int c = t + NTH * it;
    const int row = c >> 4, cc = (c & 15) * 8;
    const int64_t gm = m0 + row, gn = n0 + cc;
    if (gm >= p.M || gn >= p.N) continue;
    float v[8];
    const f32x4 lo = *(const f32x4*)(cs + row * CS_LD + cc);
    const f32x4 hi = *(const f32x4*)(cs + row * CS_LD + cc + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) { v[j] = lo[j] * p.alpha; v[4 + j] = hi[j] * p.alpha; }
    if (slab) {
      float* Cf = (float*)p.C + (int64_t)split * p.M * p.ldc + bidx * p.sC + gm * p.ldc + gn;
      *(f32x4*)Cf = f32x4{v[0], v[1], v[2], v[3]};
      *(f32x4*)(Cf + 4) = f32x4{v[4], v[5], v[6], v[7]};
      continue;
    }
    if (p.bias) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += p.bias[gn + j];
    }
    if (p.act == 6) {
      // GELU backward: C = acc * gelu'(R) with R the bf16 pre-activation (the act-1 C2), replacing
      // a bf16 dX GEMM + ctclip_gelu_bwd (one rounding fewer: acc is not rounded to bf16 first)
      float rr[8];
      unpack8(*(const u32x4*)((const u16*)p.R + bidx * p.sR + gm * p.ldr + gn), rr);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] *= gelu_erf_grad(rr[j]);
    } else if (p.R) {
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
      // C2 (if given) keeps the pre-activation for the GELU backward
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
      // the fp16 GEGLU GEMM (act 2) writes h (fp16, derivative form) in the GEGLU pass below
      if (!(H16 && p.act == 2)) *(u32x4*)Cb = pack8(v);
    }
    if (p.C2 && p.act == 0) *(u32x4*)(p.C2 + bidx * p.sC2 + gm * p.ldc2 + gn) = pack8(v);
  }
  if (p.act == 2 && p.C2) {
    // GEGLU: each 64-column group is [32 x | 32 gate] -> 32 output columns
    for (int it = 0; it < (BM * 64 / 8) / NTH; ++it) {
      const int c = t + NTH * it;
      const int row = c >> 3, oc = (c & 7) * 8;          // output column within the tile's 64
      const int grp = oc >> 5, cc = grp * 64 + (oc & 31);  // x column within the tile
      const int64_t gm = m0 + row, gn = n0 / 2 + oc;
      if (gm >= p.M || n0 + grp * 64 >= p.N) continue;
      float v[8];
      if (H16) {
        // fp16 h in the derivative form [gelu(gate) | x gelu'(gate)] (the GEGLU backward's two
        // factors; gemm256.hip EP 2), g and the factors from the fp16-rounded x / gate
        float av[8], bv[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float xb = rh(cs[row * CS_LD + cc + j] * p.alpha);
          const float gb = rh(cs[row * CS_LD + 32 + cc + j] * p.alpha);
          float ge, dge;
          gelu_erf_and_grad(gb, ge, dge);
          av[j] = ge;
          bv[j] = xb * dge;
          v[j] = ge * xb;
        }
        if (p.C) {
          u16* hr = (u16*)p.C + bidx * p.sC + gm * p.ldc + n0 + cc;
          *(u32x4*)hr = pack8h(av);
          *(u32x4*)(hr + 32) = pack8h(bv);
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float x = cs[row * CS_LD + cc + j] * p.alpha;
          const float gt = cs[row * CS_LD + 32 + cc + j] * p.alpha;
          // round h as stored (bf16) first so forward g == geglu(stored h) bit-for-bit in backward
          v[j] = gelu_erf(bf2f(f2bf(gt))) * bf2f(f2bf(x));
        }
      }
      *(u32x4*)(p.C2 + bidx * p.sC2 + gm * p.ldc2 + gn) = pack8(v);
    }
  }
}

template <bool AK, bool BK, bool H16 = false>
int launch(const P& p, int batch, hipStream_t st) {
  dim3 grid(cdiv(p.N, BN), cdiv(p.M, BM), batch * p.split_k);
  hipLaunchKernelGGL((gemm_kernel<AK, BK, H16>), grid, dim3(NTH), SMEM_BYTES, st, p);
  CT_CHECK_LAUNCH();
  return 0;
}

__global__ void reduce_slabs_kernel(const float* __restrict__ s, int64_t nslab, int64_t rows, int64_t cols,
                                    int64_t ld, void* out, int64_t ldo, int out_f32, int accumulate) {
  const int64_t n4 = cols / 4;
  const int64_t total = rows * n4;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / n4, c = (i - r * n4) * 4;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int64_t z = 0; z < nslab; ++z) acc += *(const f32x4*)(s + (z * rows + r) * ld + c);
    if (out_f32) {
      float* o = (float*)out + r * ldo + c;
      if (accumulate) acc += *(const f32x4*)o;
      *(f32x4*)o = acc;
    } else {
      u16* o = (u16*)out + r * ldo + c;
      if (accumulate) {
        acc[0] += bf2f(o[0]); acc[1] += bf2f(o[1]); acc[2] += bf2f(o[2]); acc[3] += bf2f(o[3]);
      }
      o[0] = f2bf(acc[0]); o[1] = f2bf(acc[1]); o[2] = f2bf(acc[2]); o[3] = f2bf(acc[3]);
    }
  }
}

// split-K slab reduction straight into a row-mapped, column-cropped f32 destination (the packed FF
// weight gradients: dst[map[r]][c] (+)= sum_z s[z][r][c] for c < cols, rows with map[r] < 0 dropped):
// the reduction and the unpack of the packed rows in one pass, summed in reduce_slabs_kernel's order
// (0 + s0 + s1 + ...) and added to dst as the unpack did, so bit-identical to that pair
template <bool V4>
__global__ __launch_bounds__(256) void reduce_slabs_rows_kernel(const float* __restrict__ s, int64_t nslab, int64_t rows,
                                                                int64_t cols, int64_t ld, const int32_t* __restrict__ map,
                                                                float* __restrict__ dst, int64_t ldd, int accumulate) {
  constexpr int W = V4 ? 4 : 1;
  const int64_t nw = cols / W, total = rows * nw;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / nw, c = (i - r * nw) * W;
    const int64_t dr = map ? (int64_t)map[r] : r;
    if (dr < 0) continue;
    if constexpr (V4) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      for (int64_t z = 0; z < nslab; ++z) acc += *(const f32x4*)(s + (z * rows + r) * ld + c);
      f32x4* o = (f32x4*)(dst + dr * ldd + c);
      *o = accumulate ? *o + acc : acc;
    } else {
      float acc = 0.f;
      for (int64_t z = 0; z < nslab; ++z) acc += s[(z * rows + r) * ld + c];
      float* o = dst + dr * ldd + c;
      *o = accumulate ? *o + acc : acc;
    }
  }
}

// skinny reduction (few output elements, many slabs): block = 64 float4 columns x 16 slab lanes
__global__ __launch_bounds__(1024) void reduce_slabs_skinny_kernel(const float* __restrict__ s, int64_t nslab,
                                                                   int64_t rows, int64_t cols, int64_t ld,
                                                                   void* out, int64_t ldo, int out_f32,
                                                                   int accumulate) {
  __shared__ f32x4 red[16][64];
  const int c4 = threadIdx.x & 63, lane = threadIdx.x >> 6;
  const int64_t n4 = cols / 4;
  const int64_t e = (int64_t)blockIdx.x * 64 + c4;   // float4 index over rows*cols/4
  const bool valid = e < rows * n4;
  const int64_t r = valid ? e / n4 : 0, c = valid ? (e - r * n4) * 4 : 0;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (valid) {
#pragma unroll 4
    for (int64_t z = lane; z < nslab; z += 16) acc += *(const f32x4*)(s + (z * rows + r) * ld + c);
  }
  red[lane][c4] = acc;
  __syncthreads();
  if (lane == 0 && valid) {
    for (int k = 1; k < 16; ++k) acc += red[k][c4];
    if (out_f32) {
      float* o = (float*)out + r * ldo + c;
      if (accumulate) acc += *(const f32x4*)o;
      *(f32x4*)o = acc;
    } else {
      u16* o = (u16*)out + r * ldo + c;
      if (accumulate) {
        acc[0] += bf2f(o[0]); acc[1] += bf2f(o[1]); acc[2] += bf2f(o[2]); acc[3] += bf2f(o[3]);
      }
      o[0] = f2bf(acc[0]); o[1] = f2bf(acc[1]); o[2] = f2bf(acc[2]); o[3] = f2bf(acc[3]);
    }
  }
}

// Split-K combine with the full GEMM epilogue (bias, residual, GELU + pre-activation, f32 /
// bf16 output, accumulate, bf16 shadow): out = epilogue(sum_z slabs[z]).  Each thread owns 8
// consecutive columns of one row.  Lets skinny GEMMs (M = 1024 text-tower tokens) split K over
// 4-6x more workgroups than they have output tiles.
__global__ __launch_bounds__(256) void reduce_slabs_ep_kernel(const float* __restrict__ s, int64_t nslab,
                                                              int64_t rows, int64_t cols, int64_t ld, P p,
                                                              unsigned thresh = 0u, float dscale = 1.f,
                                                              uint64_t seed = 0, int drop = 0) {
  const int64_t n8 = cols / 8;
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= rows * n8) return;
  const int64_t r = i / n8, c = (i - r * n8) * 8;
  float v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int64_t z = 0; z < nslab; ++z) {
    const float* sp = s + (z * rows + r) * ld + c;
    const f32x4 a = *(const f32x4*)sp, b = *(const f32x4*)(sp + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) { v[j] += a[j]; v[4 + j] += b[j]; }
  }
  if (p.bias) {
    const f32x4 a = *(const f32x4*)(p.bias + c), b = *(const f32x4*)(p.bias + c + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) { v[j] += a[j]; v[4 + j] += b[j]; }
  }
  if (drop) {   // BERT hidden dropout of the dense output, before the residual (ctclip_dropout's mask)
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] *= hid_keep(seed, r * cols + c + j, thresh, dscale);
  }
  if (p.R) {
    if (p.r_f32) {
      const float* Rp = (const float*)p.R + r * p.ldr + c;
      const f32x4 a = *(const f32x4*)Rp, b = *(const f32x4*)(Rp + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) { v[j] += a[j]; v[4 + j] += b[j]; }
    } else {
      float rr[8];
      unpack8(*(const u32x4*)((const u16*)p.R + r * p.ldr + c), rr);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += rr[j];
    }
  }
  if (p.act == 1) {
    if (p.C2) *(u32x4*)(p.C2 + r * p.ldc2 + c) = pack8(v);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = gelu_erf(v[j]);
  }
  if (p.c_f32) {
    float* Cf = (float*)p.C + r * p.ldc + c;
    if (p.accumulate) {
      const f32x4 a = *(const f32x4*)Cf, b = *(const f32x4*)(Cf + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) { v[j] += a[j]; v[4 + j] += b[j]; }
    }
    *(f32x4*)Cf = f32x4{v[0], v[1], v[2], v[3]};
    *(f32x4*)(Cf + 4) = f32x4{v[4], v[5], v[6], v[7]};
  } else {
    u16* Cb = (u16*)p.C + r * p.ldc + c;
    if (p.accumulate) {
      float rr[8];
      unpack8(*(const u32x4*)Cb, rr);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += rr[j];
    }
    *(u32x4*)Cb = pack8(v);
  }
  if (p.C2 && p.act == 0) *(u32x4*)(p.C2 + r * p.ldc2 + c) = pack8(v);
}

static bool s_smem_set = false;

}  // namespace

extern "C" int ctclip_gemm(const ctclip_gemm_args* a, void* stream) {
  if (!a) return CT_EINVAL;
  if (a->M <= 0 || a->N <= 0 || a->K <= 0) return a->M == 0 || a->N == 0 ? 0 : CT_ESHAPE;
  const int split = a->split_k > 0 ? a->split_k : 1;
  if (split > 1 && !a->c_f32) return CT_EINVAL;
  if (a->act == 2 && !a->C2) return CT_EINVAL;
  // 16-byte alignment of every operand row / chunk
  CT_REQUIRE(aligned16(a->A) && aligned16(a->B) && aligned16(a->C), CT_EALIGN);
  CT_REQUIRE(a->lda % 8 == 0 && a->ldb % 8 == 0, CT_EALIGN);
  CT_REQUIRE(a->a_kcontig ? (a->K % 8 == 0) : (a->M % 8 == 0), CT_EALIGN);
  CT_REQUIRE(a->b_kcontig ? (a->K % 8 == 0) : (a->N % 8 == 0), CT_EALIGN);
  if (a->act != 3) {
    CT_REQUIRE(a->N % 8 == 0 && a->ldc % 8 == 0, CT_EALIGN);
    if (a->C2) CT_REQUIRE(aligned16(a->C2) && a->ldc2 % 8 == 0, CT_EALIGN);
    if (a->R) CT_REQUIRE(aligned16(a->R) && a->ldr % 8 == 0, CT_EALIGN);
  }
  if (a->act == 2) CT_REQUIRE(a->N % 64 == 0 && a->ldc2 % 8 == 0, CT_ESHAPE);
  if (a->act == 4) CT_REQUIRE(a->N % 32 == 0 && a->R && !a->r_f32 && !a->c_f32 && a->split_k <= 1, CT_EINVAL);
  if (a->act == 6)
    CT_REQUIRE(a->R && !a->r_f32 && !a->bias && !a->accumulate && !a->C2 && split == 1 && (a->batch <= 1), CT_EINVAL);
  if (a->act == 5)
    CT_REQUIRE(a->C2 && a->bias && aligned16(a->bias) && !a->R && !a->c_f32 && !a->accumulate && split == 1 &&
                   (a->batch <= 1) && a->N % 64 == 0 && a->n2 > 0 && a->n2 % 64 == 0 && a->n2 <= a->N,
               CT_EINVAL);
  if (a->B2) CT_REQUIRE(aligned16(a->B2) && a->act != 3, CT_EINVAL);
  if (a->A_lo || a->B_lo) {
    // split-fp16 x3 operands: the 8-phase kernel only (any M / N; rows past the matrix are clamped
    // loads whose results are dropped), f32 rows or the x3 GEGLU pair
    CT_REQUIRE(a->A_lo && a->B_lo && a->ab_f16 && aligned16(a->A_lo) && aligned16(a->B_lo) && a->K % 64 == 0,
               CT_EINVAL);
    CT_REQUIRE(a->a_kcontig && a->b_kcontig && !a->B2 && split == 1 && !a->accumulate && a->batch <= 1, CT_EINVAL);
    CT_REQUIRE(a->K < (int64_t)64 * 10000, CT_ESHAPE);   // K-step index 3 k + s stays < 2^15
    if (a->act == 2)
      CT_REQUIRE(!a->c_f32 && !a->R && !a->bias && a->C3 && aligned16(a->C3) && a->ldc3 % 8 == 0 &&
                     (!a->C4 || (aligned16(a->C4) && a->ldc4 % 8 == 0)),
                 CT_EINVAL);
    else
      CT_REQUIRE(a->act == 0 && a->c_f32 && (!a->R || a->r_f32), CT_EINVAL);
    return ctclip_gemm256(a, 1, 1, stream);
  }
  if (a->ab_f16)   // fp16 operands: the 3D-ViT forward GEMMs and the VQ distance GEMM (act 3, round 6;
                   // K-contiguous A and B, no split-K / B2)
    CT_REQUIRE(a->a_kcontig && a->b_kcontig && !a->B2 && split == 1 && (a->act == 0 || a->act == 2 || a->act == 3) &&
                   !a->accumulate && (a->batch <= 1),
               CT_EINVAL);
  if (!a->B2 && a->act != 6) {   // act 6 (GELU backward): the 128-tile kernel only (text tower)
    const int b = a->batch > 0 ? a->batch : 1;
    const int64_t tiles256 = ((a->M + 255) / 256) * ((a->N + 255) / 256) * split * b;
    if (a->K % 64 == 0 && a->M >= 256 && a->N >= 256 && tiles256 >= 160 && (split == 1 || (a->K / split) >= 512) &&
        (!a->bias || aligned16(a->bias)))
      return ctclip_gemm256(a, split, b, stream);
  }
  if (a->act == 5) {
    // small shapes: the plain GEMM, then the stand-alone l2norm kernel (same rule)
    ctclip_gemm_args g = *a;
    g.act = 0;
    g.bias = nullptr;
    g.C2 = nullptr;
    const int rc = ctclip_gemm(&g, stream);
    if (rc) return rc;
    return ctclip_l2norm_scale_fwd(a->C, a->ldc, a->M, a->n2 / 32, 32, a->bias, a->C2, a->ldc2, stream);
  }
  if (!s_smem_set) {
    (void)hipFuncSetAttribute((const void*)gemm_kernel<true, true>, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM_BYTES);
    (void)hipFuncSetAttribute((const void*)gemm_kernel<true, false>, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM_BYTES);
    (void)hipFuncSetAttribute((const void*)gemm_kernel<false, true>, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM_BYTES);
    (void)hipFuncSetAttribute((const void*)gemm_kernel<false, false>, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM_BYTES);
    (void)hipFuncSetAttribute((const void*)gemm_kernel<true, true, true>, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM_BYTES);
    s_smem_set = true;
  }
  P p;
  p.M = a->M; p.N = a->N; p.K = a->K;
  p.A = (const u16*)a->A; p.lda = a->lda;
  p.B = (const u16*)a->B; p.ldb = a->ldb;
  p.B2 = (const u16*)a->B2;
  p.C = a->C; p.ldc = a->ldc; p.c_f32 = a->c_f32;
  p.C2 = (u16*)a->C2; p.ldc2 = a->ldc2;
  p.bias = a->bias;
  p.R = a->R; p.ldr = a->ldr; p.r_f32 = a->r_f32;
  p.alpha = a->alpha; p.act = a->act; p.accumulate = a->accumulate; p.split_k = split;
  p.sA = a->sA; p.sB = a->sB; p.sC = a->sC; p.sC2 = a->sC2; p.sR = a->sR;
  int64_t kper = (a->K + split - 1) / split;
  kper = (kper + BKT - 1) / BKT * BKT;
  p.kper = kper;
  p.r_f16 = a->r_f16;
  const int batch = a->batch > 0 ? a->batch : 1;
  hipStream_t st = (hipStream_t)stream;
  if (a->ab_f16) return launch<true, true, true>(p, batch, st);
  if (a->a_kcontig && a->b_kcontig) return launch<true, true>(p, batch, st);
  if (a->a_kcontig && !a->b_kcontig) return launch<true, false>(p, batch, st);
  if (!a->a_kcontig && a->b_kcontig) return launch<false, true>(p, batch, st);
  return launch<false, false>(p, batch, st);
}

extern "C" int ctclip_reduce_slabs_ep(const float* slabs, int64_t nslab, int64_t rows, int64_t cols, int64_t ld,
                                      const ctclip_gemm_args* a, void* stream) {
  if (rows == 0 || cols == 0) return 0;
  CT_REQUIRE(a && (a->act == 0 || a->act == 1), CT_EINVAL);
  CT_REQUIRE(cols % 8 == 0 && ld % 4 == 0 && a->ldc % 8 == 0 && aligned16(slabs) && aligned16(a->C), CT_EALIGN);
  if (a->bias) CT_REQUIRE(aligned16(a->bias), CT_EALIGN);
  if (a->R) CT_REQUIRE(aligned16(a->R) && a->ldr % 8 == 0, CT_EALIGN);
  if (a->C2) CT_REQUIRE(aligned16(a->C2) && a->ldc2 % 8 == 0, CT_EALIGN);
  P p{};
  p.C = a->C; p.ldc = a->ldc; p.c_f32 = a->c_f32;
  p.C2 = (u16*)a->C2; p.ldc2 = a->ldc2;
  p.bias = a->bias;
  p.R = a->R; p.ldr = a->ldr; p.r_f32 = a->r_f32;
  p.act = a->act; p.accumulate = a->accumulate;
  const int64_t total = rows * (cols / 8);
  hipLaunchKernelGGL(reduce_slabs_ep_kernel, dim3(cdiv(total, 256)), dim3(256), 0, (hipStream_t)stream, slabs, nslab,
                     rows, cols, ld, p);
  CT_CHECK_LAUNCH();
  return 0;
}

// the same with BERT's hidden dropout on (sum + bias) before the residual: C = drop(sum + bias) + R
// (the mask of ctclip_dropout on a contiguous [rows][cols] tensor; requires ldc == cols)
extern "C" int ctclip_reduce_slabs_ep_drop(const float* slabs, int64_t nslab, int64_t rows, int64_t cols, int64_t ld,
                                           const ctclip_gemm_args* a, float dp, uint64_t seed, void* stream) {
  if (rows == 0 || cols == 0) return 0;
  CT_REQUIRE(a && a->act == 0 && !a->accumulate && a->ldc == cols && dp >= 0.f && dp < 1.f, CT_EINVAL);
  CT_REQUIRE(cols % 8 == 0 && ld % 4 == 0 && aligned16(slabs) && aligned16(a->C), CT_EALIGN);
  if (a->bias) CT_REQUIRE(aligned16(a->bias), CT_EALIGN);
  if (a->R) CT_REQUIRE(aligned16(a->R) && a->ldr % 8 == 0, CT_EALIGN);
  if (a->C2) CT_REQUIRE(aligned16(a->C2) && a->ldc2 % 8 == 0, CT_EALIGN);
  P p{};
  p.C = a->C; p.ldc = a->ldc; p.c_f32 = a->c_f32;
  p.C2 = (u16*)a->C2; p.ldc2 = a->ldc2;
  p.bias = a->bias;
  p.R = a->R; p.ldr = a->ldr; p.r_f32 = a->r_f32;
  p.act = 0; p.accumulate = 0;
  const unsigned thresh = (unsigned)std::min(4294967295.0, (double)dp * 4294967296.0);
  const int64_t total = rows * (cols / 8);
  hipLaunchKernelGGL(reduce_slabs_ep_kernel, dim3(cdiv(total, 256)), dim3(256), 0, (hipStream_t)stream, slabs, nslab,
                     rows, cols, ld, p, thresh, 1.f / (1.f - dp), seed, 1);
  CT_CHECK_LAUNCH();
  return 0;
}

// batched skinny reductions: blockIdx.y = job, blockIdx.x = 64 float4 columns; 16 slab lanes
// strided as reduce_slabs_skinny_kernel (same order of additions)
constexpr int MULTI_JOBS = 32;
struct MultiJobs {
  ctclip_slab_job j[MULTI_JOBS];
};
__global__ __launch_bounds__(1024) void reduce_slabs_multi_kernel(MultiJobs jobs) {
  __shared__ f32x4 red[16][64];
  const ctclip_slab_job jb = jobs.j[blockIdx.y];
  const int c4 = threadIdx.x & 63, lane = threadIdx.x >> 6;
  const int64_t e = (int64_t)blockIdx.x * 64 + c4;
  if ((int64_t)blockIdx.x * 64 >= jb.cols / 4) return;   // uniform: this job has fewer columns
  const bool valid = e < jb.cols / 4;
  const int64_t c = valid ? e * 4 : 0;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (valid) {
#pragma unroll 4
    for (int64_t z = lane; z < jb.nslab; z += 16) acc += *(const f32x4*)(jb.slabs + z * jb.cols + c);
  }
  red[lane][c4] = acc;
  __syncthreads();
  if (lane == 0 && valid) {
    for (int k = 1; k < 16; ++k) acc += red[k][c4];
    float* o = jb.out + c;
    if (jb.accumulate) acc += *(const f32x4*)o;
    *(f32x4*)o = acc;
  }
}

extern "C" int ctclip_reduce_slabs_multi(const ctclip_slab_job* jobs, int32_t njobs, void* stream) {
  // the jobs of one call run concurrently, each read-add-writing its output: outputs must be
  // distinct (the caller splits a shared output over successive calls, kernels.flush_reductions)
  for (int32_t i = 0; i < njobs; ++i)
    for (int32_t k = 0; k < i; ++k) CT_REQUIRE(jobs[i].out != jobs[k].out, CT_EINVAL);
  for (int32_t j0 = 0; j0 < njobs; j0 += MULTI_JOBS) {
    MultiJobs mj{};
    const int n = std::min<int32_t>(MULTI_JOBS, njobs - j0);
    int64_t maxc = 0;
    for (int i = 0; i < n; ++i) {
      const ctclip_slab_job& jb = jobs[j0 + i];
      CT_REQUIRE(jb.cols % 4 == 0 && aligned16(jb.slabs) && aligned16(jb.out), CT_EALIGN);
      mj.j[i] = jb;
      maxc = std::max(maxc, jb.cols);
    }
    if (maxc == 0) continue;
    hipLaunchKernelGGL(reduce_slabs_multi_kernel, dim3((unsigned)cdiv(maxc / 4, 64), n), dim3(1024), 0,
                       (hipStream_t)stream, mj);
    CT_CHECK_LAUNCH();
  }
  return 0;
}

extern "C" int ctclip_reduce_slabs_rows(const float* slabs, int64_t nslab, int64_t rows, int64_t cols, int64_t ld,
                                        const int32_t* map, float* dst, int64_t ldd, int32_t accumulate, void* stream) {
  if (rows == 0 || cols == 0) return 0;
  CT_REQUIRE(cols <= ld, CT_EINVAL);
  const bool v4 = cols % 4 == 0 && ld % 4 == 0 && ldd % 4 == 0 && aligned16(slabs) && aligned16(dst);
  const int64_t total = rows * (v4 ? cols / 4 : cols);
  const int blocks = (int)std::min<int64_t>(4096, (total + 255) / 256);
  if (v4)
    hipLaunchKernelGGL(reduce_slabs_rows_kernel<true>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, slabs, nslab,
                       rows, cols, ld, map, dst, ldd, accumulate);
  else
    hipLaunchKernelGGL(reduce_slabs_rows_kernel<false>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, slabs, nslab,
                       rows, cols, ld, map, dst, ldd, accumulate);
  CT_CHECK_LAUNCH();
  return 0;
}

extern "C" int ctclip_reduce_slabs(const float* slabs, int64_t nslab, int64_t rows, int64_t cols, int64_t ld,
                                   void* out, int64_t ldo, int32_t out_f32, int32_t accumulate, void* stream) {
  if (rows == 0 || cols == 0) return 0;
  CT_REQUIRE(cols % 4 == 0 && ld % 4 == 0 && ldo % 4 == 0, CT_EALIGN);
  const int64_t total = rows * (cols / 4);
  if (total < 64 * 1024 && nslab >= 16) {
    hipLaunchKernelGGL(reduce_slabs_skinny_kernel, dim3(cdiv(total, 64)), dim3(1024), 0, (hipStream_t)stream, slabs,
                       nslab, rows, cols, ld, out, ldo, out_f32, accumulate);
    CT_CHECK_LAUNCH();
    return 0;
  }
  const int blocks = (int)std::min<int64_t>(4096, (total + 255) / 256);
  hipLaunchKernelGGL(reduce_slabs_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, slabs, nslab, rows, cols,
                     ld, out, ldo, out_f32, accumulate);
  CT_CHECK_LAUNCH();
  return 0;
}
