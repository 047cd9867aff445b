// MX-fp8 (OCP e4m3 elements, e8m0 scale per 32 consecutive k) GEMM for gfx950 — the
// configs[3] precision of SURVEY §8(d) ("fp8 attention and MLP GEMMs").  The reference runs these
// linears in fp32 (ct_clip/attention.py:44-52 FeedForward, :88-181 Attention projections); this
// path is compared to the build's own bf16 path with a tolerance stated per test.
//
// Quantiser (OCP MX v1.0 rule): per row and 32-element k block, X = floor(log2(amax)) - 8
// (8 = emax of e4m3), element = sat_448(RNE(x * 2^-X)), scale byte = X + 127.  k in [K, Kp) is
// zero-filled so the GEMM's K only needs to be a multiple of 128.
//
// GEMM: C[M,N] = alpha * (A . B^T) (+ bias) (+ f32 residual, bf16 copy; or the GEGLU epilogue of
// the 8-phase bf16 kernel), A [M][Kp] and B [N][Kp] fp8 K-contiguous with their
// scale planes [rows][Kp/32].  Tile 128x128x128 (k in elements = bytes), 256 threads = 2x2 waves,
// each wave a 64x64 block of 4x4 v_mfma_scale_f32_16x16x128_f8f6f4 (2x the bf16 MFMA rate per
// clock on gfx950).  Operand lane map (tools/mx_probe.hip, found on the GPU with integer data):
// lane l holds row (l & 15), k = 16g..16g+15 in bytes 0-15 and 64+16g..64+16g+15 in bytes 16-31
// (g = l>>4), and passes the e8m0 scale of (row, k block g) — block g's 32 k sit in lane groups
// 2(g&1), 2(g&1)+1 at byte half g>>1, so the scale is NOT that of the lane's own bytes.
// Register-staged double-buffered LDS (one barrier per k-step), rows padded to 144 B, scales
// staged beside the tiles; f32 tile staged through LDS for 16-B output rows (element stores for
// a ragged last column group or an unaligned ldc).
#include "common.h"
#include "../../include/ctclip_hip.h"

namespace {

typedef int i32x8 __attribute__((ext_vector_type(8)));

// BM = 128 (wave tile 64x64, 2 workgroups / CU; the default) or 256 (wave tile 128x64: 25 % fewer
// LDS bytes per flop, 1 workgroup / CU).  Measured (profiles/r01_mx_bench_v2.log): 256 is 12-27 %
// slower at every model shape — with 4-11 k-steps per tile the exposed first-load latency and
// epilogue, which a second co-resident workgroup hides, cost more than the LDS reads saved.
constexpr int BN = 128, BK = 128, NTH = 256;
constexpr int KROW = BK + 16;                      // 144-B rows
constexpr int CS_LD = 132;
template <int BM> struct Cfg {
  static constexpr int TA = BM * KROW, TB = BN * KROW;       // operand tiles
  static constexpr int SA = BM * 4, SB = BN * 4;              // scale bytes per k-step
  static constexpr int BUF = TA + TB + SA + SB;
  static constexpr int SMEM = 2 * BUF;
  static constexpr int MI = BM / 32;                         // 16-row A fragments per wave
  static constexpr int NA = BM / 32;                         // 16-B A loads per thread per k-step
  static_assert(128 * CS_LD * 4 <= SMEM, "epilogue staging fits");
};

__device__ __forceinline__ unsigned e4m3_pair(float a, float b) {
  a = fminf(fmaxf(a, -448.f), 448.f);
  b = fminf(fmaxf(b, -448.f), 448.f);
  return (unsigned)__builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false) & 0xffffu;
}

// one thread per (row, 32-k block)
__global__ __launch_bounds__(256) void quant_kernel(const void* __restrict__ x, int x_f32, int64_t rows, int64_t K,
                                                    int64_t ldx, uint8_t* __restrict__ q, int64_t ldq,
                                                    uint8_t* __restrict__ sc, int64_t nblk) {
  const int64_t id = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (id >= rows * nblk) return;
  const int64_t r = id / nblk, b = id - r * nblk, k0 = b * 32;
  float v[32];
  if (x_f32) {
    const float* xr = (const float*)x + r * ldx + k0;
    if (k0 + 32 <= K && ((ldx | k0) & 3) == 0) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const f32x4 t = ((const f32x4*)xr)[i];
        v[4 * i] = t[0]; v[4 * i + 1] = t[1]; v[4 * i + 2] = t[2]; v[4 * i + 3] = t[3];
      }
    } else {
      for (int i = 0; i < 32; ++i) v[i] = k0 + i < K ? xr[i] : 0.f;
    }
  } else {
    const u16* xr = (const u16*)x + r * ldx + k0;
    if (k0 + 32 <= K && ((ldx | k0) & 7) == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) unpack8(((const u32x4*)xr)[i], v + 8 * i);
    } else {
      for (int i = 0; i < 32; ++i) v[i] = k0 + i < K ? bf2f(xr[i]) : 0.f;
    }
  }
  float amax = 0.f;
#pragma unroll
  for (int i = 0; i < 32; ++i) amax = fmaxf(amax, fabsf(v[i]));
  int X = 0;
  if (amax > 0.f) {
    const int e = (int)((__float_as_uint(amax) >> 23) & 255);
    X = (e ? e - 127 : -127) - 8;                 // floor(log2 amax) - emax(e4m3); subnormal amax -> -135
    X = max(-127, min(127, X));
  }
  const float inv = __uint_as_float((unsigned)(127 - X) << 23 & 0x7f800000u);  // 2^-X (X in [-126, 127])
  const float mul = X == -127 ? 0x1p126f * 2.f : inv;
  unsigned w[8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
    w[i] = e4m3_pair(v[4 * i] * mul, v[4 * i + 1] * mul) | (e4m3_pair(v[4 * i + 2] * mul, v[4 * i + 3] * mul) << 16);
  u32x4* qo = (u32x4*)(q + r * ldq + k0);
  qo[0] = make_uint4(w[0], w[1], w[2], w[3]);
  qo[1] = make_uint4(w[4], w[5], w[6], w[7]);
  sc[r * nblk + b] = (uint8_t)(X + 127);
}

struct P {
  int64_t M, N, Kp;
  const uint8_t* A; int64_t lda; const uint8_t* sA;
  const uint8_t* B; int64_t ldb; const uint8_t* sB;
  void* C; int64_t ldc; int c_f32;
  const float* bias; float alpha;
  const float* R; int64_t ldr;     // f32 residual added after bias (or null)
  u16* C2; int64_t ldc2;           // act 0: bf16 copy of C; act 2: the GEGLU output g
  int act;                         // 0 none, 2 GEGLU over 32-column [x | gate] pairs (bf16 C = h)
};

__device__ __forceinline__ void xcd_remap(int& tx, int& ty) {
  const int gx = gridDim.x, nwg = gridDim.x * gridDim.y;
  const int orig = blockIdx.y * gx + blockIdx.x;
  int id = orig;
  if (nwg >= 16) {
    const int xcd = orig & 7, qq = nwg >> 3, rr = nwg & 7;
    id = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (orig >> 3);
  }
  ty = id / gx;
  tx = id - ty * gx;
}

template <int BM>
struct Stage {
  u32x4 a[Cfg<BM>::NA], b[4];
  unsigned s[BM / 128 + 1];
};

template <int BM>
__device__ __forceinline__ void gload(Stage<BM>& st, const P& p, int64_t m0, int64_t n0, int64_t k0) {
  const int t = threadIdx.x, kc = (t & 7) * 16;
#pragma unroll
  for (int i = 0; i < Cfg<BM>::NA; ++i) {
    const int64_t r = (t >> 3) + 32 * i;
    st.a[i] = m0 + r < p.M ? *(const u32x4*)(p.A + (m0 + r) * p.lda + k0 + kc) : make_uint4(0, 0, 0, 0);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t r = (t >> 3) + 32 * i;
    st.b[i] = n0 + r < p.N ? *(const u32x4*)(p.B + (n0 + r) * p.ldb + k0 + kc) : make_uint4(0, 0, 0, 0);
  }
  // scale rows: [0, BM) of A then [0, BN) of B, one u32 (4 k blocks) each
  const int64_t nb = p.Kp >> 5;
#pragma unroll
  for (int j = 0; j < BM / 128 + 1; ++j) {
    const int s = t + 256 * j;
    if (s < BM) st.s[j] = m0 + s < p.M ? *(const unsigned*)(p.sA + (m0 + s) * nb + (k0 >> 5)) : 0x7f7f7f7fu;
    else if (s < BM + BN)
      st.s[j] = n0 + (s - BM) < p.N ? *(const unsigned*)(p.sB + (n0 + s - BM) * nb + (k0 >> 5)) : 0x7f7f7f7fu;
  }
}

template <int BM>
__device__ __forceinline__ void swrite(char* buf, const Stage<BM>& st) {
  using C = Cfg<BM>;
  const int t = threadIdx.x, kc = (t & 7) * 16;
#pragma unroll
  for (int i = 0; i < C::NA; ++i) *(u32x4*)(buf + ((t >> 3) + 32 * i) * KROW + kc) = st.a[i];
#pragma unroll
  for (int i = 0; i < 4; ++i) *(u32x4*)(buf + C::TA + ((t >> 3) + 32 * i) * KROW + kc) = st.b[i];
#pragma unroll
  for (int j = 0; j < BM / 128 + 1; ++j) {
    const int s = t + 256 * j;
    if (s < BM + BN) *(unsigned*)(buf + C::TA + C::TB + s * 4) = st.s[j];   // sA rows then sB rows
  }
}

__device__ __forceinline__ i32x8 frag(const char* tile, int r0, int lane) {
  const char* src = tile + (r0 + (lane & 15)) * KROW + 16 * (lane >> 4);
  const u32x4 lo = *(const u32x4*)src, hi = *(const u32x4*)(src + 64);
  i32x8 v;
  v[0] = (int)lo.x; v[1] = (int)lo.y; v[2] = (int)lo.z; v[3] = (int)lo.w;
  v[4] = (int)hi.x; v[5] = (int)hi.y; v[6] = (int)hi.z; v[7] = (int)hi.w;
  return v;
}

template <int BM>
__global__ __launch_bounds__(NTH, BM == 128 ? 2 : 1) void mx_gemm_kernel(P p) {
  using C = Cfg<BM>;
  constexpr int MI = C::MI, WR = BM / 2;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, wr = w >> 1, wc = w & 1;
  int tx, ty;
  xcd_remap(tx, ty);
  const int64_t m0 = (int64_t)ty * BM, n0 = (int64_t)tx * BN;
  f32x4 acc[MI][4];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = (int)(p.Kp / BK);
  Stage<BM> st;
  if (nk > 0) {
    gload<BM>(st, p, m0, n0, 0);
    swrite<BM>(smem, st);
  }
  __syncthreads();
  const int kb = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    char* cur = smem + (kt & 1) * C::BUF;
    if (kt + 1 < nk) gload<BM>(st, p, m0, n0, (int64_t)(kt + 1) * BK);
    const uint8_t* sa = (const uint8_t*)(cur + C::TA + C::TB);
    const uint8_t* sb = sa + C::SA;
    i32x8 bfr[4];
    int scb[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int rb = wc * 64 + j * 16;
      bfr[j] = frag(cur + C::TA, rb, lane);
      scb[j] = sb[(rb + (lane & 15)) * 4 + kb];
    }
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int ra = wr * WR + i * 16;
      const i32x8 af = frag(cur, ra, lane);
      const int sca = sa[(ra + (lane & 15)) * 4 + kb];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af, bfr[j], acc[i][j], 0, 0, 0, sca, 0, scb[j]);
    }
    if (kt + 1 < nk) swrite<BM>(smem + ((kt + 1) & 1) * C::BUF, st);
    __syncthreads();
  }

  // epilogue in 128-row halves: stage f32 through LDS, then 16-B output rows
  float* cs = (float*)smem;
  const int t = threadIdx.x;
  const bool vec = (p.ldc & 7) == 0;
#pragma unroll
  for (int h = 0; h < BM / 128; ++h) {
    if (BM == 128 || wr == h) {
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            cs[((BM == 128 ? wr * 64 : 0) + i * 16 + (lane >> 4) * 4 + r) * CS_LD + wc * 64 + j * 16 + (lane & 15)] =
                acc[i][j][r];
    }
    __syncthreads();
    for (int it = 0; it < (128 * BN / 8) / NTH; ++it) {
      const int c = t + NTH * it;
      const int row = c >> 4, cc = (c & 15) * 8;
      const int64_t gm = m0 + h * 128 + row, gn = n0 + cc;
      if (gm >= p.M || gn >= p.N) continue;
      float v[8];
      const f32x4 lo = *(const f32x4*)(cs + row * CS_LD + cc);
      const f32x4 hi = *(const f32x4*)(cs + row * CS_LD + cc + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) { v[j] = lo[j] * p.alpha; v[4 + j] = hi[j] * p.alpha; }
      const int nv = (int)min((int64_t)8, p.N - gn);
      if (p.bias) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] += j < nv ? p.bias[gn + j] : 0.f;
      }
      if (p.act == 2) {
        // GEGLU (the 8-phase kernel's rule): h keeps both halves (bf16), g = gelu(gate) x from the
        // bf16-rounded x and gate; chunks in the x half of a 64-column group write g's 8 columns
        *(u32x4*)((u16*)p.C + gm * p.ldc + gn) = pack8(v);
        if ((cc & 63) < 32) {
          const f32x4 glo = *(const f32x4*)(cs + row * CS_LD + cc + 32);
          const f32x4 ghi = *(const f32x4*)(cs + row * CS_LD + cc + 36);
          const float gt[8] = {glo[0], glo[1], glo[2], glo[3], ghi[0], ghi[1], ghi[2], ghi[3]};
          float gg[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) gg[j] = gelu_erf(bf2f(f2bf(gt[j] * p.alpha))) * bf2f(f2bf(v[j]));
          *(u32x4*)(p.C2 + gm * p.ldc2 + (gn >> 6) * 32 + (gn & 63)) = pack8(gg);
        }
        continue;
      }
      if (p.R) {
        const float* Rp = p.R + gm * p.ldr + gn;
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] += j < nv ? Rp[j] : 0.f;
      }
      if (p.C2 && vec && nv == 8) *(u32x4*)(p.C2 + gm * p.ldc2 + gn) = pack8(v);
      if (vec && nv == 8) {
        if (p.c_f32) {
          float* Cf = (float*)p.C + gm * p.ldc + gn;
          *(f32x4*)Cf = f32x4{v[0], v[1], v[2], v[3]};
          *(f32x4*)(Cf + 4) = f32x4{v[4], v[5], v[6], v[7]};
        } else {
          *(u32x4*)((u16*)p.C + gm * p.ldc + gn) = pack8(v);
        }
      } else {
        for (int j = 0; j < nv; ++j) {
          if (p.c_f32) ((float*)p.C)[gm * p.ldc + gn + j] = v[j];
          else ((u16*)p.C)[gm * p.ldc + gn + j] = f2bf(v[j]);
        }
      }
    }
    __syncthreads();
  }
}

int g_mx_tile = 0;   // 0 = auto, 128 / 256 = forced (diagnostic)

template <int BM>
int mx_launch(const P& p, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)mx_gemm_kernel<BM>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              Cfg<BM>::SMEM);
    attr = true;
  }
  dim3 grid((unsigned)cdiv(p.N, BN), (unsigned)cdiv(p.M, BM));
  hipLaunchKernelGGL(mx_gemm_kernel<BM>, grid, dim3(NTH), Cfg<BM>::SMEM, s, p);
  CT_CHECK_LAUNCH();
  return 0;
}

}  // namespace

extern "C" int ctclip_quant_mxfp8(const void* x, int32_t x_f32, int64_t rows, int64_t K, int64_t ldx, void* q,
                                  int64_t ldq, void* scales, int64_t Kp, void* stream) {
  CT_REQUIRE(rows >= 0 && K >= 0 && Kp >= K && Kp % 128 == 0 && ldq >= Kp && ldq % 16 == 0 && ldx >= K, CT_ESHAPE);
  CT_REQUIRE(((uintptr_t)q & 15) == 0, CT_EALIGN);
  if (rows == 0 || Kp == 0) return 0;
  const int64_t n = rows * (Kp / 32);
  hipLaunchKernelGGL(quant_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, x, x_f32,
                     rows, K, ldx, (uint8_t*)q, ldq, (uint8_t*)scales, Kp / 32);
  CT_CHECK_LAUNCH();
  return 0;
}

extern "C" int ctclip_gemm_mxfp8(const ctclip_mx_gemm_args* a, void* stream) {
  CT_REQUIRE(a->M >= 0 && a->N >= 0 && a->Kp >= 0 && a->Kp % 128 == 0, CT_ESHAPE);
  CT_REQUIRE(a->lda >= a->Kp && a->ldb >= a->Kp && a->lda % 16 == 0 && a->ldb % 16 == 0, CT_ESHAPE);
  CT_REQUIRE(a->ldc >= a->N, CT_ESHAPE);
  CT_REQUIRE(((uintptr_t)a->A & 15) == 0 && ((uintptr_t)a->B & 15) == 0 && ((uintptr_t)a->C & 15) == 0, CT_EALIGN);
  CT_REQUIRE(((uintptr_t)a->sA & 3) == 0 && ((uintptr_t)a->sB & 3) == 0, CT_EALIGN);
  if (a->M == 0 || a->N == 0) return 0;
  CT_REQUIRE(a->act == 0 || a->act == 2, CT_EINVAL);
  if (a->act == 2) CT_REQUIRE(a->C2 && !a->c_f32 && !a->R && !a->bias && a->N % 64 == 0 && a->ldc % 8 == 0 && a->ldc2 % 8 == 0, CT_ESHAPE);
  if (a->C2 || a->R) CT_REQUIRE(a->ldc % 8 == 0 && a->N % 8 == 0, CT_ESHAPE);
  if (a->C2) CT_REQUIRE(((uintptr_t)a->C2 & 15) == 0 && a->ldc2 % 8 == 0, CT_EALIGN);
  P p{a->M, a->N, a->Kp, (const uint8_t*)a->A, a->lda, (const uint8_t*)a->sA, (const uint8_t*)a->B, a->ldb,
      (const uint8_t*)a->sB, a->C, a->ldc, a->c_f32, a->bias, a->alpha, a->R, a->ldr, (u16*)a->C2, a->ldc2, a->act};
  const int bm = g_mx_tile ? g_mx_tile : 128;
  return bm == 256 ? mx_launch<256>(p, (hipStream_t)stream) : mx_launch<128>(p, (hipStream_t)stream);
}

extern "C" int ctclip_gemm_mxfp8_set_tile(int bm) {
  const int prev = g_mx_tile;
  g_mx_tile = (bm == 128 || bm == 256) ? bm : 0;
  return prev;
}
