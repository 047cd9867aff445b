// Fused input normalisation + patchify + LayerNorm(patch_dim) for CTViT.to_patch_emb.
//   int16 HU -> clamp(-1000, 1000) / 1000.f      (ct_clip/data.py:150-152; f32 division is
//                                                 bit-identical to the reference's f64 path)
//   Rearrange 'b c (t pt) (h p1) (w p2) -> b t h w (c pt p1 p2)'   (ct_clip/ctvit.py:170)
//   LayerNorm(patch_dim) statistics (ctvit.py:171); the kernel writes xhat = (x-mean)*rstd in
//   bf16.  The LN affine (gamma, beta) is folded into the following Linear on the host:
//   W' = W*diag(gamma), b' = b + W.beta, so the same xhat also serves the weight gradient.
// One wave per token (patch), the patch held in registers, element -> voxel offsets from a
// small per-call table (no integer division in the loop).
#include <type_traits>

#include "common.h"
#include "../../include/ctclip_hip.h"

namespace {

constexpr int MAXC = 64;  // patch_dim <= 64*64 = 4096

__global__ __launch_bounds__(256) void patch_ln_kernel(const void* __restrict__ video, int is_f32, int is_hu,
                                                       int64_t ntok, int T, int Hg, int Wg, int64_t vol_stride,
                                                       int64_t frame_elems, int W, int PT, int P,
                                                       const int32_t* __restrict__ offs, int pd, float eps,
                                                       u16* __restrict__ out, int64_t ldo, u16* __restrict__ out16,
                                                       u16* __restrict__ out16lo) {
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
      if (is_f32) {
        x = ((const float*)video)[a];
      } else {
        x = (float)((const short*)video)[a];
      }
      if (is_hu) x = fminf(fmaxf(x, -1000.f), 1000.f) / 1000.f;
    }
    v[i] = x;
    s += x;
  }
  const float mean = warp_sum(s) / pd;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < MAXC; ++i) {
    const int e = lane + 64 * i;
    if (e < pd) { const float d = v[i] - mean; q += d * d; }
  }
  const float rstd = rsqrtf(warp_sum(q) / pd + eps);
  u16* o = out ? out + tok * ldo : nullptr;   // (bf16 xhat optional with out16: the eval forward)
  u16* oh = out16 ? out16 + tok * ldo : nullptr;
  u16* ol = out16lo ? out16lo + tok * ldo : nullptr;
#pragma unroll
  for (int i = 0; i < MAXC; ++i) {
    const int e = lane + 64 * i;
    if (e < pd) {
      const float a = (v[i] - mean) * rstd;
      if (o) o[e] = f2bf(a);
      if (oh) oh[e] = f2h(a);
      if (ol) ol[e] = f2h(a - rh(a));
    }
  }
  for (int e = pd + lane; e < ldo; e += 64) {   // K padding of the patch-embed GEMM
    if (o) o[e] = 0;
    if (oh) oh[e] = 0;
    if (ol) ol[e] = 0;
  }
}

// Row-strip form (the fast path, single-channel volumes): a workgroup owns PW = 4 horizontally
// adjacent patches of one (b, t, hg) strip.  Phase 1 reads the strip's PT x P rows of 4P voxels
// with coalesced 16-B loads and scatters the normalised voxels into LDS in patch order
// [token][pt p1 p2]; phase 2 (one wave per patch) takes the LN statistics from LDS and writes
// xhat as contiguous bf16 pairs.  Every voxel is read from HBM once in full 16-B segments
// (the gather form above reads 40-B row pieces through the cache).
constexpr int PW = 4;

// int16 volumes stay raw int16 in LDS (32 KB per workgroup -> 4 per CU) and are normalised
// when read back; all of a thread's 16-B loads are issued before the first LDS scatter.
template <bool F32>
__global__ __launch_bounds__(256) void patch_ln_strip_kernel(const void* __restrict__ video, int is_hu, int T,
                                                             int Hg, int Wg, int64_t vol_stride, int H, int W,
                                                             int PT, int P, float eps, u16* __restrict__ out,
                                                             int64_t ldo, u16* __restrict__ out16,
                                                             u16* __restrict__ out16lo) {
  using E = typename std::conditional<F32, float, short>::type;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  E* sx = (E*)smem_raw;   // [PW][pd]
  constexpr int VEC = F32 ? 4 : 8;
  constexpr int NCH = PW * 4096 / VEC / 256;   // 16-B loads per thread at pd <= 4096
  const int pd = PT * P * P;
  // patch groups of one strip are consecutive workgroups: they share the strip's cache lines
  int r = blockIdx.y;
  const int hg = r % Hg; r /= Hg;
  const int t = r % T;
  const int b = r / T;
  const int wg0 = blockIdx.x * PW;
  const int ntk = min(PW, Wg - wg0);
  const int cpr = ntk * P / VEC;   // 16-B chunks per row segment
  const int nchunk = PT * P * cpr;
  const int64_t base = (int64_t)b * vol_stride + ((int64_t)t * PT * H + (int64_t)hg * P) * W + (int64_t)wg0 * P;
  u32x4 ld[NCH];
#pragma unroll
  for (int m = 0; m < NCH; ++m) {
    const int c = threadIdx.x + m * 256;
    if (c < nchunk) {
      const int k = c % cpr, rowi = c / cpr, p1 = rowi % P, pt = rowi / P;
      ld[m] = *(const u32x4*)((const E*)video + base + ((int64_t)pt * H + p1) * W + k * VEC);
    }
  }
#pragma unroll
  for (int m = 0; m < NCH; ++m) {
    const int c = threadIdx.x + m * 256;
    if (c >= nchunk) break;
    const int k = c % cpr, rowi = c / cpr, p1 = rowi % P, pt = rowi / P;
    const E* ev = (const E*)&ld[m];
    int cr = k * VEC, tk = cr / P, p2 = cr - tk * P;
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      sx[tk * pd + (pt * P + p1) * P + p2] = ev[j];
      if (++p2 == P) { p2 = 0; ++tk; }
    }
  }
  __syncthreads();
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (w >= ntk) return;
  const E* px = sx + w * pd;
  constexpr int NP = 32;   // pairs per lane: pd <= 4096
  float v[NP][2];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const int e = 2 * (lane + 64 * i);
    v[i][0] = v[i][1] = 0.f;
    if (e < pd) {
      if constexpr (F32) {
        const float2 u = *(const float2*)(px + e);
        v[i][0] = u.x;
        v[i][1] = u.y;
      } else {
        const uint32_t u = *(const uint32_t*)(px + e);
        v[i][0] = (float)(short)(u & 0xffffu);
        v[i][1] = (float)(short)(u >> 16);
      }
      if (is_hu) {
        v[i][0] = fminf(fmaxf(v[i][0], -1000.f), 1000.f) / 1000.f;
        v[i][1] = fminf(fmaxf(v[i][1], -1000.f), 1000.f) / 1000.f;
      }
    }
    s += v[i][0] + v[i][1];
  }
  const float mean = warp_sum(s) / pd;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    if (2 * (lane + 64 * i) < pd) {
      const float d0 = v[i][0] - mean, d1 = v[i][1] - mean;
      q += d0 * d0 + d1 * d1;
    }
  }
  const float rstd = rsqrtf(warp_sum(q) / pd + eps);
  const int64_t tok = (((int64_t)b * T + t) * Hg + hg) * Wg + wg0 + w;
  uint32_t* o = out ? (uint32_t*)(out + tok * ldo) : nullptr;       // (optional with out16: eval forward)
  uint32_t* oh = out16 ? (uint32_t*)(out16 + tok * ldo) : nullptr;   // optional fp16 copy
  uint32_t* ol = out16lo ? (uint32_t*)(out16lo + tok * ldo) : nullptr;   // ... and its lo residual (x3)
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const int e = 2 * (lane + 64 * i);
    if (e < pd) {
      const float a = (v[i][0] - mean) * rstd, c = (v[i][1] - mean) * rstd;
      if (o) o[e >> 1] = (uint32_t)f2bf(a) | ((uint32_t)f2bf(c) << 16);
      if (oh) oh[e >> 1] = pack2h(a, c);
      if (ol) ol[e >> 1] = pack2h(a - rh(a), c - rh(c));
    }
  }
  for (int e = pd + 2 * lane; e < ldo; e += 128) {   // K padding of the patch-embed GEMM
    if (o) o[e >> 1] = 0u;
    if (oh) oh[e >> 1] = 0u;
    if (ol) ol[e >> 1] = 0u;
  }
}

// x / 1000.f, correctly rounded, for the clamped HU range: one reciprocal product and one fma
// correction (checked against IEEE division for every integer in [-1000, 1000]:
// tests/test_hu_divide.py) instead of the ~10-instruction division sequence
__device__ __forceinline__ float div1000(float x) {
#pragma clang fp contract(off)
  const float R = 1.0f / 1000.0f;
  const float q0 = x * R;
  const float r = __builtin_fmaf(-q0, 1000.0f, x);
  return __builtin_fmaf(r, R, q0);
}

// P = 20 strip kernel (the CT-CLIP patch): the strip stays in LDS in its natural [PT*P rows]
// [ntk*P columns] layout -- one ds_write_b128 per 16-B load instead of a per-voxel scatter --
// and phase 2 maps pair j of a patch to (row j / 10, column 2 (j % 10)) with constant divisors.
template <bool F32>
__global__ __launch_bounds__(256) void patch_ln_strip20_kernel(const void* __restrict__ video, int is_hu, int T,
                                                               int Hg, int Wg, int64_t vol_stride, int H, int W,
                                                               int PT, float eps, u16* __restrict__ out,
                                                               int64_t ldo, int g_remap, u16* __restrict__ out16,
                                                               u16* __restrict__ out16lo) {
  using E = typename std::conditional<F32, float, short>::type;
  constexpr int P = 20, VEC = F32 ? 4 : 8;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  E* sx = (E*)smem_raw;   // [PT * P][ntk * P]
  constexpr int NCH = PW * 4096 / VEC / 256;
  const int pd = PT * P * P;
  // XCD-aware block order: the gridDim.x strips of one (b, t, hg) row group share partial 128-B
  // lines at their edges (a 4-patch strip row is 160 B of int16); consecutive dispatch goes round
  // robin over the 8 XCDs, so remap the linear index to give each XCD a contiguous range and let
  // its L2 merge those lines instead of each XCD fetching them from HBM
  int bx = blockIdx.x, by = blockIdx.y;
  {
    const int nb = gridDim.x * gridDim.y, lin = by * gridDim.x + bx;
    if (nb >= 64 && g_remap) {
      const int xcd = lin & 7, q = nb >> 3, rm = nb & 7;
      const int id = (xcd < rm ? xcd * (q + 1) : rm * (q + 1) + (xcd - rm) * q) + (lin >> 3);
      by = id / gridDim.x;
      bx = id - by * gridDim.x;
    }
  }
  int r = by;
  const int hg = r % Hg; r /= Hg;
  const int t = r % T;
  const int b = r / T;
  const int wg0 = bx * PW;
  const int ntk = min(PW, Wg - wg0);
  const int sw = ntk * P, cpr = sw / VEC;
  const int nchunk = PT * P * cpr;
  const int64_t base = (int64_t)b * vol_stride + ((int64_t)t * PT * H + (int64_t)hg * P) * W + (int64_t)wg0 * P;
  // branch-free loads (clamped chunk index), all in flight before the first LDS write
  u32x4 ld[NCH];
#pragma unroll
  for (int m = 0; m < NCH; ++m) {
    const int c = min((int)threadIdx.x + m * 256, nchunk - 1);
    const int k = c % cpr, rowi = c / cpr, p1 = rowi % P, pt = rowi / P;
    ld[m] = *(const u32x4*)((const E*)video + base + ((int64_t)pt * H + p1) * W + k * VEC);
  }
  __builtin_amdgcn_sched_barrier(0);   // keep the scheduler from pairing each load with its write
  // unconditional writes (lanes past the strip rewrite the last chunk with its own bytes), so the
  // loads are not sunk into per-chunk branches and serialised behind their writes
#pragma unroll
  for (int m = 0; m < NCH; ++m) {
    const int c = min((int)threadIdx.x + m * 256, nchunk - 1);
    *(u32x4*)(sx + c * VEC) = ld[m];   // row c / cpr, column (c % cpr) * VEC
  }
  __syncthreads();
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (w >= ntk) return;
  const E* px = sx + w * P;
  constexpr int NP = 32;   // pairs per lane: pd <= 4096
  float v[NP][2];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const int j = lane + 64 * i;
    v[i][0] = v[i][1] = 0.f;
    if (2 * j < pd) {
      const int row = j / (P / 2), col = 2 * (j - row * (P / 2));
      const E* e = px + row * sw + col;
      if constexpr (F32) {
        const float2 u = *(const float2*)e;
        v[i][0] = u.x;
        v[i][1] = u.y;
      } else {
        const uint32_t u = *(const uint32_t*)e;
        v[i][0] = (float)(short)(u & 0xffffu);
        v[i][1] = (float)(short)(u >> 16);
      }
      if (is_hu) {
        v[i][0] = div1000(fminf(fmaxf(v[i][0], -1000.f), 1000.f));
        v[i][1] = div1000(fminf(fmaxf(v[i][1], -1000.f), 1000.f));
      }
    }
    s += v[i][0] + v[i][1];
  }
  const float mean = warp_sum(s) / pd;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    if (2 * (lane + 64 * i) < pd) {
      const float d0 = v[i][0] - mean, d1 = v[i][1] - mean;
      q += d0 * d0 + d1 * d1;
    }
  }
  const float rstd = rsqrtf(warp_sum(q) / pd + eps);
  const int64_t tok = (((int64_t)b * T + t) * Hg + hg) * Wg + wg0 + w;
  uint32_t* o = out ? (uint32_t*)(out + tok * ldo) : nullptr;       // (optional with out16: eval forward)
  uint32_t* oh = out16 ? (uint32_t*)(out16 + tok * ldo) : nullptr;   // optional fp16 copy
  uint32_t* ol = out16lo ? (uint32_t*)(out16lo + tok * ldo) : nullptr;   // ... and its lo residual (x3)
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const int e = 2 * (lane + 64 * i);
    if (e < pd) {
      const float a = (v[i][0] - mean) * rstd, c = (v[i][1] - mean) * rstd;
      if (o) o[e >> 1] = (uint32_t)f2bf(a) | ((uint32_t)f2bf(c) << 16);
      if (oh) oh[e >> 1] = pack2h(a, c);
      if (ol) ol[e >> 1] = pack2h(a - rh(a), c - rh(c));
    }
  }
  for (int e = pd + 2 * lane; e < ldo; e += 128) {   // K padding of the patch-embed GEMM
    if (o) o[e >> 1] = 0u;
    if (oh) oh[e >> 1] = 0u;
    if (ol) ol[e >> 1] = 0u;
  }
}

bool s_strip_attr = false;
// A/B switch of the strip20 kernel's XCD-aware block order (CTCLIP_PATCH_XCD=0: dispatch order)
int s_patch_remap = [] { const char* e = getenv("CTCLIP_PATCH_XCD"); return e ? atoi(e) != 0 : 1; }();
bool s_strip20_attr = false;

// Given G = dy^T . xhat  [N][K] (f32) and colsum(dy) cs[N], produce the grads of the folded
// LayerNorm+Linear pair: dW = G*g + cs (x) b, dgamma[k] = sum_n W[n,k] G[n,k], dbeta[k] = sum_n W[n,k] cs[n].
__global__ __launch_bounds__(1024) void patch_wgrad_kernel(const float* __restrict__ G, const float* __restrict__ cs,
                                                          const float* __restrict__ Wt, const float* __restrict__ g,
                                                          const float* __restrict__ bt, int N, int K,
                                                          float* __restrict__ dW, float* __restrict__ dg,
                                                          float* __restrict__ db, int accumulate) {
  // 64 columns x 16 row groups (one wave each: rows n = wave, wave + 16, ...); dW is elementwise,
  // the row groups' dgamma / dbeta partials fold in group order through LDS (no float atomics:
  // bit-reproducible)
  __shared__ float red[2][16][64];
  const int lane = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int k = blockIdx.x * 64 + lane;
  float sg = 0.f, sb = 0.f;
  if (k < K) {
    const float gk = g[k], bk = bt[k];
    for (int n = rg; n < N; n += 16) {
      const float Gv = G[(int64_t)n * K + k], w = Wt[(int64_t)n * K + k], c = cs[n];
      sg += w * Gv;
      sb += w * c;
      const float d = Gv * gk + c * bk;
      float* p = dW + (int64_t)n * K + k;
      *p = accumulate ? *p + d : d;
    }
  }
  red[0][rg][lane] = sg;
  red[1][rg][lane] = sb;
  __syncthreads();
  if (rg < 2 && k < K) {
    float v = red[rg][0][lane];
#pragma unroll
    for (int i = 1; i < 16; ++i) v += red[rg][i][lane];
    float* o = (rg == 0 ? dg : db) + k;
    *o = accumulate ? *o + v : v;
  }
}

}  // namespace

namespace {

// CTViT.to_pixels' Rearrange 'b t h w (c pt p1 p2) -> b c (t pt) (h p1) (w p2)' (ct_clip/ctvit.py:
// 194-197) fused with F.mse_loss(video, recon) (:451) and its gradient: one wave per token row;
// element e of the row lands at voxel base + offs[e] (the patch_ln map, inverted).  Writes the
// squared-error sum of the row (part[tok]), optionally the gradient 2 (pix - video) / n in the
// row layout and the reconstruction in the video layout.
__global__ __launch_bounds__(256) void unpatch_mse_kernel(const float* __restrict__ pix, int64_t ldp,
                                                          const void* __restrict__ video, int is_f32, int is_hu,
                                                          int64_t ntok, int T, int Hg, int Wg, int64_t vol_stride,
                                                          int64_t frame_elems, int W, int PT, int P,
                                                          const int32_t* __restrict__ offs, int pd, float gscale,
                                                          float* __restrict__ grad, int64_t ldg,
                                                          float* __restrict__ recon, float* __restrict__ part) {
  const int lane = threadIdx.x & 63;
  const int64_t tok = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (tok >= ntok) return;
  int64_t r = tok;
  const int wg = (int)(r % Wg); r /= Wg;
  const int hg = (int)(r % Hg); r /= Hg;
  const int t = (int)(r % T);
  const int64_t b = r / T;
  const int64_t base = b * vol_stride + (int64_t)t * PT * frame_elems + (int64_t)hg * P * W + (int64_t)wg * P;
  const float* row = pix + tok * ldp;
  float sq = 0.f;
  for (int e = lane; e < pd; e += 64) {
    const int64_t a = base + offs[e];
    float x = is_f32 ? ((const float*)video)[a] : (float)((const short*)video)[a];
    if (is_hu) x = fminf(fmaxf(x, -1000.f), 1000.f) / 1000.f;
    const float y = row[e], d = y - x;
    sq += d * d;
    if (grad) grad[tok * ldg + e] = gscale * d;
    if (recon) recon[a] = y;
  }
  sq = warp_sum(sq);
  if (lane == 0) part[tok] = sq;
}

// mean of the row sums (one workgroup, f64 accumulation: deterministic)
__global__ __launch_bounds__(256) void mse_finish_kernel(const float* __restrict__ part, int64_t n, double inv,
                                                         float* __restrict__ loss) {
  __shared__ double red[256];
  double s = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += 256) s += part[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) loss[0] = (float)(red[0] * inv);
}

}  // namespace

extern "C" int ctclip_unpatch_mse(const float* pix, int64_t ldp, const void* video, int32_t is_f32, int32_t is_hu,
                                  int64_t B, int32_t C, int32_t F, int32_t H, int32_t W, int32_t PT, int32_t P,
                                  const int32_t* offs, float* grad, int64_t ldg, float* recon, float* part,
                                  float* loss, void* stream) {
  const int pd = C * PT * P * P;
  CT_REQUIRE(pix && video && offs && part && loss, CT_EINVAL);
  CT_REQUIRE(F % PT == 0 && H % P == 0 && W % P == 0 && ldp >= pd && (!grad || ldg >= pd), CT_ESHAPE);
  const int T = F / PT, Hg = H / P, Wg = W / P;
  const int64_t ntok = B * T * Hg * Wg;
  if (ntok == 0) return 0;
  const int64_t frame = (int64_t)H * W, vol = (int64_t)C * F * frame;
  const int64_t n = B * vol;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(unpatch_mse_kernel, dim3(cdiv(ntok, 4)), dim3(256), 0, st, pix, ldp, video, is_f32, is_hu, ntok,
                     T, Hg, Wg, vol, frame, W, PT, P, offs, pd, (float)(2.0 / (double)n), grad, ldg, recon, part);
  hipLaunchKernelGGL(mse_finish_kernel, dim3(1), dim3(256), 0, st, part, ntok, 1.0 / (double)n, loss);
  CT_CHECK_LAUNCH();
  return 0;
}


extern "C" int ctclip_patch_ln(const void* video, int32_t is_f32, int32_t is_hu, int64_t B, int32_t C, int32_t F,
                               int32_t H, int32_t W, int32_t PT, int32_t P, const int32_t* offs, float eps,
                               void* out, int64_t ldo, void* stream) {
  return ctclip_patch_ln_x2(video, is_f32, is_hu, B, C, F, H, W, PT, P, offs, eps, out, nullptr, ldo, stream);
}

extern "C" int ctclip_patch_ln_x2(const void* video, int32_t is_f32, int32_t is_hu, int64_t B, int32_t C, int32_t F,
                                  int32_t H, int32_t W, int32_t PT, int32_t P, const int32_t* offs, float eps,
                                  void* out, void* out16, int64_t ldo, void* stream) {
  return ctclip_patch_ln_x3(video, is_f32, is_hu, B, C, F, H, W, PT, P, offs, eps, out, out16, nullptr, ldo, stream);
}

extern "C" int ctclip_patch_ln_x3(const void* video, int32_t is_f32, int32_t is_hu, int64_t B, int32_t C, int32_t F,
                                  int32_t H, int32_t W, int32_t PT, int32_t P, const int32_t* offs, float eps,
                                  void* out, void* out16, void* out16lo, int64_t ldo, void* stream) {
  if ((out16lo || !out) && !out16) return CT_EINVAL;
  const int pd = C * PT * P * P;
  CT_REQUIRE(pd <= 64 * MAXC, CT_ESHAPE);
  if (ldo <= 0) ldo = pd;
  CT_REQUIRE(ldo >= pd && ldo % 2 == 0, CT_ESHAPE);
  CT_REQUIRE(F % PT == 0 && H % P == 0 && W % P == 0, CT_ESHAPE);
  const int T = F / PT, Hg = H / P, Wg = W / P;
  const int64_t ntok = B * T * Hg * Wg;
  const int64_t frame = (int64_t)H * W;
  const int64_t vol = (int64_t)C * F * frame;
  if (ntok == 0) return 0;
  const int vec = is_f32 ? 4 : 8;
  if (C == 1 && pd % 2 == 0 && (PW * P) % vec == 0 && ((Wg % PW) * P) % vec == 0 && W % vec == 0) {
    if (!s_strip_attr) {
      (void)hipFuncSetAttribute((const void*)patch_ln_strip_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                PW * 4096 * 4);
      (void)hipFuncSetAttribute((const void*)patch_ln_strip_kernel<false>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, PW * 4096 * 4);
      s_strip_attr = true;
    }
    dim3 grid(cdiv(Wg, PW), B * T * Hg);
    const size_t sm = (size_t)PW * pd * (is_f32 ? 4 : 2);
    if (P == 20) {
      if (!s_strip20_attr) {
        (void)hipFuncSetAttribute((const void*)patch_ln_strip20_kernel<true>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, PW * 4096 * 4);
        (void)hipFuncSetAttribute((const void*)patch_ln_strip20_kernel<false>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, PW * 4096 * 4);
        s_strip20_attr = true;
      }
      if (is_f32)
        hipLaunchKernelGGL(patch_ln_strip20_kernel<true>, grid, dim3(256), sm, (hipStream_t)stream, video, is_hu, T,
                           Hg, Wg, vol, H, W, PT, eps, (u16*)out, ldo, s_patch_remap, (u16*)out16, (u16*)out16lo);
      else
        hipLaunchKernelGGL(patch_ln_strip20_kernel<false>, grid, dim3(256), sm, (hipStream_t)stream, video, is_hu, T,
                           Hg, Wg, vol, H, W, PT, eps, (u16*)out, ldo, s_patch_remap, (u16*)out16, (u16*)out16lo);
    } else if (is_f32)
      hipLaunchKernelGGL(patch_ln_strip_kernel<true>, grid, dim3(256), sm, (hipStream_t)stream, video, is_hu, T, Hg,
                         Wg, vol, H, W, PT, P, eps, (u16*)out, ldo, (u16*)out16, (u16*)out16lo);
    else
      hipLaunchKernelGGL(patch_ln_strip_kernel<false>, grid, dim3(256), sm, (hipStream_t)stream, video, is_hu, T,
                         Hg, Wg, vol, H, W, PT, P, eps, (u16*)out, ldo, (u16*)out16, (u16*)out16lo);
  } else {
    hipLaunchKernelGGL(patch_ln_kernel, dim3(cdiv(ntok, 4)), dim3(256), 0, (hipStream_t)stream, video, is_f32,
                       is_hu, ntok, T, Hg, Wg, vol, frame, W, PT, P, offs, pd, eps, (u16*)out, ldo, (u16*)out16,
                       (u16*)out16lo);
  }
  CT_CHECK_LAUNCH();
  return 0;
}

extern "C" int ctclip_patch_wgrad(const float* G, const float* cs, const float* Wt, const float* g, const float* b,
                                  int32_t N, int32_t K, float* dW, float* dg, float* db, int32_t accumulate,
                                  void* stream) {
  if (K <= 0) return 0;
  hipLaunchKernelGGL(patch_wgrad_kernel, dim3(cdiv(K, 64)), dim3(1024), 0, (hipStream_t)stream, G, cs, Wt, g, b, N, K,
                     dW, dg, db, accumulate);
  CT_CHECK_LAUNCH();
  return 0;
}
