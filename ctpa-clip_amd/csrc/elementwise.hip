// Bandwidth-bound helpers: GEGLU / GELU backward, weight packing (f32 master -> bf16
// working layout), gradient unpacking, casts, HU normalisation.
#include "common.h"
#include "../../include/ctclip_hip.h"

namespace {

// GEGLU backward on the group-interleaved pre-activation h (see gemm.hip act=2):
// group t: h[:, 64t + c] = x part, h[:, 64t + 32 + c] = gate part, g[:, 32t + c] = gelu(gate)*x.
// (ct_clip/attention.py:39-42)
__global__ __launch_bounds__(256) void geglu_bwd_kernel(const u16* __restrict__ dg, int64_t lddg,
                                                        const u16* __restrict__ h, int64_t ldh, int64_t rows,
                                                        int gcols, u16* __restrict__ dh, int64_t lddh) {
  const int nch = gcols / 8;
  const int64_t total = rows * nch;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / nch;
    const int gc = (int)(i - r * nch) * 8;
    const int t = gc >> 5, c = gc & 31;
    float d[8], x[8], gt[8], ox[8], og[8];
    unpack8(*(const u32x4*)(dg + r * lddg + gc), d);
    unpack8(*(const u32x4*)(h + r * ldh + t * 64 + c), x);
    unpack8(*(const u32x4*)(h + r * ldh + t * 64 + 32 + c), gt);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float ge, dge;
      gelu_erf_and_grad(gt[j], ge, dge);
      ox[j] = d[j] * ge;
      og[j] = d[j] * x[j] * dge;
    }
    *(u32x4*)(dh + r * lddh + t * 64 + c) = pack8(ox);
    *(u32x4*)(dh + r * lddh + t * 64 + 32 + c) = pack8(og);
  }
}

// dpre = dy * gelu'(pre)    (BERT intermediate GELU)
__global__ __launch_bounds__(256) void gelu_bwd_kernel(const u16* __restrict__ dy, const u16* __restrict__ pre,
                                                       u16* __restrict__ dx, int64_t n8) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
    float d[8], x[8], o[8];
    unpack8(((const u32x4*)dy)[i], d);
    unpack8(((const u32x4*)pre)[i], x);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = d[j] * gelu_erf_grad(x[j]);
    ((u32x4*)dx)[i] = pack8(o);
  }
}

// dst[r][c] (bf16, ld_dst) = src[map[r]][c] * (colscale ? colscale[c] : 1), zero if map[r] < 0 or c >= cols
template <typename OUT, bool H16 = false>
__global__ __launch_bounds__(256) void pack_rows_kernel(const float* __restrict__ src, int64_t ld_src,
                                                        const int32_t* __restrict__ map, int64_t rows_dst,
                                                        int cols, int cols_dst, const float* __restrict__ colscale,
                                                        OUT* __restrict__ dst, int64_t ld_dst) {
  const int64_t total = rows_dst * cols_dst;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / cols_dst;
    const int c = (int)(i - r * cols_dst);
    const int64_t sr = map ? (int64_t)map[r] : r;
    float v = 0.f;
    if (sr >= 0 && c < cols) {
      v = src[sr * ld_src + c];
      if (colscale) v *= colscale[c];
    }
    if constexpr (H16) dst[r * ld_dst + c] = f2h(v);
    else if constexpr (sizeof(OUT) == 2) dst[r * ld_dst + c] = f2bf(v);
    else dst[r * ld_dst + c] = v;
  }
}

// dst[map[r]][c] (f32) (+)= src[r][c] for r with map[r] >= 0, c < cols
__global__ __launch_bounds__(256) void unpack_rows_kernel(const float* __restrict__ src, int64_t ld_src,
                                                          const int32_t* __restrict__ map, int64_t rows_src, int cols,
                                                          float* __restrict__ dst, int64_t ld_dst, int accumulate) {
  const int64_t total = rows_src * cols;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / cols;
    const int c = (int)(i - r * cols);
    const int64_t dr = map ? (int64_t)map[r] : r;
    if (dr < 0) continue;
    const float v = src[r * ld_src + c];
    float* d = dst + dr * ld_dst + c;
    *d = accumulate ? *d + v : v;
  }
}

__global__ __launch_bounds__(256) void cast_f32_bf16_kernel(const float* __restrict__ x, u16* __restrict__ y, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    y[i] = f2bf(x[i]);
}

__global__ __launch_bounds__(256) void cast_split_kernel(const float* __restrict__ x, u16* __restrict__ hi,
                                                         u16* __restrict__ lo, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float v = x[i];
    const u16 h = f2bf(v);
    hi[i] = h;
    lo[i] = f2bf(v - bf2f(h));
  }
}

// y = a + b (f32) with optional bf16 shadow; n % 4 == 0
__global__ __launch_bounds__(256) void add_f32_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                      float* __restrict__ y, u16* __restrict__ yb, int64_t n4) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    f32x4 v = ((const f32x4*)a)[i];
    if (b) v += ((const f32x4*)b)[i];
    if (y) ((f32x4*)y)[i] = v;
    if (yb) {
      uint2 o;
      o.x = pack2(v[0], v[1]);
      o.y = pack2(v[2], v[3]);
      ((uint2*)yb)[i] = o;
    }
  }
}

inline int grid_for(int64_t n) { return (int)std::min<int64_t>(8192, std::max<int64_t>(1, (n + 255) / 256)); }

// Split-fp16 image pair of f32 values (the x3 GEMM's operands, ctclip_gemm_args.A_lo / B_lo):
// hi = fp16(v s), lo = fp16(v s - hi), 8 values per thread (16-B hi / lo stores).  A value whose
// scaled magnitude leaves fp16's range (or is NaN / inf) sets CT_STATUS_F16_RANGE.
__device__ __forceinline__ void split8(const float* v, float s, u32x4& h, u32x4& l, bool& bad) {
  float a[8], b[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float x = v[j] * s;
    bad |= !f16_ok(x);
    a[j] = rh(x);
    b[j] = x - a[j];
  }
  h = pack8h(a);
  l = pack8h(b);
}

__global__ __launch_bounds__(256) void split_f16_kernel(const float* __restrict__ x, int64_t ldx, int64_t rows,
                                                        int cols, float s, u16* __restrict__ hi,
                                                        u16* __restrict__ lo, int64_t ldo, int* status) {
  const int nch = cols / 8;
  const int64_t total = rows * nch;
  bool bad = false;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / nch;
    const int c = (int)(i - r * nch) * 8;
    const float* xp = x + r * ldx + c;
    const f32x4 a = *(const f32x4*)xp, b = *(const f32x4*)(xp + 4);
    const float v[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
    u32x4 h, l;
    split8(v, s, h, l, bad);
    *(u32x4*)(hi + r * ldo + c) = h;
    *(u32x4*)(lo + r * ldo + c) = l;
  }
  status_or(status, CT_STATUS_F16_RANGE, bad);
}

// pack_rows (row map, column scale, zero padding) into a split-fp16 pair, values scaled by s
__global__ __launch_bounds__(256) void pack_rows_x3_kernel(const float* __restrict__ src, int64_t ld_src,
                                                           const int32_t* __restrict__ map, int64_t rows_dst, int cols,
                                                           int cols_dst, const float* __restrict__ colscale, float s,
                                                           u16* __restrict__ hi, u16* __restrict__ lo, int64_t ld_dst,
                                                           int* status) {
  const int64_t total = rows_dst * cols_dst;
  bool bad = false;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / cols_dst;
    const int c = (int)(i - r * cols_dst);
    const int64_t sr = map ? (int64_t)map[r] : r;
    float v = 0.f;
    if (sr >= 0 && c < cols) {
      v = src[sr * ld_src + c];
      if (colscale) v *= colscale[c];
    }
    const float x = v * s;
    bad |= !f16_ok(x);
    const float h = rh(x);
    hi[r * ld_dst + c] = f2h(h);
    lo[r * ld_dst + c] = f2h(x - h);
  }
  status_or(status, CT_STATUS_F16_RANGE, bad);
}

}  // namespace

extern "C" int ctclip_split_f16(const float* x, int64_t ldx, int64_t rows, int32_t cols, float scale, void* hi,
                                void* lo, int64_t ldo, int32_t* status, void* stream) {
  if (rows == 0) return 0;
  CT_REQUIRE(x && hi && lo && rows > 0 && cols > 0 && cols % 8 == 0 && ldx % 4 == 0 && ldo % 8 == 0, CT_EINVAL);
  CT_REQUIRE(aligned16(x) && aligned16(hi) && aligned16(lo), CT_EALIGN);
  hipLaunchKernelGGL(split_f16_kernel, dim3(grid_for(rows * cols / 8)), dim3(256), 0, (hipStream_t)stream, x, ldx, rows,
                     cols, scale, (u16*)hi, (u16*)lo, ldo, (int*)status);
  CT_CHECK_LAUNCH();
  return 0;
}

extern "C" int ctclip_pack_rows_x3(const float* src, int64_t ld_src, const int32_t* map, int64_t rows_dst,
                                   int32_t cols, int32_t cols_dst, const float* colscale, float scale, void* hi,
                                   void* lo, int64_t ld_dst, int32_t* status, void* stream) {
  if (rows_dst == 0) return 0;
  CT_REQUIRE(src && hi && lo && cols <= cols_dst, CT_EINVAL);
  hipLaunchKernelGGL(pack_rows_x3_kernel, dim3(grid_for(rows_dst * cols_dst)), dim3(256), 0, (hipStream_t)stream, src,
                     ld_src, map, rows_dst, cols, cols_dst, colscale, scale, (u16*)hi, (u16*)lo, ld_dst, (int*)status);
  CT_CHECK_LAUNCH();
  return 0;
}

extern "C" int ctclip_geglu_bwd(const void* dg, int64_t lddg, const void* h, int64_t ldh, int64_t rows, int32_t gcols,
                                void* dh, int64_t lddh, void* stream) {
  CT_REQUIRE(gcols % 32 == 0, CT_ESHAPE);
  hipLaunchKernelGGL(geglu_bwd_kernel, dim3(grid_for(rows * gcols / 8)), dim3(256), 0, (hipStream_t)stream,
                     (const u16*)dg, lddg, (const u16*)h, ldh, rows, gcols, (u16*)dh, lddh);
  CT_CHECK_LAUNCH();
  return 0;
}

extern "C" int ctclip_gelu_bwd(const void* dy, const void* pre, void* dx, int64_t n, void* stream) {
  CT_REQUIRE(n % 8 == 0 && aligned16(dy) && aligned16(pre) && aligned16(dx), CT_EALIGN);
  hipLaunchKernelGGL(gelu_bwd_kernel, dim3(grid_for(n / 8)), dim3(256), 0, (hipStream_t)stream, (const u16*)dy,
                     (const u16*)pre, (u16*)dx, n / 8);
  CT_CHECK_LAUNCH();
  return 0;
}

extern "C" int ctclip_pack_rows(const float* src, int64_t ld_src, const int32_t* map, int64_t rows_dst, int32_t cols,
                                int32_t cols_dst, const float* colscale, void* dst, int64_t ld_dst, void* stream) {
  hipLaunchKernelGGL(pack_rows_kernel<u16>, dim3(grid_for(rows_dst * cols_dst)), dim3(256), 0, (hipStream_t)stream,
                     src, ld_src, map, rows_dst, cols, cols_dst, colscale, (u16*)dst, ld_dst);
  CT_CHECK_LAUNCH();
  return 0;
}

extern "C" int ctclip_pack_rows_h16(const float* src, int64_t ld_src, const int32_t* map, int64_t rows_dst,
                                    int32_t cols, int32_t cols_dst, const float* colscale, void* dst, int64_t ld_dst,
                                    void* stream) {
  hipLaunchKernelGGL((pack_rows_kernel<u16, true>), dim3(grid_for(rows_dst * cols_dst)), dim3(256), 0,
                     (hipStream_t)stream, src, ld_src, map, rows_dst, cols, cols_dst, colscale, (u16*)dst, ld_dst);
  CT_CHECK_LAUNCH();
  return 0;
}

extern "C" int ctclip_pack_rows_f32(const float* src, int64_t ld_src, const int32_t* map, int64_t rows_dst,
                                    int32_t cols, int32_t cols_dst, const float* colscale, float* dst, int64_t ld_dst,
                                    void* stream) {
  hipLaunchKernelGGL(pack_rows_kernel<float>, dim3(grid_for(rows_dst * cols_dst)), dim3(256), 0, (hipStream_t)stream,
                     src, ld_src, map, rows_dst, cols, cols_dst, colscale, dst, ld_dst);
  CT_CHECK_LAUNCH();
  return 0;
}

extern "C" int ctclip_unpack_rows(const float* src, int64_t ld_src, const int32_t* map, int64_t rows_src,
                                  int32_t cols, float* dst, int64_t ld_dst, int32_t accumulate, void* stream) {
  hipLaunchKernelGGL(unpack_rows_kernel, dim3(grid_for(rows_src * cols)), dim3(256), 0, (hipStream_t)stream, src,
                     ld_src, map, rows_src, cols, dst, ld_dst, accumulate);
  CT_CHECK_LAUNCH();
  return 0;
}

extern "C" int ctclip_cast_f32_bf16(const float* x, void* y, int64_t n, void* stream) {
  hipLaunchKernelGGL(cast_f32_bf16_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, x, (u16*)y, n);
  CT_CHECK_LAUNCH();
  return 0;
}

extern "C" int ctclip_cast_f32_bf16_split(const float* x, void* hi, void* lo, int64_t n, void* stream) {
  hipLaunchKernelGGL(cast_split_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, x, (u16*)hi, (u16*)lo, n);
  CT_CHECK_LAUNCH();
  return 0;
}

extern "C" int ctclip_add_f32(const float* a, const float* b, float* y, void* yb, int64_t n, void* stream) {
  CT_REQUIRE(n % 4 == 0, CT_EALIGN);
  hipLaunchKernelGGL(add_f32_kernel, dim3(grid_for(n / 4)), dim3(256), 0, (hipStream_t)stream, a, b, y, (u16*)yb,
                     n / 4);
  CT_CHECK_LAUNCH();
  return 0;
}

namespace {
__global__ __launch_bounds__(256) void gelu_f32_kernel(const float* __restrict__ x, float* __restrict__ y, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    y[i] = gelu_erf(x[i]);
}
}  // namespace

extern "C" int ctclip_gelu_f32(const float* x, float* y, int64_t n, void* stream) {
  hipLaunchKernelGGL(gelu_f32_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, x, y, n);
  CT_CHECK_LAUNCH();
  return 0;
}

// Hidden-state dropout of the BERT text tower (transformers BertEmbeddings / BertSelfOutput /
// BertOutput .dropout, p = hidden_dropout_prob in train mode): y = x * keep(seed, i) / (1 - p)
// (+ res), element i kept iff its splitmix64 hash >= p * 2^32.  The backward is the same call on
// the gradient with the same seed (res = null).
namespace {
__global__ __launch_bounds__(256) void dropout_kernel(const float* __restrict__ x, const float* __restrict__ res,
                                                      float* __restrict__ yf, u16* __restrict__ yb, int64_t n4,
                                                      unsigned thresh, float scale, uint64_t seed) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    f32x4 v = ((const f32x4*)x)[i];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] *= hid_keep(seed, 4 * i + j, thresh, scale);
    if (res) v += ((const f32x4*)res)[i];
    if (yf) ((f32x4*)yf)[i] = v;
    if (yb) {
      uint2 w;
      w.x = (unsigned)f2bf(v[0]) | ((unsigned)f2bf(v[1]) << 16);
      w.y = (unsigned)f2bf(v[2]) | ((unsigned)f2bf(v[3]) << 16);
      ((uint2*)yb)[i] = w;
    }
  }
}
}  // namespace

extern "C" int ctclip_dropout(const float* x, const float* res, float* yf, void* yb, int64_t n, float p,
                              uint64_t seed, void* stream) {
  CT_REQUIRE(n % 4 == 0, CT_EALIGN);
  CT_REQUIRE(p >= 0.f && p < 1.f, CT_EINVAL);
  const unsigned thresh = (unsigned)std::min(4294967295.0, (double)p * 4294967296.0);
  hipLaunchKernelGGL(dropout_kernel, dim3(grid_for(n / 4)), dim3(256), 0, (hipStream_t)stream, x, res, yf, (u16*)yb,
                     n / 4, thresh, 1.f / (1.f - p), seed);
  CT_CHECK_LAUNCH();
  return 0;
}
