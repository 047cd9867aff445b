// CT volume preprocessing on the GPU: the step before the contrastive
// path, done per sample on the host in the reference.
//
//   online  (mode 0, ct_clip/data.py:114-192, npz_img_to_tensor): v = slope*x + intercept ->
//           F.interpolate(trilinear, align_corners=False) to int(n * spacing/target) ->
//           clip(-1000, 1000) / 1000 -> centre crop / pad (value -1) to 480 x 480 x 240 ->
//           (1, D, H, W).  The arithmetic type is numpy's: int16 / f64 scans compute in f64 (the
//           f32 result is the f64 value rounded once), f32 scans in f32.
//   offline (mode 1, data_prep/preprocess_train.py:67-104): v = f32(clip(slope*x + intercept,
//           -1000, 1000) / 1000) (f64) -> F.interpolate in f32.  No crop / pad.
//
// Interpolation follows ATen's CPU linear upsampling: per axis src = max(scale*(dst+0.5)-0.5, 0)
// with scale = in/out, i0 = min(floor(src), in-1), l1 = clamp(src-i0, 0, 1), l0 = 1-l1, i1 = i0 +
// (i0 < in-1); out = (f_h(d0) * ld0 + f_h(d1) * ld1), f_h = f_w(h0) * lh0 + f_w(h1) * lh1, f_w =
// x(w0) * lw0 + x(w1) * lw1, in that order with no FMA contraction.
//
// Layout: the source is read through (d, h, w) strides, so the reference's (H, W, D) scan needs
// no transpose.  The kernel is HBM-bound (8 gathered + 1 written values per voxel, mostly L2 hits):
// a workgroup owns a 64 x 64 tile of one output plane.  When the source is contiguous along d
// (the npz (H, W, D) layout) the tile is computed with lanes along d (coalesced gathers) and
// transposed through LDS so the output rows are written along w (coalesced stores).
#include "common.h"
#include "../../include/ctclip_hip.h"

namespace {

struct RP {
  const void* src;
  int sdt;                      // CTCLIP_F32 / CTCLIP_I16 / CTCLIP_F64
  int64_t D, H, W;              // source extents, (d, h, w) view
  int64_t sd, sh, sw;           // source strides (elements)
  int64_t Dn, Hn, Wn;           // resized extents
  int64_t Do, Ho, Wo;           // output extents
  int64_t od, oh, ow;           // output index - resized index
  double slope, intercept;
  int mode;
  float fill;
};

template <typename T>
struct Tap {
  int64_t i0, i1;
  T l0, l1;
};

// ATen compute_source_index_and_lambda (align_corners = False)
template <typename T>
__device__ __forceinline__ Tap<T> tap(int64_t dst, int64_t in, int64_t out) {
#pragma clang fp contract(off)
  Tap<T> t;
  if (in == out) {
    t.i0 = t.i1 = dst;
    t.l0 = (T)1;
    t.l1 = (T)0;
    return t;
  }
  const T scale = (T)in / (T)out;
  T src = scale * ((T)dst + (T)0.5) - (T)0.5;
  if (src < (T)0) src = (T)0;
  const int64_t fl = (int64_t)floor(src);
  t.i0 = fl < in - 1 ? fl : in - 1;
  T l1 = src - (T)t.i0;
  l1 = l1 < (T)0 ? (T)0 : (l1 > (T)1 ? (T)1 : l1);
  t.l1 = l1;
  t.l0 = (T)1 - l1;
  t.i1 = t.i0 + (t.i0 < in - 1 ? 1 : 0);
  return t;
}

// source value after the pre-op, in the interpolation type T
template <typename T>
__device__ __forceinline__ T pre(const RP& p, int64_t idx) {
#pragma clang fp contract(off)
  double x;
  if (p.sdt == CTCLIP_I16) x = (double)((const int16_t*)p.src)[idx];
  else if (p.sdt == CTCLIP_F64) x = ((const double*)p.src)[idx];
  else x = (double)((const float*)p.src)[idx];
  if (p.mode == 1) {
    double v = p.slope * x + p.intercept;
    v = fmin(fmax(v, -1000.0), 1000.0) / 1000.0;
    return (T)(float)v;
  }
  if constexpr (sizeof(T) == 4) {
    // numpy: f32 array * python float -> f32 (the scalar is cast to f32 first), + f32
    const float v = (float)p.slope * (float)x;
    return v + (float)p.intercept;
  } else {
    return p.slope * x + p.intercept;
  }
}

template <typename T>
__device__ __forceinline__ float voxel(const RP& p, int64_t d, int64_t h, int64_t w) {
#pragma clang fp contract(off)
  const int64_t dr = d - p.od, hr = h - p.oh, wr = w - p.ow;
  if (dr < 0 || dr >= p.Dn || hr < 0 || hr >= p.Hn || wr < 0 || wr >= p.Wn) return p.fill;
  const Tap<T> td = tap<T>(dr, p.D, p.Dn), th = tap<T>(hr, p.H, p.Hn), tw = tap<T>(wr, p.W, p.Wn);
  T fd[2];
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    const int64_t di = a ? td.i1 : td.i0;
    T fh[2];
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int64_t base = di * p.sd + (b ? th.i1 : th.i0) * p.sh;
      T o = pre<T>(p, base + tw.i0 * p.sw) * tw.l0;
      o += pre<T>(p, base + tw.i1 * p.sw) * tw.l1;
      fh[b] = o;
    }
    T o = fh[0] * th.l0;
    o += fh[1] * th.l1;
    fd[a] = o;
  }
  T v = fd[0] * td.l0;
  v += fd[1] * td.l1;
  if (p.mode == 1) return (float)v;
  v = v < (T)-1000 ? (T)-1000 : (v > (T)1000 ? (T)1000 : v);
  return (float)(v / (T)1000);
}

constexpr int TILE = 64;

// DFAST: lanes along d in the compute phase (source contiguous along d), LDS transpose before
// the w-contiguous stores; otherwise lanes along w throughout.  grid (Wo/64, Ho, Do/64), 256 thr.
template <typename T, bool DFAST>
__global__ __launch_bounds__(256) void resample_kernel(RP p, float* __restrict__ out) {
  __shared__ float tile[TILE][TILE + 1];
  const int64_t w0 = (int64_t)blockIdx.x * TILE, h = blockIdx.y, d0 = (int64_t)blockIdx.z * TILE;
  const int t = threadIdx.x;
  if constexpr (DFAST) {
#pragma unroll 4
    for (int k = 0; k < TILE / 4; ++k) {
      const int dd = t & 63, ww = (t >> 6) + 4 * k;
      const int64_t d = d0 + dd, w = w0 + ww;
      tile[dd][ww] = (d < p.Do && w < p.Wo) ? voxel<T>(p, d, h, w) : 0.f;
    }
    __syncthreads();
#pragma unroll 4
    for (int k = 0; k < TILE / 4; ++k) {
      const int ww = t & 63, dd = (t >> 6) + 4 * k;
      const int64_t d = d0 + dd, w = w0 + ww;
      if (d < p.Do && w < p.Wo) out[(d * p.Ho + h) * p.Wo + w] = tile[dd][ww];
    }
  } else {
#pragma unroll 4
    for (int k = 0; k < TILE / 4; ++k) {
      const int ww = t & 63, dd = (t >> 6) + 4 * k;
      const int64_t d = d0 + dd, w = w0 + ww;
      if (d < p.Do && w < p.Wo) out[(d * p.Ho + h) * p.Wo + w] = voxel<T>(p, d, h, w);
    }
  }
}

template <typename T>
void launch(const RP& p, float* out, hipStream_t st) {
  dim3 grid((unsigned)((p.Wo + TILE - 1) / TILE), (unsigned)p.Ho, (unsigned)((p.Do + TILE - 1) / TILE));
  if (p.sd < p.sw) hipLaunchKernelGGL((resample_kernel<T, true>), grid, dim3(256), 0, st, p, out);
  else hipLaunchKernelGGL((resample_kernel<T, false>), grid, dim3(256), 0, st, p, out);
}

}  // namespace

extern "C" int ctclip_resample_volume(const ctclip_resample_args* a, float* out, void* stream) {
  CT_REQUIRE(a && a->src && out, CT_EINVAL);
  CT_REQUIRE(a->src_dtype == CTCLIP_F32 || a->src_dtype == CTCLIP_I16 || a->src_dtype == CTCLIP_F64, CT_EINVAL);
  CT_REQUIRE(a->mode == 0 || a->mode == 1, CT_EINVAL);
  CT_REQUIRE(a->D > 0 && a->H > 0 && a->W > 0 && a->Dn > 0 && a->Hn > 0 && a->Wn > 0, CT_ESHAPE);
  CT_REQUIRE(a->Do > 0 && a->Ho > 0 && a->Wo > 0 && a->Ho < 65536 && (a->Do + TILE - 1) / TILE < 65536, CT_ESHAPE);
  RP p;
  p.src = a->src; p.sdt = a->src_dtype;
  p.D = a->D; p.H = a->H; p.W = a->W;
  p.sd = a->sd; p.sh = a->sh; p.sw = a->sw;
  p.Dn = a->Dn; p.Hn = a->Hn; p.Wn = a->Wn;
  p.Do = a->Do; p.Ho = a->Ho; p.Wo = a->Wo;
  p.od = a->od; p.oh = a->oh; p.ow = a->ow;
  p.slope = a->slope; p.intercept = a->intercept;
  p.mode = a->mode; p.fill = a->fill;
  hipStream_t st = (hipStream_t)stream;
  // numpy's arithmetic type: f64 for int16 / f64 scans online; the offline path interpolates f32
  if (a->mode == 0 && a->src_dtype != CTCLIP_F32) launch<double>(p, out, st);
  else launch<float>(p, out, st);
  CT_CHECK_LAUNCH();
  return 0;
}
