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

}  // namespace

extern "C" int ctclip_peg_fwd(const void* x_bf16, const float* x_f32, int64_t B, int32_t T, int32_t H, int32_t W,
                              int32_t D, const float* weight, const float* bias, int32_t mode, float* out_f32,
                              void* out_bf16, void* stream) {
  CT_REQUIRE(D % 8 == 0, CT_EALIGN);
  Geo g{T, H, W, T * H * W, mode};
  const int64_t ntok = B * g.thw;
  dim3 grid(cdiv(ntok, 32), cdiv(D, 64));
  hipLaunchKernelGGL(peg_kernel<0>, grid, dim3(256), 0, (hipStream_t)stream, (const u16*)x_bf16, ntok, D, weight,
                     bias, x_f32, g, out_f32, (u16*)out_bf16);
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
  dim3 grid(cdiv(ntok, 32), cdiv(D, 64));
  hipLaunchKernelGGL(peg_kernel<1>, grid, dim3(256), 0, (hipStream_t)stream, (const u16*)dout_bf16, ntok, D, weight,
                     (const float*)nullptr, dout_f32, g, dx_f32, (u16*)dx_bf16);
  CT_CHECK_LAUNCH();
  return 0;
}

// part: [nblk][D][28] f32 partials (27 taps in (kt,kh,kw) order, then bias)
extern "C" int ctclip_peg_bwd_weight(const void* dout_bf16, const void* x_bf16, int64_t B, int32_t T, int32_t H,
                                     int32_t W, int32_t D, int32_t mode, float* part, int32_t nblk, void* stream) {
  CT_REQUIRE(D % 8 == 0, CT_EALIGN);
  Geo g{T, H, W, T * H * W, mode};
  const int64_t ntok = B * g.thw;
  const int64_t per = (ntok + nblk - 1) / nblk;
  dim3 grid(nblk, cdiv(D, 64));
  hipLaunchKernelGGL(peg_wgrad_kernel, grid, dim3(192), 0, (hipStream_t)stream, (const u16*)dout_bf16,
                     (const u16*)x_bf16, ntok, D, g, per, part);
  CT_CHECK_LAUNCH();
  return 0;
}
