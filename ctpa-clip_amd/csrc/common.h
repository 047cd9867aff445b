// Shared device helpers for the CT-CLIP gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <algorithm>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16;
typedef uint4 u32x4;

#define LDS_PTR(T, p) ((__attribute__((address_space(3))) T*)(p))

// ds_read_b64_tr_b16 through inline asm, for kernels that keep LDS-DMA (global_load_lds) in
// flight across fragment reads: hipcc (ROCm 7.2) puts an s_waitcnt vmcnt(0) in front of every
// intrinsic ds_read_tr while any LDS-DMA is outstanding (it cannot prove they do not alias),
// which drains the load pipeline each phase.  The asm form is invisible to that check AND to the
// compiler's lgkmcnt tracking: the caller must wait (s_waitcnt lgkmcnt) before using the result.
// 16-B LDS-DMA (global_load_lds_dwordx4) through inline asm: wave-uniform LDS base in M0, lane l
// lands at base + 16 l.  Invisible to hipcc's LDS-DMA tracking, so the compiler no longer drains
// the queue (vmcnt(0)) before LDS reads it cannot prove disjoint (every ds_read_b64_tr_b16 of an
// MN-contiguous operand); the kernel's own counted vmcnt waits order the DMA and the reads.  The
// compiler's waits for its own loads stay safe: unseen younger ops only make them stricter.
// M0 is a reserved register: it is saved and restored around the DMA, with the one wait state a
// SALU write of M0 needs before an LDS-DMA reads it.
__device__ __forceinline__ void glds16_asm(const void* g, const void* lds) {
  const unsigned l = __builtin_amdgcn_readfirstlane((unsigned)(size_t)LDS_PTR(char, lds));
  unsigned saved;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(saved)
      : "v"(g), "s"(l)
      : "memory");
}

template <int OFF>
__device__ __forceinline__ s16x4 ds_read_tr16_b64_asm(const void* p) {
  s16x4 r;
  const unsigned a = (unsigned)(size_t)LDS_PTR(char, p);
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(a), "i"(OFF));
  return r;
}

#define CT_CHECK_LAUNCH()                                  \
  do {                                                     \
    hipError_t _e = hipGetLastError();                     \
    if (_e != hipSuccess) return (int)_e;                  \
  } while (0)

#define CT_REQUIRE(cond, code) \
  do {                         \
    if (!(cond)) return (code); \
  } while (0)

// error codes returned by the C-ABI besides hipError_t values
enum { CT_EINVAL = 1001, CT_EALIGN = 1002, CT_ESHAPE = 1003 };

__device__ __forceinline__ float bf2f(u16 v) { return __uint_as_float(((unsigned)v) << 16); }
__device__ __forceinline__ u16 f2bf(float f) {
  bf16 h = (bf16)f;  // v_cvt_pk_bf16_f32, RNE, NaN-preserving
  return __builtin_bit_cast(u16, h);
}
__device__ __forceinline__ void unpack8(const u32x4& v, float* f) {
  const unsigned w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
__device__ __forceinline__ unsigned pack2(float a, float b) {
  return (unsigned)f2bf(a) | ((unsigned)f2bf(b) << 16);
}
__device__ __forceinline__ u32x4 pack8(const float* f) {
  u32x4 r;
  r.x = pack2(f[0], f[1]);
  r.y = pack2(f[2], f[3]);
  r.z = pack2(f[4], f[5]);
  r.w = pack2(f[6], f[7]);
  return r;
}
__device__ __forceinline__ uint2 pack4(const float* f) { return make_uint2(pack2(f[0], f[1]), pack2(f[2], f[3])); }

// IEEE fp16 (the 3D-ViT forward's 16-bit GEMM operands since round 5: 3 more mantissa bits than
// bf16 at the same MFMA rate).  Conversions round to nearest even.
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ u16 f2h(float f) { return __builtin_bit_cast(u16, (_Float16)f); }
__device__ __forceinline__ float h2f(u16 v) { return (float)__builtin_bit_cast(_Float16, v); }
__device__ __forceinline__ float rh(float f) { return (float)(_Float16)f; }   // f rounded to f16
__device__ __forceinline__ unsigned pack2h(float a, float b) { return (unsigned)f2h(a) | ((unsigned)f2h(b) << 16); }
__device__ __forceinline__ u32x4 pack8h(const float* f) {
  return make_uint4(pack2h(f[0], f[1]), pack2h(f[2], f[3]), pack2h(f[4], f[5]), pack2h(f[6], f[7]));
}
__device__ __forceinline__ uint2 pack4h(const float* f) { return make_uint2(pack2h(f[0], f[1]), pack2h(f[2], f[3])); }
__device__ __forceinline__ void unpack8h(const u32x4& v, float* f) {
  const unsigned w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = h2f((u16)(w[i] & 0xffffu));
    f[2 * i + 1] = h2f((u16)(w[i] >> 16));
  }
}
// 16-bit A/B MFMA step: bf16 or fp16 operands (same fragment layout), f32 accumulate
template <bool H16>
__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  if constexpr (H16)
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0,
                                                  0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ void unpack4(const uint2& v, float* f) {
  f[0] = __uint_as_float(v.x << 16);
  f[1] = __uint_as_float(v.x & 0xffff0000u);
  f[2] = __uint_as_float(v.y << 16);
  f[3] = __uint_as_float(v.y & 0xffff0000u);
}

// Branch-free erf (Abramowitz & Stegun 7.1.26, |error| <= 1.5e-7 absolute): one v_rcp, one
// v_exp and five FMAs instead of ocml's two-branch erff, whose divergent lanes pay both branches
// inside the GEGLU / GELU GEMM epilogues.  The error is below bf16 resolution of every output
// it feeds (GEGLU / GELU activations are stored in bf16).
__device__ __forceinline__ float erf_fast(float x) {
  const float a = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, a, 1.0f));
  float y = fmaf(1.061405429f, t, -1.453152027f);
  y = fmaf(y, t, 1.421413741f);
  y = fmaf(y, t, -0.284496736f);
  y = fmaf(y, t, 0.254829592f);
  y *= t;
  const float r = fmaf(-y, __expf(-a * a), 1.0f);
  return copysignf(r, x);
}
#ifdef CTCLIP_DIAG_CHEAP_GELU
// diagnostic A/B build only (tools/gelu_cost_ab.py): WRONG activations, to time what the erf costs
// inside the GEGLU / GELU GEMM epilogues
__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x; }
__device__ __forceinline__ float gelu_erf_grad(float x) { return 0.5f + 0.1f * x; }
__device__ __forceinline__ void gelu_erf_and_grad(float x, float& gelu, float& dgelu) {
  gelu = gelu_erf(x);
  dgelu = gelu_erf_grad(x);
}
#else
__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.0f + erf_fast(x * 0.70710678118654752f)); }
// GELU and its derivative together (the GEGLU backward needs both): one erf, and the pdf's
// exp(-x^2 / 2) is the erf's own exp(-a^2), a = |x| / sqrt 2.  gelu bit-identical to gelu_erf.
__device__ __forceinline__ void gelu_erf_and_grad(float x, float& gelu, float& dgelu) {
  const float a = fabsf(x * 0.70710678118654752f);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, a, 1.0f));
  float y = fmaf(1.061405429f, t, -1.453152027f);
  y = fmaf(y, t, 1.421413741f);
  y = fmaf(y, t, -0.284496736f);
  y = fmaf(y, t, 0.254829592f);
  y *= t;
  const float e = __expf(-a * a);
  const float erf = copysignf(fmaf(-y, e, 1.0f), x);
  gelu = 0.5f * x * (1.0f + erf);
  // (the fma spelled out: left to -ffp-contract, its two possible fusions differ in the last bit
  // between inlining contexts, and the fused / two-kernel GEGLU backward must agree bit for bit)
  dgelu = fmaf(x, 0.39894228040143268f * e, 0.5f * (1.0f + erf));
}
__device__ __forceinline__ float gelu_erf_grad(float x) {   // one exp (gelu_erf_and_grad)
  float ge, dge;
  gelu_erf_and_grad(x, ge, dge);
  return dge;
}
#endif

__device__ __forceinline__ float warp_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float warp_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum of one value per thread (blockDim multiple of 64, <= 1024).
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = warp_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
  for (int i = 0; i < nw; ++i) s += red[i];
  return s;
}

// Step status word (include/ctclip_hip.h CT_STATUS_*): a kernel that detects a condition ORs its
// bit in with ONE vector atomic per wave (the lowest lane that saw it); the word is sticky and the
// trainer turns it into the Adam kernel's skip guard and a host-side exception.
__device__ __forceinline__ void status_or(int* status, int bits, bool bad) {
  const unsigned long long b = __ballot(bad);
  if (status && b && (int)(threadIdx.x & 63) == __ffsll((long long)b) - 1)
    __hip_atomic_fetch_or(status, bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// fp16 range check of a value about to be stored as fp16 (false for NaN / inf / |v| > 65504)
__device__ __forceinline__ bool f16_ok(float v) { return fabsf(v) <= 65504.f; }

static inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }
static inline bool aligned16(const void* p) { return (((uintptr_t)p) & 15) == 0; }

// Hidden-state dropout keep factor of the BERT text tower (ctclip_dropout and the kernels it is
// fused into): element i (flat index of a contiguous [rows][D] tensor) is kept iff the splitmix64
// finaliser of seed ^ i*phi is >= thresh = p * 2^32; returns scale = 1 / (1 - p) or 0.
__device__ __forceinline__ float hid_keep(uint64_t seed, int64_t i, unsigned thresh, float scale) {
  uint64_t x = seed ^ ((uint64_t)i * 0x9E3779B97F4A7C15ull);
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return (unsigned)x >= thresh ? scale : 0.f;
}
