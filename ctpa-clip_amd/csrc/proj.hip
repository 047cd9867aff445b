// Skinny-M HBM-streaming GEMM for CT-CLIP's image projection ``to_visual_latent``
// (ct_clip/ct_clip.py:564 Linear(294,912 -> 512, no bias), applied at :767 to the pooled image
// tokens): C[m][n] = sum_k A[m][k] B[n][k] with M = the local batch (<= 16 rows), N = 512, K =
// 294,912.  The 302 MB bf16 weight B is the whole cost, so the kernel is a pure HBM stream: every
// workgroup owns a [64 n x ks k] block of B and moves it straight from HBM into MFMA registers once
// (no LDS on the way), with the batch rows of A as the 16-column B operand of
// v_mfma_f32_16x16x32_bf16 (columns >= M zero).
//   * wave w of the workgroup takes the w-th quarter of the k-slice for all 64 rows (four 16-row
//     MFMA groups), so A's fragment is loaded once per wave and k-step (lanes of rows >= M load
//     nothing);
//   * lane l reads 32 consecutive bytes of row (l & 15) of each group at k + 16 (l >> 4): the four
//     lanes of a row cover one 128-B line per k-step; A's fragment takes the same k permutation, so
//     the products summed are exactly the natural order's;
//   * two k-steps in flight per wave (registers double-buffered, the loop unrolled by two so the
//     compiler's vmcnt waits retire only the older step);
//   * the four waves' partial tiles are summed through LDS in wave order, one f32 slab per k-slice
//     [S][M][N] (a caller workspace), reduced in a fixed order by ctclip_reduce_slabs: deterministic.
// Grid: N / 64 row blocks x S k-slices (512 workgroups at the base shape, two per CU); the 8 row
// blocks of a k-slice run on one XCD (workgroup i -> XCD i % 8) so its A slice comes from HBM once.
#include "common.h"
#include "../../include/ctclip_hip.h"

namespace {

// Round 6: templated on the element type.  bf16: a lane's 32 bytes are 16 k, one
// v_mfma_f32_16x16x32_bf16 per half; f32 (the precise towers' projection, ctclip_skinny_sgemm): 8 k,
// four v_mfma_f32_16x16x4_f32 per half (lane group q's k = 8 q + 4 h + j, A read in the same order).
template <bool F32> struct Elt;
template <> struct Elt<false> { using T = u16; static constexpr int E = 16; };
template <> struct Elt<true> { using T = float; static constexpr int E = 8; };
template <bool F32> constexpr int kstep() { return 4 * Elt<F32>::E; }   // k per wave step: 4 lane groups
constexpr int NG = 4;       // 16-row MFMA groups per workgroup (64 rows)

struct Step {
  u32x4 w[NG][2];
  u32x4 a[2];
};

template <bool F32>
__device__ __forceinline__ void load_step(Step& s, const typename Elt<F32>::T* __restrict__ bp, int64_t ldb16,
                                          const typename Elt<F32>::T* __restrict__ ap, bool arow, int64_t o) {
  constexpr int HALF = Elt<F32>::E / 2;
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    s.w[g][0] = *(const u32x4*)(bp + g * ldb16 + o);
    s.w[g][1] = *(const u32x4*)(bp + g * ldb16 + o + HALF);
  }
  if (arow) {
    s.a[0] = *(const u32x4*)(ap + o);
    s.a[1] = *(const u32x4*)(ap + o + HALF);
  } else {
    s.a[0] = s.a[1] = u32x4{0u, 0u, 0u, 0u};
  }
}

template <bool F32>
__device__ __forceinline__ void mma_step(f32x4 (&acc)[NG], const Step& s) {
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      if constexpr (F32) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(__builtin_bit_cast(float, s.w[g][h][j]),
                                                        __builtin_bit_cast(float, s.a[h][j]), acc[g], 0, 0, 0);
      } else {
        acc[g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, s.w[g][h]),
                                                         __builtin_bit_cast(bf16x8, s.a[h]), acc[g], 0, 0, 0);
      }
    }
}

template <bool F32>
__global__ __launch_bounds__(256) void skinny_gemm_kernel(const typename Elt<F32>::T* __restrict__ A, int64_t lda,
                                                          int M, const typename Elt<F32>::T* __restrict__ B,
                                                          int64_t ldb, int nblk, int64_t ks, float* __restrict__ slabs,
                                                          int N, int S) {
  using T = typename Elt<F32>::T;
  constexpr int KSTEP = kstep<F32>();
  __shared__ f32x4 red[3][NG][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i = blockIdx.x;
  int s, nb;
  if (nblk == 8 && S % 8 == 0) {   // XCD-aware: workgroup i runs on XCD i % 8
    const int xcd = i & 7, j = i >> 3;
    s = (j >> 3) * 8 + xcd;
    nb = j & 7;
  } else {
    s = i / nblk;
    nb = i - s * nblk;
  }
  const int r = lane & 15, q = lane >> 4;
  const int64_t kq = ks / 4;                       // this wave's quarter of the slice
  const int64_t k0 = (int64_t)s * ks + w * kq;
  const T* bp = B + (int64_t)(nb * 64 + r) * ldb + k0 + q * Elt<F32>::E;
  const bool arow = r < M;
  const T* ap = A + (int64_t)(arow ? r : 0) * lda + k0 + q * Elt<F32>::E;
  const int64_t ldb16 = 16 * ldb;
  f32x4 acc[NG];
#pragma unroll
  for (int g = 0; g < NG; ++g) acc[g] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nsteps = (int)(kq / KSTEP);
  Step s0, s1;
  load_step<F32>(s0, bp, ldb16, ap, arow, 0);
  int t = 0;
  for (; t + 2 <= nsteps; t += 2) {
    load_step<F32>(s1, bp, ldb16, ap, arow, (int64_t)(t + 1) * KSTEP);
    mma_step<F32>(acc, s0);
    // the step after next, clamped to the last one (re-read, unused) so no branch merges s0
    load_step<F32>(s0, bp, ldb16, ap, arow, (int64_t)min(t + 2, nsteps - 1) * KSTEP);
    mma_step<F32>(acc, s1);
  }
  if (t < nsteps) mma_step<F32>(acc, s0);   // odd step count: s0 holds step nsteps - 1
  // acc[g][v] = C[n = nb*64 + 16g + 4q + v][m = r], this wave's k-quarter; waves 1..3 hand theirs to
  // wave 0 through LDS, which adds them in wave order
  if (w > 0) {
#pragma unroll
    for (int g = 0; g < NG; ++g) red[w - 1][g][lane] = acc[g];
  }
  __syncthreads();
  if (w == 0 && r < M) {
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      f32x4 v = acc[g];
#pragma unroll
      for (int u = 0; u < 3; ++u) v += red[u][g][lane];
      *(f32x4*)(slabs + ((int64_t)s * M + r) * N + nb * 64 + g * 16 + 4 * q) = v;
    }
  }
}

// k-slices: as many as give ~512 workgroups, each slice a multiple of 4 KSTEP (one per wave) dividing K
int pick_slices(int64_t K, int nblk, int kst) {
  const int want = std::max(1, 512 / nblk);
  for (int s = want; s >= 1; --s)
    if (K % ((int64_t)s * 4 * kst) == 0) return s;
  return 0;
}

template <bool F32>
int skinny_slices(int64_t M, int64_t N, int64_t K) {
  constexpr int KSTEP = kstep<F32>();
  if (M < 1 || M > 16 || N % 64 != 0 || N <= 0 || K <= 0 || K % (4 * KSTEP) != 0) return 0;
  return pick_slices(K, (int)(N / 64), KSTEP);
}

template <bool F32>
int skinny_launch(const void* A, int64_t lda, const void* B, int64_t ldb, int64_t M, int64_t N, int64_t K,
                  float* slabs, int32_t nslices, void* stream) {
  using T = typename Elt<F32>::T;
  constexpr int KSTEP = kstep<F32>();
  if (M == 0 || N == 0) return 0;
  CT_REQUIRE(M >= 1 && M <= 16 && N % 64 == 0 && K % (4 * KSTEP) == 0, CT_ESHAPE);
  CT_REQUIRE(nslices == skinny_slices<F32>(M, N, K) && nslices > 0, CT_EINVAL);
  constexpr int VEC = 16 / sizeof(T);
  CT_REQUIRE(aligned16(A) && aligned16(B) && aligned16(slabs) && lda % VEC == 0 && ldb % VEC == 0, CT_EALIGN);
  const int nblk = (int)(N / 64);
  hipLaunchKernelGGL(skinny_gemm_kernel<F32>, dim3(nblk * nslices), dim3(256), 0, (hipStream_t)stream, (const T*)A,
                     lda, (int)M, (const T*)B, ldb, nblk, K / nslices, slabs, (int)N, nslices);
  CT_CHECK_LAUNCH();
  return 0;
}

}  // namespace

extern "C" int ctclip_skinny_gemm_slices(int64_t M, int64_t N, int64_t K) { return skinny_slices<false>(M, N, K); }

extern "C" int ctclip_skinny_gemm(const void* A, int64_t lda, const void* B, int64_t ldb, int64_t M, int64_t N,
                                  int64_t K, float* slabs, int32_t nslices, void* stream) {
  return skinny_launch<false>(A, lda, B, ldb, M, N, K, slabs, nslices, stream);
}

extern "C" int ctclip_skinny_sgemm_slices(int64_t M, int64_t N, int64_t K) { return skinny_slices<true>(M, N, K); }

extern "C" int ctclip_skinny_sgemm(const float* A, int64_t lda, const float* B, int64_t ldb, int64_t M, int64_t N,
                                   int64_t K, float* slabs, int32_t nslices, void* stream) {
  return skinny_launch<true>(A, lda, B, ldb, M, N, K, slabs, nslices, stream);
}
