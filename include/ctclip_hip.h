/*
 * libctclip_hip.so — C-ABI of the MI355X (gfx950) CT-CLIP contrastive-step kernels.
 *
 * The reference (sharonct/CTPA-CLIP) is pure PyTorch and has no FFI layer: its boundary is
 * the nn.Module API + the state_dict layout.  This header is the
 * kernel-level boundary the build's PyTorch-ROCm host code (ctpa-clip_amd/ctclip_mi355x)
 * binds through ctypes; each entry point names the reference symbol whose arithmetic it
 * replaces (paths relative to CTPA_CLIP/).
 *
 * Conventions
 *   - All tensor pointers are DEVICE pointers owned by the caller; the library never
 *     allocates.  Scratch comes from caller-provided workspaces.
 *   - `stream` is a hipStream_t passed as void*; every call is asynchronous on it.
 *   - bf16 tensors are raw 16-bit bfloat16 (same bits as torch.bfloat16).
 *   - Return 0 on success, a hipError_t value on launch failure, or one of
 *     CT_EINVAL=1001 (bad argument), CT_EALIGN=1002 (pointer / leading-dim not 16-byte
 *     aligned), CT_ESHAPE=1003 (unsupported shape).
 */
#ifndef CTCLIP_HIP_H
#define CTCLIP_HIP_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------- version / probe */
int ctclip_version(void);          /* ABI version */
int ctclip_device_arch(char* buf, int n); /* writes gcnArchName of the current device */

/* ---------------------------------------------------------------- dense GEMM (MFMA)
 * C[m, n] = epilogue( alpha * sum_k A[m, k] * B[k, n] )   bf16 x bf16 -> f32 accumulate.
 * Replaces every nn.Linear of the path: Attention.to_q/to_kv/to_out
 * (ct_clip/attention.py:119-125), FeedForward Linears (attention.py:48,51), to_patch_emb's
 * Linear (ct_clip/ctvit.py:172), to_text_latent / to_visual_latent (ct_clip/ct_clip.py:549,564),
 * the VQ cosine-distance matmul (vector_quantize_pytorch, ctvit.py:427), BERT's Linears
 * (ct_clip/ct_clip.py:685) and all their backward GEMMs.
 *   a_kcontig = 1: A[m*lda + k]   (row-major M x K);   0: A[k*lda + m]  (K x M)
 *   b_kcontig = 1: B[n*ldb + k]   (nn.Linear weight);  0: B[k*ldb + n]  (K x N)
 *   act: 0 none, 1 gelu(erf), 2 geglu (tile-interleaved pairs), 3 argmax
 *   split_k > 1: C is an f32 slab array [split_k][M][ldc] of partial sums (no epilogue).
 */
typedef struct {
  int64_t M, N, K;
  const void* A; int64_t lda; int32_t a_kcontig;
  const void* B; int64_t ldb; int32_t b_kcontig;
  void* C; int64_t ldc; int32_t c_f32;
  void* C2; int64_t ldc2;           /* optional bf16 secondary output (shadow / geglu) */
  const float* bias;                /* optional per-column f32 bias */
  const void* R; int64_t ldr; int32_t r_f32;  /* optional residual added after alpha*acc */
  float alpha;
  int32_t act;
  int32_t accumulate;               /* C (f32) += result */
  int32_t split_k;
  int32_t batch;
  int64_t sA, sB, sC, sC2, sR;      /* batch strides in elements */
} ctclip_gemm_args;
int ctclip_gemm(const ctclip_gemm_args* a, void* stream);

/* sum f32 slabs [s][rows][ld] -> out (f32 or bf16), optional accumulate into f32 out */
int ctclip_reduce_slabs(const float* slabs, int64_t nslab, int64_t rows, int64_t cols, int64_t ld,
                        void* out, int64_t ldo, int32_t out_f32, int32_t accumulate, void* stream);

#ifdef __cplusplus
}
#endif
#endif
