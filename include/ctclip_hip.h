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
/* ABI version: bumped whenever a public struct changes layout (round 6: 2 -- ctclip_gemm_args gained
 * A_lo / B_lo / C3 / C4, and the round-5 trailing fields ab_f16 / r_f16, ctclip_ln_epilogue.Y16,
 * ctclip_attn_args.o16 now count as part of version 2).  A binding must check ctclip_version() ==
 * CTCLIP_ABI_VERSION before passing any struct: a binding built against an older header passes a
 * shorter struct, and the library would read its missing trailing fields from the caller's stack. */
#define CTCLIP_ABI_VERSION 2
/* Bits of the step status word (an int32 the caller owns; sticky, never cleared by the library):
 * the kernels that take a `status` pointer OR their bit in when they see the condition.  The
 * trainer sums the ranks' words with the last gradient bucket and passes the result to ctclip_adam
 * as its skip guard, so a step with any bit set is applied by no rank, then raises on the host. */
#define CT_STATUS_LN_TIMEOUT 1       /* a LayerNorm-fused GEMM's partner statistics never arrived */
#define CT_STATUS_F16_RANGE 2        /* a value stored as fp16 was non-finite or beyond +-65504 */
#define CT_STATUS_NONFINITE_GRAD 4   /* the gradient norm (ctclip_grad_norm) is not finite */
#define CT_STATUS_VQ_NONFINITE 8     /* a VQ token had no finite codebook score */
int ctclip_version(void);          /* returns CTCLIP_ABI_VERSION */
int ctclip_device_arch(char* buf, int n); /* writes gcnArchName of the current device */
/* test knob: nwg workgroups, each holding lds_bytes of a CU's LDS, spin for `cycles` shader clocks on
 * `stream` (a stand-in for resident RCCL kernels occupying CUs beside a persistent GEMM) */
int ctclip_debug_hold_cus(int32_t nwg, int64_t cycles, int32_t lds_bytes, void* stream);

/* ---------------------------------------------------------------- dense GEMM (MFMA)
 * C[m, n] = epilogue( alpha * sum_k A[m, k] * B[k, n] )   bf16 x bf16 -> f32 accumulate.
 * Replaces every nn.Linear of the path: Attention.to_q/to_kv/to_out
 * (ct_clip/attention.py:119-125), FeedForward Linears (attention.py:48,51), to_patch_emb's
 * Linear (ct_clip/ctvit.py:172), to_text_latent / to_visual_latent (ct_clip/ct_clip.py:549,564),
 * the VQ cosine-distance matmul (vector_quantize_pytorch, ctvit.py:427), BERT's Linears
 * (ct_clip/ct_clip.py:685) and all their backward GEMMs.
 *   a_kcontig = 1: A[m*lda + k]   (row-major M x K);   0: A[k*lda + m]  (K x M)
 *   b_kcontig = 1: B[n*ldb + k]   (nn.Linear weight);  0: B[k*ldb + n]  (K x N)
 *   act: 0 none, 1 gelu(erf), 2 geglu (tile-interleaved pairs), 3 argmax,
 *        4 geglu backward: acc = dg (N = g-space columns, N % 32 == 0), R = h (bf16, the
 *          act-2 pre-activation), C = dh (bf16, h's layout) — replaces dg + geglu_bwd,
 *        5 l2norm: C = bf16 result (N % 64 == 0), C2[:, :n2] = per 32-column head
 *          l2norm(C) * bias[c % 32] (Attention's l2norm(q) * q_scale, attention.py:152-154;
 *          bias = the [32] scale) — replaces a GEMM + ctclip_l2norm_scale_fwd
 *        6 GELU backward: C = acc * gelu'(R) with R the bf16 pre-activation (act 1's C2; no
 *          bias / C2 / split-K / accumulate) — replaces a dX GEMM + ctclip_gelu_bwd (BERT's
 *          intermediate dense, ct_clip/ct_clip.py:685)
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
  int32_t n2;                       /* act 5: normalised columns (multiple of 64, <= N) */
  const void* B2;                   /* optional: a second B with B's layout / ldb / sB, summed in:
                                     * C = epilogue(alpha * (A.B + A.B2)).  With B = bf16(W) and
                                     * B2 = bf16(W - bf16(W)) the GEMM sees W to ~16 mantissa bits
                                     * (the text tower's hi / lo split weights); 128-tile kernel only,
                                     * not with act 3 */
  int32_t ab_f16;                   /* A and B are IEEE fp16 (both K-contiguous; no B2, split-K,
                                     * act 4-6): the 3D-ViT forward GEMMs and (round 6) the act-3
                                     * VQ distance GEMM (3 more mantissa bits
                                     * than bf16 at the same MFMA rate).  With act 2 the h output
                                     * C is fp16 in the DERIVATIVE form (round 6): per 64-column
                                     * group [gelu(gate) | x gelu'(gate)] instead of [x | gate], the
                                     * two factors act 4 multiplies dg by; g from the f32 values */
  int32_t r_f16;                    /* act 4: R (h) is fp16 in that derivative form (written by an
                                     * ab_f16 act-2 GEMM): dh = [dg gelu(gate) | dg x gelu'(gate)]
                                     * by two multiplies */
  /* split-fp16 "x3" operands (round 6, ab_f16 required; K % 64 == 0, both K-contiguous, no bias-free
   * restrictions beyond act 0 / 2): A_lo / B_lo are the fp16 residual images of A / B (same ld), e.g.
   * A = fp16(x), A_lo = fp16(x - A), so the GEMM reads x to ~22 mantissa bits; every K-step runs
   * A.B + A.B_lo + A_lo.B into one f32 accumulator (3x the fp16 MFMA work) -- the f32-equivalent
   * image-tower forward of precise.set_vit_precision('split').  act 0: C f32 (c_f32 = 1) with
   * optional bias, f32 residual R and bf16 copy C2.  act 2 (GEGLU): C = h (fp16), g = gelu(gate) x
   * from the unrounded f32 h written as the fp16 pair C2 (hi, ldc2) / C3 (lo, ldc3) and, when C4 is
   * given, as bf16 C4 (ldc4).  Both NULL: an ordinary GEMM. */
  const void* A_lo;
  const void* B_lo;
  void* C3; int64_t ldc3;
  void* C4; int64_t ldc4;
} ctclip_gemm_args;
int ctclip_gemm(const ctclip_gemm_args* a, void* stream);
/* diagnostic: large-tile kernel variant (8 = 8-phase 256x256x64 default, 1 = 128x256x32,
 * 2 = 256x256x32); returns the previous one.  Every variant computes bit-identical results. */
int ctclip_gemm_set_variant(int variant);
/* diagnostic: start stagger of the 8-phase kernel (units of ~2k cycles); returns the previous */
int ctclip_gemm_set_stagger(int units);
/* A/B switch: the 8-phase kernel's transposed bf16 / GEGLU epilogues store through a wave-private
 * LDS scratch so consecutive lanes write consecutive 16 B of a row (1; 2 = the same with sc1
 * stores, which drop their lines from the XCD's L2) or straight from the transposed accumulator
 * layout (0, default; 3 = those direct stores with sc1); returns the previous setting.  Results
 * are identical. */
int ctclip_gemm_set_epi_lds(int on);
/* diagnostic: 8-phase kernel as persistent workgroups walking the tile sequence (1, default) or
 * one workgroup per tile (0); returns the previous setting.  Results are identical. */
int ctclip_gemm_set_persist(int on);
/* 8-phase persistent grid cap (workgroups) for the launches that follow; 0 = one per CU (default).
 * Two GEMMs on two streams, each capped, share the chip.  Returns the previous cap. */
int ctclip_gemm_set_grid_cap(int workgroups);

/* BERT hidden dropout (hidden_dropout_prob, train mode) fused into its neighbours, same mask as
 * ctclip_dropout (element i of a contiguous [rows][cols] tensor kept iff splitmix64(seed ^ i phi)
 * >= p 2^32, kept values scaled by 1 / (1 - p)):
 *  - split-K combine of the dense output: C = dropout(sum_z slabs[z] + bias) + R (act 0, ldc = cols)
 *    -- BertSelfOutput / BertOutput's dense -> dropout -> + input, ahead of their LayerNorm;
 *  - LayerNorm backward: dx_f32 = LN'(dy) (to the residual branch), dx_bf16 = bf16(dropout(dx))
 *    (to the dense branch), part_drop [nblocks][D] (optional) the column partials of dx_bf16
 *    (the dense bias gradient); dy, x f32, D in (512, 1024]. */
int ctclip_reduce_slabs_ep_drop(const float* slabs, int64_t nslab, int64_t rows, int64_t cols, int64_t ld,
                                const ctclip_gemm_args* ep, float p, uint64_t seed, void* stream);
int ctclip_layernorm_bwd_drop(const void* dy, int32_t dy_f32, int64_t lddy, const void* x, int32_t x_f32, int64_t ldx,
                              const float* mean, const float* rstd, const float* gamma, int64_t rows, int32_t D,
                              float* dx_f32, int64_t lddxf, void* dx_bf16, int64_t lddxb, float* part_gamma,
                              float* part_beta, float* part_drop, int32_t nblocks, float p, uint64_t seed,
                              void* stream);

/* LayerNorm fused into the epilogue of an N = 512 GEMM (the 3D-ViT's d = 512 token rows).  The
 * two 256-column tiles of a row block exchange per-row partial statistics inside the launch.
 * a: the GEMM (A K-contiguous, alpha, C f32 [M][512], optional bf16 copy C2, optional f32
 * residual R, optional bias in mode 1); act 0, no split-K / batch / accumulate / B2.
 *   mode 1, forward (replaces Linear + residual + LayerNorm: the to_out / FeedForward residual of
 *     ct_clip/attention.py:324-326 feeding the next LayerNorm, attention.py:28-35,47):
 *       C = alpha A.B (+ bias) + R;  Y = (C - mean) * rstd * gamma (+ beta) in bf16;
 *       mean / rstd [M] written (f32, eps as given).
 *   mode 2, backward (replaces the dX GEMM + ctclip_layernorm_bwd): dy = bf16(alpha A.B) is the
 *       gradient of LN(X) (X bf16, mean / rstd from the forward); C = LN'(dy) + R, C2 = bf16(C)
 *       (R and C2 required); part_gamma (required) / part_beta (optional) [M / 128][512]: per
 *       128-row block column sums of
 *       dy * xhat and dy (reduce with ctclip_reduce_slabs).  beta must be NULL.
 * Requires M % 2048 == 0, N == 512, K % 64 == 0, the default 8-phase persistent GEMM (no grid cap);
 * otherwise CT_EINVAL / CT_ESHAPE and nothing runs (call the two kernels instead).
 * xchg: >= 4 * M u64 words, zeroed once when allocated; epoch: nonzero and different from every
 * earlier launch on that buffer; launches sharing one xchg buffer must be stream-ordered.
 * status (optional): set to 1 if a partner tile's statistics never arrived (bounded wait: spin_limit
 * polls, 0 = the default ~0.1 s); the outputs of that launch are then wrong.  The status word is
 * sticky (never cleared by the library): the trainer passes it to ctclip_adam as its skip guard, so a
 * step with a timed-out exchange is never applied, and checks it on the host once per step
 * (ctclip_mi355x.trainer: the step raises).  debug != 0 (tests only): the second tile of row block 0
 * never publishes, so its partner times out. */
typedef struct {
  int32_t mode;
  const float* gamma; const float* beta; float eps;
  void* Y; int64_t ldy;
  float* mean; float* rstd;
  const void* X; int64_t ldx;
  float* part_gamma; float* part_beta;
  void* xchg; uint32_t epoch;
  int32_t* status;
  uint32_t spin_limit;
  int32_t debug;
  void* Y16;                        /* mode 1, optional: an fp16 copy of Y (same ldy) -- the next
                                     * fp16 GEMM's A operand */
} ctclip_ln_epilogue;
int ctclip_gemm_ln(const ctclip_gemm_args* a, const ctclip_ln_epilogue* ln, void* stream);

/* Q | K | V projections of one transformer layer as ONE GEMM over the raw residual rows x, with
 * the attention's pre-norm LayerNorm (bias-free, gamma) folded into the Q columns
 * (ct_clip/attention.py:139-141 norm -> to_q; 119-125 to_q / to_kv; 152-154 l2norm * scale):
 *   B = [gamma o Wq ; Wkv] bf16 K-contiguous (ctclip_pack_qkv_fold), N % 256 == 0;
 *   C (bf16 [M][N]) columns < nfold: rstd[m] * (x_m . B_n - mean[m] * fold_cs[n]) = LN(x) Wq^T,
 *   the rest x . B_n; C2 (bf16 [M][n2]) = per 32-column head l2norm(C) * scale, scale = bias[0:32]
 *   for columns < nfold (q_scale) and bias[32:64] after them (k_scale); act must be 5, A / B
 *   K-contiguous, nfold % 256 == 0, nfold < n2 <= N, no R / split-K / batch / accumulate / B2.
 * mean / rstd: the LayerNorm statistics of x (ctclip_ln_stats_merge).  Replaces ctclip_layernorm_fwd
 * + two act-5 GEMMs. */
int ctclip_gemm_qkv_lnfold(const ctclip_gemm_args* a, const float* mean, const float* rstd, const float* fold_cs,
                           int32_t nfold, void* stream);
/* ... storing only the C columns >= c_col0 (a multiple of 64; the l2norm'd C2 is written in full): the
 * eval forward keeps V and drops the raw q / k, which only the backward reads (round 6) */
int ctclip_gemm_qkv_lnfold2(const ctclip_gemm_args* a, const float* mean, const float* rstd, const float* fold_cs,
                            int32_t nfold, int32_t c_col0, void* stream);
/* B operand of ctclip_gemm_qkv_lnfold: out rows [0, nq) = bf16(Wq o gamma) (Wq f32 [nq][K]), rows
 * [nq, nq + nrest) = the bf16 rows of Wrest; cs [nq] = row sums of the bf16 folded rows (f32);
 * s_out (optional) [2 ns] = s_fold ++ s_rest (the epilogue's two l2norm scales). */
int ctclip_pack_qkv_fold(const float* Wq, int64_t ldq, const float* gamma, int64_t nq, int64_t K,
                         const void* Wrest, int64_t ldr, int64_t nrest, void* out, int64_t ldo, float* cs,
                         const float* s_fold, const float* s_rest, int32_t ns, float* s_out, void* stream);
/* fp16 B operand of the fp16 ctclip_gemm_qkv_lnfold (ab_f16): rows [0, nq) = f16(Wq o gamma), cs [nq] =
 * their row sums (of the f16 values), rows [nq, nq + nrest) = f16 of the f32 rows of Wrest */
int ctclip_pack_qkv_fold_h16(const float* Wq, int64_t ldq, const float* gamma, int64_t nq, int64_t K,
                             const float* Wrest, int64_t ldr, int64_t nrest, void* out, int64_t ldo, float* cs,
                             void* stream);
/* LayerNorm statistics from ngroups partial (mean, M2) groups of D / ngroups columns each
 * (part [ngroups][rows] float2, e.g. ctclip_peg_fwd_stats): mean, rstd = 1 / sqrt(var + eps). */
int ctclip_ln_stats_merge(const float* part, int32_t ngroups, int64_t rows, int32_t D, float eps, float* mean,
                          float* rstd, void* stream);
/* Backward of ctclip_gemm_qkv_lnfold's layer input: with A = [dq o rstd | dk | dv] (bf16, K-contiguous)
 * and B = the forward's packed [gamma o Wq ; Wkv] read as [K][N] (b_kcontig = 0),
 *   C (f32) = A B + R - c1[m] - beta[m] X[m][n]  (= LN'(dq Wq) + dkv Wkv + R),  C2 = bf16(C) if given;
 * X = the LayerNorm's bf16 input, c1 / beta from ctclip_l2norm_scale_bwd_fold.  act 0, R f32 required,
 * no bias / split-K / batch / accumulate / B2.  Replaces two dX GEMMs and ctclip_layernorm_bwd. */
int ctclip_gemm_lnfold_bwd(const ctclip_gemm_args* a, const void* X, int64_t ldx, const float* c1, const float* beta,
                           void* stream);
/* Weight gradients of the fold from G = [dq o rstd | dkv]^T X ([nq + nrest][K] f32) and
 * u = (dq o rstd)^T mean (ctclip_l2norm_scale_bwd_fold):
 *   grad_q[n][k] += gamma[k] (G[n][k] - u[n])            (n < nq: dWq = dq^T LN(X))
 *   grad_gamma[k] += sum_n Wq[n][k] (G[n][k] - u[n])    (optional: the LayerNorm gamma gradient)
 *   grad_rest[n - nq][k] += G[n][k]                     (n >= nq: dWkv = dkv^T X) */
int ctclip_lnfold_wgrad(const float* G, int64_t ldg, const float* u, const float* gamma, const float* Wq, int64_t ldw,
                        int64_t nq, int64_t nrest, int64_t K, float* grad_q, int64_t ldgq, float* grad_gamma,
                        float* grad_rest, int64_t ldgr, void* stream);

/* Skinny-M streaming GEMM: slabs[s][m][n] = sum over k-slice s of A[m][k] B[n][k], A [M][K] and B
 * [N][K] bf16 K-contiguous, 1 <= M <= 16, N % 64 == 0, K % 64 == 0; nslices must equal
 * ctclip_skinny_gemm_slices(M, N, K) (> 0); reduce the [nslices][M][N] f32 workspace with
 * ctclip_reduce_slabs.  The forward of CTCLIP's image projection to_visual_latent
 * (ct_clip/ct_clip.py:564,767: Linear(294,912 -> 512) on the pooled tokens of the local batch),
 * which streams its 302 MB bf16 weight once per step. */
int ctclip_skinny_gemm_slices(int64_t M, int64_t N, int64_t K);
int ctclip_skinny_gemm(const void* A, int64_t lda, const void* B, int64_t ldb, int64_t M, int64_t N, int64_t K,
                       float* slabs, int32_t nslices, void* stream);
/* Round 6: the f32 twin (A, B f32, K % 128 == 0, lda / ldb % 4 == 0; v_mfma_f32_16x16x4_f32, an f32
 * fma per product) for the precise image towers' projection: the 604 MB f32 weight streamed once. */
int ctclip_skinny_sgemm_slices(int64_t M, int64_t N, int64_t K);
int ctclip_skinny_sgemm(const float* A, int64_t lda, const float* B, int64_t ldb, int64_t M, int64_t N, int64_t K,
                        float* slabs, int32_t nslices, void* stream);
/* split-K slab reduction into a row-mapped, column-cropped f32 destination: dst[map[r]][c] (+)=
 * sum_z slabs[z][r][c] for c < cols <= ld (rows with map[r] < 0 dropped; map NULL = identity).
 * Bit-identical to ctclip_reduce_slabs into a temporary followed by ctclip_unpack_rows (the packed
 * GEGLU W1 / padded W2 weight gradients of attention.py:44-52). */
int ctclip_reduce_slabs_rows(const float* slabs, int64_t nslab, int64_t rows, int64_t cols, int64_t ld,
                             const int32_t* map, float* dst, int64_t ldd, int32_t accumulate, void* stream);
/* sum f32 slabs [s][rows][ld] -> out (f32 or bf16), optional accumulate into f32 out */
int ctclip_reduce_slabs(const float* slabs, int64_t nslab, int64_t rows, int64_t cols, int64_t ld,
                        void* out, int64_t ldo, int32_t out_f32, int32_t accumulate, void* stream);
/* batched [nslab][1][cols] -> [1][cols] f32 reductions (parameter-gradient partials of the LN /
 * l2norm / bias backward kernels), many jobs per launch: the host defers them to the end of the
 * backward pass or the gradient bucket's all-reduce (kernels.py) instead of one launch each.
 * Same summation order as ctclip_reduce_slabs' skinny path (bit-identical results). */
typedef struct {
  const float* slabs;  /* [nslab][cols] */
  int64_t nslab, cols; /* cols % 4 == 0 */
  float* out;          /* [cols] */
  int32_t accumulate, pad;
} ctclip_slab_job;
int ctclip_reduce_slabs_multi(const ctclip_slab_job* jobs, int32_t njobs, void* stream);
/* split-K combine with the GEMM epilogue of `ep` (C, ldc, c_f32, C2, ldc2, bias, R, ldr, r_f32,
 * act in {0, 1}, accumulate; M/N/K/A/B ignored): C = epilogue(sum_z slabs[z][rows][ld]) */
int ctclip_reduce_slabs_ep(const float* slabs, int64_t nslab, int64_t rows, int64_t cols, int64_t ld,
                           const ctclip_gemm_args* ep, void* stream);


/* ---------------------------------------------------------------- MX-fp8 GEMM (configs[3])
 * SURVEY §8(d) configs[3]: "fp8 attention and MLP GEMMs".  Replaces the fp32 nn.Linear calls of
 * ct_clip/attention.py:44-52 (FeedForward) and :88-181 (to_q / to_kv / to_out) for that config;
 * compared to the build's own bf16 path.  OCP MX: e4m3 elements, one e8m0 scale
 * per 32 consecutive k.
 * quant: x [rows][K] (bf16, or f32 if x_f32) -> q [rows][Kp] e4m3 (ldq bytes, 16-B aligned),
 *   scales [rows][Kp/32] (X + 127 with X = floor(log2 amax) - 8); k in [K, Kp) zero; Kp % 128 == 0.
 * gemm: C[M][N] = alpha * (A . B^T) (+ bias[N]) (+ R) in bf16 (or f32 if c_f32), optional bf16
 *   copy C2; or act 2: GEGLU (C = h bf16, C2 = g [M][N/2]); A [M][Kp], B [N][Kp] e4m3 with their
 *   scale planes.  Errors: CT_ESHAPE / CT_EALIGN / CT_EINVAL. */
typedef struct {
  int64_t M, N, Kp;
  const void* A; int64_t lda; const void* sA;   /* lda, ldb in bytes */
  const void* B; int64_t ldb; const void* sB;
  void* C; int64_t ldc; int32_t c_f32;
  const float* bias; float alpha;
  const float* R; int64_t ldr;   /* f32 residual added after the bias (or NULL) */
  void* C2; int64_t ldc2;        /* act 0: bf16 copy of C (or NULL); act 2: GEGLU output g (bf16) */
  int32_t act;                   /* 0 none; 2 GEGLU over 32-column [x | gate] pairs, C = h (bf16) */
} ctclip_mx_gemm_args;
int ctclip_quant_mxfp8(const void* x, int32_t x_f32, int64_t rows, int64_t K, int64_t ldx, void* q, int64_t ldq,
                       void* scales, int64_t Kp, void* stream);
int ctclip_gemm_mxfp8(const ctclip_mx_gemm_args* a, void* stream);
/* diagnostic: force the 128- or 256-row tile kernel (0 = auto); returns the previous setting.
 * Both compute identical results. */
int ctclip_gemm_mxfp8_set_tile(int bm);

/* ---------------------------------------------------------------- LayerNorm family
 * ct_clip/attention.py:28-35 (bias-less LayerNorm: gamma, beta = 0 buffer, eps 1e-5),
 * nn.LayerNorm in FeedForward / to_patch_emb (attention.py:47, ctvit.py:171,173), BERT LayerNorms.
 * x, y row-major with leading dims; f32 statistics; y in bf16 and/or f32.  D % 8 == 0. */
/* ctclip_layernorm_fwd plus an optional fp16 copy y_f16 of the output (stride ldyb): the A operand of
 * the fp16 FeedForward GEMM (round 5) */
int ctclip_layernorm_fwd_x2(const void* x, int32_t x_f32, int64_t ldx, int64_t rows, int32_t D, const float* gamma,
                            const float* beta, float eps, void* y_bf16, void* y_f16, int64_t ldyb, float* y_f32,
                            int64_t ldyf, float* mean, float* rstd, void* stream);
/* ... with, beside y_f16, its lo residual y_f16lo = fp16(y - y_f16) (the split-fp16 x3 GEMM's A pair,
 * round 6; y_f16 required) and the fp16 range check: an fp16 output beyond +-65504 or non-finite
 * sets CT_STATUS_F16_RANGE in *status (optional) */
int ctclip_layernorm_fwd_x3(const void* x, int32_t x_f32, int64_t ldx, int64_t rows, int32_t D, const float* gamma,
                            const float* beta, float eps, void* y_bf16, void* y_f16, void* y_f16lo, int64_t ldyb,
                            float* y_f32, int64_t ldyf, float* mean, float* rstd, int32_t* status, void* stream);
int ctclip_layernorm_fwd(const void* x, int32_t x_f32, int64_t ldx, int64_t rows, int32_t D,
                         const float* gamma, const float* beta, float eps,
                         void* y_bf16, int64_t ldyb, float* y_f32, int64_t ldyf,
                         float* mean, float* rstd, void* stream);
/* dx = LN'(dy) [+ dres]; per-block partial dgamma/dbeta [nblocks][D] (reduce with
 * ctclip_reduce_slabs).  D <= 1024. */
int ctclip_layernorm_bwd(const void* dy, int32_t dy_f32, int64_t lddy, const void* x, int32_t x_f32, int64_t ldx,
                         const float* mean, const float* rstd, const float* gamma, int64_t rows, int32_t D,
                         const float* dres, int64_t lddres, float* dx_f32, int64_t lddxf,
                         void* dx_bf16, int64_t lddxb, float* part_gamma, float* part_beta,
                         int32_t nblocks, void* stream);
/* per-head l2norm * scale (attention.py:152-154): y[:, h*D:(h+1)*D] = x / max(|x|,1e-12) * scale */
int ctclip_l2norm_scale_fwd(const void* x, int64_t ldx, int64_t rows, int32_t H, int32_t D,
                            const float* scale, void* y, int64_t ldy, void* stream);
int ctclip_l2norm_scale_bwd(const void* x, int64_t ldx, const void* dy, int64_t lddy, int64_t rows,
                            int32_t H, int32_t D, const float* scale, void* dx, int64_t lddx,
                            float* part_scale, int32_t nblocks, void* stream);
/* the same for the folded-LayerNorm Q (ctclip_gemm_qkv_lnfold; x = the forward's q): dx (optional)
 * as above, dx2 = bf16(dx * row_rstd[row]), part_u [nblocks][H * D] = per-block column sums of
 * dx2 * row_mean[row]; with c1_out / beta_out (and fold_cs [H * D], the LayerNorm width Dm) the
 * LayerNorm backward's row terms for ctclip_gemm_lnfold_bwd: alpha = (dx2 . fold_cs) / Dm,
 * beta = row_rstd (dx2 . x) / Dm, c1 = alpha - beta * row_mean.  H * D / 8 divides 256, <= 64. */
int ctclip_l2norm_scale_bwd_fold(const void* x, int64_t ldx, const void* dy, int64_t lddy, int64_t rows,
                                 int32_t H, int32_t D, const float* scale, void* dx, int64_t lddx,
                                 float* part_scale, int32_t nblocks, const float* row_rstd, const float* row_mean,
                                 void* dx2, int64_t lddx2, float* part_u, const float* fold_cs, int32_t Dm,
                                 float* c1_out, float* beta_out, void* stream);
/* both l2norm backwards of the folded layer in one pass (head dim 32; x = the forward's [q | k],
 * 256 + 256 columns; dy = [dq_n | dk_n]): out[:, :256] = dq o row_rstd, out[:, 256:] = dk (the
 * [dq o rstd | dk | dv] buffer), part_s [2][nblocks][32] = q / k scale-gradient partials, part_u /
 * c1 / beta as ctclip_l2norm_scale_bwd_fold.  Replaces that call + ctclip_l2norm_scale_bwd for k. */
int ctclip_l2norm_qk_bwd_fold(const void* x, int64_t ldx, const void* dy, int64_t lddy, int64_t rows,
                              const float* scale_q, const float* scale_k, void* out, int64_t ldo, float* part_s,
                              int32_t nblocks, const float* row_rstd, const float* row_mean, float* part_u,
                              const float* fold_cs, int32_t Dm, float* c1_out, float* beta_out, void* stream);
/* per-block column-sum partials [nblocks][cols] (bias gradients) */
int ctclip_colsum(const void* x, int32_t x_f32, int64_t ld, int64_t rows, int32_t cols, float* part,
                  int32_t nblocks, void* stream);

/* ---------------------------------------------------------------- elementwise / layout
 * GEGLU backward on the tile-interleaved pre-activation (FeedForward, attention.py:39-52) */
int ctclip_geglu_bwd(const void* dg, int64_t lddg, const void* h, int64_t ldh, int64_t rows, int32_t gcols,
                     void* dh, int64_t lddh, void* stream);
int ctclip_gelu_bwd(const void* dy, const void* pre, void* dx, int64_t n, void* stream);
/* bf16 working weights from f32 masters: dst[r][c] = src[map[r]][c] * colscale[c] (zero pads) */
int ctclip_pack_rows(const float* src, int64_t ld_src, const int32_t* map, int64_t rows_dst, int32_t cols,
                     int32_t cols_dst, const float* colscale, void* dst, int64_t ld_dst, void* stream);
int ctclip_unpack_rows(const float* src, int64_t ld_src, const int32_t* map, int64_t rows_src, int32_t cols,
                       float* dst, int64_t ld_dst, int32_t accumulate, void* stream);
int ctclip_gelu_f32(const float* x, float* y, int64_t n, void* stream);
/* BERT hidden dropout (BertEmbeddings / BertSelfOutput / BertOutput, train mode):
 * y = x * keep / (1 - p) (+ res) into yf (f32) and / or yb (bf16); keep = hash(seed, i) >= p * 2^32.
 * The backward is the same call on dy with the same seed.  n % 4 == 0. */
int ctclip_dropout(const float* x, const float* res, float* yf, void* yb, int64_t n, float p, uint64_t seed,
                   void* stream);
int ctclip_cast_f32_bf16(const float* x, void* y, int64_t n, void* stream);
/* hi = bf16(x), lo = bf16(x - hi) (round to nearest even both): x = hi + lo to ~16 bits */
int ctclip_cast_f32_bf16_split(const float* x, void* hi, void* lo, int64_t n, void* stream);
int ctclip_add_f32(const float* a, const float* b, float* y, void* y_bf16, int64_t n, void* stream);

/* ---------------------------------------------------------------- patch embedding
 * int16 HU (is_hu: clamp(-1000,1000)/1000.f, ct_clip/data.py:150-152) or f32 video
 * (B, C, F, H, W) -> xhat (B*T*Hg*Wg, C*PT*P*P) bf16 = LayerNorm statistics applied
 * (ctvit.py:170-171).  offs[e] = voxel offset of patch element e from the patch origin.
 * ldo = xhat row stride in elements (>= patch dim, even; <= 0 means patch dim); columns
 * [patch dim, ldo) are written as zeros (K padding for the 64-deep patch-embed GEMM). */
int ctclip_patch_ln(const void* video, int32_t is_f32, int32_t is_hu, int64_t B, int32_t C, int32_t F,
                    int32_t H, int32_t W, int32_t PT, int32_t P, const int32_t* offs, float eps,
                    void* xhat, int64_t ldo, void* stream);
/* the same, plus an optional fp16 copy xhat16 (same ldo): the fp16 patch-embed GEMM's A operand
 * (round 5; the bf16 xhat stays the weight gradient's operand) */
int ctclip_patch_ln_x2(const void* video, int32_t is_f32, int32_t is_hu, int64_t B, int32_t C, int32_t F,
                       int32_t H, int32_t W, int32_t PT, int32_t P, const int32_t* offs, float eps,
                       void* xhat, void* xhat16, int64_t ldo, void* stream);
/* ... and, with xhat16, its lo residual xhat16lo = fp16(xhat - xhat16) (same ldo): the split-fp16
 * patch-embed GEMM's A pair (round 6, precise 'split' mode) */
int ctclip_patch_ln_x3(const void* video, int32_t is_f32, int32_t is_hu, int64_t B, int32_t C, int32_t F,
                       int32_t H, int32_t W, int32_t PT, int32_t P, const int32_t* offs, float eps,
                       void* xhat, void* xhat16, void* xhat16lo, int64_t ldo, void* stream);
int ctclip_patch_wgrad(const float* G, const float* colsum_dy, const float* W, const float* gamma,
                       const float* beta, int32_t N, int32_t K, float* dW, float* dgamma, float* dbeta,
                       int32_t accumulate, void* stream);
/* reconstruction loss of the VQ-VAE path: to_pixels' Rearrange
 * 'b t h w (c pt p1 p2) -> b c (t pt) (h p1) (w p2)' (ct_clip/ctvit.py:194-197) fused with
 * F.mse_loss(video, recon) (ctvit.py:451).  pix [tokens][ldp] f32 (the to_pixels Linear output);
 * video as for ctclip_patch_ln; offs its element->voxel table.  Writes loss[0] = mean squared
 * error, part[tokens] (workspace: per-row sums), optionally grad [tokens][ldg] = d loss / d pix and
 * recon (B, C, F, H, W) f32. */
int ctclip_unpatch_mse(const float* pix, int64_t ldp, const void* video, int32_t is_f32, int32_t is_hu, int64_t B,
                       int32_t C, int32_t F, int32_t H, int32_t W, int32_t PT, int32_t P, const int32_t* offs,
                       float* grad, int64_t ldg, float* recon, float* part, float* loss, void* stream);

/* ---------------------------------------------------------------- PEG (attention.py:56-84)
 * causal depthwise 3x3x3 conv + residual on canonical (b,t,h,w) token rows; mode 0 = spatial
 * view, mode 1 = the temporal transformer's raw-reshape view (attention.py:69-70). */
int ctclip_peg_fwd(const void* x_bf16, const float* x_f32, int64_t B, int32_t T, int32_t H, int32_t W,
                   int32_t D, const float* weight, const float* bias, int32_t mode, float* out_f32,
                   void* out_bf16, void* stream);
/* the same, plus the LayerNorm statistics of every output row over each 64-channel group:
 * stats [D / 64][B T H W] float2 (mean, M2) for ctclip_ln_stats_merge (plane-streaming shapes) */
int ctclip_peg_fwd_stats(const void* x_bf16, const float* x_f32, int64_t B, int32_t T, int32_t H, int32_t W,
                         int32_t D, const float* weight, const float* bias, int32_t mode, float* out_f32,
                         void* out_bf16, float* stats, void* stream);
/* PEG forward with the conv taps read from the f32 residual stream x (not its bf16 shadow; the
 * residual is the centre tap): out_f32 = x + bias + conv(x) (ct_clip/attention.py:56-84,324),
 * out_bf16 / out_f16 (optional) its 16-bit copies, stats (optional, plane-streaming shapes:
 * D % 32 == 0, W <= 24) [D / 32][B T H W] float2 (mean, M2) per 32-channel group for
 * ctclip_ln_stats_merge.  Any D % 4 == 0 otherwise (one thread per token x 4 channels). */
int ctclip_peg_fwd_x32(const float* x_f32, int64_t B, int32_t T, int32_t H, int32_t W, int32_t D,
                       const float* weight, const float* bias, int32_t mode, float* out_f32, void* out_bf16,
                       void* out_f16, float* stats, void* stream);
/* ... with, beside out_f16, its lo residual out_f16lo = fp16(out - out_f16) (the split-fp16 x3 Q | K | V
 * GEMM's A pair, round 6; out_f16 required) and the fp16 range check: an fp16 output beyond +-65504
 * or non-finite sets CT_STATUS_F16_RANGE in *status (optional) */
int ctclip_peg_fwd_x32s(const float* x_f32, int64_t B, int32_t T, int32_t H, int32_t W, int32_t D,
                        const float* weight, const float* bias, int32_t mode, float* out_f32, void* out_bf16,
                        void* out_f16, void* out_f16lo, float* stats, int32_t* status, void* stream);
/* dx = dout + conv^T(dout) from the f32 dout alone (the conv taps in f32; no bf16 dout read): the x32
 * kernel's transposed form, fixed 24^3 grids (returns CT_ESHAPE otherwise: use ctclip_peg_bwd_data).
 * ct_clip/attention.py:56-84 backward. */
int ctclip_peg_bwd_data_x32(const float* dout_f32, int64_t B, int32_t T, int32_t H, int32_t W, int32_t D,
                            const float* weight, int32_t mode, float* dx_f32, void* dx_bf16, void* stream);
int ctclip_peg_bwd_data(const void* dout_bf16, const float* dout_f32, int64_t B, int32_t T, int32_t H,
                        int32_t W, int32_t D, const float* weight, int32_t mode, float* dx_f32,
                        void* dx_bf16, void* stream);
/* part: [nblk][D][28] f32 partial sums (27 taps in (kt,kh,kw) order, then bias); nblk must equal
   ctclip_peg_wgrad_slabs(B, T, H, W, D) (one slab per (batch, 2-row tile) on the plane-streaming path). */
int ctclip_peg_bwd_weight(const void* dout_bf16, const void* x_bf16, int64_t B, int32_t T, int32_t H,
                          int32_t W, int32_t D, int32_t mode, float* part, int32_t nblk, void* stream);
int ctclip_peg_wgrad_slabs(int64_t B, int32_t T, int32_t H, int32_t W, int32_t D);
/* Sum of the nblk [D][28] partial slabs of ctclip_peg_bwd_weight straight into the parameters'
   gradients: dweight[c][27] (+)= sum_b part[b][c][0..26], dbias[c] (+)= sum_b part[b][c][27], slabs
   summed in order (deterministic); either output may be null.  Replaces a slab reduction + two
   strided adds per layer (round 4). */
int ctclip_peg_wgrad_reduce(const float* part, int32_t nblk, int32_t D, float* dweight, float* dbias,
                            int32_t accumulate, void* stream);
/* mode 1 on a T = H = W = 24 cube runs as a canonical-order walk (the view is an axis permutation
 * there; same outputs up to f32 summation order); 0 = the view-order walk (A/B).  Returns the previous. */
int ctclip_peg_set_canon1(int32_t on);

/* ---------------------------------------------------------------- attention (attention.py:127-181)
 * softmax(scale * q.k^T + bias + mask) v per (sequence, head); q/k already l2-normalised and
 * scaled for CTViT.  Sequence rows: row(s,i) = (s/n_inner)*s_outer + (s%n_inner)*s_inner + i*s_pos.
 * bias_u: deduplicated continuous-position-bias table [H][(2gh-1)(2gw-1)] (attention.py:229-276).
 * bwd: writes dq, dk, dv (bf16), delta [H][M], accumulates dbias_u with atomics.
 * q, k, v, o, o16, dout, dq, dk, dv (those given): 16-B aligned, ld % 8 == 0, else CT_EALIGN. */
typedef struct {
  const void* q; int64_t ldq;
  const void* k; int64_t ldk;
  const void* v; int64_t ldv;
  void* o; int64_t ldo;
  const void* dout; int64_t lddo;
  void* dq; int64_t lddq;
  void* dk; int64_t lddk;
  void* dv; int64_t lddv;
  float* lse; float* delta;
  const float* bias_u; float* dbias_u;
  const int32_t* kmask;
  float scale;
  int32_t L, H, D, nseq;
  int64_t M;
  int32_t grid_h, grid_w;
  int32_t n_inner;
  int64_t s_outer, s_inner, s_pos;
  /* attention-probability dropout (transformers BertSelfAttention.dropout, train mode): P[q][k]
   * kept iff hash(dropout_seed, seq, head, q, k) >= p * 2^32, kept entries scaled by 1/(1-p);
   * the backward regenerates the mask from the same seed.  0 = off; bias_u != null: CT_EINVAL. */
  float dropout_p;
  uint64_t dropout_seed;
  /* bwd, optional: caller-provided workspace for the bias gradient's per-workgroup partial bins,
   * summed into dbias_u by one deterministic reduction instead of global float atomics; NULL =
   * atomics.  Its size in floats is ctclip_attn_bwd_ws_floats(a) (0: this shape does not use it). */
  float* dbias_ws;
  int64_t dbias_ws_floats;
  void* o16;   /* fwd, optional: an fp16 copy of O (ldo) -- the fp16 to_out GEMM's A operand; the
                * forward's o and lse may be NULL when o16 is given (the eval forward, round 6) */
} ctclip_attn_args;
int ctclip_attn_fwd(const ctclip_attn_args* a, void* stream);
int ctclip_attn_bwd(const ctclip_attn_args* a, void* stream);
int ctclip_attn_bwd_ws_floats(const ctclip_attn_args* a);
int ctclip_attn_fwd_f32(const ctclip_attn_args* a, void* stream);
/* split-fp16 x3 attention forward (precise 'split' mode, round 6; D = 32): q, k, v f32 as for
 * ctclip_attn_fwd_f32, every product on v_mfma_f32_16x16x32_f16 as hi.hi + hi.lo + lo.hi of fp16
 * (hi, lo) operand pairs (the probabilities included), f32 softmax.  O is written as the fp16 pair
 * (oh, ol) that the x3 to_out GEMM reads (ldo = a->ldo), optionally as bf16 ob and with the natural-log
 * lse [H][M] -- the operands of the bf16 backward (ctclip_attn_bwd) -- so no bf16 forward re-run. */
int ctclip_attn_fwd_x3(const ctclip_attn_args* a, void* oh, void* ol, void* ob, float* lse, void* stream);   /* f32 image tower, see below */
/* diagnostic: query blocks per wave processed together by the spatial (CPB-bias) forward kernel,
 * 1..3 (default 3); results are bit-identical.  Returns the previous setting. */
int ctclip_attn_set_fwd_qb(int qb);
/* diagnostic: static-bound softmax in the 3-block spatial forward (1) or the online max (0, default:
 * measured faster); see attn.hip.  Returns the previous setting. */
int ctclip_attn_set_fwd_smax(int on);
/* the C-init score chain of the 3-block spatial forward (1, default, round 6: the CPB bias as the
 * MFMA's accumulator input, row sums on the MFMA) or the round-5 chain (0); returns the previous. */
int ctclip_attn_set_fwd_cinit(int on);

/* ---------------------------------------------------------------- f32 image tower (opt-in)
 * Exact-f32 forward stages of functional.set_vit_precision('f32') (csrc/f32path.hip); the linears
 * of that mode run on ctclip_sgemm.  All tensors f32.
 *   patch_ln_f32: to_patch_emb's Rearrange + nn.LayerNorm(pd) with affine (ct_clip/ctvit.py:169-174)
 *   peg_fwd_f32:  out = x + PEG(x), canonical rows, mode as ctclip_peg_fwd (attention.py:56-84,324)
 *   l2norm_scale_fwd_f32: per head x / max(||x||, 1e-12) * scale (attention.py:152-154)
 *   geglu_f32:    g[:, c] = gelu_erf(h[:, inner + c]) * h[:, c] (attention.py:39-42, un-interleaved W1)
 *   attn_fwd_f32: ctclip_attn_args with f32 q / k / v / o (lse unused); no kmask, no dropout */
int ctclip_patch_ln_f32(const void* video, int32_t is_f32, int32_t is_hu, int64_t B, int32_t C, int32_t F,
                        int32_t H, int32_t W, int32_t PT, int32_t P, const int32_t* offs, float eps,
                        const float* gamma, const float* beta, float* out, int64_t ldo, void* stream);
int ctclip_peg_fwd_f32(const float* x, int64_t B, int32_t T, int32_t H, int32_t W, int32_t D,
                       const float* weight, const float* bias, int32_t mode, float* out, void* stream);
int ctclip_l2norm_scale_fwd_f32(const float* x, int64_t ldx, int64_t rows, int32_t H, int32_t D,
                                const float* scale, float* y, int64_t ldy, void* stream);
/* Round 6: the same with an optional bf16 copy y_bf16 (ldyb % 4 == 0, 8-B aligned; D = 32 or 64) --
 * the precise 'split' tower's q / k for the bf16 backward, without a separate cast pass. */
int ctclip_l2norm_scale_fwd_f32b(const float* x, int64_t ldx, int64_t rows, int32_t H, int32_t D,
                                 const float* scale, float* y, int64_t ldy, void* y_bf16, int64_t ldyb, void* stream);
int ctclip_geglu_f32(const float* h, int64_t ldh, int64_t rows, int32_t inner, float* g, int64_t ldg,
                     void* stream);
/* Round 4: the f32 tower trains (its forward feeds the bf16 backward kernels) and its Linears run on
 * a dedicated f32 MFMA GEMM (csrc/sgemm_tn.hip): C[M][N] = alpha A[M][K] . B[N][K]^T, each output one
 * f32 fma chain in ascending k (bit-identical to ctclip_sgemm).  act 0: C f32 (+ bias[N]) (+ R f32),
 * optional bf16 copy C2; act 2: GEGLU over the packed [32 x | 32 gate] pairs (N % 64 == 0): C2 = h
 * bf16 [M][N], C = g f32 [M][N/2], optional C3 = g bf16.  K, N, ld* % 4 == 0; A, B, C 16-B aligned. */
typedef struct {
  int64_t M, N, K;
  const float* A; int64_t lda;
  const float* B; int64_t ldb;
  float* C; int64_t ldc;
  void* C2; int64_t ldc2;
  void* C3; int64_t ldc3;
  const float* bias;
  const float* R; int64_t ldr;
  float alpha;
  int32_t act;
} ctclip_sgemm_tn_args;
int ctclip_sgemm_tn(const ctclip_sgemm_tn_args* a, void* stream);
/* fp16 working weights of the fp16 forward GEMMs, as ctclip_pack_rows (round 5) */
int ctclip_pack_rows_h16(const float* src, int64_t ld_src, const int32_t* map, int64_t rows_dst, int32_t cols,
                         int32_t cols_dst, const float* colscale, void* dst, int64_t ld_dst, void* stream);
/* split-fp16 operands of the x3 GEMM (ctclip_gemm_args.A_lo / B_lo; precise.set_vit_precision('split'),
 * round 6): hi = fp16(v scale), lo = fp16(v scale - hi) of every f32 value v, so hi + lo carries v
 * to ~22 mantissa bits (the dropped remainder is < 2^-22 |v| for |v scale| in [2^-3, 65504]; smaller
 * values keep an absolute 2^-25 / scale).  A value outside fp16's range after scaling sets
 * CT_STATUS_F16_RANGE in *status (optional).  The weights are scaled by 256 (the GEMM's alpha undoes
 * it, exactly: a power of two) so their ~1e-2 entries keep a normal lo part.
 *   split_f16: x [rows][cols] (ldx, f32, cols % 8 == 0) -> hi / lo [rows][cols] (ldo);
 *   pack_rows_x3: ctclip_pack_rows (row map, column scale, zero padding) into the pair. */
int ctclip_split_f16(const float* x, int64_t ldx, int64_t rows, int32_t cols, float scale, void* hi, void* lo,
                     int64_t ldo, int32_t* status, void* stream);
int ctclip_pack_rows_x3(const float* src, int64_t ld_src, const int32_t* map, int64_t rows_dst, int32_t cols,
                        int32_t cols_dst, const float* colscale, float scale, void* hi, void* lo, int64_t ld_dst,
                        int32_t* status, void* stream);
/* f32 working weights: dst[r][c] = src[map[r]][c] * colscale[c] (zero pads), as ctclip_pack_rows */
int ctclip_pack_rows_f32(const float* src, int64_t ld_src, const int32_t* map, int64_t rows_dst, int32_t cols,
                         int32_t cols_dst, const float* colscale, float* dst, int64_t ld_dst, void* stream);

/* ---------------------------------------------------------------- vector quantiser
 * vector_quantize_pytorch==1.1.2 cosine codebook (ct_clip/ctvit.py:187,421-427).
 * cand = float2[rows][ntiles] (score, index) and cand2 = float[rows][ntiles] (second-best score) of
 * each 64-code group, from ctclip_gemm(act=3, C2 = cand2) over l2norm(x).codebook_bf16^T;
 * ntiles = ceil(C / 64).  select re-scores in f32 (f32 x, f32 codebook [C][D]) every code whose bf16
 * score can lie within `margin` of the best -- group winners, and whole groups whose second-best is
 * within it -> the exact f32 argmax (first index on ties) for margin >= 2^-6 (bf16 scoring error
 * bound, see vq.hip).  cand2 = NULL re-scores group winners only.  D % 4 == 0, D <= 4096.
 * Round 6: "the f32 argmax" is the argmax of the SEQUENTIAL f32 dot product (k = 0 .. D-1, one fma
 * per term): fast slice / butterfly sums decide every row whose best two are further apart than
 * their worst-case difference, the sequential sum decides the near-ties -- so the index does not
 * depend on which codes the low-precision GEMM made candidates (codebook rows of norm <= 4). */
int ctclip_vq_select(const float* cand, const float* cand2, int32_t ntiles, const float* x, int64_t rows, int32_t D,
                     const float* codebook, int32_t C, float margin, int32_t* idx, float* xn_out, void* stream);
/* ... with the step status word: a row without any finite score (NaN / inf token) gets idx 0 and a
 * zero xn row as above AND sets CT_STATUS_VQ_NONFINITE in *status (round 6) */
int ctclip_vq_select_s(const float* cand, const float* cand2, int32_t ntiles, const float* x, int64_t rows, int32_t D,
                       const float* codebook, int32_t C, float margin, int32_t* idx, float* xn_out, int32_t* status,
                       void* stream);
/* Round 6: the fp16 scoring operand of the VQ distance GEMM: y = fp16(x / max(||x||, 1e-12)) per row
 * (x f32 [rows][ldx], D % 4 == 0).  With an fp16 image of the (unit-norm) codebook and
 * ctclip_gemm_args.ab_f16 on the act-3 GEMM, every score is within ~2^-10 of the f32 cosine, and
 * ctclip_vq_select's margin can be 4e-3 instead of 2e-2 (exact f32 argmax either way). */
int ctclip_vq_l2norm_h16(const float* x, int64_t ldx, int64_t rows, int32_t D, void* y, int64_t ldy, void* stream);
/* pooled[b][hw][:] = mean_t codebook[idx[b][t*HW+hw]]   (ct_clip/ct_clip.py:724,740) */
int ctclip_vq_pool(const int32_t* idx, const float* codebook, int64_t B, int32_t T, int32_t HW, int32_t D,
                   float* out, void* out_bf16, void* stream);
/* backward of pool + straight-through estimator: dx[b][t][hw] = dpooled[b][hw] / T */
int ctclip_vq_pool_bwd(const float* dpooled, int64_t B, int32_t T, int32_t HW, int32_t D, float* dx, void* dx_bf16,
                       void* stream);
int ctclip_vq_gather(const int32_t* idx, const float* codebook, int64_t rows, int32_t D, float* out, void* stream);
/* training-mode EMA codebook update (bins / embed_sum accumulate, then finalize).  esum [C][D]
 * holds the per-code token sums in signed 2^-40 fixed point (int64, zeroed by the caller; xn rows
 * are unit vectors): integer sums are bit-identical whatever the order of the adds, on one GPU and
 * through a SUM all-reduce across ranks (bins: f32 counts, exact below 2^24). */
int ctclip_vq_ema_accum(const int32_t* idx, const float* xn, int64_t rows, int32_t D, float* bins, int64_t* esum,
                        void* stream);
/* the same statistics, bit for bit, with the rows first bucketed by code (counting sort), so the
 * fixed-point adds go out once per (code, 32 sorted rows) instead of once per token-order run:
 * work = int32 [2 C + 2 rows] scratch whose first C entries are zero on entry and left zero. */
int ctclip_vq_ema_accum_sorted(const int32_t* idx, const float* xn, int64_t rows, int32_t D, int32_t C, float* bins,
                               int64_t* esum, int32_t* work, void* stream);
int ctclip_vq_ema_finalize(const float* bins, const int64_t* esum, int32_t C, int32_t D, float decay, float* embed,
                           float* cluster_size, void* embed_bf16, void* stream);
/* ctclip_vq_ema_finalize that also zeroes bins / esum behind its reads, so persistent statistics
 * buffers are ready for the next step's ctclip_vq_ema_accum (no fill launches). */
int ctclip_vq_ema_finalize_reset(float* bins, int64_t* esum, int32_t C, int32_t D, float decay, float* embed,
                                 float* cluster_size, void* embed_bf16, void* stream);
/* ... guarded (round 6): when *guard != 0 (the summed step status words, carried through the
 * statistics' all-reduce in the slot after the bins) the step's update is dropped on every rank --
 * embed / cluster_size untouched -- and only the statistics are zeroed.  guard NULL: unguarded. */
int ctclip_vq_ema_finalize_guard(float* bins, int64_t* esum, int32_t C, int32_t D, float decay, float* embed,
                                 float* cluster_size, void* embed_bf16, const float* guard, void* stream);

/* ---------------------------------------------------------------- contrastive loss
 * symmetric InfoNCE over the (global) batch, ct_clip/ct_clip.py:771,796,845-901; one workgroup.
 * Inputs are raw projected latents; returns loss, d loss / d raw latents, d loss / d log-temp. */
int ctclip_clip_loss(const float* t_raw, const float* i_raw, int32_t Bg, int32_t Dl, const float* log_temp,
                     float* t_norm, float* i_norm, float* loss, float* dt_raw, float* di_raw, float* dlogtemp,
                     float* sim, void* stream);
/* eval branch einsum('b d, b d -> b') * temp (ct_clip.py:805-807) */
int ctclip_clip_scores(const float* t_raw, const float* i_raw, int32_t B, int32_t Dl, const float* log_temp,
                       float* out, void* stream);
/* zero-shot pathology scoring, replaces the per-volume x per-pathology loop of
 * ct_clip/ctclip_inference.py:305-315 (CTCLIP.forward eval branch on a 2-prompt pair, softmax
 * over the pair, 'present' entry): t_raw [2P][Dl] raw prompt latents (rows 2j / 2j+1 = "present" /
 * "not present" of pathology j), i_raw [N][Dl] raw image latents -> scores [N][P][2], probs [N][P] */
int ctclip_zero_shot(const float* t_raw, const float* i_raw, int32_t P, int32_t N, int32_t Dl, const float* log_temp,
                     float* scores, float* probs, void* stream);

/* ---------------------------------------------------------------- small exact-f32 GEMM (strided)
 * CPB MLP (attention.py:247-252,271-274) and its backward; act 1 = LeakyReLU(slope),
 * act 2 = multiply by LeakyReLU'(aux).  split > 1 splits K over `split` workgroup layers writing
 * f32 slabs into `workspace` ([split][M][N]), folded in slab order (deterministic). */
int ctclip_sgemm(int64_t M, int64_t N, int64_t K, const float* A, int64_t sam, int64_t sak, const float* B,
                 int64_t sbk, int64_t sbn, float* C, int64_t scm, int64_t scn, const float* bias, float alpha,
                 int32_t act, float slope, const float* aux, int64_t sxm, int64_t sxn, int32_t accumulate,
                 float* workspace, int32_t split, void* stream);

/* ---------------------------------------------------------------- BERT embeddings */
int ctclip_embed_fwd(const int64_t* ids, int64_t B, int32_t L, int32_t Hd, const float* word, const float* pos,
                     const float* type0, float* out, void* stream);
/* accumulates into dword / dpos / dtype0 (each may be NULL) without float atomics: bit-reproducible.
 * Tokens whose id == pad_id add nothing to dword (nn.Embedding padding_idx: transformers'
 * BertEmbeddings word table, pad_token_id 0); pad_id < 0 = none.  Hd % 4 == 0, 16-byte aligned rows. */
int ctclip_embed_bwd(const int64_t* ids, int64_t B, int32_t L, int32_t Hd, const float* dx, float* dword,
                     float* dpos, float* dtype0, int64_t pad_id, void* stream);

/* ---------------------------------------------------------------- optimizer (CTCLIPTrainer.py:347-353)
 * grad norm -> out[0] = norm, out[1] = clip coef (torch clip_grad_norm_ semantics);
 * Adam over a flat arena (optimizer.py:24), grads scaled by coef[1], bf16 copy refreshed;
 * zero_grad != 0 also zeroes g in the same pass (the trainer's zero_grad, CTCLIPTrainer.py:353).
 * skip (optional device int32): when *skip != 0 the step is dropped: p, m, v unchanged, g zeroed if
 * zero_grad (the step's guard word:
 * the LayerNorm-fused GEMM status of ctclip_gemm_ln).
 * p, g, m, v must share one alignment modulo 16 B (slices of arenas with one layout): CT_EALIGN. */
int ctclip_grad_norm(const float* g, int64_t n, float max_norm, float* part, int32_t nblk, float* out, void* stream);
/* ... and a non-finite norm ORs CT_STATUS_NONFINITE_GRAD into *skip (the Adam kernels' guard word of
 * the step, round 6): a NaN / inf gradient never reaches the parameters or the moments */
int ctclip_grad_norm_s(const float* g, int64_t n, float max_norm, float* part, int32_t nblk, float* out, int32_t* skip,
                       void* stream);
int ctclip_adam(float* p, float* g, float* m, float* v, int64_t n, float lr, float b1, float b2, float eps,
                float wd, int32_t step, const float* coef, void* p_bf16, void* p_bf16_lo, int32_t zero_grad,
                const int32_t* skip, void* stream);   /* p_bf16_lo (needs p_bf16): bf16(p - bf16(p)), the
                                                       * split-weight lo image */

/* ---------------------------------------------------------------- volume preprocessing
 * Replaces the host-side per-sample loader arithmetic:
 *   mode 0 = ct_clip/data.py:114-192 (CTReportDataset.npz_img_to_tensor after the metadata
 *            lookup): slope*x + intercept -> resize_array (data.py:15-40, F.interpolate trilinear,
 *            align_corners=False) -> clip(-1000, 1000) / 1000 -> centre crop / pad (fill) ->
 *            (D, H, W) f32.  f64 arithmetic for int16 / f64 sources (numpy promotion), f32 for f32.
 *   mode 1 = data_prep/preprocess_train.py:67-104 (process_file): f32(clip(slope*x + intercept) /
 *            1000) -> resize_array in f32; output = the resized volume.
 * The source is read through (d, h, w) element strides (the npz scan is (H, W, D): sd = 1,
 * sh = W*D, sw = D).  Output voxel (d, h, w) takes resized voxel (d-od, h-oh, w-ow), or `fill`
 * outside [0,Dn) x [0,Hn) x [0,Wn).  The host computes Dn/Hn/Wn and the offsets exactly as the
 * reference does (ctclip_mi355x/preprocess.py). */
enum { CTCLIP_F32 = 0, CTCLIP_I16 = 1, CTCLIP_F64 = 2 };
typedef struct {
  const void* src; int32_t src_dtype;
  int64_t D, H, W;          /* source extents in the (d, h, w) view */
  int64_t sd, sh, sw;       /* source strides, elements */
  int64_t Dn, Hn, Wn;       /* resized extents (interpolation target) */
  int64_t Do, Ho, Wo;       /* output extents */
  int64_t od, oh, ow;       /* output index - resized index (crop / pad placement) */
  double slope, intercept;
  int32_t mode;
  float fill;
} ctclip_resample_args;
int ctclip_resample_volume(const ctclip_resample_args* a, float* out, void* stream);

#ifdef __cplusplus
}
#endif
#endif
