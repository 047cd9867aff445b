// BERT embeddings (transformers.BertModel, called at ct_clip/ct_clip.py:685): word +
// token_type(0) + absolute position, before the embedding LayerNorm (norm.hip), and the
// sparse scatter-add backward into the three tables.
#include "common.h"
#include "../../include/ctclip_hip.h"

namespace {

__global__ __launch_bounds__(256) void embed_fwd_kernel(const int64_t* __restrict__ ids, int64_t B, int L, int Hd,
                                                        const float* __restrict__ word, const float* __restrict__ pos,
                                                        const float* __restrict__ type0, float* __restrict__ out) {
  const int nch = Hd / 4;
  const int64_t total = B * L * nch;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t tok = i / nch;
    const int c = (int)(i - tok * nch) * 4;
    const int l = (int)(tok % L);
    const int64_t id = ids[tok];
    f32x4 v = *(const f32x4*)(word + id * Hd + c);
    v += *(const f32x4*)(pos + (int64_t)l * Hd + c);
    v += *(const f32x4*)(type0 + c);
    *(f32x4*)(out + tok * Hd + c) = v;
  }
}

// Backward without float atomics (bit-reproducible): the word-table gradient of an id is summed
// by ONE workgroup, the one of the id's first token, over the id's tokens in token order; the
// pad id gets none (nn.Embedding padding_idx, as transformers' BertEmbeddings builds the word
// table with padding_idx = pad_token_id).  grid = tokens, 256 threads x 4 columns per pass.
__global__ __launch_bounds__(256) void embed_word_bwd_kernel(const int64_t* __restrict__ ids, int ntok, int Hd,
                                                             const float* __restrict__ dx, float* __restrict__ dword,
                                                             int64_t pad_id) {
  __shared__ int64_t sid[1024];
  const int t = blockIdx.x, tid = threadIdx.x;
  const int64_t id = ids[t];
  if (id == pad_id) return;
  int dup = 0;
  for (int u = tid; u < t; u += 256) dup |= ids[u] == id;
  if (__syncthreads_or(dup)) return;   // an earlier token of this id owns it
  for (int c0 = 0; c0 < Hd; c0 += 1024) {
    const int c = c0 + tid * 4;
    const bool cv = c < Hd;
    f32x4 s = cv ? *(const f32x4*)(dx + (int64_t)t * Hd + c) : f32x4{0.f, 0.f, 0.f, 0.f};
    for (int u0 = t + 1; u0 < ntok; u0 += 1024) {
      const int n = min(1024, ntok - u0);
      __syncthreads();
      for (int i = tid; i < n; i += 256) sid[i] = ids[u0 + i];
      __syncthreads();
      if (cv)
        for (int i = 0; i < n; ++i)
          if (sid[i] == id) s += *(const f32x4*)(dx + (int64_t)(u0 + i) * Hd + c);
    }
    if (cv) {
      f32x4* w = (f32x4*)(dword + id * Hd + c);
      *w = *w + s;
    }
  }
}

// position rows (sum over the batch, b in order) and the token-type-0 row (sum of the position
// sums: 64 position groups per column, folded in group order).  1,024 threads = 16 column quads
// x 64 position groups; grid = Hd / 64.
__global__ __launch_bounds__(1024) void embed_pos_bwd_kernel(int B, int L, int Hd, const float* __restrict__ dx,
                                                             float* __restrict__ dpos, float* __restrict__ dtype0) {
  __shared__ f32x4 red[64][16];
  const int q = threadIdx.x & 15, lg = threadIdx.x >> 4;
  const int c = blockIdx.x * 64 + q * 4;
  const bool cv = c < Hd;
  f32x4 tsum = f32x4{0.f, 0.f, 0.f, 0.f};
  if (cv)
    for (int l = lg; l < L; l += 64) {
      f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};
      for (int b = 0; b < B; ++b) s += *(const f32x4*)(dx + ((int64_t)b * L + l) * Hd + c);
      if (dpos) {
        f32x4* w = (f32x4*)(dpos + (int64_t)l * Hd + c);
        *w = *w + s;
      }
      tsum += s;
    }
  red[lg][q] = tsum;
  __syncthreads();
  if (lg == 0 && cv && dtype0) {
    f32x4 s = red[0][q];
    for (int i = 1; i < 64; ++i) s += red[i][q];
    f32x4* w = (f32x4*)(dtype0 + c);
    *w = *w + s;
  }
}

}  // namespace

extern "C" int ctclip_embed_fwd(const int64_t* ids, int64_t B, int32_t L, int32_t Hd, const float* word,
                                const float* pos, const float* type0, float* out, void* stream) {
  CT_REQUIRE(Hd % 4 == 0, CT_EALIGN);
  const int64_t n = B * L * Hd / 4;
  hipLaunchKernelGGL(embed_fwd_kernel, dim3((int)std::min<int64_t>(4096, (n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, ids, B, L, Hd, word, pos, type0, out);
  CT_CHECK_LAUNCH();
  return 0;
}

extern "C" int ctclip_embed_bwd(const int64_t* ids, int64_t B, int32_t L, int32_t Hd, const float* dx, float* dword,
                                float* dpos, float* dtype0, int64_t pad_id, void* stream) {
  const int64_t ntok = B * L;
  if (ntok == 0) return 0;
  CT_REQUIRE(Hd % 4 == 0 && aligned16(dx) && ntok < (1 << 30), CT_EALIGN);
  CT_REQUIRE(!dword || aligned16(dword), CT_EALIGN);
  CT_REQUIRE((!dpos || aligned16(dpos)) && (!dtype0 || aligned16(dtype0)), CT_EALIGN);
  if (dword) {
    hipLaunchKernelGGL(embed_word_bwd_kernel, dim3((unsigned)ntok), dim3(256), 0, (hipStream_t)stream, ids, (int)ntok,
                       Hd, dx, dword, pad_id);
    CT_CHECK_LAUNCH();
  }
  if (dpos || dtype0) {
    hipLaunchKernelGGL(embed_pos_bwd_kernel, dim3(cdiv(Hd, 64)), dim3(1024), 0, (hipStream_t)stream, (int)B, L, Hd, dx,
                       dpos, dtype0);
    CT_CHECK_LAUNCH();
  }
  return 0;
}
