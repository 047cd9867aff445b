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

__global__ __launch_bounds__(256) void embed_bwd_kernel(const int64_t* __restrict__ ids, int64_t B, int L, int Hd,
                                                        const float* __restrict__ dx, float* __restrict__ dword,
                                                        float* __restrict__ dpos, float* __restrict__ dtype0) {
  const int64_t total = B * L * Hd;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t tok = i / Hd;
    const int c = (int)(i - tok * Hd);
    const int l = (int)(tok % L);
    const float g = dx[i];
    if (dword) atomicAdd(&dword[ids[tok] * Hd + c], g);
    if (dpos) atomicAdd(&dpos[(int64_t)l * Hd + c], g);
    if (dtype0) atomicAdd(&dtype0[c], g);
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
                                float* dpos, float* dtype0, void* stream) {
  const int64_t n = B * L * Hd;
  hipLaunchKernelGGL(embed_bwd_kernel, dim3((int)std::min<int64_t>(4096, (n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, ids, B, L, Hd, dx, dword, dpos, dtype0);
  CT_CHECK_LAUNCH();
  return 0;
}
