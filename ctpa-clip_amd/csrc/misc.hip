// Probe entry points of the C-ABI.
#include <string.h>
#include "common.h"
#include "../../include/ctclip_hip.h"

extern "C" int ctclip_version(void) { return CTCLIP_ABI_VERSION; }

extern "C" int ctclip_device_arch(char* buf, int n) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return (int)e;
  hipDeviceProp_t prop;
  e = hipGetDeviceProperties(&prop, dev);
  if (e != hipSuccess) return (int)e;
  if (buf && n > 0) {
    strncpy(buf, prop.gcnArchName, n - 1);
    buf[n - 1] = 0;
  }
  return 0;
}

// Test knob: nwg workgroups that each occupy a CU's LDS (lds_bytes) and spin for `cycles` shader
// clocks -- a stand-in for RCCL's resident kernels holding CUs while a persistent GEMM launches
// (tests/test_gpu_gemm_ln.py: the LayerNorm-fused GEMM's paired tiles beside CU-holding kernels).
namespace {
__global__ __launch_bounds__(64) void hold_cus_kernel(long long cycles) {
  extern __shared__ char lds[];
  if (threadIdx.x == 0) lds[0] = 0;
  const long long t0 = clock64();
  while (clock64() - t0 < cycles) __builtin_amdgcn_s_sleep(8);
}
}  // namespace

extern "C" int ctclip_debug_hold_cus(int32_t nwg, int64_t cycles, int32_t lds_bytes, void* stream) {
  CT_REQUIRE(nwg > 0 && nwg <= 4096 && cycles >= 0 && cycles < (1ll << 34) && lds_bytes >= 0 && lds_bytes <= 160 * 1024,
             CT_EINVAL);
  (void)hipFuncSetAttribute((const void*)hold_cus_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hipLaunchKernelGGL(hold_cus_kernel, dim3(nwg), dim3(64), lds_bytes, (hipStream_t)stream, (long long)cycles);
  CT_CHECK_LAUNCH();
  return 0;
}
