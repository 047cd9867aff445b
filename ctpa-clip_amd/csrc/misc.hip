// Probe entry points of the C-ABI.
#include <string.h>
#include "common.h"
#include "../../include/ctclip_hip.h"

extern "C" int ctclip_version(void) { return 1; }

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
