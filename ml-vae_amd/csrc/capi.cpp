// C-ABI plumbing: thread-local last-error string and library identification.
#include <stdarg.h>
#include <stdio.h>
#include <string.h>
#include <hip/hip_runtime.h>

static thread_local char g_err[512] = {0};

extern "C" void mlvae_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

extern "C" const char* mlvae_last_error(void) { return g_err; }

extern "C" int mlvae_abi_version(void) { return 1; }

// 0 = library loaded and a gfx950 device is visible; 1 = no device; 2 = wrong architecture
extern "C" int mlvae_device_check(char* name_out, int len) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
    mlvae_set_error("no HIP device visible");
    return 1;
  }
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, dev) != hipSuccess) { mlvae_set_error("hipGetDeviceProperties failed"); return 1; }
  if (name_out && len > 0) snprintf(name_out, len, "%s", p.gcnArchName);
  if (strncmp(p.gcnArchName, "gfx950", 6) != 0) {
    mlvae_set_error("device is %s, library built for gfx950", p.gcnArchName);
    return 2;
  }
  return 0;
}
