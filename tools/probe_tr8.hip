// Probe of ds_read_b64_tr_b8 (gfx950): which source lane's address and which byte of its 8 each
// destination byte comes from.  LDS bytes 0..511 hold b & 255; lane l supplies address 8 l (so
// lanes 0..31 address distinct bytes 0..255).  Prints the 8 bytes every lane of 0..31 received.
// build: hipcc --offload-arch=gfx950 -O2 tools/probe_tr8.hip -o tools/probe_tr8
#include <hip/hip_runtime.h>
#include <cstdio>

typedef int v2i __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) v2i* lds_v2i;

__global__ void probe(unsigned char* out) {
  __shared__ __attribute__((aligned(16))) unsigned char s[512];
  for (int b = threadIdx.x; b < 512; b += 64) s[b] = (unsigned char)(b & 255);
  __syncthreads();
  const v2i v = __builtin_amdgcn_ds_read_tr8_b64_v2i32((lds_v2i)(s + 8 * threadIdx.x));
  const unsigned char* p = reinterpret_cast<const unsigned char*>(&v);
  for (int j = 0; j < 8; ++j) out[threadIdx.x * 8 + j] = p[j];
}

int main() {
  unsigned char* d;
  unsigned char h[512];
  if (hipMalloc(&d, 512) != hipSuccess) return 1;
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
  if (hipMemcpy(h, d, 512, hipMemcpyDeviceToHost) != hipSuccess) return 2;
  for (int l = 0; l < 32; ++l) {
    printf("lane %2d:", l);
    for (int j = 0; j < 8; ++j) {
      const int b = h[l * 8 + j];
      printf(" %3d(l%2d+%d)", b, b / 8, b % 8);
    }
    printf("\n");
  }
  (void)hipFree(d);
  return 0;
}
