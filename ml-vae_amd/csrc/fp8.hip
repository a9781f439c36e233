// fp8 e4m3 (OCP, gfx950's native format) operand preparation for the fp8 GEMM mode
// (BASELINE.json configs[4]: "fp8 MFMA encoder/decoder GEMMs"): per-tensor scales from the
// absolute maximum and saturating casts.  The GEMM (gemm_fast.hip VAR 8) multiplies the
// quantised operands and rescales its fp32 accumulators by the device scalar these write.
//
//   mlvae_fp8_scale: amax = max |x|; q = 448 / amax (1 when amax == 0 or not finite);
//                    out[0] = q, out[1] = 1 / (q * other_scale)  (the GEMM's alpha)
//   mlvae_cast_fp8:  dst = e4m3(clamp(src * (scale ? *scale : s), -448, 448)), round to nearest
//                    even (v_cvt_pk_fp8_f32); src fp32 or bf16.
// Two-pass amax (per-block partials, then one block): no atomics.
#include "common.h"

namespace {

constexpr int RB = 256;          // threads
constexpr int RBLOCKS = 512;     // first-pass blocks

__global__ __launch_bounds__(RB) void amax_partial_kernel(size_t n, const float* x, float* part) {
  float m = 0.f;
  for (size_t i = (size_t)blockIdx.x * RB + threadIdx.x; i < n; i += (size_t)gridDim.x * RB) {
    const float v = fabsf(x[i]);
    m = v > m ? v : (v != v ? INFINITY : m);  // NaN -> inf: the scale falls back to 1
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  __shared__ float red[RB / 64];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    float r = red[0];
    for (int w = 1; w < RB / 64; ++w) r = fmaxf(r, red[w]);
    part[blockIdx.x] = r;
  }
}

__global__ __launch_bounds__(RB) void amax_final_kernel(int np, const float* part, float other, float* out) {
  float m = 0.f;
  for (int i = threadIdx.x; i < np; i += RB) m = fmaxf(m, part[i]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  __shared__ float red[RB / 64];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    float r = red[0];
    for (int w = 1; w < RB / 64; ++w) r = fmaxf(r, red[w]);
    const float q = (r > 0.f && r < INFINITY) ? E4M3_MAX / r : 1.f;
    out[0] = q;
    out[1] = 1.f / (q * other);
  }
}

template <bool BF>
__global__ __launch_bounds__(RB) void cast_fp8_kernel(size_t n8, const void* src, const float* scale_p, float scale,
                                                       u32x2* dst) {
  const float s = scale_p ? *scale_p : scale;
  for (size_t i = (size_t)blockIdx.x * RB + threadIdx.x; i < n8; i += (size_t)gridDim.x * RB) {
    float v[8];
    if constexpr (BF) {
      const u32x4 w = reinterpret_cast<const u32x4*>(src)[i];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[2 * e] = __uint_as_float(w[e] << 16);
        v[2 * e + 1] = __uint_as_float(w[e] & 0xffff0000u);
      }
    } else {
      const f32x4 a = reinterpret_cast<const f32x4*>(src)[2 * i], b = reinterpret_cast<const f32x4*>(src)[2 * i + 1];
      v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3]; v[4] = b[0]; v[5] = b[1]; v[6] = b[2]; v[7] = b[3];
    }
    dst[i] = u32x2{pack4_fp8(v[0] * s, v[1] * s, v[2] * s, v[3] * s), pack4_fp8(v[4] * s, v[5] * s, v[6] * s, v[7] * s)};
  }
}

// delayed (previous-step) scaling of an operand whose amax a producer kernel max-ed into a word
// as float bits: q = 448 / (margin * amax_prev), 1 without a usable amax; out[1] = the GEMM's
// alpha 1 / (q * other_q); the next step's amax word is cleared for its producer
__global__ void delayed_scale_kernel(const unsigned* amax_prev, unsigned* amax_next, const float* other_q,
                                     float margin, float* out) {
  if (threadIdx.x || blockIdx.x) return;
  const float am = __uint_as_float(*amax_prev) * margin;
  const float q = (am > 0.f && am < INFINITY) ? E4M3_MAX / am : 1.f;
  out[0] = q;
  out[1] = 1.f / (q * *other_q);
  if (amax_next) *amax_next = 0u;
}

int grid_for(size_t n) {
  size_t g = (n + RB - 1) / RB;
  return (int)(g > 4096 ? 4096 : (g < 1 ? 1 : g));
}

}  // namespace

extern "C" size_t mlvae_fp8_scale_workspace_size() { return RBLOCKS * sizeof(float); }

extern "C" int mlvae_fp8_scale(size_t n, const float* x, float other_scale, float* out, float* ws, size_t ws_bytes,
                               void* stream) {
  if (!x || !out || !ws || ws_bytes < mlvae_fp8_scale_workspace_size() || !(other_scale > 0.f)) {
    mlvae_set_error("mlvae_fp8_scale: bad pointer / workspace / scale");
    return 1;
  }
  hipStream_t s = (hipStream_t)stream;
  const int nb = n == 0 ? 1 : (int)((n + RB - 1) / RB < RBLOCKS ? (n + RB - 1) / RB : RBLOCKS);
  hipLaunchKernelGGL(amax_partial_kernel, dim3(nb), dim3(RB), 0, s, n, x, ws);
  MLVAE_CHECK_LAUNCH();
  hipLaunchKernelGGL(amax_final_kernel, dim3(1), dim3(RB), 0, s, nb, ws, other_scale, out);
  MLVAE_CHECK_LAUNCH();
  return 0;
}

extern "C" int mlvae_cast_fp8(size_t n, const void* src, int src_bf16, const float* scale_p, float scale,
                              void* dst, void* stream) {
  if (n == 0) return 0;
  if (!src || !dst || n % 8 || ((uintptr_t)src % 16) || ((uintptr_t)dst % 8)) {
    mlvae_set_error("mlvae_cast_fp8: n %% 8 and 16-byte aligned src / 8-byte aligned dst");
    return 1;
  }
  hipStream_t s = (hipStream_t)stream;
  const size_t n8 = n / 8;
  if (src_bf16)
    hipLaunchKernelGGL(cast_fp8_kernel<true>, dim3(grid_for(n8)), dim3(RB), 0, s, n8, src, scale_p, scale,
                       static_cast<u32x2*>(dst));
  else
    hipLaunchKernelGGL(cast_fp8_kernel<false>, dim3(grid_for(n8)), dim3(RB), 0, s, n8, src, scale_p, scale,
                       static_cast<u32x2*>(dst));
  MLVAE_CHECK_LAUNCH();
  return 0;
}

extern "C" int mlvae_fp8_delayed_scale(const unsigned* amax_prev, unsigned* amax_next, const float* other_q,
                                       float margin, float* out, void* stream) {
  if (!amax_prev || !other_q || !out || !(margin >= 1.f) || amax_prev == amax_next) {
    mlvae_set_error("mlvae_fp8_delayed_scale: amax words (distinct), other scale, out, margin >= 1");
    return 1;
  }
  hipLaunchKernelGGL(delayed_scale_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, amax_prev, amax_next,
                     other_q, margin, out);
  MLVAE_CHECK_LAUNCH();
  return 0;
}
