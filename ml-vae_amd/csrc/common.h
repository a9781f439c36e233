// Shared device helpers for the ML-VAE CDNA4 (gfx950) kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>
#include <stddef.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef int i32x8 __attribute__((ext_vector_type(8)));  // fp8 MFMA operand (32 e4m3 per lane)
typedef int i32x4 __attribute__((ext_vector_type(4)));  // raw buffer-resource words (asm operands)

// Compute precision of a matrix product (operands; accumulation is always fp32).
enum MlvaePrec { PREC_F32 = 0, PREC_BF16 = 1 };

#define MLVAE_NEG_SLOPE 0.01f  // nn.LeakyReLU default (ref:src/modules/fc_block.py:11)

// Record an error string for mlvae_last_error() (capi.cpp).
extern "C" void mlvae_set_error(const char* fmt, ...);

#define MLVAE_CHECK_LAUNCH()                                               \
  do {                                                                     \
    hipError_t e__ = hipGetLastError();                                    \
    if (e__ != hipSuccess) {                                               \
      mlvae_set_error("%s: launch failed: %s", __func__, hipGetErrorString(e__)); \
      return 2;                                                            \
    }                                                                      \
  } while (0)

__device__ __forceinline__ float lrelu(float x) { return x > 0.f ? x : MLVAE_NEG_SLOPE * x; }
__device__ __forceinline__ float lrelu_d(float post) { return post > 0.f ? 1.f : MLVAE_NEG_SLOPE; }
__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + __expf(-x)); }
// sigmoid / tanh on the hardware exp + rcp (|err| ~1e-7): the cell update is on the
// recurrence's serial path
__device__ __forceinline__ float sigmoid_fast(float x) {
  return __builtin_amdgcn_rcpf(1.f + __expf(-x));
}
__device__ __forceinline__ float tanh_fast(float x) {
  // tanh(x) = 1 - 2/(1+e^{2x}); saturates cleanly for |x| large
  return 1.f - 2.f * __builtin_amdgcn_rcpf(1.f + __expf(2.f * x));
}
// The fp32 parity mode's cell math: libm-accurate.  tanh_fast loses relative accuracy near 0
// (1 - 2/(2 + 2x) cancels: |err| ~ 1e-7 absolute, not relative), which made the fp32 mode's
// rnn_out 6x further from fp64 than the fp32 oracle's (round 5, tools/parity_heads_dw1.py).
// (With sigmoid_fast, a few ulp, and libm tanh only, one heads LeakyReLU-derivative flip came
// back at the c3 test seed: both stay libm; the recurrence's time does not change measurably.)
template <int PREC> __device__ __forceinline__ float sigmoid_p(float x) {
  if constexpr (PREC == PREC_F32) return 1.f / (1.f + expf(-x)); else return sigmoid_fast(x);
}
template <int PREC> __device__ __forceinline__ float tanh_p(float x) {
  if constexpr (PREC == PREC_F32) return tanhf(x); else return tanh_fast(x);
}

// bf16 round-to-nearest-even, NaN-preserving (plain cast -> v_cvt_pk_bf16_f32).
__device__ __forceinline__ short f2bf(float x) {
  __hip_bfloat16 h = __float2bfloat16(x);
  return *reinterpret_cast<short*>(&h);
}
// IEEE fp16 (round to nearest even): the wide-batch recurrence's gate buffer G
__device__ __forceinline__ unsigned short f2h(float x) {
  _Float16 h = (_Float16)x;
  return __builtin_bit_cast(unsigned short, h);
}
__device__ __forceinline__ float h2f(unsigned short s) {
  return (float)__builtin_bit_cast(_Float16, s);
}
__device__ __forceinline__ u32x2 f2h4(f32x4 v) {
  return u32x2{(unsigned)f2h(v[0]) | ((unsigned)f2h(v[1]) << 16),
               (unsigned)f2h(v[2]) | ((unsigned)f2h(v[3]) << 16)};
}
__device__ __forceinline__ float bf2f(short s) {
  unsigned u = ((unsigned)(unsigned short)s) << 16;
  return __uint_as_float(u);
}
// the low half of a split-bf16 pair: x ~ bf2f(f2bf(x)) + bf2f(f2bf_lo(x)) to ~2^-17 relative
// (the split forward's operands: a product a_hi b_hi + a_hi b_lo + a_lo b_hi on the bf16 MFMA)
__device__ __forceinline__ short f2bf_lo(float x) {
  return f2bf(x - bf2f(f2bf(x)));
}

// ---- write-through (sc1) hand-off primitives (MI355X_MICROARCH.md "Valid forms" row 1)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, bytes, 0x00020000);
}
__device__ __forceinline__ u32x4 ld_sc1_b128(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16 /*sc1*/);
}
__device__ __forceinline__ void st_sc1_b128(__amdgpu_buffer_rsrc_t r, unsigned off, u32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 16 /*sc1*/);
}
__device__ __forceinline__ void st_sc1_b32(__amdgpu_buffer_rsrc_t r, unsigned off, unsigned v) {
  __builtin_amdgcn_raw_buffer_store_b32(v, r, off, 0, 16 /*sc1*/);
}
__device__ __forceinline__ void st_sc1_b16(__amdgpu_buffer_rsrc_t r, unsigned off, unsigned short v) {
  __builtin_amdgcn_raw_buffer_store_b16(v, r, off, 0, 16 /*sc1*/);
}
__device__ __forceinline__ unsigned ld_flag(const unsigned* p) {
  return __hip_atomic_load(const_cast<unsigned*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_flag(unsigned* p, unsigned v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Number of valid frames of one utterance under SpeechBrain length_to_mask semantics
// (ref:src/utils/data_utils.py:86-87): t valid iff (float)t < fp32(rel_len * T).
__device__ __forceinline__ int valid_frames(float rel_len, int T) {
  float lim = rel_len * (float)T;
  if (!(lim > 0.f)) return 0;
  float c = ceilf(lim);
  return c >= (float)T ? T : (int)c;
}

// Total valid frames for a workgroup: *count when given (data parallel: the all-reduced global
// count), else summed by the whole workgroup -- integers, so exact in any order.  Every thread
// must call it (two barriers); all get the result.  (A single thread walking B lengths serially
// held every workgroup of the heads / encoder-backward kernels for ~128 dependent scalar loads.)
__device__ __forceinline__ int block_frames(const float* lens, int B, int T, const int* count, int* sh) {
  if (count) return *count;
  if (threadIdx.x == 0) *sh = 0;
  __syncthreads();
  int c = 0;
  for (int b = threadIdx.x; b < B; b += blockDim.x) c += valid_frames(lens[b], T);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(sh, c);
  __syncthreads();
  return *sh;
}

// DPP lane move of a float (row_mask = bank_mask = 0xf, bound_ctrl: out-of-row lanes read 0)
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, true));
}

// Wave-level sum (64 lanes) with a fixed butterfly order (deterministic).
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Counter-based Philox-4x32-10 (four 32-bit words per counter), keyed by a 64-bit seed.
__device__ __forceinline__ void philox4(unsigned long long seed, unsigned long long ctr,
                                        unsigned out[4]) {
  unsigned c0 = (unsigned)ctr, c1 = (unsigned)(ctr >> 32), c2 = 0x243F6A88u, c3 = 0x85A308D3u;
  unsigned k0 = (unsigned)seed, k1 = (unsigned)(seed >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const unsigned long long p0 = (unsigned long long)0xD2511F53u * c0;
    const unsigned long long p1 = (unsigned long long)0xCD9E8D57u * c2;
    const unsigned n0 = (unsigned)(p1 >> 32) ^ c1 ^ k0, n2 = (unsigned)(p0 >> 32) ^ c3 ^ k1;
    c0 = n0; c1 = (unsigned)p1; c2 = n2; c3 = (unsigned)p0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

// Inter-layer LSTM dropout mask of flat element i (train mode, ref:src/modules/decoder.py:14):
// keep iff u < 1-p, u = the 16-bit uniform in bits [16 (i & 3), +16) of
//     r(q) = mix64(drop_key(seed) + q * 0x9E3779B97F4A7C15),  q = i >> 2
// (SplitMix64: the generator's output function over a Weyl sequence; 8 32-bit multiplies per
// four elements against Philox-4x32-10's 40, which sat on the forward recurrence's poll path and
// in the dgrad epilogue); kept elements are scaled by 1/(1-p) (nn.Dropout).  The forward (dropout
// kernel / recurrence store path) and the backward (dgrad GEMM epilogue) evaluate the same
// function: no stored mask.  tests/philox_np.py dropout_mask restates it.
__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ unsigned long long drop_key(unsigned long long seed) {
  return mix64(seed ^ 0x6A09E667F3BCC909ull);
}
// the 64 random bits of element quad q under key k = drop_key(seed)
__device__ __forceinline__ unsigned long long drop_quad(unsigned long long k, unsigned long long q) {
  return mix64(k + q * 0x9E3779B97F4A7C15ull);
}
// element e (0..3) of a quad: scale if kept, else 0
__device__ __forceinline__ float drop_elem_scale(unsigned long long r, int e, float keep, float scale) {
  return ((float)((unsigned)(r >> (16 * e)) & 0xffffu) * (1.f / 65536.f)) < keep ? scale : 0.f;
}
__device__ __forceinline__ float dropout_scale(unsigned long long seed, unsigned long long i,
                                               float keep, float scale) {
  return drop_elem_scale(drop_quad(drop_key(seed), i >> 2), (int)(i & 3), keep, scale);
}

// ---- fp8 e4m3 (OCP, gfx950's native format): saturating pack of four floats, round to nearest
// even (v_cvt_pk_fp8_f32).  Shared by the casts (fp8.hip) and the recurrences' fused fp8 outputs.
constexpr float E4M3_MAX = 448.f;
__device__ __forceinline__ unsigned pack4_fp8(float a, float b, float c, float d) {
  a = fminf(fmaxf(a, -E4M3_MAX), E4M3_MAX);
  b = fminf(fmaxf(b, -E4M3_MAX), E4M3_MAX);
  c = fminf(fmaxf(c, -E4M3_MAX), E4M3_MAX);
  d = fminf(fmaxf(d, -E4M3_MAX), E4M3_MAX);
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
  return (unsigned)w;
}

// eight e4m3 (two dwords) -> eight bf16, exactly (every e4m3 value is a bf16 value: 3 of bf16's 7
// mantissa bits, exponents inside its range), through v_cvt_pk_f32_fp8 (OCP, as pack4_fp8)
__device__ __forceinline__ bf16x8 fp8x8_to_bf16(unsigned lo, unsigned hi) {
  const auto a = __builtin_amdgcn_cvt_pk_f32_fp8((int)lo, false), b = __builtin_amdgcn_cvt_pk_f32_fp8((int)lo, true);
  const auto c = __builtin_amdgcn_cvt_pk_f32_fp8((int)hi, false), d = __builtin_amdgcn_cvt_pk_f32_fp8((int)hi, true);
  auto t = [](float x) { return (short)(__float_as_uint(x) >> 16); };
  return bf16x8{t(a[0]), t(a[1]), t(b[0]), t(b[1]), t(c[0]), t(c[1]), t(d[0]), t(d[1])};
}

// Workgroup barrier for LDS reuse only: the LDS operations done, the global stores left in flight.
// (__syncthreads() also waits for every outstanding global store: in the 256-squared GEMM's staged
// epilogue that put four HBM write round trips of the chip-wide store burst into every tile -- the
// projection's per-tile fixed cost was 13.0 us, 2.35 us without the epilogue, tools/gemm_kscan.py.)
// Register data a thread loaded from global memory before the barrier is waited for by the
// compiler's own counted vmcnt where it is used.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}

