// InputNormalization(norm_type='global') inside the fused train step.
//
// Reference: SpeechBrain's InputNormalization (un-vendored, SpeechBrain 0.5 semantics; parity
// unpinned), built at ref:src/models/test_vanilla_vae/model.yaml:14-15 and called on every batch
// at ref:src/models/test_vanilla_vae/model.py:24-25, before the encoder.  Restated host-side in
// brain/features.py (the checker of these kernels):
//   n_b      = round(rel_len_b * T) frames of utterance b
//   mean_b   = sum_{t<n_b} x[b,t,:] / n_b,  std_b = max(sqrt(sum (x - mean_b)^2 / (n_b - 1)), eps)
//   cur      = average of mean_b / std_b over the utterances with n_b > 0 (all ranks: the sums
//              and the count are what a data-parallel run all-reduces)
//   global   = cur (first batch) | (1 - w) global + w cur (training, epoch < update_until_epoch)
//   out      = (x - global_mean) / global_std
//
// Three launches, all HBM-streaming, deterministic (fixed-order reductions, no atomics):
//   norm_stats_kernel   one workgroup per utterance, two passes over its rows (the second
//                       re-reads them from L2): per-utterance mean / std
//   norm_sums_kernel    one workgroup: the fixed-order sums over utterances + the count
//   norm_update_kernel  one workgroup: set / running-average update of the global statistics
//   norm_apply_kernel   grid-stride, 16-byte accesses: out = (x - mean) / std
#include "common.h"

namespace {

constexpr int NT = 256;

__device__ __forceinline__ int norm_frames(float rel, int T) {
  // torch.round(lengths * T): fp32 product, round half to even
  const float n = rintf(rel * (float)T);
  return n <= 0.f ? 0 : (n >= (float)T ? T : (int)n);
}

// block = one utterance; thread (rl, q): column quad q (4 features), row lane rl
__global__ __launch_bounds__(NT) void norm_stats_kernel(int T, int F, const float* __restrict__ x,
                                                        const float* __restrict__ lens,
                                                        float* __restrict__ stats, float eps) {
  extern __shared__ f32x4 red[];  // [RL][FQ]
  const int b = blockIdx.x, FQ = F / 4, RL = NT / FQ;
  const int q = threadIdx.x % FQ, rl = threadIdx.x / FQ;
  const int n = norm_frames(lens[b], T);
  const f32x4* xb = reinterpret_cast<const f32x4*>(x + (size_t)b * T * F);
  const bool act = rl < RL;
  // four independent rows in flight per thread (a dependent load per row would make the
  // pass latency-bound: ~40 HBM round trips per thread at T = 500)
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  if (act) {
    int r = rl;
    for (; r + 3 * RL < n; r += 4 * RL) {
      const f32x4 a0 = xb[(size_t)r * FQ + q], a1 = xb[(size_t)(r + RL) * FQ + q];
      const f32x4 a2 = xb[(size_t)(r + 2 * RL) * FQ + q], a3 = xb[(size_t)(r + 3 * RL) * FQ + q];
      s += a0; s += a1; s += a2; s += a3;
    }
    for (; r < n; r += RL) s += xb[(size_t)r * FQ + q];
    red[rl * FQ + q] = s;
  }
  __syncthreads();
  f32x4 mean = {0.f, 0.f, 0.f, 0.f};
  if (n > 0) {
    f32x4 t = red[q];
    for (int i = 1; i < RL; ++i) t += red[i * FQ + q];
    mean = t / (float)n;
  }
  __syncthreads();
  f32x4 v = {0.f, 0.f, 0.f, 0.f};
  if (act) {
    int r = rl;
    for (; r + 3 * RL < n; r += 4 * RL) {
      const f32x4 d0 = xb[(size_t)r * FQ + q] - mean, d1 = xb[(size_t)(r + RL) * FQ + q] - mean;
      const f32x4 d2 = xb[(size_t)(r + 2 * RL) * FQ + q] - mean, d3 = xb[(size_t)(r + 3 * RL) * FQ + q] - mean;
      v += d0 * d0; v += d1 * d1; v += d2 * d2; v += d3 * d3;
    }
    for (; r < n; r += RL) {
      const f32x4 d = xb[(size_t)r * FQ + q] - mean;
      v += d * d;
    }
    red[rl * FQ + q] = v;
  }
  __syncthreads();
  if (rl == 0) {
    f32x4 t = red[q];
    for (int i = 1; i < RL; ++i) t += red[i * FQ + q];
    f32x4 sd;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float var = t[e] / (float)(n - 1);
      const float st = sqrtf(var);
      sd[e] = n > 0 ? (st < eps ? eps : st) : 0.f;  // clamp(min=eps); a NaN (n = 1) propagates
    }
    float* o = stats + (size_t)b * 2 * F;
    *reinterpret_cast<f32x4*>(o + 4 * q) = mean;
    *reinterpret_cast<f32x4*>(o + F + 4 * q) = sd;
  }
}

// sums[f] = sum_b valid_b stats[b][f] (f < 2F), sums[2F] = number of valid utterances.  Block =
// 64 columns x 4 utterance lanes (lane l sums b = l, l + 4, ... with four loads in flight), the
// four lane sums folded in a fixed order: deterministic, and no 256-long dependent load chain
// (one thread per column walking every utterance took 80 us at B = 256).
__global__ __launch_bounds__(NT) void norm_sums_kernel(int B, int T, int F, const float* __restrict__ lens,
                                                       const float* __restrict__ stats,
                                                       float* __restrict__ sums) {
  __shared__ float red[4][64];
  const int c = threadIdx.x & 63, lb = threadIdx.x >> 6, f = blockIdx.x * 64 + c;
  float s = 0.f;
  if (f <= 2 * F) {
    int b = lb;
    for (; b + 12 < B; b += 16) {
      float v[4], m[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        m[i] = norm_frames(lens[b + 4 * i], T) > 0 ? 1.f : 0.f;
        v[i] = f < 2 * F ? stats[(size_t)(b + 4 * i) * 2 * F + f] : 1.f;
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) s += m[i] * v[i];
    }
    for (; b < B; b += 4)
      if (norm_frames(lens[b], T) > 0) s += f < 2 * F ? stats[(size_t)b * 2 * F + f] : 1.f;
  }
  red[lb][c] = s;
  __syncthreads();
  if (lb == 0 && f <= 2 * F) sums[f] = ((red[0][c] + red[1][c]) + red[2][c]) + red[3][c];
}

// mode 0: keep; 1: set to the batch's; 2: global = (1 - w) global + w cur
__global__ __launch_bounds__(NT) void norm_update_kernel(int F, const float* __restrict__ sums,
                                                         float* __restrict__ gmean, float* __restrict__ gstd,
                                                         int mode, float w1, float w) {
  const float cnt = sums[2 * F] > 0.f ? sums[2 * F] : 1.f;
  for (int f = threadIdx.x; f < F; f += NT) {
    const float cm = sums[f] / cnt, cs = sums[F + f] / cnt;
    if (mode == 1) { gmean[f] = cm; gstd[f] = cs; }
    else if (mode == 2) { gmean[f] = w1 * gmean[f] + w * cm; gstd[f] = w1 * gstd[f] + w * cs; }
  }
}

__global__ __launch_bounds__(NT) void norm_apply_kernel(size_t nq, int FQ, const f32x4* __restrict__ x,
                                                        const float* __restrict__ gmean,
                                                        const float* __restrict__ gstd,
                                                        f32x4* __restrict__ out) {
  for (size_t i = (size_t)blockIdx.x * NT + threadIdx.x; i < nq; i += (size_t)gridDim.x * NT) {
    const int q = (int)(i % FQ);
    const f32x4 m = *reinterpret_cast<const f32x4*>(gmean + 4 * q);
    const f32x4 s = *reinterpret_cast<const f32x4*>(gstd + 4 * q);
    out[i] = (x[i] - m) / s;  // (x - mean) / std: the restatement's two fp32 ops, IEEE division
  }
}

}  // namespace

extern "C" int mlvae_norm_supported(int F) { return F > 0 && F % 4 == 0 && F / 4 <= NT; }

extern "C" int mlvae_norm_stats(int B, int T, int F, const float* x, const float* rel_lens,
                                float* utt_stats, float* sums, float eps, void* stream) {
  if (!mlvae_norm_supported(F) || B <= 0 || T <= 0) {
    mlvae_set_error("norm_stats: B=%d T=%d F=%d unsupported (F %% 4 == 0, F <= 1024)", B, T, F);
    return 1;
  }
  if (((uintptr_t)x | (uintptr_t)utt_stats) & 15) {
    mlvae_set_error("norm_stats: x / utt_stats must be 16-byte aligned");
    return 1;
  }
  hipStream_t s = (hipStream_t)stream;
  const int FQ = F / 4, RL = NT / FQ;
  norm_stats_kernel<<<B, NT, (size_t)RL * FQ * sizeof(f32x4), s>>>(T, F, x, rel_lens, utt_stats, eps);
  norm_sums_kernel<<<(2 * F + 1 + 63) / 64, NT, 0, s>>>(B, T, F, rel_lens, utt_stats, sums);
  MLVAE_CHECK_LAUNCH();
  return 0;
}

// w_old / w_new: the weights (1 - w) and w as the host computes them (fp32 casts of its doubles)
extern "C" int mlvae_norm_update(int F, const float* sums, float* glob_mean, float* glob_std, int mode,
                                 float w_old, float w_new, void* stream) {
  if (mode < 0 || mode > 2) { mlvae_set_error("norm_update: mode %d", mode); return 1; }
  if (mode == 0) return 0;
  norm_update_kernel<<<1, NT, 0, (hipStream_t)stream>>>(F, sums, glob_mean, glob_std, mode, w_old, w_new);
  MLVAE_CHECK_LAUNCH();
  return 0;
}

extern "C" int mlvae_norm_apply(size_t rows, int F, const float* x, const float* glob_mean,
                                const float* glob_std, float* out, void* stream) {
  if (!mlvae_norm_supported(F)) { mlvae_set_error("norm_apply: F=%d unsupported", F); return 1; }
  if (((uintptr_t)x | (uintptr_t)out | (uintptr_t)glob_mean | (uintptr_t)glob_std) & 15) {
    mlvae_set_error("norm_apply: buffers must be 16-byte aligned");
    return 1;
  }
  const size_t nq = rows * (size_t)(F / 4);
  size_t g = (nq + NT - 1) / NT;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  norm_apply_kernel<<<(unsigned)g, NT, 0, (hipStream_t)stream>>>(
      nq, F / 4, reinterpret_cast<const f32x4*>(x), glob_mean, glob_std, reinterpret_cast<f32x4*>(out));
  MLVAE_CHECK_LAUNCH();
  return 0;
}
