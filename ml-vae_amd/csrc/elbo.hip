// ELBO kernels: reparameterisation + KL (encoder side) and Gaussian-NLL / MSE reconstruction
// (decoder side), each fused with its masked partial sums and, in training, its gradient.
//
//   reparameterize   ref:src/modules/vanilla_vae.py:37-40   z = eps * exp(0.5 lv) + mu
//   compute_kld_loss ref:src/modules/vanilla_vae.py:42-45   kl = -0.5 (1 + lv - mu^2 - e^lv)
//   compute_recon    ref:src/modules/decoder.py:37-53       likelihood: 0.5(log2pi + lv + (x-mu)^2/(e^lv+1e-5))
//                                                           mse: (x - mu)^2
//   apply_lens_to_loss ref:src/utils/data_utils.py:67-104   sum(loss*mask)/sum(mask)
//   compute_and_save_losses ref:src/models/md_model.py:189-213 (weights applied in finalize)
//
// Layout: every tensor is row-major [B*T, C] (row n = b*T + t).  Masked sums are reduced per
// block in a fixed order (wave butterfly, then waves in index order) into `partials[block]`;
// `mlvae_elbo_finalize` folds the partials in index order in fp64: deterministic run to run.
#include "common.h"

namespace {

constexpr float LOG_2PI = 1.8378770351409912f;  // fp32(log(2*pi)) as ref:src/modules/decoder.py:42

__device__ float block_sum(float v, float* sm) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) sm[w] = v;
  __syncthreads();
  float s = 0.f;
  if (threadIdx.x == 0)
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) s += sm[i];
  __syncthreads();
  return s;  // valid in thread 0
}

// total valid frames (SpeechBrain fp32 length_to_mask semantics)
__device__ int total_frames(const float* lens, int B, int T) {
  int n = 0;
  for (int b = 0; b < B; ++b) n += valid_frames(lens[b], T);
  return n;
}

__global__ __launch_bounds__(256) void reparam_kl_fwd_kernel(
    int B, int T, int Z, const float* __restrict__ ml, int ldml, const float* __restrict__ eps,
    const float* __restrict__ lens, float* __restrict__ z, float* __restrict__ kl_out,
    float* __restrict__ partials) {
  __shared__ float sm[4];
  const size_t total = (size_t)B * T * Z;
  float acc = 0.f;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (size_t)gridDim.x * 256) {
    const size_t n = i / Z;
    const int k = (int)(i % Z);
    const int b = (int)(n / T), t = (int)(n % T);
    const float mu = ml[n * ldml + k], lv = ml[n * ldml + Z + k];
    const float sd = expf(0.5f * lv);
    z[n * Z + k] = eps[n * Z + k] * sd + mu;
    const float kl = -0.5f * (1.f + lv - mu * mu - expf(lv));
    if (kl_out) kl_out[n * Z + k] = kl;
    if (t < valid_frames(lens[b], T)) acc += kl;
  }
  float s = block_sum(acc, sm);
  if (threadIdx.x == 0 && partials) partials[blockIdx.x] = s;
}

// dml[:, :Z] = dz + s*mu ; dml[:, Z:] = dz*0.5*eps*exp(0.5 lv) + s*0.5*(exp(lv) - 1)
// s = dkl (elementwise upstream grad) or kl_scale * mask / (valid_frames*Z)
__global__ __launch_bounds__(256) void reparam_kl_bwd_kernel(
    int B, int T, int Z, const float* __restrict__ ml, int ldml, const float* __restrict__ eps,
    const float* __restrict__ lens, const int* __restrict__ count, const float* __restrict__ dz,
    const float* __restrict__ dkl, float kl_scale, float* __restrict__ dml, int lddml) {
  __shared__ float inv_count;
  if (threadIdx.x == 0 && !dkl) {  // the mask normaliser is only needed without dkl
    const int c = count ? *count : total_frames(lens, B, T);
    inv_count = c > 0 ? 1.f / ((float)c * (float)Z) : 0.f;
  }
  __syncthreads();
  const size_t total = (size_t)B * T * Z;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (size_t)gridDim.x * 256) {
    const size_t n = i / Z;
    const int k = (int)(i % Z);
    const int b = (int)(n / T), t = (int)(n % T);
    const float mu = ml[n * ldml + k], lv = ml[n * ldml + Z + k];
    float s;
    if (dkl) s = dkl[n * Z + k];
    else s = (t < valid_frames(lens[b], T)) ? kl_scale * inv_count : 0.f;
    const float g = dz ? dz[n * Z + k] : 0.f;
    dml[n * lddml + k] = g + s * mu;
    dml[n * lddml + Z + k] = g * 0.5f * eps[n * Z + k] * expf(0.5f * lv) + s * 0.5f * (expf(lv) - 1.f);
  }
}

// Reconstruction term, its masked partial sums and (optionally) its gradient wrt mu_x, lv_x.
__global__ __launch_bounds__(256) void recon_kernel(
    int B, int T, int F, int loss_type, const float* __restrict__ mux, int ldmu,
    const float* __restrict__ lvx, int ldlv, const float* __restrict__ x, int ldx,
    const float* __restrict__ lens, const int* __restrict__ count, float* __restrict__ rec_out,
    float* __restrict__ partials, const float* __restrict__ drec, float rec_scale,
    float* __restrict__ dmux, float* __restrict__ dlvx) {
  __shared__ float sm[4];
  __shared__ float inv_count;
  if (threadIdx.x == 0 && dmux && !drec) {  // only the fused-gradient mode needs it
    const int c = count ? *count : total_frames(lens, B, T);
    inv_count = c > 0 ? 1.f / ((float)c * (float)F) : 0.f;
  }
  __syncthreads();
  const size_t total = (size_t)B * T * F;
  float acc = 0.f;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (size_t)gridDim.x * 256) {
    const size_t n = i / F;
    const int k = (int)(i % F);
    const int b = (int)(n / T), t = (int)(n % T);
    const bool m = t < valid_frames(lens[b], T);
    const float mu = mux[n * ldmu + k], xv = x[n * ldx + k];
    const float d = xv - mu;
    float r, gmu = 0.f, glv = 0.f;
    if (loss_type == 0) {
      const float lv = lvx[n * ldlv + k];
      const float ev = expf(lv) + 1e-5f;
      r = 0.5f * (LOG_2PI + lv + d * d / ev);
      // dr/dmu = -(x-mu)/ev ; dr/dlv = 0.5 (1 - (x-mu)^2 e^lv / ev^2)
      gmu = -d / ev;
      glv = 0.5f * (1.f - d * d * expf(lv) / (ev * ev));
    } else {
      r = d * d;
      gmu = -2.f * d;
    }
    if (rec_out) rec_out[n * F + k] = r;
    if (m) acc += r;
    if (dmux) {
      const float s = drec ? drec[n * F + k] : (m ? rec_scale * inv_count : 0.f);
      dmux[n * ldmu + k] = s * gmu;
      if (dlvx) dlvx[n * ldlv + k] = s * glv;
    }
  }
  float s = block_sum(acc, sm);
  if (threadIdx.x == 0 && partials) partials[blockIdx.x] = s;
}

// out = [kld_loss, recon_loss, total] = [sum_kl/(cnt*Z), sum_rec/(cnt*F), w_kl*kld + w_rec*rec]
// one 256-thread block; partials folded in a fixed order (strided fp64 + tree): deterministic
__global__ __launch_bounds__(256) void finalize_kernel(const float* pk, int nk, const float* pr,
                                                       int nr, const float* lens, const int* count,
                                                       int B, int T, int Z, int F, float w_kl,
                                                       float w_rec, float* out) {
  __shared__ double sk[256], sr[256];
  __shared__ int sc[256];
  double a = 0.0, b = 0.0;
  int cnt = 0;
  for (int i = threadIdx.x; i < nk; i += 256) a += pk[i];
  for (int i = threadIdx.x; i < nr; i += 256) b += pr[i];
  for (int i = threadIdx.x; i < B; i += 256) cnt += valid_frames(lens[i], T);
  sk[threadIdx.x] = a; sr[threadIdx.x] = b; sc[threadIdx.x] = cnt;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      sk[threadIdx.x] += sk[threadIdx.x + o];
      sr[threadIdx.x] += sr[threadIdx.x + o];
      sc[threadIdx.x] += sc[threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x != 0) return;
  const int c = count ? *count : sc[0];
  const float kld = (float)(sk[0] / ((double)c * Z));
  const float rec = (float)(sr[0] / ((double)c * F));
  out[0] = kld;
  out[1] = rec;
  float tot = 0.f;  // ref:src/models/md_model.py:191-202 accumulates in dict order (kld, recon)
  tot = tot + w_kl * kld;
  tot = tot + w_rec * rec;
  out[2] = tot;
}

// Generic apply_lens_to_loss over a [B,T,C] tensor: reduction 0 mean, 1 batchmean, 2 batch.
__global__ __launch_bounds__(256) void masked_mean_kernel(int B, int T, int C,
                                                          const float* __restrict__ loss,
                                                          const float* __restrict__ lens,
                                                          int reduction, float* __restrict__ out) {
  // one block per utterance; block partial in a fixed order
  __shared__ float sm[4];
  const int b = blockIdx.x;
  const int vf = valid_frames(lens[b], T);
  float acc = 0.f;
  for (int i = threadIdx.x; i < vf * C; i += 256) acc += loss[(size_t)b * T * C + i];
  float s = block_sum(acc, sm);
  if (threadIdx.x == 0) out[B + b] = s;  // scratch: per-utterance sums after the B outputs
  (void)reduction;
}

__global__ void masked_mean_final(int B, int T, int C, const float* lens, int reduction,
                                  float* out) {
  if (threadIdx.x != 0) return;
  if (reduction == 2) {
    for (int b = 0; b < B; ++b) {
      const int vf = valid_frames(lens[b], T);
      out[b] = out[B + b] / (float)(vf * C);
    }
    return;
  }
  double s = 0.0;
  int cnt = 0;
  for (int b = 0; b < B; ++b) { s += out[B + b]; cnt += valid_frames(lens[b], T); }
  out[0] = reduction == 0 ? (float)(s / ((double)cnt * C)) : (float)(s / B);
}

__global__ void count_frames_kernel(const float* lens, int B, int T, int* out) {
  if (threadIdx.x || blockIdx.x) return;
  *out = total_frames(lens, B, T);
}

// Counter-based standard normals: Philox-4x32-10 (common.h) keyed by seed, counter = global
// element index (so a data-parallel shard that passes its global offset draws the same eps as
// one GPU would).
__global__ __launch_bounds__(256) void randn_kernel(size_t n, unsigned long long seed,
                                                    unsigned long long offset, float* out) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    unsigned r[4];
    philox4(seed, offset + i, r);
    const float u1 = ((r[0] >> 8) + 1u) * (1.f / 16777217.f);  // (0, 1]
    const float u2 = (r[1] >> 8) * (1.f / 16777216.f);
    out[i] = sqrtf(-2.f * logf(u1)) * cospif(2.f * u2);
  }
}

int grid_for(size_t total) {
  size_t g = (total + 255) / 256;
  if (g > 1024) g = 1024;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace

extern "C" int mlvae_elbo_partials_count(int B, int T, int C) { return grid_for((size_t)B * T * C); }

extern "C" int mlvae_reparam_kl_fwd(int B, int T, int Z, const float* ml, int ldml,
                                    const float* eps, const float* lens, float* z, float* kl_out,
                                    float* partials, void* stream) {
  if (B * T * Z == 0) return 0;
  if (!ml || !eps || !lens || !z) { mlvae_set_error("reparam_kl_fwd: null pointer"); return 1; }
  reparam_kl_fwd_kernel<<<grid_for((size_t)B * T * Z), 256, 0, (hipStream_t)stream>>>(
      B, T, Z, ml, ldml, eps, lens, z, kl_out, partials);
  MLVAE_CHECK_LAUNCH();
  return 0;
}

extern "C" int mlvae_reparam_kl_bwd(int B, int T, int Z, const float* ml, int ldml,
                                    const float* eps, const float* lens, const int* count,
                                    const float* dz, const float* dkl, float kl_scale, float* dml,
                                    int lddml, void* stream) {
  if (B * T * Z == 0) return 0;
  if (!ml || !eps || !lens || !dml) { mlvae_set_error("reparam_kl_bwd: null pointer"); return 1; }
  reparam_kl_bwd_kernel<<<grid_for((size_t)B * T * Z), 256, 0, (hipStream_t)stream>>>(
      B, T, Z, ml, ldml, eps, lens, count, dz, dkl, kl_scale, dml, lddml);
  MLVAE_CHECK_LAUNCH();
  return 0;
}

extern "C" int mlvae_recon(int B, int T, int F, int loss_type, const float* mux, int ldmu,
                           const float* lvx, int ldlv, const float* x, int ldx, const float* lens,
                           const int* count, float* rec_out, float* partials, const float* drec,
                           float rec_scale, float* dmux, float* dlvx, void* stream) {
  if (B * T * F == 0) return 0;
  if (loss_type != 0 && loss_type != 1) { mlvae_set_error("Invalid loss type: %d", loss_type); return 1; }
  if (!mux || !x || !lens || (loss_type == 0 && !lvx)) { mlvae_set_error("recon: null pointer"); return 1; }
  recon_kernel<<<grid_for((size_t)B * T * F), 256, 0, (hipStream_t)stream>>>(
      B, T, F, loss_type, mux, ldmu, lvx, ldlv, x, ldx, lens, count, rec_out, partials, drec,
      rec_scale, dmux, dlvx);
  MLVAE_CHECK_LAUNCH();
  return 0;
}

extern "C" int mlvae_elbo_finalize(const float* pk, int nk, const float* pr, int nr,
                                   const float* lens, const int* count, int B, int T, int Z, int F,
                                   float w_kl, float w_rec, float* out, void* stream) {
  finalize_kernel<<<1, 256, 0, (hipStream_t)stream>>>(pk, nk, pr, nr, lens, count, B, T, Z, F,
                                                     w_kl, w_rec, out);
  MLVAE_CHECK_LAUNCH();
  return 0;
}

// out must hold 2*B floats (first B: results; next B: scratch)
extern "C" int mlvae_masked_mean(int B, int T, int C, const float* loss, const float* lens,
                                 int reduction, float* out, void* stream) {
  if (reduction < 0 || reduction > 2) { mlvae_set_error("masked_mean: bad reduction"); return 1; }
  if (B == 0) return 0;
  masked_mean_kernel<<<B, 256, 0, (hipStream_t)stream>>>(B, T, C, loss, lens, reduction, out);
  masked_mean_final<<<1, 64, 0, (hipStream_t)stream>>>(B, T, C, lens, reduction, out);
  MLVAE_CHECK_LAUNCH();
  return 0;
}

extern "C" int mlvae_count_frames(const float* lens, int B, int T, int* out, void* stream) {
  count_frames_kernel<<<1, 64, 0, (hipStream_t)stream>>>(lens, B, T, out);
  MLVAE_CHECK_LAUNCH();
  return 0;
}

extern "C" int mlvae_randn(size_t n, unsigned long long seed, unsigned long long offset, float* out,
                           void* stream) {
  if (n == 0) return 0;
  size_t g = (n + 255) / 256;
  if (g > 2048) g = 2048;
  randn_kernel<<<(int)g, 256, 0, (hipStream_t)stream>>>(n, seed, offset, out);
  MLVAE_CHECK_LAUNCH();
  return 0;
}

// ---- autograd helpers for the module-level (drop-in nn.Module) path -------------------------
__global__ __launch_bounds__(256) void lrelu_bwd_kernel(size_t n, const float* __restrict__ dy,
                                                        const float* __restrict__ y,
                                                        float* __restrict__ dx) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    dx[i] = dy[i] * lrelu_d(y[i]);
}

// d/dloss of apply_lens_to_loss: dloss[b,t,c] = g * mask / denom  (reduction mean/batchmean)
// or g[b] * mask / (valid_b * C) (batch); g = upstream grad (1 or B floats, device)
__global__ __launch_bounds__(256) void masked_mean_bwd_kernel(int B, int T, int C,
                                                              const float* __restrict__ lens,
                                                              int reduction,
                                                              const float* __restrict__ g,
                                                              float* __restrict__ dloss) {
  __shared__ int cnt_sh;
  const int cnt = block_frames(lens, B, T, nullptr, &cnt_sh);
  const size_t total = (size_t)B * T * C;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (size_t)gridDim.x * 256) {
    const int b = (int)(i / ((size_t)T * C)), t = (int)((i / C) % T);
    const int vf = valid_frames(lens[b], T);
    float v = 0.f;
    if (t < vf) {
      if (reduction == 0) v = g[0] / ((float)cnt * C);
      else if (reduction == 1) v = g[0] / (float)B;
      else v = g[b] / ((float)vf * C);
    }
    dloss[i] = v;
  }
}

extern "C" int mlvae_lrelu_bwd(size_t n, const float* dy, const float* y, float* dx, void* stream) {
  if (n == 0) return 0;
  lrelu_bwd_kernel<<<grid_for(n), 256, 0, (hipStream_t)stream>>>(n, dy, y, dx);
  MLVAE_CHECK_LAUNCH();
  return 0;
}

extern "C" int mlvae_masked_mean_bwd(int B, int T, int C, const float* lens, int reduction,
                                     const float* g, float* dloss, void* stream) {
  if ((size_t)B * T * C == 0) return 0;
  if (reduction < 0 || reduction > 2) { mlvae_set_error("masked_mean_bwd: bad reduction"); return 1; }
  masked_mean_bwd_kernel<<<grid_for((size_t)B * T * C), 256, 0, (hipStream_t)stream>>>(
      B, T, C, lens, reduction, g, dloss);
  MLVAE_CHECK_LAUNCH();
  return 0;
}
