// GMM-VAE latent block and the mixture weighting of the Hierarchical VAE.
//
//   GMMVAE.forward           ref:src/modules/gmm_vae.py:24-48
//     gumbel_softmax(tau=0.1, hard=True)  ref:src/modules/gmm_vae.py:31 (straight-through)
//   GMMVAE.reparameterize    ref:src/modules/gmm_vae.py:50-55   z = eps * exp(0.5 lv) + m
//   GMMVAE.compute_kld_loss  ref:src/modules/gmm_vae.py:57-67
//     kl = -0.5 (1 + lv - plv - (e^lv + (m - pm)^2) / (e^plv + 1e-5))
//   apply_weight             ref:src/utils/data_utils.py:32-64  y[r,c] = sum_n w[r,n] x[r,n*C+c]
//
// Layout.  The five heads of GMMVAE are ONE stacked GEMM output P, row-major [rows, ldp] with
// columns [prior_mean | prior_log_var | mean | log_var] (N*Z each) then the N gmm logits.
// Every kernel here is an HBM-streaming elementwise pass (no reuse to stage in LDS): consecutive
// lanes take consecutive columns of a row, so each wave's loads and stores are coalesced.
#include "common.h"

namespace {

struct GmmArgs {
  int rows, N, Z, ldp;
  const float* P;
  const float* eps;    // [rows, N*Z]
  const float* expo;   // [rows, N] Exp(1) draws, or NULL: Philox(seed, offset + r*N + n)
  unsigned long long seed, offset;
  float tau;
  float* z;            // [rows, N*Z]
  float* kl;           // [rows, N*Z]
  float* w;            // [rows, N]  straight-through hard weights
  float* ysoft;        // [rows, N]  softmax((logits + g) / tau), kept for the backward
  // backward
  const float* dz;     // NULL = 0
  const float* dkl;    // NULL = 0
  const float* dw;     // NULL = 0
  float* dP;           // [rows, lddp] same column layout as P
  int lddp;
};

constexpr int GMM_MAX_N = 64;

// Exp(1) sample as torch's exponential_: -log(u), u in (0, 1) (strictly positive, finite)
__device__ __forceinline__ float exp1(unsigned long long seed, unsigned long long i) {
  unsigned r[4];
  philox4(seed, i, r);
  const float u = ((float)(r[0] >> 8) + 0.5f) * (1.f / 16777216.f);
  return -logf(u);
}

__global__ __launch_bounds__(256) void gmm_latent_fwd_kernel(GmmArgs a) {
  const int NZ = a.N * a.Z;
  const size_t total = (size_t)a.rows * NZ;
  const size_t stride = (size_t)gridDim.x * 256;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < total; i += stride) {
    const size_t r = i / NZ;
    const int k = (int)(i % NZ);
    const float* p = a.P + r * a.ldp;
    const float pm = p[k], plv = p[NZ + k], m = p[2 * NZ + k], lv = p[3 * NZ + k];
    a.z[i] = a.eps[i] * expf(0.5f * lv) + m;
    const float d = m - pm;
    a.kl[i] = -0.5f * (1.f + lv - plv - (expf(lv) + d * d) / (expf(plv) + 1e-5f));
  }
  // Gumbel-softmax, one thread per row (N is the number of mixture components: small)
  for (size_t r = (size_t)blockIdx.x * 256 + threadIdx.x; r < (size_t)a.rows; r += stride) {
    const float* lg = a.P + r * a.ldp + 4 * NZ;
    float u[GMM_MAX_N];
    float mx = -INFINITY;
    int arg = 0;
    for (int n = 0; n < a.N; ++n) {
      const float e = a.expo ? a.expo[r * a.N + n] : exp1(a.seed, a.offset + r * a.N + n);
      u[n] = (lg[n] + -logf(e)) / a.tau;
      if (u[n] > mx) mx = u[n];
    }
    float s = 0.f;
    for (int n = 0; n < a.N; ++n) { u[n] = expf(u[n] - mx); s += u[n]; }
    float best = -1.f;
    for (int n = 0; n < a.N; ++n) {
      u[n] = u[n] / s;
      if (u[n] > best) { best = u[n]; arg = n; }  // first maximum, as torch.max
    }
    for (int n = 0; n < a.N; ++n) {
      const float hard = n == arg ? 1.f : 0.f;
      a.w[r * a.N + n] = (hard - u[n]) + u[n];
      a.ysoft[r * a.N + n] = u[n];
    }
  }
}

__global__ __launch_bounds__(256) void gmm_latent_bwd_kernel(GmmArgs a) {
  const int NZ = a.N * a.Z;
  const size_t total = (size_t)a.rows * NZ;
  const size_t stride = (size_t)gridDim.x * 256;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < total; i += stride) {
    const size_t r = i / NZ;
    const int k = (int)(i % NZ);
    const float* p = a.P + r * a.ldp;
    const float pm = p[k], plv = p[NZ + k], m = p[2 * NZ + k], lv = p[3 * NZ + k];
    const float g = a.dz ? a.dz[i] : 0.f, s = a.dkl ? a.dkl[i] : 0.f;
    const float D = expf(plv) + 1e-5f, ev = expf(lv), d = m - pm;
    float* q = a.dP + r * a.lddp;
    q[k] = -s * d / D;                                        // d/d prior_mean
    q[NZ + k] = s * 0.5f * (1.f - (ev + d * d) * expf(plv) / (D * D));  // d/d prior_log_var
    q[2 * NZ + k] = g + s * d / D;                            // d/d mean
    q[3 * NZ + k] = g * 0.5f * a.eps[i] * expf(0.5f * lv) - s * 0.5f * (1.f - ev / D);  // d/d lv
  }
  // straight-through Gumbel-softmax: the gradient flows through y_soft only
  for (size_t r = (size_t)blockIdx.x * 256 + threadIdx.x; r < (size_t)a.rows; r += stride) {
    const float* y = a.ysoft + r * a.N;
    float* q = a.dP + r * a.lddp + 4 * NZ;
    float sg = 0.f;
    for (int n = 0; n < a.N; ++n) sg += (a.dw ? a.dw[r * a.N + n] : 0.f) * y[n];
    for (int n = 0; n < a.N; ++n)
      q[n] = y[n] * ((a.dw ? a.dw[r * a.N + n] : 0.f) - sg) / a.tau;
  }
}

// y[r, c] = sum_n w[r, n] x[r, n*C + c]
__global__ __launch_bounds__(256) void apply_weight_fwd_kernel(int rows, int N, int C,
                                                               const float* __restrict__ x, int ldx,
                                                               const float* __restrict__ w,
                                                               float* __restrict__ y, int ldy) {
  const size_t total = (size_t)rows * C;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (size_t)gridDim.x * 256) {
    const size_t r = i / C;
    const int c = (int)(i % C);
    const float* xr = x + r * ldx + c;
    const float* wr = w + r * N;
    float acc = 0.f;
    for (int n = 0; n < N; ++n) acc += wr[n] * xr[(size_t)n * C];
    y[r * ldy + c] = acc;
  }
}

// dx[r, n*C + c] = w[r, n] dy[r, c];  dw[r, n] = sum_c dy[r, c] x[r, n*C + c]
// one wave per row: lanes over c, a wave reduction per component
__global__ __launch_bounds__(256) void apply_weight_bwd_kernel(int rows, int N, int C,
                                                               const float* __restrict__ x, int ldx,
                                                               const float* __restrict__ w,
                                                               const float* __restrict__ dy, int lddy,
                                                               float* __restrict__ dx, int lddx,
                                                               float* __restrict__ dw) {
  const int lane = threadIdx.x & 63;
  const size_t nw = (size_t)gridDim.x * 4;
  for (size_t r = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < (size_t)rows; r += nw) {
    for (int n = 0; n < N; ++n) {
      const float wn = w[r * N + n];
      float acc = 0.f;
      for (int c = lane; c < C; c += 64) {
        const float g = dy[r * lddy + c];
        if (x) acc += g * x[r * ldx + (size_t)n * C + c];
        if (dx) dx[r * lddx + (size_t)n * C + c] = wn * g;
      }
      if (dw) {
        acc = wave_sum(acc);
        if (lane == 0) dw[r * N + n] = acc;
      }
    }
  }
}

int grid_of(size_t total, int per_block = 256) {
  size_t g = (total + per_block - 1) / per_block;
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace

extern "C" int mlvae_gmm_latent_fwd(int rows, int N, int Z, const float* P, int ldp,
                                    const float* eps, const float* expo, unsigned long long seed,
                                    unsigned long long offset, float tau, float* z, float* kl,
                                    float* w, float* ysoft, void* stream) {
  if (rows < 0 || N < 1 || N > GMM_MAX_N || Z < 1 || ldp < 4 * N * Z + N) {
    mlvae_set_error("gmm_latent_fwd: bad shape rows=%d N=%d Z=%d ldp=%d", rows, N, Z, ldp);
    return 1;
  }
  if (!P || !eps || !z || !kl || !w || !ysoft) { mlvae_set_error("gmm_latent_fwd: null pointer"); return 1; }
  if (rows == 0) return 0;
  GmmArgs a{};
  a.rows = rows; a.N = N; a.Z = Z; a.ldp = ldp; a.P = P; a.eps = eps; a.expo = expo;
  a.seed = seed; a.offset = offset; a.tau = tau; a.z = z; a.kl = kl; a.w = w; a.ysoft = ysoft;
  gmm_latent_fwd_kernel<<<grid_of((size_t)rows * N * Z), 256, 0, (hipStream_t)stream>>>(a);
  MLVAE_CHECK_LAUNCH();
  return 0;
}

extern "C" int mlvae_gmm_latent_bwd(int rows, int N, int Z, const float* P, int ldp,
                                    const float* eps, const float* ysoft, float tau,
                                    const float* dz, const float* dkl, const float* dw, float* dP,
                                    int lddp, void* stream) {
  if (rows < 0 || N < 1 || N > GMM_MAX_N || Z < 1 || ldp < 4 * N * Z + N || lddp < 4 * N * Z + N) {
    mlvae_set_error("gmm_latent_bwd: bad shape rows=%d N=%d Z=%d ldp=%d lddp=%d", rows, N, Z, ldp, lddp);
    return 1;
  }
  if (!P || !eps || !ysoft || !dP) { mlvae_set_error("gmm_latent_bwd: null pointer"); return 1; }
  if (rows == 0) return 0;
  GmmArgs a{};
  a.rows = rows; a.N = N; a.Z = Z; a.ldp = ldp; a.P = P; a.eps = eps; a.ysoft = const_cast<float*>(ysoft);
  a.tau = tau; a.dz = dz; a.dkl = dkl; a.dw = dw; a.dP = dP; a.lddp = lddp;
  gmm_latent_bwd_kernel<<<grid_of((size_t)rows * N * Z), 256, 0, (hipStream_t)stream>>>(a);
  MLVAE_CHECK_LAUNCH();
  return 0;
}

extern "C" int mlvae_apply_weight_fwd(int rows, int N, int C, const float* x, int ldx,
                                      const float* w, float* y, int ldy, void* stream) {
  if (rows < 0 || N < 1 || C < 1 || ldx < N * C || ldy < C) {
    mlvae_set_error("apply_weight_fwd: bad shape rows=%d N=%d C=%d", rows, N, C);
    return 1;
  }
  if (!x || !w || !y) { mlvae_set_error("apply_weight_fwd: null pointer"); return 1; }
  if (rows == 0) return 0;
  apply_weight_fwd_kernel<<<grid_of((size_t)rows * C), 256, 0, (hipStream_t)stream>>>(
      rows, N, C, x, ldx, w, y, ldy);
  MLVAE_CHECK_LAUNCH();
  return 0;
}

extern "C" int mlvae_apply_weight_bwd(int rows, int N, int C, const float* x, int ldx,
                                      const float* w, const float* dy, int lddy, float* dx,
                                      int lddx, float* dw, void* stream) {
  if (rows < 0 || N < 1 || C < 1 || ldx < N * C || lddy < C || (dx && lddx < N * C)) {
    mlvae_set_error("apply_weight_bwd: bad shape rows=%d N=%d C=%d", rows, N, C);
    return 1;
  }
  if (!w || !dy || (dw && !x)) { mlvae_set_error("apply_weight_bwd: null pointer"); return 1; }
  if (rows == 0) return 0;
  apply_weight_bwd_kernel<<<grid_of((size_t)rows, 4), 256, 0, (hipStream_t)stream>>>(
      rows, N, C, x, ldx, w, dy, lddy, dx, lddx, dw);
  MLVAE_CHECK_LAUNCH();
  return 0;
}
