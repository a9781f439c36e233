// MD-VAE upstream-LSTM losses on gfx950.
//
//   phn_bce_kernel       PhonemeRecognizer.compute_losses (ref:src/modules/phoneme_recognizer.py:35-81):
//                        BCE-with-logits of the recogniser's [B,T,C] output against the canonical
//                        phoneme sequence expanded by the forced-alignment boundaries, and its
//                        gradient.  The reference loops over utterances on the host (a
//                        torch.where(...).tolist() sync per utterance); here one workgroup per
//                        utterance scans the boundary flags (block prefix sum) so frame t reads
//                        phoneme (boundaries in [0, t]) - 1 -- the same repeat_interleave
//                        expansion -- with no host round trip.  The reference's asserts
//                        (boundary count == L_i, sum of durations == T_i) become bits of a device
//                        error word the caller checks at its next sync.
//   boundary_fwd/bwd     BoundaryDetector after its two FC heads (ref:src/modules/boundary_detector.py:
//                        42-86): alpha, beta = Softplus(head) + 1e-5, KL(Beta(alpha, beta) ||
//                        Beta(1, 9)), ten Kumaraswamy draws v = (1 - u^(1/beta))^(1/alpha) (u =
//                        0.01 + 0.98 U(0,1): injected, or Philox keyed by element index), their
//                        mean and mean BCE; the backward gives d/d(head outputs) in closed form
//                        (trigamma for the KL, the Kumaraswamy chain rule for the draws).
// Both are elementwise / per-utterance HBM passes over [B,T,C] or [B,T] (bytes below).
#include "common.h"

namespace {

// ---- phoneme-recogniser BCE ----------------------------------------------------------------
constexpr int PB = 256;  // frames per scan chunk = threads

__device__ __forceinline__ float bce_logits(float x, float y) {
  // torch binary_cross_entropy_with_logits (no weights): (1-y) x + m + log(e^-m + e^(-x-m)), m = max(-x, 0)
  const float m = fmaxf(-x, 0.f);
  return (1.f - y) * x + m + logf(expf(-m) + expf(-x - m));
}

__global__ __launch_bounds__(PB) void phn_bce_kernel(int T, int C, const float* __restrict__ logits, int ldl,
                                                     const float* __restrict__ feat_lens,
                                                     const long long* __restrict__ phn, int L,
                                                     const float* __restrict__ phn_lens,
                                                     const float* __restrict__ boundary,
                                                     float* __restrict__ loss,
                                                     const float* __restrict__ dloss,
                                                     float* __restrict__ dlogits, int* err) {
  __shared__ int cls[PB];
  __shared__ int wsum[PB / 64];
  __shared__ int carry_s;
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // torch.round(T * rel).int(): fp32 product, round half to even
  int Ti = (int)rintf((float)T * feat_lens[b]);
  Ti = Ti < 0 ? 0 : (Ti > T ? T : Ti);
  const int Li = (int)rintf((float)L * phn_lens[b]);
  if (tid == 0) carry_s = 0;
  __syncthreads();
  int bad = 0;
  for (int t0 = 0; t0 < T; t0 += PB) {
    const int t = t0 + tid;
    const int f = (t < Ti && boundary[(size_t)b * T + t] == 1.f) ? 1 : 0;
    // inclusive block scan of the boundary flags
    int v = f;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int u = __shfl_up(v, o, 64);
      if (lane >= o) v += u;
    }
    if (lane == 63) wsum[wave] = v;
    __syncthreads();
    int pre = carry_s;
    for (int w = 0; w < wave; ++w) pre += wsum[w];
    const int idx = pre + v - 1;  // position of this frame's phoneme in the canonical sequence
    int c = -1;
    if (t < Ti) {
      if (idx < 0 || idx >= Li || idx >= L) {
        bad |= 2;  // no boundary at frame 0, or more boundaries than phonemes
      } else {
        const long long p = phn[(size_t)b * L + idx];
        if (p < 0 || p >= C) bad |= 4;  // one_hot(num_classes = C) would raise
        else c = (int)p;
      }
    }
    cls[tid] = c;
    __syncthreads();
    if (tid == 0) {
      int tot = 0;
      for (int w = 0; w < PB / 64; ++w) tot += wsum[w];
      carry_s += tot;
    }
    const int nf = min(PB, T - t0);
    for (int e = tid; e < nf * C; e += PB) {
      const int tt = e / C, cc = e % C, tf = t0 + tt;
      const size_t row = (size_t)b * T + tf;
      const int k = cls[tt];
      const float x = logits[row * ldl + cc];
      const float y = k == cc ? 1.f : 0.f;
      if (loss) loss[row * C + cc] = k >= 0 ? bce_logits(x, y) : 0.f;
      if (dlogits) {
        const float s = 1.f / (1.f + expf(-x));
        dlogits[row * C + cc] = k >= 0 ? dloss[row * C + cc] * (s - y) : 0.f;
      }
    }
    __syncthreads();  // cls / wsum / carry reused by the next chunk
  }
  if (tid == 0 && carry_s != Li) bad |= 2;  // boundary count != L_i (phoneme_recognizer.py:65)
  if (bad) atomicOr(err, bad);
}

// ---- boundary detector heads -----------------------------------------------------------------
constexpr float PRIOR_A = 1.f, PRIOR_B = 9.f;  // ref:src/modules/boundary_detector.py:91-92
constexpr float EPS_AB = 1e-5f, EPS_V = 1e-5f;  // :46-48, :66-67
constexpr int NS = 10;                          // draws, :55

__device__ __forceinline__ float softplus(float z) {  // torch Softplus (beta 1, threshold 20)
  return z > 20.f ? z : log1pf(expf(z));
}
__device__ __forceinline__ float softplus_d(float z) { return z > 20.f ? 1.f : 1.f / (1.f + expf(-z)); }

// digamma / trigamma for x > 0: recurrence to x >= 8, then the asymptotic series (double)
__device__ double digamma_d(double x) {
  double r = 0.0;
  while (x < 8.0) { r -= 1.0 / x; x += 1.0; }
  const double i2 = 1.0 / (x * x);
  return r + log(x) - 0.5 / x - i2 * (1.0 / 12 - i2 * (1.0 / 120 - i2 * (1.0 / 252 - i2 * (1.0 / 240 - i2 / 132))));
}
__device__ double trigamma_d(double x) {
  double r = 0.0;
  while (x < 8.0) { r += 1.0 / (x * x); x += 1.0; }
  const double i = 1.0 / x, i2 = i * i;
  return r + i + 0.5 * i2 + i * i2 * (1.0 / 6 - i2 * (1.0 / 30 - i2 * (1.0 / 42 - i2 / 30)));
}

// U(0,1) draw s of element i: injected (u[s*n + i]) or Philox(seed, offset + s*n + i), 24 bits
__device__ __forceinline__ float draw(const float* u, unsigned long long seed, unsigned long long off,
                                      size_t n, int s, size_t i) {
  if (u) return u[(size_t)s * n + i];
  const unsigned long long k = off + (unsigned long long)s * n + i;
  unsigned w[4];
  philox4(seed, k >> 2, w);
  return (w[k & 3] >> 8) * (1.f / 16777216.f);
}

struct BndArgs {
  size_t n;
  const float *za, *zb, *y, *u;
  unsigned long long seed, off;
  float *v, *bce, *kld;                 // forward outputs (any may be NULL)
  const float *dv, *dbce, *dkld;        // backward cotangents (NULL = 0)
  float *dza, *dzb;                     // backward outputs
};

template <bool BWD>
__global__ __launch_bounds__(256) void boundary_kernel(BndArgs g) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < g.n; i += (size_t)gridDim.x * 256) {
    const float za = g.za[i], zb = g.zb[i], y = g.y[i];
    const float a = softplus(za) + EPS_AB, b = softplus(zb) + EPS_AB;
    const double ad = a, bd = b, A0 = PRIOR_A, B0 = PRIOR_B;
    if (!BWD) {
      if (g.kld) {
        const double kl = lgamma(A0) + lgamma(B0) + lgamma(ad + bd) - lgamma(ad) - lgamma(bd) -
                          lgamma(A0 + B0) + (ad - A0) * digamma_d(ad) + (bd - B0) * digamma_d(bd) +
                          (A0 + B0 - ad - bd) * digamma_d(ad + bd);
        g.kld[i] = (float)kl;
      }
      float vs = 0.f, bs = 0.f;
      for (int s = 0; s < NS; ++s) {
        const float u = draw(g.u, g.seed, g.off, g.n, s, i) * 0.98f + 0.01f;
        float v = powf(1.f - powf(u, 1.f / b), 1.f / a);
        v = v * (1.f - 2.f * EPS_V) + EPS_V;
        vs += v;
        // torch binary_cross_entropy: logs clamped at -100
        bs += -(y * fmaxf(logf(v), -100.f) + (1.f - y) * fmaxf(logf(1.f - v), -100.f));
      }
      if (g.v) g.v[i] = vs / NS;
      if (g.bce) g.bce[i] = bs / NS;
    } else {
      double da = 0.0, db = 0.0;
      if (g.dkld) {
        const double k = g.dkld[i], tab = trigamma_d(ad + bd);
        da += k * ((ad - A0) * trigamma_d(ad) + (A0 + B0 - ad - bd) * tab);
        db += k * ((bd - B0) * trigamma_d(bd) + (A0 + B0 - ad - bd) * tab);
      }
      const float gv = g.dv ? g.dv[i] / NS : 0.f, gb = g.dbce ? g.dbce[i] / NS : 0.f;
      if (gv != 0.f || gb != 0.f) {
        for (int s = 0; s < NS; ++s) {
          const float u = draw(g.u, g.seed, g.off, g.n, s, i) * 0.98f + 0.01f;
          const float lu = logf(u);
          const float w = expf(lu / b);          // u^(1/b)
          const float sm = 1.f - w;
          const float vr = powf(sm, 1.f / a);    // (1 - w)^(1/a)
          const float v = vr * (1.f - 2.f * EPS_V) + EPS_V;
          // d v / d a, d v / d b through the Kumaraswamy inverse CDF
          const float dva = (1.f - 2.f * EPS_V) * vr * (-logf(sm) / (a * a));
          const float dvb = (1.f - 2.f * EPS_V) * vr / (a * sm) * w * lu / (b * b);
          // torch BCE backward: (v - y) / max(v (1 - v), 1e-12)
          const float dl = (v - y) / fmaxf(v * (1.f - v), 1e-12f);
          const float gtot = gb * dl + gv;
          da += (double)(gtot * dva);
          db += (double)(gtot * dvb);
        }
      }
      g.dza[i] = (float)da * softplus_d(za);
      g.dzb[i] = (float)db * softplus_d(zb);
    }
  }
}

int grid_n(size_t n) {
  size_t b = (n + 255) / 256;
  return (int)(b > 4096 ? 4096 : (b < 1 ? 1 : b));
}

}  // namespace

extern "C" int mlvae_phn_bce(int B, int T, int C, const float* logits, int ldl, const float* feat_lens,
                             const long long* phn, int L, const float* phn_lens, const float* boundary,
                             float* loss, const float* dloss, float* dlogits, int* err, void* stream) {
  if (B <= 0 || T <= 0) return 0;
  if (C <= 0 || L <= 0 || ldl < C || !logits || !feat_lens || !phn || !phn_lens || !boundary || !err ||
      (dlogits && !dloss)) {
    mlvae_set_error("mlvae_phn_bce: bad shape/pointer");
    return 1;
  }
  phn_bce_kernel<<<B, PB, 0, (hipStream_t)stream>>>(T, C, logits, ldl, feat_lens, phn, L, phn_lens,
                                                    boundary, loss, dloss, dlogits, err);
  MLVAE_CHECK_LAUNCH();
  return 0;
}

extern "C" int mlvae_boundary_fwd(size_t n, const float* za, const float* zb, const float* y,
                                  const float* u, unsigned long long seed, unsigned long long offset,
                                  float* v, float* bce, float* kld, void* stream) {
  if (n == 0) return 0;
  if (!za || !zb || !y) { mlvae_set_error("mlvae_boundary_fwd: null input"); return 1; }
  BndArgs g{};
  g.n = n; g.za = za; g.zb = zb; g.y = y; g.u = u; g.seed = seed; g.off = offset;
  g.v = v; g.bce = bce; g.kld = kld;
  boundary_kernel<false><<<grid_n(n), 256, 0, (hipStream_t)stream>>>(g);
  MLVAE_CHECK_LAUNCH();
  return 0;
}

extern "C" int mlvae_boundary_bwd(size_t n, const float* za, const float* zb, const float* y,
                                  const float* u, unsigned long long seed, unsigned long long offset,
                                  const float* dv, const float* dbce, const float* dkld, float* dza,
                                  float* dzb, void* stream) {
  if (n == 0) return 0;
  if (!za || !zb || !y || !dza || !dzb) { mlvae_set_error("mlvae_boundary_bwd: null pointer"); return 1; }
  BndArgs g{};
  g.n = n; g.za = za; g.zb = zb; g.y = y; g.u = u; g.seed = seed; g.off = offset;
  g.dv = dv; g.dbce = dbce; g.dkld = dkld; g.dza = dza; g.dzb = dzb;
  boundary_kernel<true><<<grid_n(n), 256, 0, (hipStream_t)stream>>>(g);
  MLVAE_CHECK_LAUNCH();
  return 0;
}
