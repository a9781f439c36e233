// Fused VanillaVAE encoder of the bf16 train step: the forward (three FC layers, the
// reparameterisation and the KL partial sums) and the backward (reparam/KL gradient, two
// LeakyReLU dgrads and all six weight/bias gradients) are ONE launch each (+ a fixed-order
// reduce of the per-workgroup weight-gradient slabs).  The encoder is narrow (E = 64, z = 32):
// as separate GEMMs it was a dozen launches of a few % MFMA occupancy each; here the
// activations stay in registers between layers and the weights sit in registers as ready
// MFMA fragments, so HBM sees each frame's x, activations and gradients once.
//
//   VanillaVAE.fc = Seq(FCBlock([F, E, E]), LeakyReLU)   ref:src/modules/vanilla_vae.py:13-16,22
//     E1 = lrelu(x W0^T + b0), E2 = lrelu(E1 W1^T + b1)   (FCBlock ref:src/modules/fc_block.py:4-21)
//   mean_fc / log_var_fc                                  ref:src/modules/vanilla_vae.py:18-19,23-24
//     [mu | lv] = E2 [Wm; Wv]^T + [bm; bv]
//   reparameterize  z = eps * exp(0.5 lv) + mu            ref:src/modules/vanilla_vae.py:37-40
//   compute_kld_loss  -0.5 (1 + lv - mu^2 - e^lv)         ref:src/modules/vanilla_vae.py:42-45
//   masked sum over valid frames                          ref:src/utils/data_utils.py:67-104
//
// v_mfma_f32_16x16x32_bf16 with swapped operands (D^T = W X^T): a wave owns 16 frames; lane
// (l15 = frame, q = lane >> 4) ends every layer holding columns 16 j + 4 q + r (tiles j, r < 4).
// Those 16 values ARE the next layer's operand fragment under the k permutation
//   perm(kk, q, e) = 32 kk + (e < 4 ? 4 q + e : 16 + 4 q + e - 4),
// with which the next layer's resident weight fragments are built: no LDS hop between layers.
// The backward's weight gradients (sums over frames) read the 64-frame tile's activations and
// gradients back through LDS with transposing reads (ds_read_b64_tr_b16).
#include "common.h"
#include <stdlib.h>

namespace {

constexpr int EW = 64;   // encoder width E
constexpr int ZW = 32;   // latent width z
typedef __attribute__((address_space(3))) bf16x4* lds_b4_p;

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ int perm_k(int kk, int q, int e) {
  return 32 * kk + (e < 4 ? 4 * q + e : 12 + 4 * q + e);
}

// weight fragment (first MFMA operand): element (n, k) = W[n][k], W row-major [.][ld]
template <bool PERM>
__device__ __forceinline__ bf16x8 wfrag(const float* W, int ld, int kmax, int n, int kk, int q) {
  bf16x8 r;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int k = PERM ? perm_k(kk, q, e) : 32 * kk + 8 * q + e;
    r[e] = k < kmax ? f2bf(W[(size_t)n * ld + k]) : (short)0;
  }
  return r;
}
// transposed weight fragment: element (n, k) = W[k][n], W row-major [K][ldn]
template <bool PERM>
__device__ __forceinline__ bf16x8 wfrag_t(const float* W, int ldn, int n, int kk, int q) {
  bf16x8 r;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int k = PERM ? perm_k(kk, q, e) : 32 * kk + 8 * q + e;
    r[e] = f2bf(W[(size_t)k * ldn + n]);
  }
  return r;
}

// the low halves of wfrag's elements (split-bf16 forward)
template <bool PERM>
__device__ __forceinline__ bf16x8 wfrag_lo(const float* W, int ld, int kmax, int n, int kk, int q) {
  bf16x8 r;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int k = PERM ? perm_k(kk, q, e) : 32 * kk + 8 * q + e;
    r[e] = k < kmax ? f2bf_lo(W[(size_t)n * ld + k]) : (short)0;
  }
  return r;
}

__device__ __forceinline__ bf16x8 pack8(const float* v) {
  return bf16x8{f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3]),
                f2bf(v[4]), f2bf(v[5]), f2bf(v[6]), f2bf(v[7])};
}
__device__ __forceinline__ bf16x4 pack4(const float* v) {
  return bf16x4{f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3])};
}
// next layer's operand fragment of k-step kk from this layer's output tiles 2kk, 2kk+1
__device__ __forceinline__ bf16x8 next_frag(float (*h)[4], int kk) {
  return bf16x8{f2bf(h[2 * kk][0]), f2bf(h[2 * kk][1]), f2bf(h[2 * kk][2]), f2bf(h[2 * kk][3]),
                f2bf(h[2 * kk + 1][0]), f2bf(h[2 * kk + 1][1]), f2bf(h[2 * kk + 1][2]),
                f2bf(h[2 * kk + 1][3])};
}
__device__ __forceinline__ bf16x8 next_frag_lo(float (*h)[4], int kk) {
  return bf16x8{f2bf_lo(h[2 * kk][0]), f2bf_lo(h[2 * kk][1]), f2bf_lo(h[2 * kk][2]), f2bf_lo(h[2 * kk][3]),
                f2bf_lo(h[2 * kk + 1][0]), f2bf_lo(h[2 * kk + 1][1]), f2bf_lo(h[2 * kk + 1][2]),
                f2bf_lo(h[2 * kk + 1][3])};
}

// operand fragment (m or n = base + (lane & 15), k = kk + 8 (lane >> 4) + e) of an LDS image
// stored [k rows][ld], read transposed (the MC fragment of gemm_fast.hip, unswizzled)
__device__ __forceinline__ bf16x8 trfrag(const short* img, int ld, int base, int kk, int lane) {
  const int g = lane >> 4, i4 = lane & 15, qq = i4 >> 2, pp = i4 & 3;
  const int r1 = kk + 8 * g + qq, r2 = r1 + 4;
  const bf16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_b4_p)(img + r1 * ld + base + 4 * pp));
  const bf16x4 v2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_b4_p)(img + r2 * ld + base + 4 * pp));
  return bf16x8{v1[0], v1[1], v1[2], v1[3], v2[0], v2[1], v2[2], v2[3]};
}

// standard normal of counter i: the same draw as mlvae_randn (elbo.hip randn_kernel)
__device__ __forceinline__ float philox_normal(unsigned long long seed, unsigned long long i) {
  unsigned r[4];
  philox4(seed, i, r);
  const float u1 = ((r[0] >> 8) + 1u) * (1.f / 16777217.f);
  const float u2 = (r[1] >> 8) * (1.f / 16777216.f);
  return sqrtf(-2.f * logf(u1)) * cospif(2.f * u2);
}

__device__ __forceinline__ bool frame_valid(const float* lens, int row, int T) {
  const int b = row / T, t = row - b * T;
  return t < valid_frames(lens[b], T);
}

struct EncFwdArgs {
  int N, T, zld;
  const float *x, *w0, *b0, *w1, *b1, *wml, *bml, *eps_in, *lens;
  unsigned long long seed, offset;
  unsigned short *e1, *e2, *zb;
  float *ml, *z, *eps_out, *partials;
};

int fwd_grid(int N) {
  const int waves = (N + 15) / 16;
  int g = (waves + 3) / 4;
  return g > 256 ? 256 : (g < 1 ? 1 : g);
}

// SPL (split-bf16 forward): every product a W^T runs as a_hi W_hi + a_hi W_lo + a_lo W_hi (three
// bf16 MFMAs, fp32 accumulation), with the fp32 x / E1 / E2 / weights split into bf16 hi + lo pairs
// in registers -- fp32-grade mu / log_var (and so z, KL) for the same HBM traffic.  The saved
// E1 / E2 (the backward's operands) stay bf16.  The bf16 rounding of the encoder's weights is a
// fixed per-step perturbation, not a per-frame one, so it does not average out over the batch:
// tools/elbo_budget.py attributes to it (with the heads' weights) most of the bf16 step's ELBO error.
template <int F, bool SPL>
__global__ __launch_bounds__(256) void encoder_fwd_kernel(EncFwdArgs a) {
  constexpr int KS0 = (F + 31) / 32;
  __shared__ float red[4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, l15 = lane & 15, q = lane >> 4;
  bf16x8 w0f[4][KS0], w1f[4][2], wmf[4][2];
  // SPL: the weights' lo fragments live in LDS (every wave holds the same fragments; in registers
  // beside the hi ones they spilled): [fragment][lane], fragment = w0 (j, kk) | w1 (j, kk) | wml (j, kk)
  constexpr int NLF = SPL ? 4 * KS0 + 16 : 1;
  __shared__ bf16x8 wlo[NLF][64];
  if constexpr (SPL) {
    for (int idx = threadIdx.x; idx < NLF * 64; idx += 256) {
      const int f = idx >> 6, ln = idx & 63, n_ = ln & 15, q_ = ln >> 4;
      bf16x8 v;
      if (f < 4 * KS0) v = wfrag_lo<false>(a.w0, F, F, 16 * (f / KS0) + n_, f % KS0, q_);
      else if (f < 4 * KS0 + 8) v = wfrag_lo<true>(a.w1, EW, EW, 16 * ((f - 4 * KS0) / 2) + n_, (f - 4 * KS0) % 2, q_);
      else v = wfrag_lo<true>(a.wml, EW, EW, 16 * ((f - 4 * KS0 - 8) / 2) + n_, (f - 4 * KS0 - 8) % 2, q_);
      wlo[f][ln] = v;
    }
    __syncthreads();
  }
  auto w0l = [&](int j, int kk) { return wlo[j * KS0 + kk][lane]; };
  auto w1l = [&](int j, int kk) { return wlo[4 * KS0 + 2 * j + kk][lane]; };
  auto wmlo = [&](int j, int kk) { return wlo[4 * KS0 + 8 + 2 * j + kk][lane]; };
  float b0v[4][4], b1v[4][4], bmv[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = 16 * j + l15;
#pragma unroll
    for (int kk = 0; kk < KS0; ++kk) w0f[j][kk] = wfrag<false>(a.w0, F, F, n, kk, q);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      w1f[j][kk] = wfrag<true>(a.w1, EW, EW, n, kk, q);
      wmf[j][kk] = wfrag<true>(a.wml, EW, EW, n, kk, q);
    }

#pragma unroll
    for (int r = 0; r < 4; ++r) {
      b0v[j][r] = a.b0[16 * j + 4 * q + r];
      b1v[j][r] = a.b1[16 * j + 4 * q + r];
      bmv[j][r] = a.bml[16 * j + 4 * q + r];
    }
  }
  float kl_acc = 0.f;
  const int ntiles = (a.N + 15) / 16;
  // the wave's next tile's x row pieces and utterance length are loaded one tile ahead
  // (unconditional loads from clamped addresses: rows past N, columns past F read valid data that
  // is zeroed / unused), so they are in flight while this tile's MFMAs and stores run
  f32x4 px[KS0][2];
  float plen;
  auto prefetch = [&](int tile_) {
    const int row_ = tile_ * 16 + l15;
    const bool rv_ = tile_ < ntiles && row_ < a.N;
    const size_t rr_ = rv_ ? row_ : 0;
#pragma unroll
    for (int kk = 0; kk < KS0; ++kk) {
      const int k0 = 32 * kk + 8 * q, kc = k0 < F ? k0 : F - 8;
      px[kk][0] = *reinterpret_cast<const f32x4*>(a.x + rr_ * F + kc);
      px[kk][1] = *reinterpret_cast<const f32x4*>(a.x + rr_ * F + kc + 4);
    }
    plen = a.lens[rr_ / a.T];
  };
  prefetch(blockIdx.x * 4 + wave);
  for (int tile = blockIdx.x * 4 + wave; tile < ntiles; tile += gridDim.x * 4) {
    const int row = tile * 16 + l15;
    const bool rv = row < a.N;
    const size_t rr = rv ? row : 0;
    bf16x8 xa[KS0], xl[SPL ? KS0 : 1];
#pragma unroll
    for (int kk = 0; kk < KS0; ++kk) {
      const int k0 = 32 * kk + 8 * q;
      const float v[8] = {px[kk][0][0], px[kk][0][1], px[kk][0][2], px[kk][0][3],
                          px[kk][1][0], px[kk][1][1], px[kk][1][2], px[kk][1][3]};
      xa[kk] = k0 < F ? pack8(v) : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
      if constexpr (SPL) {
        bf16x8 lo;
#pragma unroll
        for (int e = 0; e < 8; ++e) lo[e] = f2bf_lo(v[e]);
        xl[kk] = k0 < F ? lo : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
      }
    }
    const float clen = plen;
    prefetch(tile + gridDim.x * 4);
    // E1 = lrelu(x W0^T + b0)
    float h[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < KS0; ++kk) {
        acc = mfma16(w0f[j][kk], xa[kk], acc);
        if constexpr (SPL) {
          acc = mfma16(w0l(j, kk), xa[kk], acc);
          acc = mfma16(w0f[j][kk], xl[kk], acc);
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) h[j][r] = lrelu(acc[r] + b0v[j][r]);
      if (rv) *reinterpret_cast<bf16x4*>(a.e1 + rr * EW + 16 * j + 4 * q) = pack4(h[j]);
    }
    bf16x8 ha[2] = {next_frag(h, 0), next_frag(h, 1)};
    bf16x8 hl[2];
    if constexpr (SPL) { hl[0] = next_frag_lo(h, 0); hl[1] = next_frag_lo(h, 1); }
    // E2 = lrelu(E1 W1^T + b1)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        acc = mfma16(w1f[j][kk], ha[kk], acc);
        if constexpr (SPL) {
          acc = mfma16(w1l(j, kk), ha[kk], acc);
          acc = mfma16(w1f[j][kk], hl[kk], acc);
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) h[j][r] = lrelu(acc[r] + b1v[j][r]);
      if (rv) *reinterpret_cast<bf16x4*>(a.e2 + rr * EW + 16 * j + 4 * q) = pack4(h[j]);
    }
    ha[0] = next_frag(h, 0);
    ha[1] = next_frag(h, 1);
    if constexpr (SPL) { hl[0] = next_frag_lo(h, 0); hl[1] = next_frag_lo(h, 1); }
    // [mu | lv] = E2 [Wm; Wv]^T + [bm; bv]: tiles 0-1 mu, 2-3 lv (column 16 j + 4 q + r of ML)
    float ml[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        acc = mfma16(wmf[j][kk], ha[kk], acc);
        if constexpr (SPL) {
          acc = mfma16(wmlo(j, kk), ha[kk], acc);
          acc = mfma16(wmf[j][kk], hl[kk], acc);
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) ml[j][r] = acc[r] + bmv[j][r];
      if (rv) *reinterpret_cast<f32x4*>(a.ml + rr * 2 * ZW + 16 * j + 4 * q) =
                  f32x4{ml[j][0], ml[j][1], ml[j][2], ml[j][3]};
    }
    if (rv) {
      const bool fv = row % a.T < valid_frames(clen, a.T);
#pragma unroll
      for (int jz = 0; jz < 2; ++jz) {
        const int z0 = 16 * jz + 4 * q;
        float ev[4], zz[4];
        if (a.eps_in) {
          const f32x4 e4 = *reinterpret_cast<const f32x4*>(a.eps_in + rr * ZW + z0);
#pragma unroll
          for (int r = 0; r < 4; ++r) ev[r] = e4[r];
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) ev[r] = philox_normal(a.seed, a.offset + rr * ZW + z0 + r);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float mu = ml[jz][r], lv = ml[jz + 2][r];
          zz[r] = ev[r] * expf(0.5f * lv) + mu;
          const float kl = -0.5f * (1.f + lv - mu * mu - expf(lv));
          if (fv) kl_acc += kl;
        }
        *reinterpret_cast<f32x4*>(a.z + rr * ZW + z0) = f32x4{zz[0], zz[1], zz[2], zz[3]};
        *reinterpret_cast<bf16x4*>(a.zb + rr * a.zld + z0) = pack4(zz);
        if (a.eps_out)
          *reinterpret_cast<f32x4*>(a.eps_out + rr * ZW + z0) = f32x4{ev[0], ev[1], ev[2], ev[3]};
      }
      // bias column of the bottom layer's skinny weight-gradient product: [z | 1 | 0 ...]
      if (a.zld >= ZW + 16 && q < 2) {
        const short one = 0x3F80;
        *reinterpret_cast<bf16x8*>(a.zb + rr * a.zld + ZW + 8 * q) =
            q == 0 ? bf16x8{one, 0, 0, 0, 0, 0, 0, 0} : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
      }
    }
  }
  kl_acc = wave_sum(kl_acc);
  if (lane == 0) red[wave] = kl_acc;
  __syncthreads();
  if (threadIdx.x == 0) a.partials[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// ---------------------------------------------------------------------------------------
// backward
// ---------------------------------------------------------------------------------------
struct EncBwdArgs {
  int N, T, B;
  const float *dz, *ml, *eps, *x, *wml, *w1, *lens;
  const int* count;
  float kl_scale;
  const unsigned short *e1, *e2;
  float* ws;  // [gridDim.x][slab]
};

template <int F>
constexpr int slab_floats() { return 2 * EW * EW + EW * F + 3 * EW; }

int bwd_grid(int N) {
  // cap on workgroups (each folds its tiles into one weight-gradient slab); MLVAE_ENC_BWD_GRID
  // overrides it for A/B timing
  // default: 128 workgroups, which leave CUs to the weight-gradient GEMM beside it when the
  // recurrence does not fill the chip (c2: 128 -> 256 costs 0.03 ms/step); 256 at B*T >= 64K
  // frames, where the tail runs serialised on the whole chip (round 5, c3 same box: 512 / 256 /
  // 1024 workgroups 75 / 65 / 97 us -- per-workgroup fixed costs (resident weight fragments,
  // the slab) against the tiles each folds in; round 3 had measured 512 over 128)
  static const int env = [] {
    const char* e = getenv("MLVAE_ENC_BWD_GRID");
    return e ? atoi(e) : 0;
  }();
  const int tiles = (N + 63) / 64;
  const int cap = env >= 1 ? env : (tiles >= 1024 ? 256 : 128);
  return tiles > cap ? cap : (tiles < 1 ? 1 : tiles);
}

template <int F>
__global__ __launch_bounds__(256) void encoder_bwd_kernel(EncBwdArgs a) {
  constexpr int LA = EW + 8;   // LDS row stride (bf16) of the 64-wide images
  constexpr int LX = F + 8;    // of the x image
  constexpr int NF = F / 16;   // dW0 column tiles
  constexpr int SLAB = slab_floats<F>();
  __shared__ __attribute__((aligned(16))) short sDML[64 * LA], sE2[64 * LA], sDE2[64 * LA];
  __shared__ __attribute__((aligned(16))) short sE1[64 * LA], sDE1[64 * LA], sX[64 * LX];
  __shared__ float sb[4][3 * EW];
  __shared__ float inv_count;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l15 = lane & 15, q = lane >> 4;

  // resident transposed weights (first MFMA operand, n = input unit):
  //   dE2 = dML Wml: (n = e, k = o) = Wml[o][e];  dE1 = dE2 W1: (n = e_in, k = e_out) = W1[e_out][e_in]
  bf16x8 wmT[4][2], w1T[4][2];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      wmT[j][kk] = wfrag_t<false>(a.wml, EW, 16 * j + l15, kk, q);
      w1T[j][kk] = wfrag_t<true>(a.w1, EW, 16 * j + l15, kk, q);
    }
  {
    __shared__ int cnt_sh;
    const int c = block_frames(a.lens, a.B, a.T, a.count, &cnt_sh);
    if (tid == 0) inv_count = c > 0 ? 1.f / ((float)c * (float)ZW) : 0.f;
  }
  __syncthreads();
  const float s_kl = a.kl_scale * inv_count;

  f32x4 gml[4], g1[4], g0[NF];
#pragma unroll
  for (int j = 0; j < 4; ++j) gml[j] = g1[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < NF; ++j) g0[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bml[16], bb1[16], bb0[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) bml[i] = bb1[i] = bb0[i] = 0.f;

  const int ntiles = (a.N + 63) / 64;
  // A tile's HBM inputs -- this lane's dz / mu / log var / eps (z index 8 q + e), E2 / E1 channels
  // and the thread's pieces of the x tile -- are loaded one tile ahead, so they are in flight
  // while the previous tile's MFMAs run (loaded at the point of use, every tile paid the full
  // load latency: the kernel sat at 1.3 TB/s at c3).
  constexpr int XP = (64 * F / 8 + 255) / 256;   // x pieces (8 floats) per thread
  const int lrow = 16 * wave + l15;
  f32x4 pg[2], pmu[2], plv[2], pep[2], px[XP][2];
  unsigned long long pe2[4], pe1[4];   // bf16x4 bit patterns (scalar words: no stack copy)
  float plen;   // the row's utterance length (read in the loop, its wait included the prefetch)
  auto prefetch = [&](int tile_) __attribute__((always_inline)) {
    const int row_ = tile_ * 64 + lrow;
    const bool rv_ = tile_ < ntiles && row_ < a.N;
    const size_t rr_ = rv_ ? row_ : 0;
    plen = rv_ ? a.lens[row_ / a.T] : 0.f;
#pragma unroll
    for (int h2 = 0; h2 < 2; ++h2) {
      const int z0 = 8 * q + 4 * h2;
      pg[h2] = pmu[h2] = plv[h2] = pep[h2] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (rv_) {
        pg[h2] = *reinterpret_cast<const f32x4*>(a.dz + rr_ * ZW + z0);
        pmu[h2] = *reinterpret_cast<const f32x4*>(a.ml + rr_ * 2 * ZW + z0);
        plv[h2] = *reinterpret_cast<const f32x4*>(a.ml + rr_ * 2 * ZW + ZW + z0);
        pep[h2] = *reinterpret_cast<const f32x4*>(a.eps + rr_ * ZW + z0);
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      pe2[j] = rv_ ? *reinterpret_cast<const unsigned long long*>(a.e2 + rr_ * EW + 16 * j + 4 * q) : 0ull;
      pe1[j] = rv_ ? *reinterpret_cast<const unsigned long long*>(a.e1 + rr_ * EW + 16 * j + 4 * q) : 0ull;
    }
#pragma unroll
    for (int i = 0; i < XP; ++i) {
      const int p_ = tid + 256 * i, r = p_ / (F / 8), c8 = p_ - r * (F / 8), grow = tile_ * 64 + r;
      px[i][0] = px[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (p_ < 64 * F / 8 && tile_ < ntiles && grow < a.N) {
        px[i][0] = *reinterpret_cast<const f32x4*>(a.x + (size_t)grow * F + 8 * c8);
        px[i][1] = *reinterpret_cast<const f32x4*>(a.x + (size_t)grow * F + 8 * c8 + 4);
      }
    }
  };
  prefetch(blockIdx.x);
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int row = tile * 64 + lrow;
    const bool rv = row < a.N;
    // this tile's inputs out of the prefetch registers, the next tile's loads issued behind them
    f32x4 cg[2], cmu[2], clv[2], cep[2], cx[XP][2];
    unsigned long long ce2[4], ce1[4];
    const float clen = plen;
#pragma unroll
    for (int h2 = 0; h2 < 2; ++h2) { cg[h2] = pg[h2]; cmu[h2] = pmu[h2]; clv[h2] = plv[h2]; cep[h2] = pep[h2]; }
#pragma unroll
    for (int j = 0; j < 4; ++j) { ce2[j] = pe2[j]; ce1[j] = pe1[j]; }
#pragma unroll
    for (int i = 0; i < XP; ++i) { cx[i][0] = px[i][0]; cx[i][1] = px[i][1]; }
    prefetch(tile + gridDim.x);
    // reparameterisation + KL gradient (as reparam_kl_bwd in elbo.hip), z index 8 q + e
    float dmu[8], dlv[8];
    if (rv) {
      const float s = row % a.T < valid_frames(clen, a.T) ? s_kl : 0.f;
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          dmu[4 * h2 + r] = cg[h2][r] + s * cmu[h2][r];
          dlv[4 * h2 + r] = cg[h2][r] * 0.5f * cep[h2][r] * expf(0.5f * clv[h2][r]) + s * 0.5f * (expf(clv[h2][r]) - 1.f);
        }
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) dmu[e] = dlv[e] = 0.f;
    }
    const bf16x8 dmla[2] = {pack8(dmu), pack8(dlv)};
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      bml[e] += dmu[e];
      bml[8 + e] += dlv[e];
    }
    *reinterpret_cast<bf16x8*>(sDML + lrow * LA + 8 * q) = dmla[0];
    *reinterpret_cast<bf16x8*>(sDML + lrow * LA + ZW + 8 * q) = dmla[1];

    // dE2 = (dML Wml) * lrelu'(E2)
    float d2[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) acc = mfma16(wmT[j][kk], dmla[kk], acc);
      const bf16x4 ev = __builtin_bit_cast(bf16x4, ce2[j]);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        d2[j][r] = rv ? acc[r] * lrelu_d(bf2f(ev[r])) : 0.f;
        bb1[4 * j + r] += d2[j][r];
      }
      *reinterpret_cast<bf16x4*>(sE2 + lrow * LA + 16 * j + 4 * q) = ev;
      *reinterpret_cast<bf16x4*>(sDE2 + lrow * LA + 16 * j + 4 * q) = pack4(d2[j]);
    }
    const bf16x8 d2a[2] = {next_frag(d2, 0), next_frag(d2, 1)};
    // dE1 = (dE2 W1) * lrelu'(E1)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) acc = mfma16(w1T[j][kk], d2a[kk], acc);
      const bf16x4 ev = __builtin_bit_cast(bf16x4, ce1[j]);
      float d1[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        d1[r] = rv ? acc[r] * lrelu_d(bf2f(ev[r])) : 0.f;
        bb0[4 * j + r] += d1[r];
      }
      *reinterpret_cast<bf16x4*>(sE1 + lrow * LA + 16 * j + 4 * q) = ev;
      *reinterpret_cast<bf16x4*>(sDE1 + lrow * LA + 16 * j + 4 * q) = pack4(d1);
    }
    // x tile as bf16 (zero rows past N: zero-filled by the prefetch)
#pragma unroll
    for (int i = 0; i < XP; ++i) {
      const int p = tid + 256 * i, r = p / (F / 8), c8 = p - r * (F / 8);
      if (p < 64 * F / 8) {
        *reinterpret_cast<bf16x8*>(sX + r * LX + 8 * c8) =
            bf16x8{f2bf(cx[i][0][0]), f2bf(cx[i][0][1]), f2bf(cx[i][0][2]), f2bf(cx[i][0][3]),
                   f2bf(cx[i][1][0]), f2bf(cx[i][1][1]), f2bf(cx[i][1][2]), f2bf(cx[i][1][3])};
      }
    }
    __syncthreads();
    // weight gradients of output-row tile `wave` over the tile's 64 frames (swapped operands:
    // lane holds dW[16 wave + l15][16 j + 4 q + r])
#pragma unroll
    for (int kk = 0; kk < 64; kk += 32) {
      const bf16x8 a_ml = trfrag(sDML, LA, 16 * wave, kk, lane);
      const bf16x8 a_e2 = trfrag(sDE2, LA, 16 * wave, kk, lane);
      const bf16x8 a_e1 = trfrag(sDE1, LA, 16 * wave, kk, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        gml[j] = mfma16(trfrag(sE2, LA, 16 * j, kk, lane), a_ml, gml[j]);
        g1[j] = mfma16(trfrag(sE1, LA, 16 * j, kk, lane), a_e2, g1[j]);
      }
#pragma unroll
      for (int j = 0; j < NF; ++j) g0[j] = mfma16(trfrag(sX, LX, 16 * j, kk, lane), a_e1, g0[j]);
    }
    __syncthreads();  // the images are rewritten by the next tile
  }

  // bias partials: sum over the 16 frame lanes (fixed butterfly), then the 4 waves in order
#pragma unroll
  for (int i = 0; i < 16; ++i)
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      bml[i] += __shfl_xor(bml[i], o, 64);
      bb1[i] += __shfl_xor(bb1[i], o, 64);
      bb0[i] += __shfl_xor(bb0[i], o, 64);
    }
  if (l15 == 0) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int cm = i < 8 ? 8 * q + i : ZW + 8 * q + (i - 8);
      const int cj = 16 * (i >> 2) + 4 * q + (i & 3);
      sb[wave][cm] = bml[i];
      sb[wave][EW + cj] = bb1[i];
      sb[wave][2 * EW + cj] = bb0[i];
    }
  }
  float* slab = a.ws + (size_t)blockIdx.x * SLAB;
  const int orow = 16 * wave + l15;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    *reinterpret_cast<f32x4*>(slab + orow * EW + 16 * j + 4 * q) = gml[j];
    *reinterpret_cast<f32x4*>(slab + EW * EW + orow * EW + 16 * j + 4 * q) = g1[j];
  }
#pragma unroll
  for (int j = 0; j < NF; ++j)
    *reinterpret_cast<f32x4*>(slab + 2 * EW * EW + orow * F + 16 * j + 4 * q) = g0[j];
  __syncthreads();
  if (tid < 3 * EW)
    slab[2 * EW * EW + EW * F + tid] = (sb[0][tid] + sb[1][tid]) + (sb[2][tid] + sb[3][tid]);
}

// sum the per-workgroup slabs into the gradients: a block covers 64 slab elements with four
// threads each (slab quarters, summed in order), combined in a fixed order through LDS
template <int F>
__global__ __launch_bounds__(256) void encoder_reduce(int G, const float* __restrict__ ws,
                                                      float* __restrict__ dwml, float* __restrict__ dbml,
                                                      float* __restrict__ dw1, float* __restrict__ db1,
                                                      float* __restrict__ dw0, float* __restrict__ db0) {
  constexpr int SLAB = slab_floats<F>();
  __shared__ float part[4][64];
  const int e = threadIdx.x & 63, qtr = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + e;
  const int g0 = qtr * G / 4, g1 = (qtr + 1) * G / 4;
  float v = 0.f;
  if (i < SLAB)
#pragma unroll 8  // eight slab loads in flight per thread; the adds keep their order
    for (int g = g0; g < g1; ++g) v += ws[(size_t)g * SLAB + i];
  part[qtr][e] = v;
  __syncthreads();
  if (qtr != 0 || i >= SLAB) return;
  v = ((part[0][e] + part[1][e]) + part[2][e]) + part[3][e];
  if (i < EW * EW) dwml[i] = v;
  else if (i < 2 * EW * EW) dw1[i - EW * EW] = v;
  else if (i < 2 * EW * EW + EW * F) dw0[i - 2 * EW * EW] = v;
  else {
    const int c = i - (2 * EW * EW + EW * F);
    if (c < EW) dbml[c] = v;
    else if (c < 2 * EW) db1[c - EW] = v;
    else db0[c - 2 * EW] = v;
  }
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace

extern "C" int mlvae_encoder_supported(int F, int E, int Z) {
  return E == EW && Z == ZW && (F == 64 || F == 80);
}

extern "C" int mlvae_encoder_partials_count(int B, int T) { return fwd_grid(B * T); }

extern "C" size_t mlvae_encoder_workspace_size(int B, int T, int F, int E, int Z) {
  if (!mlvae_encoder_supported(F, E, Z)) return 0;
  return (size_t)bwd_grid(B * T) * (2 * EW * EW + EW * F + 3 * EW) * sizeof(float);
}

// Forward.  x [B*T, F] fp32; w0 [E, F], w1 [E, E], wml [2Z, E] (mean rows then log_var rows),
// biases fp32; eps_in [B*T, Z] or NULL (then eps = Philox normals at counter offset + n*Z + k,
// the mlvae_randn stream, written to eps_out if given).  Outputs: e1/e2 bf16 [B*T, E],
// ml [B*T, 2Z] = [mu | log_var], z [B*T, Z] fp32, z_bf16 [B*T, z_ld] (z_ld = Z, or >= Z + 16:
// then columns Z..Z+15 = [1, 0, ...]), kl_partials [mlvae_encoder_partials_count] (masked KL sums).
extern "C" int mlvae_encoder_fwd_ex(int B, int T, int F, int E, int Z, const float* x, const float* w0,
                                    const float* b0, const float* w1, const float* b1, const float* wml,
                                    const float* bml, const float* eps_in, unsigned long long seed,
                                    unsigned long long offset, const float* lens, void* e1_bf16,
                                    void* e2_bf16, float* ml, float* z, void* z_bf16, int z_ld,
                                    float* eps_out, float* kl_partials, int split, void* stream);
extern "C" int mlvae_encoder_fwd(int B, int T, int F, int E, int Z, const float* x, const float* w0,
                                 const float* b0, const float* w1, const float* b1, const float* wml,
                                 const float* bml, const float* eps_in, unsigned long long seed,
                                 unsigned long long offset, const float* lens, void* e1_bf16,
                                 void* e2_bf16, float* ml, float* z, void* z_bf16, int z_ld,
                                 float* eps_out, float* kl_partials, void* stream) {
  return mlvae_encoder_fwd_ex(B, T, F, E, Z, x, w0, b0, w1, b1, wml, bml, eps_in, seed, offset, lens, e1_bf16,
                              e2_bf16, ml, z, z_bf16, z_ld, eps_out, kl_partials, 0, stream);
}
extern "C" int mlvae_encoder_fwd_ex(int B, int T, int F, int E, int Z, const float* x, const float* w0,
                                    const float* b0, const float* w1, const float* b1, const float* wml,
                                    const float* bml, const float* eps_in, unsigned long long seed,
                                    unsigned long long offset, const float* lens, void* e1_bf16,
                                    void* e2_bf16, float* ml, float* z, void* z_bf16, int z_ld,
                                    float* eps_out, float* kl_partials, int split, void* stream) {
  const int N = B * T;
  if (N <= 0) return 0;
  if (!mlvae_encoder_supported(F, E, Z)) {
    mlvae_set_error("mlvae_encoder_fwd: needs E = 64, Z = 32, F in {64, 80} (got %d, %d, %d)", E, Z, F);
    return 1;
  }
  if (!x || !w0 || !b0 || !w1 || !b1 || !wml || !bml || !lens || !e1_bf16 || !e2_bf16 || !ml || !z ||
      !z_bf16 || !kl_partials || !aligned16(x) || !aligned16(ml) || !aligned16(z) || !aligned16(z_bf16) ||
      !aligned16(e1_bf16) || !aligned16(e2_bf16) || (eps_in && !aligned16(eps_in)) ||
      (eps_out && !aligned16(eps_out)) || !(z_ld == Z || z_ld >= Z + 16) || z_ld % 8) {
    mlvae_set_error("mlvae_encoder_fwd: null or misaligned pointer, or bad z_ld %d", z_ld);
    return 1;
  }
  EncFwdArgs a;
  a.N = N; a.T = T; a.zld = z_ld;
  a.x = x; a.w0 = w0; a.b0 = b0; a.w1 = w1; a.b1 = b1; a.wml = wml; a.bml = bml;
  a.eps_in = eps_in; a.lens = lens; a.seed = seed; a.offset = offset;
  a.e1 = static_cast<unsigned short*>(e1_bf16);
  a.e2 = static_cast<unsigned short*>(e2_bf16);
  a.zb = static_cast<unsigned short*>(z_bf16);
  a.ml = ml; a.z = z; a.eps_out = eps_out; a.partials = kl_partials;
  hipStream_t st = (hipStream_t)stream;
  auto k = F == 80 ? (split ? encoder_fwd_kernel<80, true> : encoder_fwd_kernel<80, false>)
                   : (split ? encoder_fwd_kernel<64, true> : encoder_fwd_kernel<64, false>);
  k<<<fwd_grid(N), 256, 0, st>>>(a);
  MLVAE_CHECK_LAUNCH();
  return 0;
}

// Backward.  dz [B*T, Z] (gradient reaching z from the decoder), ml/eps/e1/e2/x as saved by the
// forward; count = global valid-frame count or NULL (then counted from lens); kl_scale = the
// KL loss weight.  Writes (overwrites) the six encoder gradients.
extern "C" int mlvae_encoder_bwd(int B, int T, int F, int E, int Z, const float* dz, const float* ml,
                                 const float* eps, const void* e1_bf16, const void* e2_bf16,
                                 const float* x, const float* wml, const float* w1, const float* lens,
                                 const int* count, float kl_scale, float* dwml, float* dbml, float* dw1,
                                 float* db1, float* dw0, float* db0, float* ws, size_t ws_bytes,
                                 void* stream) {
  const int N = B * T;
  if (N <= 0) return 0;
  if (!mlvae_encoder_supported(F, E, Z)) {
    mlvae_set_error("mlvae_encoder_bwd: needs E = 64, Z = 32, F in {64, 80} (got %d, %d, %d)", E, Z, F);
    return 1;
  }
  if (!dz || !ml || !eps || !e1_bf16 || !e2_bf16 || !x || !wml || !w1 || !lens || !dwml || !dbml ||
      !dw1 || !db1 || !dw0 || !db0 || !aligned16(dz) || !aligned16(ml) || !aligned16(eps) ||
      !aligned16(x) || ((uintptr_t)e1_bf16 & 7) || ((uintptr_t)e2_bf16 & 7)) {
    mlvae_set_error("mlvae_encoder_bwd: null or misaligned pointer");
    return 1;
  }
  const int G = bwd_grid(N);
  if (!ws || ws_bytes < mlvae_encoder_workspace_size(B, T, F, E, Z)) {
    mlvae_set_error("mlvae_encoder_bwd: workspace too small");
    return 1;
  }
  EncBwdArgs a;
  a.N = N; a.T = T; a.B = B;
  a.dz = dz; a.ml = ml; a.eps = eps; a.x = x; a.wml = wml; a.w1 = w1; a.lens = lens;
  a.count = count; a.kl_scale = kl_scale;
  a.e1 = static_cast<const unsigned short*>(e1_bf16);
  a.e2 = static_cast<const unsigned short*>(e2_bf16);
  a.ws = ws;
  hipStream_t st = (hipStream_t)stream;
  const int slab = 2 * EW * EW + EW * F + 3 * EW;
  const int rblocks = (slab + 63) / 64;
  if (F == 80) {
    encoder_bwd_kernel<80><<<G, 256, 0, st>>>(a);
    MLVAE_CHECK_LAUNCH();
    encoder_reduce<80><<<rblocks, 256, 0, st>>>(G, ws, dwml, dbml, dw1, db1, dw0, db0);
  } else {
    encoder_bwd_kernel<64><<<G, 256, 0, st>>>(a);
    MLVAE_CHECK_LAUNCH();
    encoder_reduce<64><<<rblocks, 256, 0, st>>>(G, ws, dwml, dbml, dw1, db1, dw0, db0);
  }
  MLVAE_CHECK_LAUNCH();
  return 0;
}
