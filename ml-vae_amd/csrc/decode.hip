// MD-VAE Viterbi decode on gfx950.
//
// Replaces decode_plvl_md_lbl_seqs_full (ref:src/utils/decode_utils.py:374-565), which the MD-VAE
// training forward runs on the host through joblib (ref:src/models/MD_VAE/model.py:20,133-141):
// one workgroup per utterance, the DP over (canonical phoneme l, state beta in {correct,
// mispronounced}) advanced frame by frame as a wavefront -- column t is a function of column t-1
// only, so all l of a frame run in parallel (the reference's l-major loop order gives the same
// values) -- with the argmax paths in a byte map and the backtrack done from LDS windows of it.
//
// Numerics follow the reference exactly where it matters for the argmax decisions:
//   * the log terms are fp32: log of the eps-clamped fp32 probabilities (decode_utils.log, :8-14):
//     sigmoid(logits), 1 - sigmoid, softmax(pi_logits), the boundary posterior and the prior;
//   * the DP values are float64 sums in the reference's left-to-right order; the weighted pi term
//     is a float32 product (NumPy 2: Python float * float32 stays float32) and the first column
//     is all-float32 arithmetic;
//   * ties keep the first candidate in (hold, from-correct, from-mispronounced), as np.argmax.
// Bytes per utterance: the gathered logits T_i*L_i*4 + T_i*16 + the path map T_i*Lmax (write +
// read); latency-bound on the T_i serial frames.
#include "common.h"

namespace {

constexpr int DT = 256;          // threads
constexpr int MAXL = 1024;       // canonical phonemes per utterance (LDS columns)
constexpr int BW = 16;           // backtrack window (frames) staged in LDS
constexpr float LEPS = 1e-5f;

__device__ __forceinline__ float clog(float p) {  // decode_utils.log: [0, eps) -> eps
  return logf(p >= 0.f && p < LEPS ? LEPS : p);
}
__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + expf(-x)); }

struct DecArgs {
  int T, N, L;
  const float* logits; int ldl;    // [B, T, N] (row stride ldl)
  const float* bv;                 // [B, T] boundary posterior
  const float* pil;                // [B, T, 2] pi logits
  const float* prior;              // [N]
  const long long* seqs;           // [B, L] canonical phoneme ids
  const float* feat_lens;          // [B] relative
  const float* seq_lens;           // [B] relative
  float weight;
  unsigned char* path;             // [B, T, L] workspace: bits 0-1 beta = 0, bits 2-3 beta = 1
  int* bnd_out;                    // [B, T] 0/1, -1 past T_i
  int* flvl_out;                   // [B, T] frame labels, -1 past T_i
  int* plvl_out;                   // [B, L] phoneme labels, -1 past L_i
  int* lens_out;                   // [B, 2] (T_i, L_i)
  int* err;
};

__global__ __launch_bounds__(DT) void viterbi_kernel(DecArgs a) {
  __shared__ double val[2][MAXL][2];
  __shared__ unsigned char win[BW * MAXL];
  __shared__ float lt[4];  // per-frame terms: log p_b(0), log p_b(1), w*log p_pi(0), w*log p_pi(1)
  const int b = blockIdx.x, tid = threadIdx.x;
  const int T = a.T, L = a.L;
  int Ti = (int)rintf(a.feat_lens[b] * (float)T);
  int Li = (int)rintf(a.seq_lens[b] * (float)L);
  Ti = Ti > T ? T : Ti;
  Li = Li > L ? L : Li;
  for (int t = tid; t < T; t += DT) {
    a.bnd_out[(size_t)b * T + t] = -1;
    a.flvl_out[(size_t)b * T + t] = -1;
  }
  for (int l = tid; l < L; l += DT) a.plvl_out[(size_t)b * L + l] = -1;
  if (tid == 0) { a.lens_out[2 * b] = Ti; a.lens_out[2 * b + 1] = Li; }
  if (Ti <= 0 || Li <= 0 || Li > MAXL) {
    if (tid == 0) atomicOr(a.err, 16);
    return;  // the whole workgroup leaves before any barrier
  }
  const float w32 = a.weight;
  const float* lg = a.logits + (size_t)b * T * a.ldl;
  const long long* y = a.seqs + (size_t)b * L;
  unsigned char* path = a.path + (size_t)b * T * L;
  auto lyx = [&](int t, long long yl, int beta) {
    const float p = sigm(lg[(size_t)t * a.ldl + yl]);
    return clog(beta ? 1.f - p : p);
  };
  auto lpy = [&](long long yl, int beta) {
    const float p = a.prior[yl];
    return clog(beta ? 1.f - p : p);
  };
  auto frame_terms = [&](int t) {  // thread 0: the frame's shared log terms
    const float v = a.bv[(size_t)b * T + t];
    const float x0 = a.pil[((size_t)b * T + t) * 2], x1 = a.pil[((size_t)b * T + t) * 2 + 1];
    const float m = fmaxf(x0, x1);
    const float e0 = expf(x0 - m), e1 = expf(x1 - m), s = e0 + e1;
    lt[0] = clog(v);
    lt[1] = clog(1.f - v);
    lt[2] = w32 * clog(e0 / s);
    lt[3] = w32 * clog(e1 / s);
  };
  // column t = 0
  if (tid == 0) frame_terms(0);
  __syncthreads();
  for (int l = tid; l < Li; l += DT) {
    for (int be = 0; be < 2; ++be) {
      if (l == 0) {
        const long long y0 = y[0];
        val[0][0][be] = (double)((lt[2 + be] + lyx(0, y0, be)) - lpy(y0, be));  // all fp32
      } else {
        val[0][l][be] = -INFINITY;
      }
    }
  }
  __syncthreads();
  for (int t = 1; t < Ti; ++t) {
    const int cur = t & 1, prv = cur ^ 1;
    if (tid == 0) frame_terms(t);
    __syncthreads();
    const double lb0 = lt[0], lb1 = lt[1];
    for (int l = tid; l < Li; l += DT) {
      const long long yl = y[l];
      unsigned char pbits = 0;
      for (int be = 0; be < 2; ++be) {
        const double ex = lyx(t, yl, be), py = lpy(yl, be);
        const double hold = ((val[prv][l][be] + lb0) + ex) - py;
        double m = hold;
        int arg = 0;
        if (l > 0) {
          const double wp = lt[2 + be];
          const double fc = (((val[prv][l - 1][0] + lb1) + wp) + ex) - py;
          const double fi = (((val[prv][l - 1][1] + lb1) + wp) + ex) - py;
          if (fc > m) { m = fc; arg = 1; }
          if (fi > m) { m = fi; arg = 2; }
        }
        val[cur][l][be] = m;
        pbits |= (unsigned char)(arg << (2 * be));
      }
      path[(size_t)t * L + l] = pbits;
    }
    __syncthreads();  // column t complete; lt / the other column free
  }
  // backtracking (ref:src/utils/decode_utils.py:500-537), windows of BW frames staged in LDS
  __shared__ int bl, bbeta, bframe, nph;
  if (tid == 0) {
    const int c = (Ti - 1) & 1;
    bl = Li - 1;
    bbeta = val[c][Li - 1][0] > val[c][Li - 1][1] ? 0 : 1;
    bframe = bbeta;
    nph = 1;
    a.flvl_out[(size_t)b * T + Ti - 1] = bbeta;
    a.plvl_out[(size_t)b * L + Li - 1] = bbeta;
  }
  __syncthreads();
  for (int hi = Ti - 1; hi > 0; hi -= BW) {
    const int lo = hi - BW + 1 > 1 ? hi - BW + 1 : 1;  // frames [lo, hi]
    for (int e = tid; e < (hi - lo + 1) * Li; e += DT) {
      const int tt = e / Li, l = e % Li;
      win[tt * MAXL + l] = path[(size_t)(lo + tt) * L + l];
    }
    __syncthreads();
    if (tid == 0) {
      int l = bl, beta = bbeta, fr = bframe, n = nph;
      for (int t = hi; t >= lo; --t) {
        const int p = (win[(t - lo) * MAXL + l] >> (2 * beta)) & 3;
        if (p == 1 || p == 2) {
          a.bnd_out[(size_t)b * T + t] = 1;
          l -= 1;
          beta = p - 1;
          fr = beta;
          if (l >= 0) a.plvl_out[(size_t)b * L + l] = beta;
          ++n;
        }
        // the label this step appends (reversed: it belongs to frame t - 1)
        a.flvl_out[(size_t)b * T + t - 1] = fr;
        if (l < 0) break;
      }
      bl = l; bbeta = beta; bframe = fr; nph = n;
    }
    __syncthreads();
    if (bl < 0) break;
  }
  if (tid == 0) {
    a.bnd_out[(size_t)b * T] = 1;  // boundary at frame 0 (appended after the loop)
    if (bl != 0 || nph != Li) atomicOr(a.err, 8);  // assert l == t == 0 (decode_utils.py:529)
  }
  __syncthreads();
  for (int t = tid; t < Ti; t += DT)
    if (a.bnd_out[(size_t)b * T + t] < 0) a.bnd_out[(size_t)b * T + t] = 0;
}

}  // namespace

extern "C" size_t mlvae_viterbi_workspace_size(int B, int T, int L) { return (size_t)B * T * L; }

extern "C" int mlvae_viterbi_md(int B, int T, int N, int L, const float* logits, int ldl, const float* boundary_v,
                                const float* pi_logits, const float* prior, const long long* seqs,
                                const float* feat_lens, const float* seq_lens, float weight, void* ws,
                                size_t ws_bytes, int* boundary_out, int* flvl_out, int* plvl_out,
                                int* lens_out, int* err, void* stream) {
  if (B <= 0 || T <= 0) return 0;
  if (N <= 0 || L <= 0 || L > MAXL || ldl < N || !logits || !boundary_v || !pi_logits || !prior || !seqs ||
      !feat_lens || !seq_lens || !boundary_out || !flvl_out || !plvl_out || !lens_out || !err) {
    mlvae_set_error("mlvae_viterbi_md: bad shape/pointer (L <= %d)", MAXL);
    return 1;
  }
  if (!ws || ws_bytes < mlvae_viterbi_workspace_size(B, T, L)) {
    mlvae_set_error("mlvae_viterbi_md: workspace too small");
    return 1;
  }
  DecArgs a;
  a.T = T; a.N = N; a.L = L; a.logits = logits; a.ldl = ldl; a.bv = boundary_v; a.pil = pi_logits;
  a.prior = prior; a.seqs = seqs; a.feat_lens = feat_lens; a.seq_lens = seq_lens; a.weight = weight;
  a.path = static_cast<unsigned char*>(ws); a.bnd_out = boundary_out; a.flvl_out = flvl_out;
  a.plvl_out = plvl_out; a.lens_out = lens_out; a.err = err;
  viterbi_kernel<<<B, DT, 0, (hipStream_t)stream>>>(a);
  MLVAE_CHECK_LAUNCH();
  return 0;
}
