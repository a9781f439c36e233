// MFMA GEMM for every Linear / LSTM-projection product of the VAE train step.
//
//   C[M,N] = epi( alpha * op(A)[M,K] . op(B)[K,N] + bias1[N] + bias2[N] + beta * C )
//
// One kernel family covers the three shapes the step needs (row-major, fp32 in HBM):
//   forward Linear  Y = X W^T      TA=0 TB=1   (ref:src/modules/fc_block.py:10,14; decoder.py:14 input proj)
//   dgrad           dX = dY W      TA=0 TB=0
//   wgrad           dW = dY^T X    TA=1 TB=0   (K = B*T rows: split-K, deterministic reduce)
// plus a time-shifted B operand for the recurrent weight gradient dW_hh = sum_t dG_t^T h_{t-1}.
//
// Operands are staged global -> registers -> LDS (k-contiguous per row, padded) and consumed by
//   PREC_F32 : v_mfma_f32_32x32x2_f32  (exact fp32, the parity mode)
//   PREC_BF16: v_mfma_f32_32x32x16_bf16 (operands rounded to bf16 while staging, fp32 accumulate)
// 256 threads = 4 waves in a 2x2 grid; each wave owns (BM/2)x(BN/2) as 32x32 MFMA blocks.
#include "common.h"

namespace {

constexpr int BK = 32;

struct GemmArgs {
  int M, N, K;
  const float* A; int lda;
  const float* B; int ldb;
  float* C; int ldc;
  float alpha, beta;
  const float* bias1; const float* bias2;
  int epi;               // 0 none, 1 leaky-relu, 2 multiply by lrelu'(aux)
  const float* aux; int ldaux;
  int kshiftT, kshift;   // B row k -> k+kshift if 0 <= (k%T)+kshift < T else 0 (TB=0 only)
  int splits, kchunk;
  float* ws;             // split-K partials [splits][M][N]
  int vecA, vecB;        // 16-byte vector loads allowed
};

enum { EPI_NONE = 0, EPI_LRELU = 1, EPI_DLRELU = 2 };

template <int PREC> struct Lds;
template <> struct Lds<PREC_F32> { typedef float T; static constexpr int PAD = 4; };
template <> struct Lds<PREC_BF16> { typedef short T; static constexpr int PAD = 8; };

__device__ __forceinline__ float ld_guard(const float* p, bool ok) { return ok ? *p : 0.f; }

// Load one 4-element chunk of the logical A tile (rows i.., k..) into registers.
// KCONT: element (r, k) at base[r*ld + k] (k contiguous); else at base[k*ld + r].
template <bool KCONT>
__device__ __forceinline__ f32x4 load_chunk(const float* base, int ld, int r, int k, int R, int K,
                                            bool vec, int kshiftT, int kshift, bool shiftK) {
  f32x4 v = {0.f, 0.f, 0.f, 0.f};
  if (KCONT) {  // 4 consecutive k for one row r
    if (r >= R) return v;
    const float* p = base + (size_t)r * ld + k;
    if (vec && k + 3 < K) {
      v = *reinterpret_cast<const f32x4*>(p);
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = ld_guard(p + e, k + e < K);
    }
  } else {  // 4 consecutive r for one k
    if (k >= K) return v;
    int kk = k;
    if (shiftK) {
      int t = k % kshiftT + kshift;
      if (t < 0 || t >= kshiftT) return v;
      kk = k + kshift;
    }
    const float* p = base + (size_t)kk * ld + r;
    if (vec && r + 3 < R) {
      v = *reinterpret_cast<const f32x4*>(p);
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = ld_guard(p + e, r + e < R);
    }
  }
  return v;
}

template <int PREC>
__device__ __forceinline__ void store4_kcont(typename Lds<PREC>::T* dst, f32x4 v) {
  if constexpr (PREC == PREC_F32) {
    *reinterpret_cast<f32x4*>(dst) = v;
  } else {
    bf16x4 b = {f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3])};
    *reinterpret_cast<bf16x4*>(dst) = b;
  }
}
template <int PREC>
__device__ __forceinline__ void store1(typename Lds<PREC>::T* dst, float v) {
  if constexpr (PREC == PREC_F32) *dst = v; else *dst = f2bf(v);
}

// TWO: the fp32 weight gradients' two-level accumulation (below); the extra accumulator set
// would take the kernel past 256 VGPRs (one wave per SIMD: the fp32 mode's step 112 -> 141 ms),
// so those instances are bounded to two workgroups per CU
template <int BM, int BN, int PREC, bool TA, bool TB>
__global__ __launch_bounds__(256, (PREC == PREC_F32 && TA) ? 2 : 1) void gemm_kernel(GemmArgs g) {
  typedef typename Lds<PREC>::T LT;
  constexpr int LDK = BK + Lds<PREC>::PAD;
  constexpr int WM = BM / 2, WN = BN / 2, MB = WM / 32, NB = WN / 32;
  constexpr int NCA = BM * BK / 4 / 256, NCB = BN * BK / 4 / 256;  // chunks per thread
  static_assert(NCA >= 1 && NCB >= 1 && NCA <= 4 && NCB <= 4, "tile size");
  __shared__ __attribute__((aligned(16))) LT As[BM * LDK];
  __shared__ __attribute__((aligned(16))) LT Bs[BN * LDK];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  // XCD-aware tile order (bijective): blocks b, b+8, ... share an XCD's L2, so each XCD gets a
  // contiguous run of tiles; consecutive tiles share the A row-panel (all n for one m).
  const int TM = (g.M + BM - 1) / BM, TN = (g.N + BN - 1) / BN, ntiles = TM * TN;
  int tile;
  {
    const int b = blockIdx.x, xcd = b % 8, local = b / 8, q = ntiles / 8, r = ntiles % 8;
    tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + local;
  }
  const int m0 = (tile / TN) * BM, n0 = (tile % TN) * BN;
  const int kbeg = blockIdx.z * g.kchunk;
  const int kend = min(g.K, kbeg + g.kchunk);
  const bool shiftK = (!TB) && g.kshift != 0;

  f32x16 acc[MB][NB];
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[i][j][v] = 0.f;
  // fp32 parity mode: two-level accumulation over long K (the weight gradients sum over B*T
  // frames).  The MFMA chain runs over KBLK = 256 of K, then folds into `tot`: a sequential fp32
  // chain of kc / 2 accumulations (kc = 10,667 at B = 256) rounds ~sqrt(kc / 256) times worse
  // than the fp32 oracle's blocked sums (round 5, fp64-anchored whole-step test: dW_ih_l1 3.5x
  // the oracle's error at B = 32 before, tests/test_gpu_trajectory.py)
  // Only the TA instances (the weight gradients: K = frames) run it -- the projections' and
  // dgrads' K is the feature width (<= 4H)
  constexpr int KBLK = 256;
  constexpr bool TWO = PREC == PREC_F32 && TA;
  f32x16 tot[TWO ? MB : 1][TWO ? NB : 1];
  if constexpr (TWO) {
#pragma unroll
    for (int i = 0; i < MB; ++i)
#pragma unroll
      for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int v = 0; v < 16; ++v) tot[i][j][v] = 0.f;
  }

  // K-contiguous operand: float4 chunks along k (NC per thread).
  // M-contiguous operand (stored [K][rows]): 4k x 4r blocks, transposed in registers so the
  // LDS image stays [row][k] and every LDS store is one 8/16-byte write.
  constexpr int NBA = (BK / 4) * (BM / 4), NBB = (BK / 4) * (BN / 4);  // 4x4 blocks per tile
  f32x4 ra[4], rb[4];
  auto load_kc = [&](f32x4* r, const float* base, int ld, int r0, int R, int k0, bool vec, int NC) {
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      int idx = tid + 256 * c;
      int rr = idx / (BK / 4), kc = (idx % (BK / 4)) * 4;
      r[c] = load_chunk<true>(base, ld, r0 + rr, k0 + kc, R, kend, vec, 0, 0, false);
    }
  };
  auto load_mc = [&](f32x4* r, const float* base, int ld, int r0, int R, int k0, bool vec, int NB_,
                     bool shift) {
    if (tid < NB_) {
      // lanes sweep k first: 8 lanes cover one 4-row x 32-k strip -> conflict-free LDS stores,
      // and every load instruction still reads whole 128-byte row segments
      const int kq = (tid % (BK / 4)) * 4;
      const int rq = (tid / (BK / 4)) * 4;
#pragma unroll
      for (int e = 0; e < 4; ++e)
        r[e] = load_chunk<false>(base, ld, r0 + rq, k0 + kq + e, R, kend, vec, g.kshiftT, g.kshift, shift);
    }
  };
  auto store_kc = [&](LT* L, const f32x4* r, int NC) {
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      int idx = tid + 256 * c;
      int rr = idx / (BK / 4), kc = (idx % (BK / 4)) * 4;
      store4_kcont<PREC>(&L[rr * LDK + kc], r[c]);
    }
  };
  auto store_mc = [&](LT* L, const f32x4* r, int NB_) {
    if (tid < NB_) {
      const int kq = (tid % (BK / 4)) * 4;
      const int rq = (tid / (BK / 4)) * 4;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        f32x4 t = {r[0][e], r[1][e], r[2][e], r[3][e]};
        store4_kcont<PREC>(&L[(rq + e) * LDK + kq], t);
      }
    }
  };
  auto gload = [&](int k0) {
    if (!TA) load_kc(ra, g.A, g.lda, m0, g.M, k0, g.vecA, NCA);
    else load_mc(ra, g.A, g.lda, m0, g.M, k0, g.vecA, NBA, false);
    if (TB) load_kc(rb, g.B, g.ldb, n0, g.N, k0, g.vecB, NCB);
    else load_mc(rb, g.B, g.ldb, n0, g.N, k0, g.vecB, NBB, shiftK);
  };
  auto lstore = [&]() {
    if (!TA) store_kc(As, ra, NCA); else store_mc(As, ra, NBA);
    if (TB) store_kc(Bs, rb, NCB); else store_mc(Bs, rb, NBB);
  };

  const int l32 = lane & 31, h = lane >> 5;
  if (kbeg < kend) gload(kbeg);
  for (int k0 = kbeg; k0 < kend; k0 += BK) {
    lstore();
    __syncthreads();
    if (k0 + BK < kend) gload(k0 + BK);
    if constexpr (PREC == PREC_F32) {
#pragma unroll
      for (int kk = 0; kk < BK; kk += 8) {
        f32x4 a4[MB], b4[NB];
#pragma unroll
        for (int i = 0; i < MB; ++i)
          a4[i] = *reinterpret_cast<const f32x4*>(&As[(wm * WM + i * 32 + l32) * LDK + kk + 4 * h]);
#pragma unroll
        for (int j = 0; j < NB; ++j)
          b4[j] = *reinterpret_cast<const f32x4*>(&Bs[(wn * WN + j * 32 + l32) * LDK + kk + 4 * h]);
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int i = 0; i < MB; ++i)
#pragma unroll
            for (int j = 0; j < NB; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a4[i][e], b4[j][e], acc[i][j], 0, 0, 0);
      }
      if (TWO && ((k0 - kbeg + BK) % KBLK == 0 || k0 + BK >= kend)) {  // fold the block (uniform)
#pragma unroll
        for (int i = 0; i < MB; ++i)
#pragma unroll
          for (int j = 0; j < NB; ++j)
#pragma unroll
            for (int v = 0; v < 16; ++v) { tot[i][j][v] += acc[i][j][v]; acc[i][j][v] = 0.f; }
      }
    } else {
#pragma unroll
      for (int kk = 0; kk < BK; kk += 16) {
        bf16x8 a8[MB], b8[NB];
#pragma unroll
        for (int i = 0; i < MB; ++i)
          a8[i] = *reinterpret_cast<const bf16x8*>(&As[(wm * WM + i * 32 + l32) * LDK + kk + 8 * h]);
#pragma unroll
        for (int j = 0; j < NB; ++j)
          b8[j] = *reinterpret_cast<const bf16x8*>(&Bs[(wn * WN + j * 32 + l32) * LDK + kk + 8 * h]);
#pragma unroll
        for (int i = 0; i < MB; ++i)
#pragma unroll
          for (int j = 0; j < NB; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a8[i], b8[j], acc[i][j], 0, 0, 0);
      }
    }
    __syncthreads();
  }

  if constexpr (TWO) {
#pragma unroll
    for (int i = 0; i < MB; ++i)
#pragma unroll
      for (int j = 0; j < NB; ++j) acc[i][j] = tot[i][j];
  }
  // epilogue: C/D layout col = lane&31, row = (v&3) + 8*(v>>2) + 4*(lane>>5)
  const bool split = g.splits > 1;
  float* wsz = split ? g.ws + (size_t)blockIdx.z * g.M * g.N : nullptr;
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int col = n0 + wn * WN + j * 32 + l32;
      if (col >= g.N) continue;
      float b = 0.f;
      if (!split) {
        if (g.bias1) b += g.bias1[col];
        if (g.bias2) b += g.bias2[col];
      }
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int row = m0 + wm * WM + i * 32 + (v & 3) + 8 * (v >> 2) + 4 * h;
        if (row >= g.M) continue;
        if (split) {
          wsz[(size_t)row * g.N + col] = acc[i][j][v];
          continue;
        }
        float val = g.alpha * acc[i][j][v] + b;
        float* cp = g.C + (size_t)row * g.ldc + col;
        if (g.beta != 0.f) val += g.beta * *cp;
        if (g.epi == EPI_LRELU) val = lrelu(val);
        else if (g.epi == EPI_DLRELU) val *= lrelu_d(g.aux[(size_t)row * g.ldaux + col]);
        *cp = val;
      }
    }
}

// Deterministic split-K combine: C = epi(alpha * sum_z ws[z] + bias + beta*C), fixed z order.
__global__ __launch_bounds__(256) void splitk_reduce(GemmArgs g) {
  const size_t MN = (size_t)g.M * g.N;
  for (size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x; idx < MN; idx += (size_t)gridDim.x * 256) {
    float s = 0.f;
    for (int z = 0; z < g.splits; ++z) s += g.ws[z * MN + idx];
    const int row = (int)(idx / g.N), col = (int)(idx % g.N);
    float val = g.alpha * s;
    if (g.bias1) val += g.bias1[col];
    if (g.bias2) val += g.bias2[col];
    float* cp = g.C + (size_t)row * g.ldc + col;
    if (g.beta != 0.f) val += g.beta * *cp;
    if (g.epi == EPI_LRELU) val = lrelu(val);
    else if (g.epi == EPI_DLRELU) val *= lrelu_d(g.aux[(size_t)row * g.ldaux + col]);
    *cp = val;
  }
}

template <int BM, int BN, int PREC>
void launch_t(const GemmArgs& g, dim3 grid, bool ta, bool tb, hipStream_t s) {
  if (!ta && tb) gemm_kernel<BM, BN, PREC, false, true><<<grid, 256, 0, s>>>(g);
  else if (!ta && !tb) gemm_kernel<BM, BN, PREC, false, false><<<grid, 256, 0, s>>>(g);
  else if (ta && !tb) gemm_kernel<BM, BN, PREC, true, false><<<grid, 256, 0, s>>>(g);
  else gemm_kernel<BM, BN, PREC, true, true><<<grid, 256, 0, s>>>(g);
}

inline bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace

// Split-K plan shared by the launcher and the workspace query.
static void gemm_plan(int M, int N, int K, int* bm, int* bn, int* splits, int* kchunk) {
  const bool big = (M >= 128 && N >= 128);
  *bm = big ? 128 : 64;
  *bn = big ? 128 : 64;
  const long tiles = (long)((M + *bm - 1) / *bm) * ((N + *bn - 1) / *bn);
  int s = 1;
  // long-K products (weight gradients over B*T rows): split K until ~3 blocks per CU are
  // resident, so the load latency of one block hides behind the MFMAs of the others
  if (tiles < 768 && K >= 4 * BK * 8) {
    s = (int)((768 + tiles - 1) / tiles);
    int maxs = K / (BK * 8);  // keep >= 8 k-tiles per split
    if (s > maxs) s = maxs;
    if (s > 64) s = 64;
    if (s < 1) s = 1;
  }
  int kc = (K + s - 1) / s;
  kc = (kc + BK - 1) / BK * BK;
  s = (K + kc - 1) / kc;
  *splits = s;
  *kchunk = kc;
}

extern "C" size_t mlvae_gemm_workspace_size(int M, int N, int K) {
  int bm, bn, s, kc;
  gemm_plan(M, N, K, &bm, &bn, &s, &kc);
  return s > 1 ? (size_t)s * M * N * sizeof(float) : 0;
}

extern "C" int mlvae_gemm(int prec, int trans_a, int trans_b, int M, int N, int K, float alpha,
                          const float* A, int lda, const float* B, int ldb, float beta, float* C,
                          int ldc, const float* bias1, const float* bias2, int epi,
                          const float* aux, int ldaux, int kshift_T, int kshift, float* ws,
                          size_t ws_bytes, void* stream) {
  if (M < 0 || N < 0 || K < 0 || !C) { mlvae_set_error("mlvae_gemm: bad shape/ptr"); return 1; }
  if (M == 0 || N == 0) return 0;
  if (prec != PREC_F32 && prec != PREC_BF16) { mlvae_set_error("mlvae_gemm: bad prec %d", prec); return 1; }
  if (epi == EPI_DLRELU && !aux) { mlvae_set_error("mlvae_gemm: DLRELU needs aux"); return 1; }
  if (kshift != 0 && (trans_b || kshift_T <= 0)) { mlvae_set_error("mlvae_gemm: kshift needs TB=0, T>0"); return 1; }
  GemmArgs g;
  g.M = M; g.N = N; g.K = K; g.A = A; g.lda = lda; g.B = B; g.ldb = ldb; g.C = C; g.ldc = ldc;
  g.alpha = alpha; g.beta = beta; g.bias1 = bias1; g.bias2 = bias2; g.epi = epi; g.aux = aux;
  g.ldaux = ldaux; g.kshiftT = kshift_T; g.kshift = kshift; g.ws = ws;
  g.vecA = aligned16(A) && (lda % 4 == 0);
  g.vecB = aligned16(B) && (ldb % 4 == 0);
  int bm, bn, s, kc;
  gemm_plan(M, N, K, &bm, &bn, &s, &kc);
  if (K == 0) { s = 1; kc = BK; }
  if (s > 1 && (!ws || ws_bytes < (size_t)s * M * N * sizeof(float))) {
    s = 1; kc = ((K + BK - 1) / BK) * BK;  // no workspace: single pass
  }
  g.splits = s; g.kchunk = kc;
  hipStream_t st = (hipStream_t)stream;
  dim3 grid(((N + bn - 1) / bn) * ((M + bm - 1) / bm), 1, s);
  if (bm == 128) {
    if (prec == PREC_F32) launch_t<128, 128, PREC_F32>(g, grid, trans_a, trans_b, st);
    else launch_t<128, 128, PREC_BF16>(g, grid, trans_a, trans_b, st);
  } else {
    if (prec == PREC_F32) launch_t<64, 64, PREC_F32>(g, grid, trans_a, trans_b, st);
    else launch_t<64, 64, PREC_BF16>(g, grid, trans_a, trans_b, st);
  }
  MLVAE_CHECK_LAUNCH();
  if (s > 1) {
    size_t MN = (size_t)M * N;
    int blocks = (int)((MN + 255) / 256);
    if (blocks > 2048) blocks = 2048;
    splitk_reduce<<<blocks, 256, 0, st>>>(g);
    MLVAE_CHECK_LAUNCH();
  }
  return 0;
}
