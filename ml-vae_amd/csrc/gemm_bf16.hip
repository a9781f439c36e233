// bf16-MFMA GEMM with bf16 or fp32 operands in HBM, software-pipelined (gfx950).
//
//   C[M,N] = epi( alpha * op(A)[M,K] . op(B)[K,N] + bias1[N] + bias2[N] + beta * C )   (C fp32)
//
// The bf16 precision mode's GEMMs (gemm.hip keeps the exact-fp32 parity kernel).  Operands
// may be stored as bf16 (the step writes bf16 copies of its GEMM operands: half the HBM/L2
// bytes of fp32, and a 16-byte load carries 8 k) or fp32 (rounded to bf16 while staging).
//   tile 128x128, BK = 64, 256 threads = 4 waves (2x2, 64x64 each as 2x2 v_mfma_f32_32x32x16_bf16)
//   LDS: two [row][k] bf16 images per operand (row stride 72: 16-byte aligned fragment reads,
//   2-way at most), ONE barrier per K-step: tile k+1 is written from registers into the idle
//   buffer and tile k+2's global loads are issued before the MFMAs of tile k.
//   K-contiguous operands load 16 B along k; M/N-contiguous ones (A^T of a weight gradient,
//   a [K][N] weight) load 4k x 8r (bf16) or 4k x 4r (fp32) blocks and transpose in registers,
//   lanes sweeping k first so the 8-byte LDS stores of a wave stay within two bank rows.
// Same epilogues, time-shifted B rows (kshift) and deterministic split-K as gemm.hip.
#include "common.h"

namespace {

constexpr int BM = 128, BN = 128, BK = 64, LDK = BK + 8;
constexpr int TILE_ELEMS = BM * LDK;              // one operand image (BM == BN)
constexpr size_t LDS_BYTES = (size_t)2 * 2 * TILE_ELEMS * sizeof(short);

struct G2Args {
  int M, N, K;
  const void* A; int lda;
  const void* B; int ldb;
  float* C; int ldc;
  float alpha, beta;
  const float* bias1; const float* bias2;
  int epi;
  const float* aux; int ldaux;
  int kshiftT, kshift;
  int splits, kchunk;
  float* ws;
  unsigned long long dseed;   // EPI_DROPOUT: mask of flat element doff + row*ldc + col
  unsigned long long doff;
  float dkeep, dscale;
};

enum { EPI_NONE = 0, EPI_LRELU = 1, EPI_DLRELU = 2, EPI_DROPOUT = 3 };

// shared epilogue: bias already added; beta * C, then the activation / mask
__device__ __forceinline__ float epi_apply(const G2Args& g, float val, int row, int col, float* cp) {
  if (g.beta != 0.f) val += g.beta * *cp;
  if (g.epi == EPI_LRELU) val = lrelu(val);
  else if (g.epi == EPI_DLRELU) val *= lrelu_d(g.aux[(size_t)row * g.ldaux + col]);
  else if (g.epi == EPI_DROPOUT) val *= dropout_scale(g.dseed, g.doff + (size_t)row * g.ldc + col, g.dkeep, g.dscale);
  return val;
}

__device__ __forceinline__ unsigned short bf_bits(float x) { return (unsigned short)f2bf(x); }

// ---- staging of one operand tile (128 rows x 64 k) ---------------------------------------
// KC = k-contiguous in HBM (element (r,k) at p[r*ld + k]); else (r,k) at p[k*ld + r].
// Register image per thread: NV u32x4 (bf16 source) or f32x4 (fp32 source).
template <bool KC, bool BF> struct Stage;

// k-contiguous, bf16: 1024 chunks of 8 k -> 4 per thread
template <> struct Stage<true, true> {
  static constexpr int NV = 4;
  typedef u32x4 V;
  __device__ static void load(V* r, const void* base, int ld, int r0, int R, int k0, int kend,
                              int, int, bool) {
    const unsigned short* p = static_cast<const unsigned short*>(base);
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      const int idx = threadIdx.x + 256 * c, rr = idx >> 3, kc = (idx & 7) * 8;
      const int row = r0 + rr, k = k0 + kc;
      if (row < R && k + 7 < kend) {
        r[c] = *reinterpret_cast<const u32x4*>(p + (size_t)row * ld + k);
      } else {
        unsigned short e[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) e[j] = (row < R && k + j < kend) ? p[(size_t)row * ld + k + j] : 0;
        r[c] = u32x4{e[0] | ((unsigned)e[1] << 16), e[2] | ((unsigned)e[3] << 16),
                     e[4] | ((unsigned)e[5] << 16), e[6] | ((unsigned)e[7] << 16)};
      }
    }
  }
  __device__ static void store(short* L, const V* r) {
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      const int idx = threadIdx.x + 256 * c, rr = idx >> 3, kc = (idx & 7) * 8;
      *reinterpret_cast<u32x4*>(L + rr * LDK + kc) = r[c];
    }
  }
};

// k-contiguous, fp32: 2048 chunks of 4 k -> 8 per thread
template <> struct Stage<true, false> {
  static constexpr int NV = 8;
  typedef f32x4 V;
  __device__ static void load(V* r, const void* base, int ld, int r0, int R, int k0, int kend,
                              int, int, bool) {
    const float* p = static_cast<const float*>(base);
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      const int idx = threadIdx.x + 256 * c, rr = idx >> 4, kc = (idx & 15) * 4;
      const int row = r0 + rr, k = k0 + kc;
      if (row < R && k + 3 < kend) {
        r[c] = *reinterpret_cast<const f32x4*>(p + (size_t)row * ld + k);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) r[c][j] = (row < R && k + j < kend) ? p[(size_t)row * ld + k + j] : 0.f;
      }
    }
  }
  __device__ static void store(short* L, const V* r) {
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      const int idx = threadIdx.x + 256 * c, rr = idx >> 4, kc = (idx & 15) * 4;
      bf16x4 b = {f2bf(r[c][0]), f2bf(r[c][1]), f2bf(r[c][2]), f2bf(r[c][3])};
      *reinterpret_cast<bf16x4*>(L + rr * LDK + kc) = b;
    }
  }
};

// row-contiguous, bf16: 256 blocks of 4k x 8r -> 1 per thread (lanes sweep k first)
template <> struct Stage<false, true> {
  static constexpr int NV = 4;
  typedef u32x4 V;
  __device__ static void load(V* r, const void* base, int ld, int r0, int R, int k0, int kend,
                              int shiftT, int shift, bool shiftK) {
    const unsigned short* p = static_cast<const unsigned short*>(base);
    const int kb = (threadIdx.x & 15) * 4, rb = (threadIdx.x >> 4) * 8;
    const int row = r0 + rb;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      int k = k0 + kb + e;
      bool ok = k < kend;
      if (shiftK && ok) {
        const int t = k % shiftT + shift;
        ok = t >= 0 && t < shiftT;
        k += shift;
      }
      if (ok && row + 7 < R) {
        r[e] = *reinterpret_cast<const u32x4*>(p + (size_t)k * ld + row);
      } else {
        unsigned short v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (ok && row + j < R) ? p[(size_t)k * ld + row + j] : 0;
        r[e] = u32x4{v[0] | ((unsigned)v[1] << 16), v[2] | ((unsigned)v[3] << 16),
                     v[4] | ((unsigned)v[5] << 16), v[6] | ((unsigned)v[7] << 16)};
      }
    }
  }
  __device__ static void store(short* L, const V* r) {
    const int kb = (threadIdx.x & 15) * 4, rb = (threadIdx.x >> 4) * 8;
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const int d = m >> 1, sh = (m & 1) * 16;
      const unsigned lo = ((r[0][d] >> sh) & 0xffffu) | (((r[1][d] >> sh) & 0xffffu) << 16);
      const unsigned hi = ((r[2][d] >> sh) & 0xffffu) | (((r[3][d] >> sh) & 0xffffu) << 16);
      *reinterpret_cast<u32x2*>(L + (rb + m) * LDK + kb) = u32x2{lo, hi};
    }
  }
};

// row-contiguous, fp32: 512 blocks of 4k x 4r -> 2 per thread
template <> struct Stage<false, false> {
  static constexpr int NV = 8;
  typedef f32x4 V;
  __device__ static void load(V* r, const void* base, int ld, int r0, int R, int k0, int kend,
                              int shiftT, int shift, bool shiftK) {
    const float* p = static_cast<const float*>(base);
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int blk = threadIdx.x + 256 * b;
      const int kb = (blk & 15) * 4, rb = (blk >> 4) * 4;
      const int row = r0 + rb;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        int k = k0 + kb + e;
        bool ok = k < kend;
        if (shiftK && ok) {
          const int t = k % shiftT + shift;
          ok = t >= 0 && t < shiftT;
          k += shift;
        }
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (ok && row + 3 < R) {
          v = *reinterpret_cast<const f32x4*>(p + (size_t)k * ld + row);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = (ok && row + j < R) ? p[(size_t)k * ld + row + j] : 0.f;
        }
        r[b * 4 + e] = v;
      }
    }
  }
  __device__ static void store(short* L, const V* r) {
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int blk = threadIdx.x + 256 * b;
      const int kb = (blk & 15) * 4, rb = (blk >> 4) * 4;
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        bf16x4 t = {f2bf(r[b * 4 + 0][m]), f2bf(r[b * 4 + 1][m]), f2bf(r[b * 4 + 2][m]),
                    f2bf(r[b * 4 + 3][m])};
        *reinterpret_cast<bf16x4*>(L + (rb + m) * LDK + kb) = t;
      }
    }
  }
};

template <bool TA, bool TB, bool ABF, bool BBF>
__global__ __launch_bounds__(256) void gemm_bf16_kernel(G2Args g) {
  typedef Stage<!TA, ABF> SA;
  typedef Stage<TB, BBF> SB;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  short* lds = reinterpret_cast<short*>(smem);  // [2 bufs][A image, B image]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int TM = (g.M + BM - 1) / BM, TN = (g.N + BN - 1) / BN, ntiles = TM * TN;
  int tile;
  {  // XCD-aware bijective order: each XCD works a contiguous run of tiles (shared A panels)
    const int b = blockIdx.x, xcd = b % 8, local = b / 8, q = ntiles / 8, r = ntiles % 8;
    tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + local;
  }
  const int m0 = (tile / TN) * BM, n0 = (tile % TN) * BN;
  const int kbeg = blockIdx.z * g.kchunk;
  const int kend = min(g.K, kbeg + g.kchunk);
  const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;
  const bool shiftK = (!TB) && g.kshift != 0;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[i][j][v] = 0.f;

  typename SA::V ra[SA::NV];
  typename SB::V rb[SB::NV];
  auto gload = [&](int k0) {
    SA::load(ra, g.A, g.lda, m0, g.M, k0, kend, 0, 0, false);
    SB::load(rb, g.B, g.ldb, n0, g.N, k0, kend, g.kshiftT, g.kshift, shiftK);
  };
  auto lstore = [&](int buf) {
    SA::store(lds + (buf * 2 + 0) * TILE_ELEMS, ra);
    SB::store(lds + (buf * 2 + 1) * TILE_ELEMS, rb);
  };

  const int l32 = lane & 31, h = lane >> 5;
  if (nk > 0) {
    gload(kbeg);
    lstore(0);
    if (nk > 1) gload(kbeg + BK);
    __syncthreads();
  }
  for (int it = 0; it < nk; ++it) {
    const int cur = it & 1;
    if (it + 1 < nk) lstore(cur ^ 1);               // tile it+1 -> idle buffer
    if (it + 2 < nk) gload(kbeg + (it + 2) * BK);   // tile it+2 in flight during the MFMAs
    const short* As = lds + (cur * 2 + 0) * TILE_ELEMS;
    const short* Bs = lds + (cur * 2 + 1) * TILE_ELEMS;
#pragma unroll
    for (int kk = 0; kk < BK; kk += 16) {
      bf16x8 a8[2], b8[2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
        a8[i] = *reinterpret_cast<const bf16x8*>(As + (wm * 64 + i * 32 + l32) * LDK + kk + 8 * h);
#pragma unroll
      for (int j = 0; j < 2; ++j)
        b8[j] = *reinterpret_cast<const bf16x8*>(Bs + (wn * 64 + j * 32 + l32) * LDK + kk + 8 * h);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a8[i], b8[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }

  // epilogue: C/D layout col = lane&31, row = (v&3) + 8*(v>>2) + 4*(lane>>5)
  const bool split = g.splits > 1;
  float* wsz = split ? g.ws + (size_t)blockIdx.z * g.M * g.N : nullptr;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = n0 + wn * 64 + j * 32 + l32;
      if (col >= g.N) continue;
      float b = 0.f;
      if (!split) {
        if (g.bias1) b += g.bias1[col];
        if (g.bias2) b += g.bias2[col];
      }
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int row = m0 + wm * 64 + i * 32 + (v & 3) + 8 * (v >> 2) + 4 * h;
        if (row >= g.M) continue;
        if (split) {
          wsz[(size_t)row * g.N + col] = acc[i][j][v];
          continue;
        }
        float* cp = g.C + (size_t)row * g.ldc + col;
        *cp = epi_apply(g, g.alpha * acc[i][j][v] + b, row, col, cp);
      }
    }
}

// Deterministic split-K reduce: a block takes 64 consecutive elements; its four 64-thread groups
// sum the splits z = g, g + 4, ... in order, then the four partials combine in a fixed order
// (a tiny-output weight gradient over 250 splits had one thread walking all of them)
__global__ __launch_bounds__(256) void splitk_reduce2(G2Args g) {
  __shared__ float part[4][64];
  const size_t MN = (size_t)g.M * g.N;
  const int e = threadIdx.x & 63, grp = threadIdx.x >> 6;
  for (size_t base = (size_t)blockIdx.x * 64; base < MN; base += (size_t)gridDim.x * 64) {
    const size_t idx = base + e;
    float s = 0.f;
    if (idx < MN)
#pragma unroll 8  // loads in flight; the adds keep their order
      for (int z = grp; z < g.splits; z += 4) s += g.ws[z * MN + idx];
    part[grp][e] = s;
    __syncthreads();
    if (grp == 0 && idx < MN) {
      const int row = (int)(idx / g.N), col = (int)(idx % g.N);
      float val = g.alpha * ((part[0][e] + part[1][e]) + (part[2][e] + part[3][e]));
      if (g.bias1) val += g.bias1[col];
      if (g.bias2) val += g.bias2[col];
      float* cp = g.C + (size_t)row * g.ldc + col;
      *cp = epi_apply(g, val, row, col, cp);
    }
    __syncthreads();
  }
}

template <bool TA, bool TB, bool ABF, bool BBF>
int launch4(const G2Args& g, dim3 grid, hipStream_t s) {
  auto k = gemm_bf16_kernel<TA, TB, ABF, BBF>;
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)LDS_BYTES) != hipSuccess) {
      mlvae_set_error("gemm_bf16: cannot reserve %zu B LDS", LDS_BYTES);
      return 2;
    }
    attr = true;
  }
  k<<<grid, 256, LDS_BYTES, s>>>(g);
  return 0;
}

template <bool TA, bool TB>
int launch2(const G2Args& g, dim3 grid, bool abf, bool bbf, hipStream_t s) {
  if (abf && bbf) return launch4<TA, TB, true, true>(g, grid, s);
  if (abf) return launch4<TA, TB, true, false>(g, grid, s);
  if (bbf) return launch4<TA, TB, false, true>(g, grid, s);
  return launch4<TA, TB, false, false>(g, grid, s);
}

}  // namespace

// Split-K plan: split long-K products (weight gradients over B*T rows) until ~3 blocks per
// CU are in flight, keeping >= 8 K-steps per split.  Up to 256 splits for one- or two-tile
// products: the decoder heads' weight gradients (M, N <= 128, K = B*T = 128,000 at c3) on 64
// splits ran on 64 CUs streaming their fp32 operands (108 vs 36 us per launch for 74 MB)
static void gemm2_plan(int M, int N, int K, int* splits, int* kchunk) {
  const long tiles = (long)((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  int s = 1;
  if (tiles < 768 && K >= BK * 16) {
    s = (int)((768 + tiles - 1) / tiles);
    int maxs = K / (BK * 8);
    if (s > maxs) s = maxs;
    if (s > (tiles <= 2 ? 256 : 64)) s = tiles <= 2 ? 256 : 64;
    if (s < 1) s = 1;
  }
  int kc = (K + s - 1) / s;
  kc = (kc + BK - 1) / BK * BK;
  s = kc > 0 ? (K + kc - 1) / kc : 1;
  *splits = s < 1 ? 1 : s;
  *kchunk = kc > 0 ? kc : BK;
}

extern "C" size_t mlvae_gemm_ex_workspace_size(int M, int N, int K) {
  int s, kc;
  gemm2_plan(M, N, K, &s, &kc);
  return s > 1 ? (size_t)s * M * N * sizeof(float) : 0;
}

extern "C" int mlvae_gemm_ex_drop(int trans_a, int trans_b, int M, int N, int K, float alpha,
                                  const void* A, int a_bf16, int lda, const void* B, int b_bf16,
                                  int ldb, float beta, float* C, int ldc, const float* bias1,
                                  const float* bias2, int epi, const float* aux, int ldaux,
                                  int kshift_T, int kshift, unsigned long long drop_seed,
                                  unsigned long long drop_offset, float drop_p, float* ws,
                                  size_t ws_bytes, void* stream) {
  if (M < 0 || N < 0 || K < 0 || !C || (K > 0 && (!A || !B))) {
    mlvae_set_error("mlvae_gemm_ex: bad shape/ptr");
    return 1;
  }
  if (M == 0 || N == 0) return 0;
  if (epi == EPI_DLRELU && !aux) { mlvae_set_error("mlvae_gemm_ex: DLRELU needs aux"); return 1; }
  if (epi == EPI_DROPOUT && !(drop_p >= 0.f && drop_p < 1.f)) {
    mlvae_set_error("mlvae_gemm_ex: dropout p=%f out of range", drop_p);
    return 1;
  }
  if (epi < EPI_NONE || epi > EPI_DROPOUT) { mlvae_set_error("mlvae_gemm_ex: bad epilogue %d", epi); return 1; }
  if (kshift != 0 && (trans_b || kshift_T <= 0)) {
    mlvae_set_error("mlvae_gemm_ex: kshift needs trans_b = 0, T > 0");
    return 1;
  }
  // vector loads need 16-byte aligned rows along the contiguous dimension
  const size_t ea = a_bf16 ? 2 : 4, eb = b_bf16 ? 2 : 4;
  const int va = (int)(16 / ea), vb = (int)(16 / eb);
  if (((uintptr_t)A % 16) || (lda % va) || ((uintptr_t)B % 16) || (ldb % vb)) {
    mlvae_set_error("mlvae_gemm_ex: operands need 16-byte aligned rows (lda %% %d, ldb %% %d)", va, vb);
    return 1;
  }
  G2Args g;
  g.M = M; g.N = N; g.K = K; g.A = A; g.lda = lda; g.B = B; g.ldb = ldb; g.C = C; g.ldc = ldc;
  g.alpha = alpha; g.beta = beta; g.bias1 = bias1; g.bias2 = bias2; g.epi = epi; g.aux = aux;
  g.ldaux = ldaux; g.kshiftT = kshift_T; g.kshift = kshift; g.ws = ws;
  g.dseed = drop_seed; g.doff = drop_offset; g.dkeep = 1.f - drop_p; g.dscale = 1.f / (1.f - drop_p);
  int s, kc;
  gemm2_plan(M, N, K, &s, &kc);
  if (s > 1 && (!ws || ws_bytes < (size_t)s * M * N * sizeof(float))) {
    s = 1;
    kc = ((K + BK - 1) / BK) * BK;
  }
  if (K == 0) { s = 1; kc = BK; }
  g.splits = s; g.kchunk = kc;
  hipStream_t st = (hipStream_t)stream;
  dim3 grid(((N + BN - 1) / BN) * ((M + BM - 1) / BM), 1, s);
  int rc;
  if (!trans_a && trans_b) rc = launch2<false, true>(g, grid, a_bf16, b_bf16, st);
  else if (!trans_a && !trans_b) rc = launch2<false, false>(g, grid, a_bf16, b_bf16, st);
  else if (trans_a && !trans_b) rc = launch2<true, false>(g, grid, a_bf16, b_bf16, st);
  else rc = launch2<true, true>(g, grid, a_bf16, b_bf16, st);
  if (rc) return rc;
  MLVAE_CHECK_LAUNCH();
  if (s > 1) {
    size_t MN = (size_t)M * N;
    int blocks = (int)((MN + 63) / 64);
    if (blocks > 4096) blocks = 4096;
    splitk_reduce2<<<blocks, 256, 0, st>>>(g);
    MLVAE_CHECK_LAUNCH();
  }
  return 0;
}

extern "C" int mlvae_gemm_ex(int trans_a, int trans_b, int M, int N, int K, float alpha,
                             const void* A, int a_bf16, int lda, const void* B, int b_bf16,
                             int ldb, float beta, float* C, int ldc, const float* bias1,
                             const float* bias2, int epi, const float* aux, int ldaux,
                             int kshift_T, int kshift, float* ws, size_t ws_bytes, void* stream) {
  if (epi == EPI_DROPOUT) { mlvae_set_error("mlvae_gemm_ex: dropout epilogue needs mlvae_gemm_ex_drop"); return 1; }
  return mlvae_gemm_ex_drop(trans_a, trans_b, M, N, K, alpha, A, a_bf16, lda, B, b_bf16, ldb, beta,
                            C, ldc, bias1, bias2, epi, aux, ldaux, kshift_T, kshift, 0ull, 0ull, 0.f, ws,
                            ws_bytes, stream);
}

// fp32 -> bf16 (round to nearest even), n elements, 16-byte aligned buffers.
__global__ __launch_bounds__(256) void cast_bf16_kernel(size_t n, const float* __restrict__ x,
                                                        unsigned short* __restrict__ y) {
  const size_t n4 = n / 4;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
    const f32x4 v = reinterpret_cast<const f32x4*>(x)[i];
    u32x2 o = {(unsigned)bf_bits(v[0]) | ((unsigned)bf_bits(v[1]) << 16),
               (unsigned)bf_bits(v[2]) | ((unsigned)bf_bits(v[3]) << 16)};
    reinterpret_cast<u32x2*>(y)[i] = o;
  }
  for (size_t i = n4 * 4 + (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    y[i] = bf_bits(x[i]);
}

extern "C" int mlvae_cast_bf16(size_t n, const float* x, void* y, void* stream) {
  if (n == 0) return 0;
  if (!x || !y || ((uintptr_t)x % 16) || ((uintptr_t)y % 8)) {
    mlvae_set_error("mlvae_cast_bf16: needs 16-byte aligned x, 8-byte aligned y");
    return 1;
  }
  size_t blocks = (n / 4 + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  cast_bf16_kernel<<<(unsigned)blocks, 256, 0, (hipStream_t)stream>>>(n, x,
                                                                       static_cast<unsigned short*>(y));
  MLVAE_CHECK_LAUNCH();
  return 0;
}

// y[c][r] (bf16) = x[r][c] (fp32): transposed bf16 copy of a [rows, cols] weight (ld = cols),
// so a dgrad dX = dG W reads W^T k-contiguous.  32 x 32 tiles through LDS.
__global__ __launch_bounds__(256) void cast_bf16_t_kernel(int rows, int cols, const float* __restrict__ x,
                                                          unsigned short* __restrict__ y) {
  __shared__ float t[32][33];
  const int r0 = blockIdx.y * 32, c0 = blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 8 rows per pass
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int r = r0 + ty + 8 * k, c = c0 + tx;
    t[ty + 8 * k][tx] = (r < rows && c < cols) ? x[(size_t)r * cols + c] : 0.f;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int c = c0 + ty + 8 * k, r = r0 + tx;
    if (c < cols && r < rows) y[(size_t)c * rows + r] = bf_bits(t[tx][ty + 8 * k]);
  }
}

extern "C" int mlvae_cast_bf16_t(int rows, int cols, const float* x, void* y, void* stream) {
  if (rows <= 0 || cols <= 0) return 0;
  if (!x || !y) { mlvae_set_error("mlvae_cast_bf16_t: null pointer"); return 1; }
  dim3 grid((cols + 31) / 32, (rows + 31) / 32);
  cast_bf16_t_kernel<<<grid, 256, 0, (hipStream_t)stream>>>(rows, cols, x, static_cast<unsigned short*>(y));
  MLVAE_CHECK_LAUNCH();
  return 0;
}
