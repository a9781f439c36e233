// Conv1d encoder layers (BASELINE.json configs[3], "Conv1d encoder variant, long utterances
// T=2000, B=64"): y[b, t, :] = act(bias + sum_{j<K} W[:, :, j] x[b, t + j - p, :]), p = (K-1)/2,
// zero padding at each utterance's ends (torch.nn.Conv1d(Cin, Cout, K, padding=p) on the
// [B, C, T] transpose of the batch-first frames).  The reference has no Conv1d (SURVEY.md
// Appendix A): the module surface is modules/conv_vae.py, the oracle oracle/vae_cpu.py
// (torch conv1d) cross-checked by an explicit numpy restatement (tests/test_oracle_conv.py).
//
// Forward and input gradient are one implicit-GEMM kernel: a workgroup owns BM = 64 frames of
// ONE utterance (tiles never straddle utterances, so the zero halo is a staging rule), stages
// the (BM + K - 1)-frame halo window of x as bf16 in LDS once and the packed weights
// [Cout][K * CinP] once per (persistent) workgroup; the K shifted windows are then plain row
// offsets into the same LDS image.  v_mfma_f32_16x16x32_bf16 with swapped operands (D^T = W X^T)
// leaves 4 consecutive output channels of one frame per lane: 16-byte stores.  The input
// gradient is the same product over the transposed, time-flipped weights
//   dx[t, i] = sum_{j', o} dy[t + j' - p, o] W[o, i, K - 1 - j'],
// with the LeakyReLU derivative of the layer below fused into the epilogue.
//
// Weight gradient dW[o, i, j] = sum_{b,t} dy[b, t, o] x[b, t + j - p, i]: persistent
// workgroups accumulate whole-tile products (K = frames) in registers over their tiles (both
// operands read transposed from LDS with ds_read_b64_tr_b16), plus the bias gradient in fp32,
// write one slab each, and a fixed-order reduce sums the slabs (deterministic).
//
// Bytes per frame (HBM, fp32 activations): forward Cin * 4 read + Cout * 4 written; input
// gradient Cin' * 4 + Cout' * 4 (+ aux Cout' * 4); weight gradient (Cin + Cout) * 4 read.
#include "common.h"

namespace {

constexpr int BM = 64;     // frames per tile (4 waves x 16)
constexpr int CT = 256;    // threads
constexpr int SKEW = 8;    // shorts of row padding in the LDS images
constexpr int MTW = 8;     // weight-gradient m-tiles per wave (K * Cin16 <= 512)
typedef __attribute__((address_space(3))) bf16x4* lds_b4_p;

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// operand fragment (m = base + (lane & 15), k = kk + 8 (lane >> 4) + e) of an LDS image stored
// [k rows][ld] (k = frames), read transposed
__device__ __forceinline__ bf16x8 trfrag(const short* img, int ld, int base, int kk, int lane) {
  const int g = lane >> 4, i4 = lane & 15, qq = i4 >> 2, pp = i4 & 3;
  const int r1 = kk + 8 * g + qq, r2 = r1 + 4;
  const bf16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_b4_p)(img + r1 * ld + base + 4 * pp));
  const bf16x4 v2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_b4_p)(img + r2 * ld + base + 4 * pp));
  return bf16x8{v1[0], v1[1], v1[2], v1[3], v2[0], v2[1], v2[2], v2[3]};
}

// Rows [t_first, t_first + R) of utterance b (zero outside [0, T) and for channels >= C) of an
// fp32 source [N][lds], element group e = tid + j * CT (row e / (CP / 4), channels 4 (e % (CP / 4))
// ...): NL 16-byte loads per thread, all issued before any is used, so a tile's rows are in
// flight together -- and the next tile's while this one's MFMAs run (the one-load-at-a-time
// staging loop held a few KB in flight per CU: 12 % of HBM).  C % 4 == 0, CP % 4 == 0.
template <int NL>
__device__ __forceinline__ void load_rows(f32x4 (&v)[NL], const float* src, int lds, int b, int T, int t_first,
                                          int R, int C, int CP) {
  const int c4n = CP / 4, n = R * c4n;
#pragma unroll
  for (int j = 0; j < NL; ++j) {
    const int e = threadIdx.x + j * CT, r = e / c4n, c = (e - r * c4n) * 4, t = t_first + r;
    v[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (e < n && t >= 0 && t < T && c < C) v[j] = *(const f32x4*)(src + ((size_t)b * T + t) * lds + c);
  }
}

// ... then as bf16 into img[R][ld].  SUM: add the thread's values to colsum (its column group is
// fixed when CT % (CP / 4) == 0).
template <bool SUM, int NL>
__device__ __forceinline__ void store_rows(short* img, int ld, const f32x4 (&v)[NL], int R, int CP,
                                           float (&colsum)[4]) {
  const int c4n = CP / 4, n = R * c4n;
#pragma unroll
  for (int j = 0; j < NL; ++j) {
    const int e = threadIdx.x + j * CT, r = e / c4n, c = (e - r * c4n) * 4;
    if (e < n) {
      if (SUM) {
        colsum[0] += v[j][0]; colsum[1] += v[j][1]; colsum[2] += v[j][2]; colsum[3] += v[j][3];
      }
      *(bf16x4*)(img + r * ld + c) = bf16x4{f2bf(v[j][0]), f2bf(v[j][1]), f2bf(v[j][2]), f2bf(v[j][3])};
    }
  }
}

constexpr int NLW = 9;   // window loads per thread: (BM + K - 1) * CinP / 4 <= 72 * 32 = 9 * CT
constexpr int NLD = 4;   // weight gradient: dy rows, BM * Cout / 4 <= 4 * CT
constexpr int NLX = 8;   // weight gradient: x window, (BM + K - 1) * Cin16 / 4 <= 8 * CT (host-checked)

struct ConvArgs {
  int T, Cin, Cout, K, CinP;   // product dims (dgrad: Cin = the layer's Cout, Cout = its Cin)
  int Lc;                      // the layer's input channels (weight row length / K)
  const float* x; int ldx;
  const float* w;              // the layer's weight, torch layout [layer Cout][layer Cin][K]
  const float* bias;
  const float* aux; int ldaux; // dgrad: LeakyReLU output whose derivative multiplies dx
  float* y; int ldy;
  int act, tpu, ntiles;
};

template <int NT, bool DG>  // DG: input gradient (transposed, time-flipped weights)
__global__ __launch_bounds__(CT) void conv_kernel(ConvArgs a) {
  extern __shared__ __attribute__((aligned(16))) short smem[];
  const int K = a.K, CinP = a.CinP, KC = K * CinP;
  const int ldw = KC + SKEW, ldxl = CinP + SKEW, p = (K - 1) / 2;
  short* Wl = smem;                          // [Cout][K * CinP]
  short* Xl = smem + a.Cout * ldw;           // [BM + K - 1][CinP]
  // packed bf16 weights, once per workgroup: Wl[o][j * CinP + c].  The fp32 weight is read in
  // its own order (coalesced 16-byte loads) and scattered into the LDS image; the padding
  // channels c in [Cin, CinP) are zeroed first.
  if (a.Cin < CinP) {  // padding channels [Cin, CinP) of every (o, tap) row: zero
    const int padc = CinP - a.Cin;
    for (int r = threadIdx.x; r < a.Cout * K; r += CT) {
      const int o = r / K, jt = r - o * K;
      short* dst = Wl + o * ldw + jt * CinP + a.Cin;
      for (int c = 0; c < padc; ++c) dst[c] = 0;
    }
  }
  {
    // the layer weight [Lo][Li][K]: one thread per (lo, li) pair reads its K contiguous taps --
    // one integer division per pair (per element, three had made this prologue most of a
    // workgroup's time at c4's 4 tiles per workgroup)
    const int npair = a.Cout * a.Cin;  // Lo * Li
    for (int pr = threadIdx.x; pr < npair; pr += CT) {
      const int lo = pr / a.Lc, li = pr - lo * a.Lc;  // layer (out, in) channel
      // forward: product row o = lo, column c = li, tap j; input gradient: o = li, c = lo,
      // tap K - 1 - j (transposed, time-flipped)
      const int o = DG ? li : lo, c = DG ? lo : li;
      const float* wp = a.w + (size_t)pr * K;
      short* dst = Wl + o * ldw + c;
      for (int j = 0; j < K; ++j) dst[(DG ? K - 1 - j : j) * CinP] = f2bf(wp[j]);
    }
  }
  const int lane = threadIdx.x & 63, l15 = lane & 15, q = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int f = 16 * wave + l15;  // this lane's frame in the tile (B operand column)
  float unused[4];
  f32x4 win[NLW];
  // input gradient: the LeakyReLU output of the layer below at this lane's frame and channels,
  // loaded with the tile's window (a load in the epilogue would wait for the next tile's window
  // loads issued before it: vmcnt counts in issue order)
  f32x4 axc[NT], axn[NT];
  auto load_aux = [&](int tile_) {
    const int b_ = tile_ / a.tpu, t_ = (tile_ - b_ * a.tpu) * BM + f;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      axn[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (t_ < a.T) axn[nt] = *(const f32x4*)(a.aux + ((size_t)b_ * a.T + t_) * a.ldaux + 16 * nt + 4 * q);
    }
  };
  if (blockIdx.x < a.ntiles) {
    const int b = blockIdx.x / a.tpu, t0 = (blockIdx.x - b * a.tpu) * BM;
    load_rows(win, a.x, a.ldx, b, a.T, t0 - p, BM + K - 1, a.Cin, CinP);
    if (DG && a.aux) load_aux(blockIdx.x);
  }
  for (int tile = blockIdx.x; tile < a.ntiles; tile += gridDim.x) {
    const int b = tile / a.tpu, t0 = (tile - b * a.tpu) * BM;
    lds_barrier();  // weights staged / the previous tile's reads done (its stores stay in flight)
    store_rows<false>(Xl, ldxl, win, BM + K - 1, CinP, unused);
    if (DG && a.aux) {
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) axc[nt] = axn[nt];
    }
    lds_barrier();
    const int nx = tile + gridDim.x;  // the next tile's window streams in under this tile's MFMAs
    if (nx < a.ntiles) {
      const int nb = nx / a.tpu, nt0 = (nx - nb * a.tpu) * BM;
      load_rows(win, a.x, a.ldx, nb, a.T, nt0 - p, BM + K - 1, a.Cin, CinP);
      if (DG && a.aux) load_aux(nx);
    }
    f32x4 acc[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int kc32 = CinP / 32;
    for (int ks = 0; ks < K * kc32; ++ks) {
      const int j = ks / kc32, c0 = (ks - j * kc32) * 32;
      const bf16x8 xb = *(const bf16x8*)(Xl + (f + j) * ldxl + c0 + 8 * q);
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const bf16x8 wa = *(const bf16x8*)(Wl + (16 * nt + l15) * ldw + ks * 32 + 8 * q);
        acc[nt] = mfma16(wa, xb, acc[nt]);
      }
    }
    const int t = t0 + f;
    if (t < a.T) {
      const size_t row = (size_t)b * a.T + t;
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const int o = 16 * nt + 4 * q;
        f32x4 v = acc[nt];
        if (a.bias) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] += a.bias[o + r];
        }
        if (a.act) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = lrelu(v[r]);
        }
        if (DG && a.aux) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] *= lrelu_d(axc[nt][r]);
        }
        *(f32x4*)(a.y + row * a.ldy + o) = v;
      }
    }
  }
}

struct WgArgs {
  int T, Cin, Cout, K, Cin16, tpu, ntiles;
  const float* dy; int lddy;
  const float* x; int ldx;
  float* slabs;                // [gridDim.x][Cout * Cin * K + Cout]
};

template <int NT>
__global__ __launch_bounds__(CT) void conv_wgrad_kernel(WgArgs a) {
  extern __shared__ __attribute__((aligned(16))) short smem[];
  constexpr int Cout = 16 * NT;
  const int K = a.K, Cin16 = a.Cin16, p = (K - 1) / 2;
  const int lddy = Cout + SKEW, ldxl = Cin16 + SKEW;
  short* DYl = smem;                     // [BM][Cout]
  short* Xl = smem + BM * lddy;          // [BM + K - 1][Cin16]
  __shared__ float red[CT * 4];
  const int lane = threadIdx.x & 63, l15 = lane & 15, q = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int mpj = Cin16 / 16, MT = K * mpj;
  f32x4 acc[MTW][NT];
#pragma unroll
  for (int u = 0; u < MTW; ++u)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[u][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bsum[4] = {0.f, 0.f, 0.f, 0.f};
  f32x4 vdy[NLD], vx[NLX];
  auto load_tile = [&](int tile) {
    const int b = tile / a.tpu, t0 = (tile - b * a.tpu) * BM;
    load_rows(vdy, a.dy, a.lddy, b, a.T, t0, BM, Cout, Cout);
    load_rows(vx, a.x, a.ldx, b, a.T, t0 - p, BM + K - 1, a.Cin, Cin16);
  };
  if (blockIdx.x < a.ntiles) load_tile(blockIdx.x);
  for (int tile = blockIdx.x; tile < a.ntiles; tile += gridDim.x) {
    lds_barrier();
    store_rows<true>(DYl, lddy, vdy, BM, Cout, bsum);
    store_rows<false>(Xl, ldxl, vx, BM + K - 1, Cin16, bsum);
    lds_barrier();
    if (tile + (int)gridDim.x < a.ntiles) load_tile(tile + gridDim.x);  // in flight under the MFMAs
#pragma unroll
    for (int kk = 0; kk < BM; kk += 32) {
      bf16x8 bf[NT];
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) bf[nt] = trfrag(DYl, lddy, 16 * nt, kk, lane);
#pragma unroll
      for (int u = 0; u < MTW; ++u) {
        const int mt = wave + 4 * u;
        if (mt < MT) {  // wave-uniform
          const int j = mt / mpj, i0 = (mt - j * mpj) * 16;
          const bf16x8 af = trfrag(Xl + j * ldxl, ldxl, i0, kk, lane);
#pragma unroll
          for (int nt = 0; nt < NT; ++nt) acc[u][nt] = mfma16(af, bf[nt], acc[u][nt]);
        }
      }
    }
  }
  // slab: dW in the accumulators' own order -- [m-tile][n-tile][lane][4], one 16-byte store per
  // lane and tile pair (1 KB per wave instruction; the torch-layout scatter of 4-byte stores
  // was the kernel's slowest part) -- then db [Cout]; the reduce writes the torch layout
  const int NW = MT * NT * 256;
  const size_t S = (size_t)NW + Cout;
  float* slab = a.slabs + (size_t)blockIdx.x * S;
#pragma unroll
  for (int u = 0; u < MTW; ++u) {
    const int mt = wave + 4 * u;
    if (mt < MT) {
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
        *reinterpret_cast<f32x4*>(slab + ((size_t)(mt * NT + nt) * 64 + lane) * 4) = acc[u][nt];
    }
  }
  // bias: thread tid summed columns 4 (tid % (Cout / 4)) .. + 3 of its rows
#pragma unroll
  for (int r = 0; r < 4; ++r) red[r * CT + threadIdx.x] = bsum[r];
  __syncthreads();
  const int c4n = Cout / 4;
  if (threadIdx.x < Cout) {
    const int c = threadIdx.x, g = c / 4, r = c - 4 * g;
    float s = 0.f;
    for (int t = g; t < CT; t += c4n) s += red[r * CT + t];
    slab[(size_t)NW + c] = s;
  }
}

// The slabs are summed in two fixed-order stages (deterministic): block (column chunk, z) sums
// slabs [z G / NZ, (z + 1) G / NZ) into part[z]; then the NZ partial rows in order.  (One pass
// with a thread per column walked all G = 256 slabs alone: ~25 K threads, each a 256-deep chain
// of dependent-address loads -- latency-bound.)
constexpr int NZ = 16;
__global__ __launch_bounds__(256) void slab_reduce_kernel(const float* slabs, int G, size_t S, float* part) {
  const size_t e = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= S) return;
  const int z = blockIdx.y, g0 = z * G / NZ, g1 = (z + 1) * G / NZ;
  float s = 0.f;
#pragma unroll 8  // loads in flight; the adds keep their order
  for (int g = g0; g < g1; ++g) s += slabs[(size_t)g * S + e];
  part[(size_t)z * S + e] = s;
}

// e < nw: slab order ((m-tile * NT + n-tile) * 64 + lane) * 4 + r -> dW[o][i][j] (torch layout) with
// o = 16 n-tile + (lane & 15), m = 16 m-tile + 4 (lane >> 4) + r = j * Cin16 + i (i < Cin)
__global__ __launch_bounds__(256) void slab_reduce2_kernel(const float* part, size_t S, size_t nw, int NT, int Cin,
                                                           int Cin16, int K, float* dw, float* db) {
  const size_t e = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= S) return;
  float s = 0.f;
#pragma unroll
  for (int z = 0; z < NZ; ++z) s += part[(size_t)z * S + e];
  if (e < nw) {
    const int r = (int)(e & 3), lane = (int)((e >> 2) & 63), tp = (int)(e >> 8);
    const int mt = tp / NT, nt = tp - mt * NT;
    const int o = 16 * nt + (lane & 15), m = 16 * mt + 4 * (lane >> 4) + r, j = m / Cin16, i = m - j * Cin16;
    if (i < Cin) dw[((size_t)o * Cin + i) * K + j] = s;
  } else if (db) {
    db[e - nw] = s;
  }
}

int device_cus() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  }
  return n;
}

int round_up(int v, int m) { return (v + m - 1) / m * m; }

bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

template <typename Kern, typename Args>
int launch_lds(Kern k, int grid, size_t lds, hipStream_t s, const Args& a) {
  if (lds > 64 * 1024 &&
      hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) {
    mlvae_set_error("conv1d: cannot reserve %zu bytes of LDS", lds);
    return 1;
  }
  hipLaunchKernelGGL(k, dim3(grid), dim3(CT), lds, s, a);
  MLVAE_CHECK_LAUNCH();
  return 0;
}

template <bool DG>
int launch_conv(ConvArgs& a, int B, hipStream_t s) {
  a.tpu = (a.T + BM - 1) / BM;
  a.ntiles = B * a.tpu;
  const size_t lds = ((size_t)a.Cout * (a.K * a.CinP + SKEW) + (size_t)(BM + a.K - 1) * (a.CinP + SKEW)) * 2;
  if (lds > 160 * 1024) {
    mlvae_set_error("conv1d: LDS image %zu bytes > 160 KB", lds);
    return 1;
  }
  // persistent workgroups per CU (each stages the weights once): MLVAE_CONV_MULT (A/B; default 2)
  static const int mult = [] {
    const char* e = getenv("MLVAE_CONV_MULT");
    const int m = e ? atoi(e) : 2;
    return m < 1 ? 1 : (m > 4 ? 4 : m);
  }();
  int g = a.ntiles < mult * device_cus() ? a.ntiles : mult * device_cus();
  switch (a.Cout / 16) {
#define CASE(n) case n: return launch_lds(conv_kernel<n, DG>, g, lds, s, a);
    CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8)
#undef CASE
    default: mlvae_set_error("conv1d: output channels %d", a.Cout); return 1;
  }
}

bool dims_ok(int B, int T, int Cin, int Cout, int K) {
  return B > 0 && T > 0 && K >= 1 && K <= 9 && (K & 1) && Cin >= 4 && Cin <= 128 && Cin % 4 == 0 &&
         Cout >= 16 && Cout <= 128 && Cout % 16 == 0;
}

}  // namespace

extern "C" int mlvae_conv1d_supported(int Cin, int Cout, int K) {
  return dims_ok(1, 1, Cin, Cout, K) && dims_ok(1, 1, Cout, Cin, K) && (Cout == 16 || Cout == 32 || Cout == 64) &&
         K * round_up(Cin, 16) <= 16 * 4 * MTW && (BM + K - 1) * round_up(Cin, 16) / 4 <= NLX * CT;
}

extern "C" int mlvae_conv1d_fwd(int B, int T, int Cin, int Cout, int K, const float* x, int ldx, const float* w,
                                const float* bias, int act, float* y, int ldy, void* stream) {
  if (B <= 0 || T <= 0) return 0;
  if (!dims_ok(B, T, Cin, Cout, K) || !x || !w || !y || ldx < Cin || ldy < Cout || ldx % 4 || ldy % 4 ||
      !aligned16(x) || !aligned16(y) || !aligned16(w)) {
    mlvae_set_error("mlvae_conv1d_fwd: unsupported shape/stride/alignment (Cin %d Cout %d K %d)", Cin, Cout, K);
    return 1;
  }
  ConvArgs a{};
  a.T = T; a.Cin = Cin; a.Cout = Cout; a.K = K; a.CinP = round_up(Cin, 32); a.Lc = Cin;
  a.x = x; a.ldx = ldx; a.w = w; a.bias = bias; a.aux = nullptr; a.ldaux = 0; a.y = y; a.ldy = ldy;
  a.act = act ? 1 : 0;
  return launch_conv<false>(a, B, (hipStream_t)stream);
}

extern "C" int mlvae_conv1d_dgrad(int B, int T, int Cin, int Cout, int K, const float* dy, int lddy,
                                  const float* w, const float* aux, int ldaux, float* dx, int lddx,
                                  void* stream) {
  if (B <= 0 || T <= 0) return 0;
  if (!dims_ok(B, T, Cout, Cin, K) || !dy || !w || !dx || lddy < Cout || lddx < Cin || lddy % 4 || lddx % 4 ||
      (aux && (ldaux < Cin || ldaux % 4 || !aligned16(aux))) || !aligned16(dy) || !aligned16(dx) || !aligned16(w)) {
    mlvae_set_error("mlvae_conv1d_dgrad: unsupported shape/stride/alignment (Cin %d Cout %d K %d)", Cin, Cout, K);
    return 1;
  }
  ConvArgs a{};
  a.T = T; a.Cin = Cout; a.Cout = Cin; a.K = K; a.CinP = round_up(Cout, 32); a.Lc = Cin;
  a.x = dy; a.ldx = lddy; a.w = w; a.bias = nullptr; a.aux = aux; a.ldaux = ldaux; a.y = dx; a.ldy = lddx;
  a.act = 0;
  return launch_conv<true>(a, B, (hipStream_t)stream);
}

// weight-gradient workgroups (one slab each): MLVAE_CONV_WG_MULT per CU (A/B; default 1)
static int wgrad_grid(int B, int T) {
  static const int mult = [] {
    const char* e = getenv("MLVAE_CONV_WG_MULT");
    const int m = e ? atoi(e) : 1;
    return m < 1 ? 1 : (m > 4 ? 4 : m);
  }();
  const int tiles = B * ((T + BM - 1) / BM), g = mult * device_cus();
  return tiles < g ? tiles : g;
}

// slab floats: the accumulators (K * Cin16 / 16 m-tiles x Cout / 16 n-tiles x 256) + the bias row
static size_t wgrad_slab(int Cin, int Cout, int K) { return (size_t)K * round_up(Cin, 16) * Cout + Cout; }

extern "C" size_t mlvae_conv1d_wgrad_workspace_size(int B, int T, int Cin, int Cout, int K) {
  if (B <= 0 || T <= 0) return 0;
  return ((size_t)wgrad_grid(B, T) + NZ) * wgrad_slab(Cin, Cout, K) * sizeof(float);  // slabs + partials
}

extern "C" int mlvae_conv1d_wgrad(int B, int T, int Cin, int Cout, int K, const float* dy, int lddy,
                                  const float* x, int ldx, float* dw, float* db, void* ws, size_t ws_bytes,
                                  void* stream) {
  if (B <= 0 || T <= 0) return 0;
  if (!mlvae_conv1d_supported(Cin, Cout, K) || !dy || !x || !dw || lddy < Cout || ldx < Cin || lddy % 4 ||
      ldx % 4 || !aligned16(dy) || !aligned16(x)) {
    mlvae_set_error("mlvae_conv1d_wgrad: unsupported shape/stride/alignment (Cin %d Cout %d K %d)", Cin, Cout, K);
    return 1;
  }
  if (!ws || ws_bytes < mlvae_conv1d_wgrad_workspace_size(B, T, Cin, Cout, K)) {
    mlvae_set_error("mlvae_conv1d_wgrad: workspace too small");
    return 1;
  }
  hipStream_t s = (hipStream_t)stream;
  WgArgs a{};
  a.T = T; a.Cin = Cin; a.Cout = Cout; a.K = K; a.Cin16 = round_up(Cin, 16);
  a.tpu = (T + BM - 1) / BM; a.ntiles = B * a.tpu;
  a.dy = dy; a.lddy = lddy; a.x = x; a.ldx = ldx; a.slabs = static_cast<float*>(ws);
  const int g = wgrad_grid(B, T);
  const size_t lds = ((size_t)BM * (Cout + SKEW) + (size_t)(BM + K - 1) * (a.Cin16 + SKEW)) * 2;
  const int rc = Cout == 16 ? launch_lds(conv_wgrad_kernel<1>, g, lds, s, a)
               : Cout == 32 ? launch_lds(conv_wgrad_kernel<2>, g, lds, s, a)
                            : launch_lds(conv_wgrad_kernel<4>, g, lds, s, a);
  if (rc) return rc;
  const size_t S = wgrad_slab(Cin, Cout, K);
  const int rb = (int)((S + 255) / 256);
  float* part = static_cast<float*>(ws) + (size_t)g * S;
  hipLaunchKernelGGL(slab_reduce_kernel, dim3(rb, NZ), dim3(256), 0, s, static_cast<const float*>(ws), g, S, part);
  MLVAE_CHECK_LAUNCH();
  hipLaunchKernelGGL(slab_reduce2_kernel, dim3(rb), dim3(256), 0, s, static_cast<const float*>(part), S, S - Cout,
                     Cout / 16, Cin, a.Cin16, K, dw, db);
  MLVAE_CHECK_LAUNCH();
  return 0;
}

