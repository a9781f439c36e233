// Skinny products of the bottom LSTM layer (bf16 mode), where one GEMM side is the latent
// width Z (16-64): on a 256-wide GEMM tile 7/8 of every MFMA and B load is padding.
//
//   dZ = dG W_ih           [B*T, Z]  = [B*T, 8H] . [8H, Z]        (dgrad into the encoder)
//   dW_ih | db = dG^T [Z | 1]   [8H, Z+1] = [8H, B*T] . [B*T, Z+1] (weight + bias gradients:
//                                 the ones column turns the bias column sum into MFMA work)
// ref:src/modules/decoder.py:14-15,22 (nn.LSTM input projection of layer 0, its autograd).
//
// skinny_nt: C[M, NB] = A[M, K] . Bt[NB, K]^T, A and Bt k-contiguous bf16.  A wave owns 16 rows
//   and all NB columns; fragments are loaded straight from global (16 B per lane, four K-steps
//   in flight); operands swapped so a lane stores 4 consecutive columns.
// skinny_proj: C[M, N] = A[M, K] . B[N, K]^T + bias1 + bias2 with K <= 32 (fp32 C): the layer-0
//   input projection G = z W_ih^T + b_ih + b_hh, whose K is the latent width.  One MFMA per
//   16 x 16 output block, fragments straight from global (W_ih is L2-resident), no LDS, small
//   register footprint: many waves per CU keep the 16-byte stores of the write-bound output
//   in flight (the 256-wide LDS tile ran one workgroup per CU and serialised its epilogue).
// skinny_tn: P_s[M, NB] = A[Ks, M]^T . B[Ks, NB] over one frame range Ks per split s; A and B
//   m/n-contiguous bf16, staged through LDS (64 frames per chunk) and read with
//   ds_read_b64_tr_b16; fp32 partial slabs per split, reduced in a fixed order by
//   skinny_reduce into the weight columns and (optionally) two bias vectors.
#include "common.h"

namespace {

typedef __attribute__((address_space(3))) bf16x4* lds_b4_p;

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

template <int NT>  // NB = 16 * NT
__global__ __launch_bounds__(256) void skinny_nt_kernel(int M, int K, const unsigned short* __restrict__ A,
                                                        int lda, const unsigned short* __restrict__ Bt,
                                                        int ldb, float* __restrict__ C, int ldc) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int l15 = lane & 15, q = lane >> 4;
  const int row = (blockIdx.x * 4 + wave) * 16 + l15;
  const bool rv = row < M;
  const unsigned short* ap = A + (size_t)(rv ? row : 0) * lda + 8 * q;
  const unsigned short* bp = Bt + (size_t)l15 * ldb + 8 * q;
  const bf16x8 z8 = {0, 0, 0, 0, 0, 0, 0, 0};
  f32x4 acc[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  constexpr int U = 4;  // K-steps of 32 in flight
  int k = 0;
  for (; k + 32 * U <= K; k += 32 * U) {
    bf16x8 af[U], bf[U][NT];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      af[u] = rv ? *reinterpret_cast<const bf16x8*>(ap + k + 32 * u) : z8;
#pragma unroll
      for (int j = 0; j < NT; ++j)
        bf[u][j] = *reinterpret_cast<const bf16x8*>(bp + (size_t)16 * j * ldb + k + 32 * u);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[j] = mfma16(bf[u][j], af[u], acc[j]);
  }
  for (; k < K; k += 32) {  // K % 32 == 0 (checked on the host)
    const bf16x8 a1 = rv ? *reinterpret_cast<const bf16x8*>(ap + k) : z8;
#pragma unroll
    for (int j = 0; j < NT; ++j)
      acc[j] = mfma16(*reinterpret_cast<const bf16x8*>(bp + (size_t)16 * j * ldb + k), a1, acc[j]);
  }
  if (!rv) return;
  // swapped operands: lane holds C[row][16j + 4q + r]
#pragma unroll
  for (int j = 0; j < NT; ++j) *reinterpret_cast<f32x4*>(C + (size_t)row * ldc + 16 * j + 4 * q) = acc[j];
}

// K split over the four waves of a 16-row workgroup (4x the loads in flight per row tile;
// the NT loop above is latency-bound at B*T = 16,000 rows: 67 us), partials summed in LDS in
// a fixed order.  K % 128 == 0.
template <int NT>
__global__ __launch_bounds__(256) void skinny_nt_ks_kernel(int M, int K, const unsigned short* __restrict__ A,
                                                           int lda, const unsigned short* __restrict__ Bt,
                                                           int ldb, float* __restrict__ C, int ldc) {
  __shared__ f32x4 red[3][NT][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int l15 = lane & 15, q = lane >> 4;
  const int row = blockIdx.x * 16 + l15;
  const bool rv = row < M;
  const int kq = K / 4, kb = wave * kq;
  const unsigned short* ap = A + (size_t)(rv ? row : 0) * lda + kb + 8 * q;
  const unsigned short* bp = Bt + (size_t)l15 * ldb + kb + 8 * q;
  const bf16x8 z8 = {0, 0, 0, 0, 0, 0, 0, 0};
  f32x4 acc[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  constexpr int U = 4;
  int k = 0;
  for (; k + 32 * U <= kq; k += 32 * U) {
    bf16x8 af[U], bf[U][NT];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      af[u] = rv ? *reinterpret_cast<const bf16x8*>(ap + k + 32 * u) : z8;
#pragma unroll
      for (int j = 0; j < NT; ++j)
        bf[u][j] = *reinterpret_cast<const bf16x8*>(bp + (size_t)16 * j * ldb + k + 32 * u);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[j] = mfma16(bf[u][j], af[u], acc[j]);
  }
  for (; k < kq; k += 32) {
    const bf16x8 a1 = rv ? *reinterpret_cast<const bf16x8*>(ap + k) : z8;
#pragma unroll
    for (int j = 0; j < NT; ++j)
      acc[j] = mfma16(*reinterpret_cast<const bf16x8*>(bp + (size_t)16 * j * ldb + k), a1, acc[j]);
  }
  if (wave > 0) {
#pragma unroll
    for (int j = 0; j < NT; ++j) red[wave - 1][j][lane] = acc[j];
  }
  __syncthreads();
  if (wave != 0 || !rv) return;
#pragma unroll
  for (int j = 0; j < NT; ++j)
    *reinterpret_cast<f32x4*>(C + (size_t)row * ldc + 16 * j + 4 * q) =
        ((acc[j] + red[0][j][lane]) + red[1][j][lane]) + red[2][j][lane];
}

// 128-row workgroups (8 waves x 16 rows, each over the whole K) with Bt streamed through LDS in
// 256-wide K-chunks that all eight waves share: the ks form above re-read Bt from L2 for every
// 16 rows (twice the bytes of its A stream) and held 2.5 TB/s on the 1 GB dG of c3 (409 us).
// A chunk c+1 (16 B x 8 per lane, 64 KB per workgroup in flight) and Bt chunk c+1 are loaded
// while chunk c's MFMAs run.  K % 256 == 0.
// F8: A is e4m3 (fp8 mode's layer-0 dG, lda in bytes) converted to bf16 in registers (exact; the
// kernel streams A, so half its bytes is half its time) and C scaled by *alpha (1 / dG's scale).
constexpr int NTL_KC = 256, NTL_LB = NTL_KC + 8;  // K-chunk, LDS row stride (shorts)
template <int NT, bool F8 = false>
__global__ __launch_bounds__(512) void skinny_nt_lds_kernel(int M, int K, const void* __restrict__ Av,
                                                            int lda, const unsigned short* __restrict__ Bt,
                                                            int ldb, float* __restrict__ C, int ldc,
                                                            const float* __restrict__ alpha) {
  constexpr int NB = 16 * NT, BPT = (NB * NTL_KC / 8 + 511) / 512;  // 16-byte Bt pieces per thread
  __shared__ __attribute__((aligned(16))) short sb[2][NB * NTL_LB];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l15 = lane & 15, q = lane >> 4;
  const int row = blockIdx.x * 128 + wave * 16 + l15;
  const bool rv = row < M;
  const unsigned short* ap = static_cast<const unsigned short*>(Av) + (size_t)(rv ? row : 0) * lda + 8 * q;
  const unsigned char* ap8 = static_cast<const unsigned char*>(Av) + (size_t)(rv ? row : 0) * lda + 8 * q;
  const bf16x8 z8 = {0, 0, 0, 0, 0, 0, 0, 0};
  bf16x8 ac[8], an[8];
  u32x2 a8[8];  // F8: the next chunk's raw e4m3 (converted when it becomes current)
  u32x4 br[BPT];
  auto aload = [&](int k0, bf16x8 (&d)[8]) {
    if constexpr (F8) {
#pragma unroll
      for (int u = 0; u < 8; ++u) a8[u] = rv ? *reinterpret_cast<const u32x2*>(ap8 + k0 + 32 * u) : u32x2{0u, 0u};
    } else {
#pragma unroll
      for (int u = 0; u < 8; ++u) d[u] = rv ? *reinterpret_cast<const bf16x8*>(ap + k0 + 32 * u) : z8;
    }
  };
  auto aconv = [&](bf16x8 (&d)[8]) {
    if constexpr (F8) {
#pragma unroll
      for (int u = 0; u < 8; ++u) d[u] = fp8x8_to_bf16(a8[u][0], a8[u][1]);
    }
  };
  auto bload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < BPT; ++i) {
      const int idx = tid + 512 * i, r = idx / (NTL_KC / 8), c8 = idx % (NTL_KC / 8);
      if (idx < NB * NTL_KC / 8) br[i] = *reinterpret_cast<const u32x4*>(Bt + (size_t)r * ldb + k0 + 8 * c8);
    }
  };
  auto bstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < BPT; ++i) {
      const int idx = tid + 512 * i, r = idx / (NTL_KC / 8), c8 = idx % (NTL_KC / 8);
      if (idx < NB * NTL_KC / 8) *reinterpret_cast<u32x4*>(&sb[buf][r * NTL_LB + 8 * c8]) = br[i];
    }
  };
  f32x4 acc[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nc = K / NTL_KC;
  aload(0, ac);
  aconv(ac);
  bload(0);
  bstore(0);
  __syncthreads();
  for (int c = 0; c < nc; ++c) {
    const bool more = c + 1 < nc;
    if (more) { aload((c + 1) * NTL_KC, an); bload((c + 1) * NTL_KC); }
    const short* b = sb[c & 1];
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int j = 0; j < NT; ++j)
        acc[j] = mfma16(*reinterpret_cast<const bf16x8*>(b + (16 * j + l15) * NTL_LB + 32 * u + 8 * q), ac[u], acc[j]);
    if (more) bstore((c + 1) & 1);
    __syncthreads();
    if constexpr (F8) {
      if (more) aconv(ac);
    } else {
#pragma unroll
      for (int u = 0; u < 8; ++u) ac[u] = an[u];
    }
  }
  if (!rv) return;
  if constexpr (F8) {
    const float al = *alpha;
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[j] *= al;
  }
  // swapped operands: lane holds C[row][16j + 4q + r]
#pragma unroll
  for (int j = 0; j < NT; ++j) *reinterpret_cast<f32x4*>(C + (size_t)row * ldc + 16 * j + 4 * q) = acc[j];
}

// LDS images: A [64 frames][64 m + 8], B [64 frames][NB + 8] (bf16); transposed fragment reads.
// F8: A is e4m3 (fp8 mode's layer-0 dG, lda in bytes), converted to bf16 on its way into the LDS
// image (exact), the partial slabs scaled by *alpha (1 / dG's scale).
template <int NT, bool F8 = false>
__global__ __launch_bounds__(256) void skinny_tn_kernel(int M, int K, int kchunk, const void* __restrict__ Av,
                                                        int lda, const unsigned short* __restrict__ B, int ldb,
                                                        float* __restrict__ ws, const float* __restrict__ alpha) {
  const unsigned short* A = static_cast<const unsigned short*>(Av);
  const unsigned char* A8 = static_cast<const unsigned char*>(Av);
  constexpr int NB = 16 * NT, LA = 64 + 8, LB = NB + 8;
  __shared__ __attribute__((aligned(16))) short sa[64 * LA];
  __shared__ __attribute__((aligned(16))) short sb[64 * LB];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m0 = blockIdx.x * 64, s = blockIdx.y;
  const int kbeg = s * kchunk, kend = min(K, kbeg + kchunk);
  f32x4 acc[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // staging roles: A chunk = 64 frames x 8 pieces of 16 B; B chunk = 64 frames x NB/8 pieces.
  // The next chunk's loads are issued before this chunk's MFMAs (one register set ahead): with a
  // load -> LDS -> MFMA loop each chunk cost one exposed HBM round trip (c5's 32,000 frames:
  // 142 us for 262 MB, 1.8 TB/s)
  constexpr int PB = 64 * NB / 8;
  constexpr int NVB = (PB + 255) / 256;
  u32x4 va[2], vb[NVB];
  auto load = [&](int k0) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int idx = tid + 256 * i, fr = idx >> 3, c8 = idx & 7;
      const int f = k0 + fr;
      if constexpr (F8) {
        const u32x2 r = f < kend ? *reinterpret_cast<const u32x2*>(A8 + (size_t)f * lda + m0 + 8 * c8) : u32x2{0u, 0u};
        va[i] = u32x4{r[0], r[1], 0u, 0u};
      } else {
        va[i] = f < kend ? *reinterpret_cast<const u32x4*>(A + (size_t)f * lda + m0 + 8 * c8) : u32x4{0u, 0u, 0u, 0u};
      }
    }
#pragma unroll
    for (int i = 0; i < NVB; ++i) {
      const int idx = tid + 256 * i, fr = idx / (NB / 8), c8 = idx % (NB / 8);
      const int f = k0 + fr;
      vb[i] = (idx < PB && f < kend) ? *reinterpret_cast<const u32x4*>(B + (size_t)f * ldb + 8 * c8)
                                     : u32x4{0u, 0u, 0u, 0u};
    }
  };
  if (kbeg < kend) load(kbeg);
  for (int k0 = kbeg; k0 < kend; k0 += 64) {
    __syncthreads();  // previous chunk's fragments are consumed
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int idx = tid + 256 * i, fr = idx >> 3, c8 = idx & 7;
      if constexpr (F8) *reinterpret_cast<bf16x8*>(sa + fr * LA + 8 * c8) = fp8x8_to_bf16(va[i][0], va[i][1]);
      else *reinterpret_cast<u32x4*>(sa + fr * LA + 8 * c8) = va[i];
    }
#pragma unroll
    for (int i = 0; i < NVB; ++i) {
      const int idx = tid + 256 * i, fr = idx / (NB / 8), c8 = idx % (NB / 8);
      if (idx < PB) *reinterpret_cast<u32x4*>(sb + fr * LB + 8 * c8) = vb[i];
    }
    __syncthreads();
    if (k0 + 64 < kend) load(k0 + 64);  // in flight under this chunk's MFMAs
    // wave w: m rows 16w .. 16w+15 (A^T fragment by transposed reads), all NB columns
    const int g = lane >> 4, i4 = lane & 15, qq = i4 >> 2, pp = i4 & 3;
#pragma unroll
    for (int kk = 0; kk < 64; kk += 32) {
      const int r1 = kk + 8 * g + qq, r2 = r1 + 4;
      const bf16x4 a1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_b4_p)(sa + r1 * LA + 16 * wave + 4 * pp));
      const bf16x4 a2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_b4_p)(sa + r2 * LA + 16 * wave + 4 * pp));
      const bf16x8 af = {a1[0], a1[1], a1[2], a1[3], a2[0], a2[1], a2[2], a2[3]};
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const bf16x4 b1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_b4_p)(sb + r1 * LB + 16 * j + 4 * pp));
        const bf16x4 b2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_b4_p)(sb + r2 * LB + 16 * j + 4 * pp));
        const bf16x8 bfr = {b1[0], b1[1], b1[2], b1[3], b2[0], b2[1], b2[2], b2[3]};
        acc[j] = mfma16(bfr, af, acc[j]);  // swapped: lane holds P[m][16j + 4q + r]
      }
    }
  }
  const int m = m0 + 16 * wave + (lane & 15), q = lane >> 4;
  if (m >= M) return;
  if constexpr (F8) {
    const float al = *alpha;
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[j] *= al;
  }
  float* out = ws + ((size_t)s * M + m) * NB;
#pragma unroll
  for (int j = 0; j < NT; ++j) *reinterpret_cast<f32x4*>(out + 16 * j + 4 * q) = acc[j];
}

// skinny_dzw: dZ = dG W_ih (as skinny_nt) AND the slabs of dW_ih | db = dG^T [z | 1] (as
// skinny_tn) from ONE pass over dG -- the two kernels each streamed the whole 1 GB dG of c3.
// A workgroup (8 waves) owns NRB 128-frame row blocks and walks dG in 256-column chunks (chunks
// outer, its row blocks inner): each [128 x 256] tile goes through LDS once and feeds both
// products -- dZ by row-major fragments (accumulated over the chunks in registers), dW^T by
// transposed reads (accumulated over the row blocks, one slab row-range per chunk).  The next
// tile's 16-byte loads are issued before this tile's MFMAs.  Slabs [G][8H][NB] reduce in a
// fixed order (skinny_reduce).  Z == 32, NB == 48 (z | 1 | pad), K8 % 256 == 0.
constexpr int DZW_KC = 256, DZW_LA = DZW_KC + 8, DZW_NB = 48, DZW_LZ = DZW_NB + 8, DZW_Z = 32, DZW_NRB = 4;
__global__ __launch_bounds__(512) void skinny_dzw_kernel(int M, int K8, const unsigned short* __restrict__ A, int lda,
                                                         const unsigned short* __restrict__ Wt, int ldw,
                                                         const unsigned short* __restrict__ Zb, int ldz,
                                                         float* __restrict__ dZ, int lddz, float* __restrict__ slabs) {
  extern __shared__ __attribute__((aligned(16))) short smem[];
  short* sa = smem;                             // [128 frames][DZW_LA]: the dG tile
  short* sw = sa + 128 * DZW_LA;                // [32 z][DZW_LA]: W_ih^T chunk
  short* sz = sw + DZW_Z * DZW_LA;              // [NRB][128 frames][DZW_LZ]: z | 1 | pad
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l15 = lane & 15, q = lane >> 4;
  const int rb0 = blockIdx.x * DZW_NRB;         // first 128-row block of this workgroup
  const int nrb_all = (M + 127) / 128;
  const int nrb = min(DZW_NRB, nrb_all - rb0);  // >= 1
  const int nch = K8 / DZW_KC;
  // z blocks (bf16, NB columns), once
  for (int i = tid; i < nrb * 128 * (DZW_NB / 8); i += 512) {
    const int r = i / (DZW_NB / 8), c8 = i % (DZW_NB / 8), f = rb0 * 128 + r;
    u32x4 v = {0u, 0u, 0u, 0u};
    if (f < M) v = *reinterpret_cast<const u32x4*>(Zb + (size_t)f * ldz + 8 * c8);
    *reinterpret_cast<u32x4*>(sz + r * DZW_LZ + 8 * c8) = v;
  }
  // dG tile loads: 128 rows x 32 16-byte pieces = 4096 pieces, 8 per thread.  Tiles in the order
  // (chunk c, row block rb), two register buffers: tile i+2's loads are issued while tile i is
  // multiplied (one tile ahead left each tile waiting ~one HBM latency: 3.9 TB/s at c3)
  const int ntl = nch * nrb;
  auto aload = [&](u32x4 (&va)[8], int ti) {
    const int c = ti / nrb, rb = ti - c * nrb;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int idx = tid + 512 * i, r = idx >> 5, c8 = idx & 31, f = (rb0 + rb) * 128 + r;
      va[i] = f < M ? *reinterpret_cast<const u32x4*>(A + (size_t)f * lda + c * DZW_KC + 8 * c8) : u32x4{0u, 0u, 0u, 0u};
    }
  };
  auto astore = [&](const u32x4 (&va)[8]) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int idx = tid + 512 * i, r = idx >> 5, c8 = idx & 31;
      *reinterpret_cast<u32x4*>(sa + r * DZW_LA + 8 * c8) = va[i];
    }
  };
  f32x4 adz[DZW_NRB][2];
#pragma unroll
  for (int b = 0; b < DZW_NRB; ++b) adz[b][0] = adz[b][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int g = lane >> 4, i4 = lane & 15, qq = i4 >> 2, pp = i4 & 3;
  f32x4 aw[2][3];  // dW^T tiles of the current chunk: m-tiles wave, wave + 8 of its 16; n-tiles 0..2
  auto tile = [&](int ti, u32x4 (&va)[8]) {
    const int c = ti / nrb, rb = ti - c * nrb;
    if (rb == 0) {
#pragma unroll
      for (int t = 0; t < 2; ++t) aw[t][0] = aw[t][1] = aw[t][2] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    __syncthreads();  // the previous tile's (and chunk's) LDS reads are done
    astore(va);
    if (rb == 0) {  // this chunk's W_ih^T rows: 32 x 256
      for (int i = tid; i < DZW_Z * (DZW_KC / 8); i += 512) {
        const int r = i / (DZW_KC / 8), c8 = i % (DZW_KC / 8);
        *reinterpret_cast<u32x4*>(sw + r * DZW_LA + 8 * c8) =
            *reinterpret_cast<const u32x4*>(Wt + (size_t)r * ldw + c * DZW_KC + 8 * c8);
      }
    }
    __syncthreads();
    if (ti + 2 < ntl) aload(va, ti + 2);  // two tiles ahead, into the buffer just staged
    // dZ[rows 16 wave .. +15 of block rb][32] += tile . W_ih  (swapped: lane holds z 16 j + 4 q + r)
#pragma unroll
    for (int u = 0; u < DZW_KC / 32; ++u) {
      const bf16x8 af = *reinterpret_cast<const bf16x8*>(sa + (16 * wave + l15) * DZW_LA + 32 * u + 8 * q);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const bf16x8 bw = *reinterpret_cast<const bf16x8*>(sw + (16 * j + l15) * DZW_LA + 32 * u + 8 * q);
#pragma unroll
        for (int b = 0; b < DZW_NRB; ++b)
          if (b == rb) adz[b][j] = mfma16(bw, af, adz[b][j]);
      }
    }
    // dW^T[chunk cols][NB] += tile^T . [z | 1]  (transposed reads over the 128 frames)
    const short* zb = sz + rb * 128 * DZW_LZ;
#pragma unroll
    for (int kk = 0; kk < 128; kk += 32) {
      const int r1 = kk + 8 * g + qq, r2 = r1 + 4;
      bf16x8 bz[3];
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const bf16x4 b1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_b4_p)(zb + r1 * DZW_LZ + 16 * j + 4 * pp));
        const bf16x4 b2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_b4_p)(zb + r2 * DZW_LZ + 16 * j + 4 * pp));
        bz[j] = bf16x8{b1[0], b1[1], b1[2], b1[3], b2[0], b2[1], b2[2], b2[3]};
      }
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int m0 = 16 * (wave + 8 * t);
        const bf16x4 a1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_b4_p)(sa + r1 * DZW_LA + m0 + 4 * pp));
        const bf16x4 a2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_b4_p)(sa + r2 * DZW_LA + m0 + 4 * pp));
        const bf16x8 af = {a1[0], a1[1], a1[2], a1[3], a2[0], a2[1], a2[2], a2[3]};
#pragma unroll
        for (int j = 0; j < 3; ++j) aw[t][j] = mfma16(bz[j], af, aw[t][j]);  // lane: P[m][16 j + 4 q + r]
      }
    }
    if (rb == nrb - 1) {  // this chunk's slab rows: slab[blockIdx.x][c * 256 + m][NB]
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int m = c * DZW_KC + 16 * (wave + 8 * t) + l15;
        float* out = slabs + ((size_t)blockIdx.x * K8 + m) * DZW_NB;
#pragma unroll
        for (int j = 0; j < 3; ++j) *reinterpret_cast<f32x4*>(out + 16 * j + 4 * q) = aw[t][j];
      }
    }
  };
  u32x4 v0[8], v1[8];
  aload(v0, 0);
  if (ntl > 1) aload(v1, 1);
  for (int ti = 0; ti < ntl; ti += 2) {
    tile(ti, v0);
    if (ti + 1 < ntl) tile(ti + 1, v1);
  }
#pragma unroll
  for (int b = 0; b < DZW_NRB; ++b) {
    const int f = (rb0 + b) * 128 + 16 * wave + l15;
    if (b < nrb && f < M) {
#pragma unroll
      for (int j = 0; j < 2; ++j) *reinterpret_cast<f32x4*>(dZ + (size_t)f * lddz + 16 * j + 4 * q) = adz[b][j];
    }
  }
}

// W[m][n] = sum_s P_s[m][n] for n < nw; bias1[m] = bias2[m] = sum_s P_s[m][nw] (if given)
__global__ __launch_bounds__(256) void skinny_reduce(int M, int NB, int S, int nw, const float* __restrict__ ws,
                                                     float* __restrict__ W, float* __restrict__ b1,
                                                     float* __restrict__ b2) {
  const int ncol = nw + ((b1 || b2) ? 1 : 0);
  const size_t total = (size_t)M * ncol;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (size_t)gridDim.x * 256) {
    const int m = (int)(i / ncol), n = (int)(i % ncol);
    float v = 0.f;
#pragma unroll 8  // loads in flight; the adds keep their order
    for (int s = 0; s < S; ++s) v += ws[((size_t)s * M + m) * NB + n];
    if (n < nw) W[(size_t)m * nw + n] = v;
    else {
      if (b1) b1[m] = v;
      if (b2) b2[m] = v;
    }
  }
}

constexpr int PROJ_CN = 512;  // output columns per workgroup (64 rows x 512 cols)

// Each wave stages its own 16 rows x 128 columns (wave-private LDS: no workgroup barrier) and
// stores them as 16-byte lanes, 256 contiguous bytes per row of fp16 (the 64-column form with a
// workgroup barrier per chunk wrote 2.8 TB/s at c3)
template <bool F16>  // C stored as fp16 (the wide-batch recurrence's gate buffer) or fp32
__global__ __launch_bounds__(256) void skinny_proj_kernel(int M, int N, int K,
                                                          const unsigned short* __restrict__ A, int lda,
                                                          const unsigned short* __restrict__ B, int ldb,
                                                          const float* __restrict__ b1,
                                                          const float* __restrict__ b2,
                                                          void* __restrict__ C, int ldc) {
  constexpr int CW = 128, LS = CW + 4;  // columns per pass, staging row stride (floats)
  __shared__ __attribute__((aligned(16))) float stg[4][16 * LS];  // per wave: 16 rows x 128 cols
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int rr = lane & 15, kq = lane >> 4;
  // column block fastest: concurrent workgroups write whole rows, not one 1 KB column slice of
  // many 8 KB rows
  const int r0 = blockIdx.y * 64 + wave * 16;
  const int n0 = blockIdx.x * PROJ_CN;
  const bool kin = 8 * kq < K;  // K % 8 == 0 (checked on the host)
  bf16x8 a = {0, 0, 0, 0, 0, 0, 0, 0};
  if (kin && r0 + rr < M) a = *reinterpret_cast<const bf16x8*>(A + (size_t)(r0 + rr) * lda + 8 * kq);
  float* sw = stg[wave];
  for (int c0 = n0; c0 < n0 + PROJ_CN && c0 < N; c0 += CW) {  // N % 16 == 0
#pragma unroll
    for (int jb = 0; jb < CW / 16; ++jb) {
      const int cb = c0 + 16 * jb;
      if (cb < N) {
        bf16x8 b = {0, 0, 0, 0, 0, 0, 0, 0};
        if (kin) b = *reinterpret_cast<const bf16x8*>(B + (size_t)(cb + rr) * ldb + 8 * kq);
        // operands swapped: lane holds C[r0 + rr][cb + 4 kq + r], r = 0..3
        const f32x4 acc = mfma16(b, a, f32x4{0.f, 0.f, 0.f, 0.f});
        *reinterpret_cast<f32x4*>(sw + rr * LS + 16 * jb + 4 * kq) = acc;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // one wave: its LDS ops complete in order
    // read back row-contiguous: lane (row 4i + lane / 16, 8 columns at 8 (lane % 16))
    const int col = c0 + 8 * (lane & 15);
    if (col < N) {
      f32x4 bl = {0.f, 0.f, 0.f, 0.f}, bh = {0.f, 0.f, 0.f, 0.f};
      if (b1) { bl += *reinterpret_cast<const f32x4*>(b1 + col); bh += *reinterpret_cast<const f32x4*>(b1 + col + 4); }
      if (b2) { bl += *reinterpret_cast<const f32x4*>(b2 + col); bh += *reinterpret_cast<const f32x4*>(b2 + col + 4); }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = 4 * i + (lane >> 4);
        const f32x4 lo = *reinterpret_cast<const f32x4*>(sw + r * LS + 8 * (lane & 15)) + bl;
        const f32x4 hi = *reinterpret_cast<const f32x4*>(sw + r * LS + 8 * (lane & 15) + 4) + bh;
        if (r0 + r >= M) continue;
        if constexpr (F16) {
          const u32x2 l2 = f2h4(lo), h2 = f2h4(hi);
          *reinterpret_cast<u32x4*>(static_cast<unsigned short*>(C) + (size_t)(r0 + r) * ldc + col) =
              u32x4{l2[0], l2[1], h2[0], h2[1]};
        } else {
          float* cp = static_cast<float*>(C) + (size_t)(r0 + r) * ldc + col;
          *reinterpret_cast<f32x4*>(cp) = lo;
          *reinterpret_cast<f32x4*>(cp + 4) = hi;
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // staging read before the next pass rewrites it
  }
}

// frame splits: ~2048 workgroups (several per CU: each holds only 8 KB of A in flight, so the
// bytes in flight chip-wide -- not the CU count -- set the stream rate; 512 ran at 1.8 TB/s)
int tn_splits(int M, int K) {
  const int mb = (M + 63) / 64;
  int s = (2048 + mb - 1) / mb;
  const int maxs = (K + 255) / 256;  // >= 4 chunks of 64 frames per split
  if (s > maxs) s = maxs;
  return s < 1 ? 1 : s;
}

}  // namespace

extern "C" int mlvae_skinny_nt(int M, int N, int K, const void* A, int lda, const void* Bt, int ldb,
                               float* C, int ldc, void* stream) {
  if (M <= 0) return 0;
  if (!A || !Bt || !C || N % 16 || N < 16 || N > 64 || K % 32 || lda % 8 || ldb % 8 || ldc % 4 ||
      ((uintptr_t)A % 16) || ((uintptr_t)Bt % 16) || ((uintptr_t)C % 16)) {
    mlvae_set_error("mlvae_skinny_nt: N in {16..64} %% 16, K %% 32, aligned 16-byte rows");
    return 1;
  }
  const unsigned short* a = static_cast<const unsigned short*>(A);
  const unsigned short* b = static_cast<const unsigned short*>(Bt);
  hipStream_t st = (hipStream_t)stream;
  if (K % NTL_KC == 0 && M >= 4096) {  // row streams of >= 32 workgroups: Bt shared through LDS
                                         // (c3 409 -> 210 us, c2 52 -> 49 us)
    dim3 g128((M + 127) / 128);
    switch (N / 16) {
      case 1: skinny_nt_lds_kernel<1><<<g128, 512, 0, st>>>(M, K, a, lda, b, ldb, C, ldc, nullptr); break;
      case 2: skinny_nt_lds_kernel<2><<<g128, 512, 0, st>>>(M, K, a, lda, b, ldb, C, ldc, nullptr); break;
      case 3: skinny_nt_lds_kernel<3><<<g128, 512, 0, st>>>(M, K, a, lda, b, ldb, C, ldc, nullptr); break;
      default: skinny_nt_lds_kernel<4><<<g128, 512, 0, st>>>(M, K, a, lda, b, ldb, C, ldc, nullptr); break;
    }
    MLVAE_CHECK_LAUNCH();
    return 0;
  }
  if (K % 128 == 0) {
    dim3 g16((M + 15) / 16);
    switch (N / 16) {
      case 1: skinny_nt_ks_kernel<1><<<g16, 256, 0, st>>>(M, K, a, lda, b, ldb, C, ldc); break;
      case 2: skinny_nt_ks_kernel<2><<<g16, 256, 0, st>>>(M, K, a, lda, b, ldb, C, ldc); break;
      case 3: skinny_nt_ks_kernel<3><<<g16, 256, 0, st>>>(M, K, a, lda, b, ldb, C, ldc); break;
      default: skinny_nt_ks_kernel<4><<<g16, 256, 0, st>>>(M, K, a, lda, b, ldb, C, ldc); break;
    }
    MLVAE_CHECK_LAUNCH();
    return 0;
  }
  dim3 grid((M + 63) / 64);
  switch (N / 16) {
    case 1: skinny_nt_kernel<1><<<grid, 256, 0, st>>>(M, K, a, lda, b, ldb, C, ldc); break;
    case 2: skinny_nt_kernel<2><<<grid, 256, 0, st>>>(M, K, a, lda, b, ldb, C, ldc); break;
    case 3: skinny_nt_kernel<3><<<grid, 256, 0, st>>>(M, K, a, lda, b, ldb, C, ldc); break;
    default: skinny_nt_kernel<4><<<grid, 256, 0, st>>>(M, K, a, lda, b, ldb, C, ldc); break;
  }
  MLVAE_CHECK_LAUNCH();
  return 0;
}

// fp8 mode (configs[4]), layer 0: dZ = alpha dG8 W_ih with dG8 e4m3 [M][lda bytes] (the fp8 BPTT's
// copy, alpha = 1 / its scale) and W_ih^T bf16 -- skinny_nt's LDS form (K % 256, M >= 4096)
extern "C" int mlvae_skinny_nt_fp8(int M, int N, int K, const void* A8, int lda, const void* Bt, int ldb,
                                   float* C, int ldc, const float* alpha, void* stream) {
  if (M <= 0) return 0;
  if (!A8 || !Bt || !C || !alpha || N % 16 || N < 16 || N > 64 || K % NTL_KC || M < 4096 || lda % 16 ||
      ldb % 8 || ldc % 4 || ((uintptr_t)A8 % 16) || ((uintptr_t)Bt % 16) || ((uintptr_t)C % 16)) {
    mlvae_set_error("mlvae_skinny_nt_fp8: N in {16..64} %% 16, K %% 256, M >= 4096, aligned rows (lda %% 16 B)");
    return 1;
  }
  const unsigned short* b = static_cast<const unsigned short*>(Bt);
  hipStream_t st = (hipStream_t)stream;
  dim3 g128((M + 127) / 128);
  switch (N / 16) {
    case 1: skinny_nt_lds_kernel<1, true><<<g128, 512, 0, st>>>(M, K, A8, lda, b, ldb, C, ldc, alpha); break;
    case 2: skinny_nt_lds_kernel<2, true><<<g128, 512, 0, st>>>(M, K, A8, lda, b, ldb, C, ldc, alpha); break;
    case 3: skinny_nt_lds_kernel<3, true><<<g128, 512, 0, st>>>(M, K, A8, lda, b, ldb, C, ldc, alpha); break;
    default: skinny_nt_lds_kernel<4, true><<<g128, 512, 0, st>>>(M, K, A8, lda, b, ldb, C, ldc, alpha); break;
  }
  MLVAE_CHECK_LAUNCH();
  return 0;
}

extern "C" int mlvae_skinny_proj_ex(int M, int N, int K, const void* A, int lda, const void* B,
                                    int ldb, const float* bias1, const float* bias2, void* C,
                                    int ldc, int c_fp16, void* stream) {
  if (M <= 0 || N <= 0) return 0;
  if (!A || !B || !C || K < 8 || K > 32 || K % 8 || N % 16 || lda % 8 || ldb % 8 || ldc % (c_fp16 ? 8 : 4) ||
      ((uintptr_t)A % 16) || ((uintptr_t)B % 16) || ((uintptr_t)C % 16) ||
      ((uintptr_t)bias1 % 16) || ((uintptr_t)bias2 % 16)) {
    mlvae_set_error("mlvae_skinny_proj: K in {8,16,24,32}, N %% 16, aligned 16-byte rows");
    return 1;
  }
  dim3 grid((N + PROJ_CN - 1) / PROJ_CN, (M + 63) / 64);
  auto k = c_fp16 ? skinny_proj_kernel<true> : skinny_proj_kernel<false>;
  k<<<grid, 256, 0, (hipStream_t)stream>>>(
      M, N, K, static_cast<const unsigned short*>(A), lda, static_cast<const unsigned short*>(B),
      ldb, bias1, bias2, C, ldc);
  MLVAE_CHECK_LAUNCH();
  return 0;
}

extern "C" int mlvae_skinny_proj(int M, int N, int K, const void* A, int lda, const void* B,
                                 int ldb, const float* bias1, const float* bias2, float* C, int ldc,
                                 void* stream) {
  return mlvae_skinny_proj_ex(M, N, K, A, lda, B, ldb, bias1, bias2, C, ldc, 0, stream);
}

extern "C" size_t mlvae_skinny_tn_workspace_size(int M, int NB, int K) {
  return (size_t)tn_splits(M, K) * M * NB * sizeof(float);
}

// W [M, nw] (+ bias1/bias2 [M] = column nw) = A^T B over K frames; B carries NB >= nw + 1
// columns when biases are wanted (column nw all ones), else NB >= nw.
extern "C" int mlvae_skinny_tn(int M, int NB, int K, const void* A, int lda, const void* B, int ldb,
                               int nw, float* W, float* bias1, float* bias2, float* ws,
                               size_t ws_bytes, void* stream) {
  if (M <= 0) return 0;
  if (!A || !B || !W || M % 64 || NB % 16 || NB < 16 || NB > 64 || nw < 1 ||
      nw + ((bias1 || bias2) ? 1 : 0) > NB || lda % 8 || ldb % 8 || ((uintptr_t)A % 16) ||
      ((uintptr_t)B % 16)) {
    mlvae_set_error("mlvae_skinny_tn: M %% 64, NB in {16..64} %% 16, nw (+1) <= NB, aligned rows");
    return 1;
  }
  const int S = tn_splits(M, K);
  if (!ws || ws_bytes < (size_t)S * M * NB * sizeof(float)) {
    mlvae_set_error("mlvae_skinny_tn: workspace too small");
    return 1;
  }
  int kc = (K + S - 1) / S;
  kc = (kc + 63) / 64 * 64;
  const unsigned short* a = static_cast<const unsigned short*>(A);
  const unsigned short* b = static_cast<const unsigned short*>(B);
  hipStream_t st = (hipStream_t)stream;
  dim3 grid(M / 64, S);
  switch (NB / 16) {
    case 1: skinny_tn_kernel<1><<<grid, 256, 0, st>>>(M, K, kc, a, lda, b, ldb, ws, nullptr); break;
    case 2: skinny_tn_kernel<2><<<grid, 256, 0, st>>>(M, K, kc, a, lda, b, ldb, ws, nullptr); break;
    case 3: skinny_tn_kernel<3><<<grid, 256, 0, st>>>(M, K, kc, a, lda, b, ldb, ws, nullptr); break;
    default: skinny_tn_kernel<4><<<grid, 256, 0, st>>>(M, K, kc, a, lda, b, ldb, ws, nullptr); break;
  }
  MLVAE_CHECK_LAUNCH();
  const size_t total = (size_t)M * (nw + 1);
  int blocks = (int)((total + 255) / 256);
  if (blocks > 1024) blocks = 1024;
  skinny_reduce<<<blocks, 256, 0, st>>>(M, NB, S, nw, ws, W, bias1, bias2);
  MLVAE_CHECK_LAUNCH();
  return 0;
}

// fp8 mode, layer 0: W [M, nw] (+ biases) = alpha A8^T B as mlvae_skinny_tn, A8 the e4m3 dG [K][lda
// bytes] (workspace: mlvae_skinny_tn_workspace_size)
extern "C" int mlvae_skinny_tn_fp8(int M, int NB, int K, const void* A8, int lda, const void* B, int ldb,
                                   int nw, float* W, float* bias1, float* bias2, const float* alpha, float* ws,
                                   size_t ws_bytes, void* stream) {
  if (M <= 0) return 0;
  if (!A8 || !B || !W || !alpha || M % 64 || NB % 16 || NB < 16 || NB > 64 || nw < 1 ||
      nw + ((bias1 || bias2) ? 1 : 0) > NB || lda % 16 || ldb % 8 || ((uintptr_t)A8 % 16) || ((uintptr_t)B % 16)) {
    mlvae_set_error("mlvae_skinny_tn_fp8: M %% 64, NB in {16..64} %% 16, nw (+1) <= NB, aligned rows (lda %% 16 B)");
    return 1;
  }
  const int S = tn_splits(M, K);
  if (!ws || ws_bytes < (size_t)S * M * NB * sizeof(float)) {
    mlvae_set_error("mlvae_skinny_tn_fp8: workspace too small");
    return 1;
  }
  int kc = (K + S - 1) / S;
  kc = (kc + 63) / 64 * 64;
  const unsigned short* b = static_cast<const unsigned short*>(B);
  hipStream_t st = (hipStream_t)stream;
  dim3 grid(M / 64, S);
  switch (NB / 16) {
    case 1: skinny_tn_kernel<1, true><<<grid, 256, 0, st>>>(M, K, kc, A8, lda, b, ldb, ws, alpha); break;
    case 2: skinny_tn_kernel<2, true><<<grid, 256, 0, st>>>(M, K, kc, A8, lda, b, ldb, ws, alpha); break;
    case 3: skinny_tn_kernel<3, true><<<grid, 256, 0, st>>>(M, K, kc, A8, lda, b, ldb, ws, alpha); break;
    default: skinny_tn_kernel<4, true><<<grid, 256, 0, st>>>(M, K, kc, A8, lda, b, ldb, ws, alpha); break;
  }
  MLVAE_CHECK_LAUNCH();
  const size_t total = (size_t)M * (nw + 1);
  int blocks = (int)((total + 255) / 256);
  if (blocks > 1024) blocks = 1024;
  skinny_reduce<<<blocks, 256, 0, st>>>(M, NB, S, nw, ws, W, bias1, bias2);
  MLVAE_CHECK_LAUNCH();
  return 0;
}

// dZ = dG W_ih and dW_ih | b_ih = b_hh grads = dG^T [z | 1] in one pass over dG (skinny_dzw_kernel):
// dG [M][lda] bf16 (K8 = 8H columns), Wt = W_ih^T [32][ldw] bf16, zb = [z | 1 | 0] [M][ldz] bf16 with
// 48 columns, dZ [M][lddz] fp32; W [K8][32], bias1 / bias2 [K8] (both optional).
extern "C" size_t mlvae_skinny_dzw_workspace_size(int M, int K8) {
  const int G = ((M + 127) / 128 + DZW_NRB - 1) / DZW_NRB;
  return (size_t)G * K8 * DZW_NB * sizeof(float);
}

extern "C" int mlvae_skinny_dzw(int M, int K8, const void* A, int lda, const void* Wt, int ldw, const void* zb, int ldz,
                                int Z, float* dZ, int lddz, float* W, float* bias1, float* bias2, float* ws,
                                size_t ws_bytes, void* stream) {
  if (M <= 0) return 0;
  if (!A || !Wt || !zb || !dZ || !W || Z != DZW_Z || K8 % DZW_KC || K8 <= 0 || lda % 8 || ldw % 8 || ldz % 8 ||
      ldz < DZW_NB || lddz % 4 || lddz < Z || ((uintptr_t)A % 16) || ((uintptr_t)Wt % 16) || ((uintptr_t)zb % 16) ||
      ((uintptr_t)dZ % 16)) {
    mlvae_set_error("mlvae_skinny_dzw: Z = 32, 8H %% 256, z rows of >= 48 bf16 (z | 1 | 0), aligned 16-byte rows");
    return 1;
  }
  const int G = ((M + 127) / 128 + DZW_NRB - 1) / DZW_NRB;
  if (!ws || ws_bytes < mlvae_skinny_dzw_workspace_size(M, K8)) {
    mlvae_set_error("mlvae_skinny_dzw: workspace too small");
    return 1;
  }
  const size_t lds = ((size_t)(128 + DZW_Z) * DZW_LA + (size_t)DZW_NRB * 128 * DZW_LZ) * sizeof(short);
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute((const void*)skinny_dzw_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
        hipSuccess) {
      mlvae_set_error("mlvae_skinny_dzw: cannot reserve %zu B LDS", lds);
      return 2;
    }
    attr = true;
  }
  hipStream_t st = (hipStream_t)stream;
  skinny_dzw_kernel<<<G, 512, lds, st>>>(M, K8, static_cast<const unsigned short*>(A), lda,
                                         static_cast<const unsigned short*>(Wt), ldw,
                                         static_cast<const unsigned short*>(zb), ldz, dZ, lddz, ws);
  MLVAE_CHECK_LAUNCH();
  const size_t total = (size_t)K8 * (Z + 1);
  int blocks = (int)((total + 255) / 256);
  if (blocks > 1024) blocks = 1024;
  skinny_reduce<<<blocks, 256, 0, st>>>(K8, DZW_NB, G, Z, ws, W, bias1, bias2);
  MLVAE_CHECK_LAUNCH();
  return 0;
}
