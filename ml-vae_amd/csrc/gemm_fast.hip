// Large bf16 GEMMs of the bf16 train step on gfx950: 256 x 256 tiles, LDS-DMA staging.
//
//   C[M,N] = epi( op(A)[M,K] . op(B)[K,N] + bias1[N] + bias2[N] + beta * C )     (C fp32)
//
// The products this serves (bf16 operands in HBM, written by the step itself):
//   input projection  G = X W_ih^T      A [N_fr, din] k-contig, B = W_ih [8H, din] k-contig
//                     (ref:src/modules/decoder.py:14-15,22, nn.LSTM input part)
//   dgrad             dX = dG W_ih      A = dG [N_fr, 8H] k-contig, B = W_ih [8H, din] n-contig
//   weight gradients  dW = dG^T X       A = dG [N_fr, 8H] m-contig, B = X [N_fr, din] n-contig
//                     (K = B*T frames: split-K; the recurrent dW_hh reads B time-shifted)
//
// Structure (cdna_hip_programming.md §5: 256² tile, BK = 64, 8 waves as 2 (M) x 4 (N), each wave
// 128 x 64 as 8 x 4 v_mfma_f32_16x16x32_bf16 tiles):
//   * operands go HBM -> LDS with buffer_load ... lds (16 B per lane; the LDS image is lane-linear,
//     so the bank swizzle is applied to the per-lane SOURCE address); out-of-range chunks read as
//     zero through the buffer descriptor's range check (offset 0x80000000);
//   * two LDS buffers (2 x 64 KB): tile k+1 streams in while tile k feeds the MFMAs; one
//     vmcnt(0) + barrier per K-step;
//   * k-contiguous operands: [rows][64 k] image (128-B rows), 16-B chunk c of row r stored at slot
//     c ^ (r & 7); fragments by ds_read_b128;
//   * m/n-contiguous operands: [64 k][256 m] image (512-B rows), chunk c of k-row r at slot
//     c ^ f(r), f(r) = 2 * ((r & 3) | ((r >> 3) & 1) << 2); fragments by ds_read_b64_tr_b16 (the
//     hardware transpose read): conflict-free per 32-lane half;
//   * XCD-aware bijective tile order; optional batch (gridDim.y) and split-K (gridDim.z, fp32
//     partial slabs + a fixed-order reduce: deterministic).
#include "common.h"
#include <stdlib.h>
#include <algorithm>
#include <cstdlib>

namespace {

constexpr int TBM = 256, TBN = 256, TBK = 64;
constexpr int IMG = TBM * TBK;                               // elements per operand image
constexpr size_t FAST_LDS = (size_t)2 * 2 * IMG * sizeof(short);  // 128 KB
constexpr unsigned OOB = 0x80000000u;

struct GFArgs {
  int M, N, K;
  const short* A; int lda; long long a_bs;
  const short* B; int ldb; long long b_bs;
  float* C; int ldc; long long c_bs;
  float beta;
  const float* bias1; const float* bias2;
  int epi;
  const float* aux; int ldaux;
  int kshiftT, kshift, kshift_bstep;
  unsigned long long dseed, doff; float dkeep, dscale;  // mask of doff + row*ldc + col
  int splits, kchunk;
  int group_m;        // > 1: tiles walk groups of group_m M-panels column-major (L2 reuse)
  int c16;            // C stored as 16-bit: 1 fp16 (epi bit EPI_OUT_F16), 2 bf16 (EPI_OUT_BF16)
  const float* alpha; // device scalar multiplying A.B (fp8 operand scales), or null
  int abl;            // ablation bits (MLVAE_GEMM_ABL, timing only): 1 no MFMA, 2 no staging loads (VAR 6),
                      // 4 the direct (unstaged) epilogue, 8 no epilogue, 64 4-column 16-bit C stores
  float* ws;
};

enum { EPI_NONE = 0, EPI_LRELU = 1, EPI_DLRELU = 2, EPI_DROPOUT = 3 };
constexpr int EPI_OUT_F16 = 16;  // flag bit of the ABI's epi: C is fp16 (staged epilogue only)
constexpr int EPI_OUT_BF16 = 32; // flag bit of the ABI's epi: C is bf16 (staged epilogue only)

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(3))) bf16x4* lds_b4_t;


// The raw words of make_rsrc()'s buffer descriptor (stride 0, flags 0x00020000) for inline asm.
__device__ __forceinline__ i32x4 rsrc_words(const void* base, unsigned bytes) {
  const unsigned long long b = (unsigned long long)(uintptr_t)base;
  return i32x4{(int)(unsigned)b, (int)((unsigned)(b >> 32) & 0xffffu), (int)bytes, 0x00020000};
}

// One 16-byte-per-lane LDS-DMA piece.  ADMA: issued from inline asm.  The compiler tracks a
// buffer_load ... lds builtin as a pending LDS write and, before any ds_read_b64_tr_b16 /
// ds_read_b64_tr_b8 builtin (whose aliasing it cannot resolve), inserts s_waitcnt vmcnt(0): the
// K-step it has just staged then lands before the current one's fragments are read, and the
// m/n-contiguous loops lost all load/compute overlap.  Issued from asm the DMA is invisible to it;
// the kernels' own counted vmcnt waits and barriers order every LDS access (as in the
// k-contiguous loops, where the compiler never inserted such waits).  m0 is set in the same
// statement (and is the only thing these kernels use m0 for).
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
template <bool ADMA>
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rs, i32x4 rw, short* dst, unsigned off) {
  if constexpr (ADMA) {
    // the low 32 bits of a generic pointer into LDS are its LDS address (the aperture is the high
    // half): no addrspacecast, whose null check cost three scalar instructions per piece
    const unsigned la = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)dst);
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds"
                 :: "v"(off), "s"(rw), "s"(la) : "memory", "m0");
  } else {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)dst, 16, off, 0, 0, 0);
  }
}
#pragma clang diagnostic pop

__device__ __forceinline__ unsigned mc_swz(int r) { return 2u * ((r & 3) | (((r >> 3) & 1) << 2)); }

// Time-shifted K rows (the recurrent dW_hh: row k reads k + sh when 0 <= k % T + sh < T).
// Byte offset of the 16-byte chunk of an m/n-contiguous operand at k-row k0 + kr, column gr, or OOB.
// 32-bit arithmetic (the host bounds every operand below 2 GB): the lane part is loop-invariant and
// the K-step adds one wave-uniform term.  tk = k0 % T is wave-uniform (one scalar division per
// stage); a lane then needs one unsigned-min wrap when T >= span (wgrad hh: 1.6x faster staging
// than a per-lane modulo).
__device__ __forceinline__ unsigned mc_off(int kr, int gr, int ld, int R, int k0, int kend, int shT, int sh, int tk,
                                           int span) {
  bool ok = k0 + kr < kend && gr < R;
  const unsigned e = (unsigned)(k0 + sh) * (unsigned)ld + (unsigned)(kr * ld + gr);
  if (sh != 0) {
    int t = tk + kr;
    t = shT >= span ? (int)min((unsigned)t, (unsigned)(t - shT)) : t % shT;
    ok = ok && (unsigned)(t + sh) < (unsigned)shT;
  }
  return ok ? e * 2u : OOB;
}

// m/n-contiguous staging with the lane-invariant part computed once per tile: per piece and K-step
// a lane then spends a compare, an add and a select (plus the wrap test for time-shifted rows)
// instead of re-deriving its column, swizzle and bounds -- the ping-pong loop's fragment-read slot
// has ~512 MFMA cycles of the other group to hide the staging in.  Pieces pb .. pb + NP - 1 of a
// [span k][256 cols] image (piece = 2 k-rows of 512 B).
template <int NP>
struct McLanes {
  unsigned off2[NP];  // 2 (kr ld + gr), or OOB for a column >= R
  int kr0;            // this lane's k-row in piece pb (piece pb + j: kr0 + 2 j)
  __device__ __forceinline__ void init(int pb, int lane, int ld, int r0, int R) {
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      const int p = (pb + j) * 64 + lane, kr = p >> 5, c = (p & 31) ^ (int)mc_swz(kr), gr = r0 + 8 * c;
      off2[j] = gr < R ? 2u * (unsigned)(kr * ld + gr) : OOB;
    }
    kr0 = (pb * 64 + lane) >> 5;
  }
  // SH: 0 no time shift; 1 rows read k + sh inside each length-shT sequence with shT >= the image
  // depth (one unsigned-min wrap); 2 any shT (per-lane modulo)
  template <int SH, bool ADMA>
  __device__ __forceinline__ void stage(short* img, __amdgpu_buffer_rsrc_t rs, i32x4 rw, int ld, int k0, int kend,
                                        int shT, int sh, int pb) const {
    const unsigned base = 2u * (unsigned)(k0 + sh) * (unsigned)ld;  // wraps for k0 + sh < 0: those rows fail
    const int lim = kend - k0;
    const int tk = SH ? k0 % shT : 0;
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      const int kr = kr0 + 2 * j;
      bool ok = kr < lim && off2[j] < OOB;
      if constexpr (SH == 1) {
        const int t = tk + kr;
        ok = ok && (unsigned)((int)min((unsigned)t, (unsigned)(t - shT)) + sh) < (unsigned)shT;
      } else if constexpr (SH == 2) {
        ok = ok && (unsigned)((tk + kr) % shT + sh) < (unsigned)shT;
      }
      dma16<ADMA>(rs, rw, img + (pb + j) * 512, ok ? off2[j] + base : OOB);
    }
  }
  template <bool ADMA>
  __device__ __forceinline__ void stage_any(short* img, __amdgpu_buffer_rsrc_t rs, i32x4 rw, int ld, int k0, int kend,
                                            int shT, int sh, int pb, int span) const {
    if (sh == 0) stage<0, ADMA>(img, rs, rw, ld, k0, kend, shT, 0, pb);
    else if (shT >= span) stage<1, ADMA>(img, rs, rw, ld, k0, kend, shT, sh, pb);
    else stage<2, ADMA>(img, rs, rw, ld, k0, kend, shT, sh, pb);
  }
};

// Issue this wave's 4 LDS-DMA pieces (1 KB each) of one 256 x 64 operand tile.
//   KC: element (row, k) at p[row * ld + k];   MC: element (row, k) at p[k * ld + row]
// rows [r0, r0 + 256) bounded by R; k [k0, k0 + 64) bounded by kend (and by the time shift).
template <bool KC, bool ADMA = false>
__device__ __forceinline__ void stage(short* img, __amdgpu_buffer_rsrc_t rs, i32x4 rw, int ld, int r0, int R,
                                      int k0, int kend, int shT, int sh, int wave, int lane) {
  const int tk = (!KC && sh != 0) ? k0 % shT : 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int piece = wave * 4 + j;
    const int p = piece * 64 + lane;
    unsigned off;
    if constexpr (KC) {
      const int row = p >> 3, c = (p & 7) ^ (row & 7);
      const int gr = r0 + row, gk = k0 + 8 * c;
      off = (gr < R && gk < kend) ? (unsigned)(((size_t)gr * ld + gk) * 2) : OOB;
    } else {
      const int kr = p >> 5, c = (p & 31) ^ (int)mc_swz(kr);
      off = mc_off(kr, r0 + 8 * c, ld, R, k0, kend, shT, sh, tk, TBK);
    }
    dma16<ADMA>(rs, rw, img + piece * 512, off);
  }
}

// MFMA 16x16x32 operand fragment: lane l gets rows/cols (base + (l & 15)), k = kk + 8 (l >> 4) + j.
template <bool KC>
__device__ __forceinline__ bf16x8 frag(const short* img, int base, int kk, int lane) {
  if constexpr (KC) {
    const int row = base + (lane & 15), c = (kk >> 3) + (lane >> 4);
    return *reinterpret_cast<const bf16x8*>(img + row * TBK + ((c ^ (row & 7)) << 3));
  } else {
    const int g = lane >> 4, i4 = lane & 15, q = i4 >> 2, pp = i4 & 3;
    const int r1 = kk + 8 * g + q, r2 = r1 + 4;
    const int c = (base >> 3) + (pp >> 1);
    const short* a1 = img + r1 * TBM + ((c ^ (int)mc_swz(r1)) << 3) + 4 * (pp & 1);
    const short* a2 = img + r2 * TBM + ((c ^ (int)mc_swz(r2)) << 3) + 4 * (pp & 1);
    const bf16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_b4_t)a1);
    const bf16x4 v2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_b4_t)a2);
    return bf16x8{v1[0], v1[1], v1[2], v1[3], v2[0], v2[1], v2[2], v2[3]};
  }
}

// ---- BK = 32 ring (VAR 12): four LDS buffers (4 x 32 KB), three K-steps in flight behind a
// counted vmcnt (raw s_barrier: no implicit drain).  The 2-buffer loop drains vmcnt(0) at every
// K-step, so each 64-deep step waits for loads issued only one step earlier.
constexpr int DBK = 32, DNB = 4;
constexpr int DIMG = TBM * DBK;  // elements per operand image (16 KB)

__device__ __forceinline__ int kc_swz(int row) { return ((row >> 2) & 1) << 1; }  // 32-k rows

// NP pieces (1 KB each) per wave: 2 with all 8 waves staging, 4 with one 4-wave group
template <bool KC, int NP = 2, bool ADMA = false>
__device__ __forceinline__ void stage32(short* img, __amdgpu_buffer_rsrc_t rs, i32x4 rw, int ld, int r0, int R,
                                        int k0, int kend, int shT, int sh, int wave, int lane) {
  const int tk = (!KC && sh != 0) ? k0 % shT : 0;
#pragma unroll
  for (int j = 0; j < NP; ++j) {
    const int piece = wave * NP + j;
    const int p = piece * 64 + lane;
    unsigned off;
    if constexpr (KC) {  // [256 rows][32 k]: 4 chunks per row, chunk c at slot c ^ kc_swz(row)
      const int row = p >> 2, c = (p & 3) ^ kc_swz(row);
      const int gr = r0 + row, gk = k0 + 8 * c;
      off = (gr < R && gk < kend) ? (unsigned)(((size_t)gr * ld + gk) * 2) : OOB;
    } else {             // [32 k][256 rows]: 32 chunks per k-row, as the 64-deep image
      const int kr = p >> 5, c = (p & 31) ^ (int)mc_swz(kr);
      off = mc_off(kr, r0 + 8 * c, ld, R, k0, kend, shT, sh, tk, DBK);
    }
    dma16<ADMA>(rs, rw, img + piece * 512, off);
  }
}

template <bool KC>
__device__ __forceinline__ bf16x8 frag32(const short* img, int base, int lane) {
  if constexpr (KC) {
    const int row = base + (lane & 15), c = lane >> 4;
    return *reinterpret_cast<const bf16x8*>(img + row * DBK + ((c ^ kc_swz(row)) << 3));
  } else {
    const int g = lane >> 4, i4 = lane & 15, q = i4 >> 2, pp = i4 & 3;
    const int r1 = 8 * g + q, r2 = r1 + 4;
    const int c = (base >> 3) + (pp >> 1);
    const short* a1 = img + r1 * TBM + ((c ^ (int)mc_swz(r1)) << 3) + 4 * (pp & 1);
    const short* a2 = img + r2 * TBM + ((c ^ (int)mc_swz(r2)) << 3) + 4 * (pp & 1);
    const bf16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_b4_t)a1);
    const bf16x4 v2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_b4_t)a2);
    return bf16x8{v1[0], v1[1], v1[2], v1[3], v2[0], v2[1], v2[2], v2[3]};
  }
}

__device__ __forceinline__ float epi_apply(const GFArgs& g, float val, int row, int col, float* cp) {
  if (g.beta != 0.f) val += g.beta * *cp;
  if (g.epi == EPI_LRELU) val = lrelu(val);
  else if (g.epi == EPI_DLRELU) val *= lrelu_d(g.aux[(size_t)row * g.ldaux + col]);
  else if (g.epi == EPI_DROPOUT) val *= dropout_scale(g.dseed, g.doff + (size_t)row * g.ldc + col, g.dkeep, g.dscale);
  return val;
}

// fp8 e4m3 operand fragment of v_mfma_scale_f32_16x16x128_f8f6f4 from a k-contiguous image of
// 128-byte rows (128 fp8 = the K-tile; the same bytes as a 64-deep bf16 image, same swizzle):
// lane l holds row base + (l & 15), k = 32 (l >> 4) + j, j < 32 (two 16-byte chunks).  Any
// k-slot assignment is exact as long as A and B use the same one.
__device__ __forceinline__ i32x8 frag8(const short* img, int base, int lane) {
  const int row = base + (lane & 15), c = 2 * (lane >> 4);
  const u32x4 lo = *reinterpret_cast<const u32x4*>(img + row * TBK + ((c ^ (row & 7)) << 3));
  const u32x4 hi = *reinterpret_cast<const u32x4*>(img + row * TBK + (((c + 1) ^ (row & 7)) << 3));
  return i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
}

// ---- fp8 e4m3 operands stored m/n-contiguous (VAR 9: the weight gradients dW = dG^T X over
// frames, both operands [frames][columns] as the recurrences write them).  Image: [128 k][256 m]
// bytes (one K-tile = 128 frames, the same 32 KB as a 64-deep bf16 image); the 16-byte chunk c of
// k-row kr at slot c ^ swz8(kr).  Fragments by ds_read_b64_tr_b8 (profiles/r04_probe_tr8.txt: in
// each 16-lane group, lane 2r + h supplies row r's bytes 8h .. 8h + 7 of a 16-column segment and
// lane i receives column i of the 8 rows), conflict-free: the 16 rows of a 32-lane half (r < 8 of
// k-rows 8s + r and 32 + 8s + r) take 16 distinct slots.
__device__ __forceinline__ int swz8(int kr) { return (kr & 7) | (((kr >> 5) & 1) << 3); }

// this wave's 4 LDS-DMA pieces (1 KB each) of one [128 k][256 m] fp8 image; element (m, k) at byte
// p[k * ld + m]; rows [r0, r0 + 256) bounded by R (R % 16 == 0), k [k0, k0 + 128) by kend.
// Time-shifted k-rows (sh != 0, the recurrent dW_hh): row k reads k + sh when 0 <= k % shT + sh
// < shT, else zeros (as mc_off: one scalar division per stage, one wrap per lane when shT >= 128)
__device__ __forceinline__ void stage8_mc(short* img, __amdgpu_buffer_rsrc_t rs, i32x4 rw, int ld, int r0, int R, int k0,
                                          int kend, int shT, int sh, int wave, int lane) {
  const int tk = sh != 0 ? k0 % shT : 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int piece = wave * 4 + j;
    const int p = piece * 64 + lane;
    const int kr = p >> 4, c = (p & 15) ^ swz8(kr);
    const int gk = k0 + kr, gm = r0 + 16 * c;
    bool ok = gk < kend && gm < R;
    if (sh != 0) {
      int t = tk + kr;
      t = shT >= 128 ? (int)min((unsigned)t, (unsigned)(t - shT)) : t % shT;
      ok = ok && (unsigned)(t + sh) < (unsigned)shT;
    }
    const unsigned off = ok ? (unsigned)(gk + sh) * (unsigned)ld + (unsigned)gm : OOB;
    dma16<true>(rs, rw, img + piece * 512, off);
  }
}

// operand fragment of v_mfma_scale_f32_16x16x128_f8f6f4 from such an image: lane l holds row
// base + (l & 15) at k = 32 (l >> 4) + j, j < 32 -- four transposed 8-row reads
typedef int v2i_t __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) v2i_t* lds_v2i_t;
__device__ __forceinline__ i32x8 frag8_mc(const short* img, int base, int lane) {
  const char* im = reinterpret_cast<const char*>(img);
  const int g = lane >> 4, i = lane & 15, r = i >> 1, h = i & 1, cb = base >> 4;
  i32x8 o;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int kr = 32 * g + 8 * s + r;
    const v2i_t v = __builtin_amdgcn_ds_read_tr8_b64_v2i32((lds_v2i_t)(im + kr * 256 + ((cb ^ swz8(kr)) << 4) + 8 * h));
    o[2 * s] = v[0];
    o[2 * s + 1] = v[1];
  }
  return o;
}

// VAR 0: stage the next K-tile's 8 pieces per wave at the top of the K-step (two buffers);
// 4: VAR 0 with both k-halves' fragments read up front; 12: ping-pong over a BK-32 ring;
// 8: fp8 e4m3 operands (both k-contiguous), one 16x16x128 block-scaled MFMA (unit scales) per
// tile pair and K-tile of 128 -- twice the bf16 MFMA rate, the same staging bytes per K-tile
template <bool AKC, bool BKC, int VAR>
__global__ __launch_bounds__(512) void gemm256_kernel(GFArgs g) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  short* lds = reinterpret_cast<short*>(smem);   // [buf][A image, B image]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const int TM = (g.M + TBM - 1) / TBM, TN = (g.N + TBN - 1) / TBN, ntiles = TM * TN;
  int tile, bz = blockIdx.y, kz = blockIdx.z;
  if (gridDim.y * gridDim.z == 1) {  // XCD-aware bijective order: each XCD works a contiguous run of tiles
    const int b = blockIdx.x, xcd = b % 8, local = b / 8, q = ntiles / 8, r = ntiles % 8;
    tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + local;
  } else {
    // batched / split-K: the same over the flat (split, batch, tile) space, split-major, so an
    // XCD works whole K-ranges -- every A and B chunk of a K-range comes from HBM once into that
    // XCD's L2 (wgrad hh at c3: 16 tiles x 16 splits read the h operand 8x before)
    const int nb = gridDim.x * gridDim.y * gridDim.z;
    const int b = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    const int xcd = b % 8, local = b / 8, q = nb / 8, r = nb % 8;
    const int w = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + local;
    tile = w % (int)gridDim.x;
    bz = (w / (int)gridDim.x) % (int)gridDim.y;
    kz = w / ((int)gridDim.x * (int)gridDim.y);
  }
  int mt = tile / TN, nt = tile % TN;
  if (g.group_m > 1) {  // grouped order: concurrent tiles share group_m A panels and fewer B panels
    const int grp = tile / (g.group_m * TN), mfirst = grp * g.group_m;
    const int gsz = min(TM - mfirst, g.group_m), in = tile - grp * g.group_m * TN;
    mt = mfirst + in % gsz;
    nt = in / gsz;
  }
  const int m0 = mt * TBM, n0 = nt * TBN;
  const short* Ap = g.A + bz * g.a_bs;
  const short* Bp = g.B + bz * g.b_bs;
  const int sh = g.kshift + bz * g.kshift_bstep;
  const auto ra = make_rsrc(Ap, OOB);
  const auto rb = make_rsrc(Bp, OOB);
  const i32x4 rwa = rsrc_words(Ap, OOB), rwb = rsrc_words(Bp, OOB);
  constexpr bool ADMA = !(AKC && BKC);  // a transposed-read operand: LDS-DMA from asm (dma16)
  const int kbeg = kz * g.kchunk;
  const int kend = min(g.K, kbeg + g.kchunk);
  constexpr int SBK = (VAR == 12 || VAR == 13) ? DBK : (VAR == 9 ? 128 : TBK);  // K per main-loop step
  const int nk = kend > kbeg ? (kend - kbeg + SBK - 1) / SBK : 0;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if constexpr (VAR == 4) {
    // VAR 4: both k-halves' fragments (24 ds_reads) issued right after the barrier, so the
    // second half's MFMAs never wait on an LDS round trip in mid-step
    auto stage_both = [&](int buf, int k0) {
      stage<AKC, ADMA>(lds + (buf * 2 + 0) * IMG, ra, rwa, g.lda, m0, g.M, k0, kend, 0, 0, wave, lane);
      stage<BKC, ADMA>(lds + (buf * 2 + 1) * IMG, rb, rwb, g.ldb, n0, g.N, k0, kend, g.kshiftT, sh, wave, lane);
    };
    if (nk > 0) {
      stage_both(0, kbeg);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
    for (int it = 0; it < nk; ++it) {
      const int cur = it & 1;
      if (it + 1 < nk) stage_both(cur ^ 1, kbeg + (it + 1) * TBK);
      const short* As = lds + (cur * 2 + 0) * IMG;
      const short* Bs = lds + (cur * 2 + 1) * IMG;
      bf16x8 af0[8], bf0[4], af1[8], bf1[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) bf0[j] = frag<BKC>(Bs, wn * 64 + j * 16, 0, lane);
#pragma unroll
      for (int i = 0; i < 8; ++i) af0[i] = frag<AKC>(As, wm * 128 + i * 16, 0, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) bf1[j] = frag<BKC>(Bs, wn * 64 + j * 16, 32, lane);
#pragma unroll
      for (int i = 0; i < 8; ++i) af1[i] = frag<AKC>(As, wm * 128 + i * 16, 32, lane);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf0[j], af0[i], acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf1[j], af1[i], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  } else if constexpr (VAR == 12 || VAR == 13) {
    // (VAR 13: this loop with timing ablations, MLVAE_GEMM_ABL bit 1 no MFMAs, bit 2 no staging)
    constexpr bool ABLV = VAR == 13;
    // VAR 12: ping-pong.  Two groups of four waves -- waves 0-3 and 4-7, one of each on every
    // SIMD -- run one barrier apart over a ring of four BK-32 buffers: while one group's waves
    // issue their 32 MFMAs, the other group's read their next fragments from LDS and stage a
    // future K-step, so each SIMD's MFMA pipe is fed by one wave or the other at every moment
    // (the 8-phase idea of cdna_hip_programming.md §5, two slots per K-step).  Slot sequence of
    // a wave: M(it) = fragment reads of step it + its group's half of step it+3 (group 0 the A
    // image, group 1 the B image) + waits, barrier, C(it) = 32 MFMAs, barrier.  Group 1 starts
    // one barrier late.  RAW: step it+1 is waited for (counted vmcnt: it+2, it+3 stay in
    // flight) before the barrier that ends each group's M(it), and the other group reads it
    // only after that barrier.  WAR: step it+3 goes into the buffer of step it-1, whose reads
    // both groups retired (lgkmcnt(0)) before their barriers of the previous slots.
    const int wv = __builtin_amdgcn_readfirstlane(wave);
    const int grpw = wv >> 2, w4 = wv & 3;
    // operands of one layout: each group's staging parameters selected once (one code path and
    // one scalar set in the loop; two had spilled SGPRs into the m/n-contiguous loop)
    const auto rs1 = grpw ? rb : ra;
    const i32x4 rw1 = grpw ? rwb : rwa;
    const int ld1 = grpw ? g.ldb : g.lda, r01 = grpw ? n0 : m0, R1 = grpw ? g.N : g.M;
    const int shT1 = grpw ? g.kshiftT : 0, sh1 = grpw ? sh : 0;
    McLanes<4> ml1;
    if constexpr (!AKC && !BKC) ml1.init(w4 * 4, lane, ld1, r01, R1);
    auto share = [&](int it) {
      const int buf = it & (DNB - 1), k0 = kbeg + it * DBK;
      if constexpr (!AKC && !BKC)
        ml1.stage_any<ADMA>(lds + (buf * 2 + grpw) * DIMG, rs1, rw1, ld1, k0, kend, shT1, sh1, w4 * 4, DBK);
      else if constexpr (AKC == BKC)
        stage32<AKC, 4, ADMA>(lds + (buf * 2 + grpw) * DIMG, rs1, rw1, ld1, r01, R1, k0, kend, shT1, sh1, w4, lane);
      else if (grpw == 0)
        stage32<AKC, 4, ADMA>(lds + (buf * 2 + 0) * DIMG, ra, rwa, g.lda, m0, g.M, k0, kend, 0, 0, w4, lane);
      else
        stage32<BKC, 4, ADMA>(lds + (buf * 2 + 1) * DIMG, rb, rwb, g.ldb, n0, g.N, k0, kend, g.kshiftT, sh, w4, lane);
    };
    auto wait_younger = [&](int n) {  // this wave's shares: all but the n youngest landed
      if (n >= 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else if (n == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    };
    const int npre = min(3, nk);
    for (int it = 0; it < npre; ++it) share(it);
    if (nk > 0) wait_younger(npre - 1);
    __builtin_amdgcn_s_barrier();
    if (grpw == 1) __builtin_amdgcn_s_barrier();  // group 1 runs one slot behind
    bf16x8 af[8], bfr[4];
    for (int it = 0; it < nk; ++it) {
      {
        const short* As = lds + ((it & (DNB - 1)) * 2 + 0) * DIMG;
        const short* Bs = lds + ((it & (DNB - 1)) * 2 + 1) * DIMG;
#pragma unroll
        for (int j = 0; j < 4; ++j) bfr[j] = frag32<BKC>(Bs, wn * 64 + j * 16, lane);
#pragma unroll
        for (int i = 0; i < 8; ++i) af[i] = frag32<AKC>(As, wm * 128 + i * 16, lane);
      }
      if (it + 3 < nk && !(ABLV && (g.abl & 2))) share(it + 3);
      if (it + 1 < nk) wait_younger(min(2, nk - it - 2));
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);  // the MFMAs stay in their slot
      __builtin_amdgcn_s_setprio(1);
      if (ABLV && (g.abl & 1)) {
#pragma unroll
        for (int i = 0; i < 8; ++i) asm volatile("" ::"v"(af[i]));
#pragma unroll
        for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(bfr[j]));
      } else {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
      }
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
    }
    if (grpw == 0) __builtin_amdgcn_s_barrier();  // both groups pass the same number of barriers
    __syncthreads();  // every wave's last fragment reads are done: the LDS is the epilogue's
  } else if constexpr (VAR == 16) {
    // VAR 16: eight phases per two 64-deep K-tiles (two LDS buffers, BK = 64), k-contiguous A and
    // B.  Two groups of four waves (0-3, 4-7: one of each per SIMD) run one barrier apart; a phase
    // of a group is [its fragment reads + one staged half-tile (2 LDS-DMA pieces per wave) +
    // counted waits] barrier [16 MFMAs: one quadrant of its 128 x 64 output, K = 64] barrier, so a
    // SIMD's MFMA pipe is fed by one group while the other reads and stages, in quarter-size
    // slices (VAR 12: 32-MFMA slots over BK = 32).  Quadrants (64-row sub sa, 32-col sub qb):
    // Q1 (0,0) reads B qb 0 + A sub 0 (12 ds_read_b128), Q2 (0,1) B qb 1 (4), Q3 (1,1) A sub 1 (8),
    // Q4 (1,0) none.  Half-tiles: A rows 0-127 / 128-255, B rows 0-127 / 128-255 of a buffer.
    // Staging slots (phase: buffer half, K-tile): 1: b1 A0 t+1, 2: b1 A1 t+1, 3: b0 B0 t+2,
    // 4: b0 B1 t+2, 5: b0 A0 t+2, 6: b0 A1 t+2, 7: b1 B0 t+3, 8: b1 B1 t+3 (t = 2 x iteration).
    // RAW: every half-tile is issued >= 3 phases before its first read, and each phase waits
    // vmcnt(4) (its last two phases' pieces may fly) before its first barrier: the reader's own
    // pieces and the other group's are then retired before a barrier it has passed.  WAR: a half
    // is restaged >= 1 phase after its last read, whose lgkmcnt(0) precedes that phase's first
    // barrier.  K-tiles past the end stage as zeros (OOB), so every phase issues its pieces and
    // the counted wait stays exact; an odd last K-tile multiplies zeros.
    // (the same schedule over fp8 operands, 8 block-scaled 16x16x128 MFMAs per quadrant, measured
    // no faster than VAR 8 and spilled: profiles/ab/r06_fp8_var20.txt)
    static_assert(AKC && BKC, "VAR 16: k-contiguous operands");
    const int wv = __builtin_amdgcn_readfirstlane(wave);
    const int grpw = wv >> 2;
    auto img = [&](int buf, int ab) -> short* { return lds + (buf * 2 + ab) * IMG; };
    // this wave's 2 pieces of half h (128 rows) of a 256 x 64 k-contiguous image.  Piece 16 h +
    // 2 wave + j holds rows 128 h + 16 wave + 8 j + lane / 8, 16-byte chunk (lane ^ lane / 8) & 7 at
    // slot lane & 7: the lane part of the source offset is computed once
    const int lrow = 16 * wv + (lane >> 3), lc8 = 8 * ((lane ^ (lane >> 3)) & 7);
    const unsigned baseA = 2u * ((unsigned)(m0 + lrow) * (unsigned)g.lda + (unsigned)lc8);
    const unsigned baseB = 2u * ((unsigned)(n0 + lrow) * (unsigned)g.ldb + (unsigned)lc8);
    auto stage_half = [&](int buf, int ab, int h, int kt) {
      const int k0 = kbeg + kt * TBK;
      const bool kok = kt < nk && lc8 < kend - k0;
      const int R = (ab ? g.N - n0 : g.M - m0) - lrow;  // rows left below this lane's row
      const unsigned ld2 = 2u * (unsigned)(ab ? g.ldb : g.lda);
      const unsigned base = (ab ? baseB : baseA) + 2u * (unsigned)k0;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int dr = 128 * h + 8 * j;
        const unsigned off = (kok && dr < R) ? base + (unsigned)dr * ld2 : OOB;
        dma16<false>(ab ? rb : ra, ab ? rwb : rwa, img(buf, ab) + (16 * h + wv * 2 + j) * 512, off);
      }
    };
    // B qb 0 of a K-tile is read in the LAST phase of the K-tile before (into the other of two
    // register sets), so the phases read 8 / 4 / 8 / 4 fragments: Q1 A sub 0, Q2 B qb 1, Q3 A sub 1,
    // Q4 the next K-tile's B qb 0 (its halves are staged >= 3 phases before, and the current
    // K-tile's B halves are last read in Q2: the staging windows above still hold)
    bf16x8 afr[4][2], b1r[2][2], b0r[2][2][2];
    auto read_a = [&](const short* As, int sa) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int kh = 0; kh < 2; ++kh) afr[i][kh] = frag<true>(As, wm * 128 + sa * 64 + i * 16, kh * 32, lane);
    };
    auto read_b = [&](const short* Bs, int qb, bf16x8 (&dst)[2][2]) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int kh = 0; kh < 2; ++kh) dst[j][kh] = frag<true>(Bs, wn * 64 + qb * 32 + j * 16, kh * 32, lane);
    };
    auto mfma_q = [&](int sa, int qb, const bf16x8 (&bq)[2][2]) {
#pragma unroll
      for (int kh = 0; kh < 2; ++kh)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[4 * sa + i][2 * qb + j] =
                __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[j][kh], afr[i][kh], acc[4 * sa + i][2 * qb + j], 0, 0, 0);
    };
    // one phase: reads (issued by the caller), the half-tile, waits, barrier, MFMAs, barrier
    auto phase_tail = [&](int buf, int ab, int h, int kt, int sa, int qb, const bf16x8 (&bq)[2][2]) {
      stage_half(buf, ab, h, kt);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
      mfma_q(sa, qb, bq);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
    };
    // prologue: K-tile 0 whole (buffer 0), K-tile 1's B halves (buffer 1); K-tile 0's B qb 0
    stage_half(0, 0, 0, 0); stage_half(0, 0, 1, 0); stage_half(0, 1, 0, 0); stage_half(0, 1, 1, 0);
    stage_half(1, 1, 0, 1); stage_half(1, 1, 1, 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (grpw == 1) __builtin_amdgcn_s_barrier();  // group 1 runs one barrier behind
    read_b(img(0, 1), 0, b0r[0]);
    const int niter = (nk + 1) / 2;
    for (int itr = 0; itr < niter; ++itr) {
      const int t = 2 * itr;
#pragma unroll
      for (int b = 0; b < 2; ++b) {  // K-tile t + b in buffer b
        const short* As = img(b, 0);
        const short* Bs = img(b, 1);
        read_a(As, 0);
        if (b == 0) phase_tail(1, 0, 0, t + 1, 0, 0, b0r[0]);   // phase 1: b1 A0 (t+1)
        else phase_tail(0, 0, 0, t + 2, 0, 0, b0r[1]);          // phase 5: b0 A0 (t+2)
        read_b(Bs, 1, b1r);
        if (b == 0) phase_tail(1, 0, 1, t + 1, 0, 1, b1r);      // phase 2: b1 A1 (t+1)
        else phase_tail(0, 0, 1, t + 2, 0, 1, b1r);             // phase 6: b0 A1 (t+2)
        read_a(As, 1);
        if (b == 0) phase_tail(0, 1, 0, t + 2, 1, 1, b1r);      // phase 3: b0 B0 (t+2)
        else phase_tail(1, 1, 0, t + 3, 1, 1, b1r);             // phase 7: b1 B0 (t+3)
        read_b(img(b ^ 1, 1), 0, b0r[b ^ 1]);                   // the next K-tile's B qb 0
        if (b == 0) phase_tail(0, 1, 1, t + 2, 1, 0, b0r[0]);   // phase 4: b0 B1 (t+2)
        else phase_tail(1, 1, 1, t + 3, 1, 0, b0r[1]);          // phase 8: b1 B1 (t+3)
      }
    }
    if (grpw == 0) __builtin_amdgcn_s_barrier();  // both groups pass the same number of barriers
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the zero-fill stages past the end land
    __syncthreads();                                   // before the epilogue reuses the LDS
  } else if constexpr (VAR == 18) {
    // VAR 18: VAR 16's eight-phase loop for m/n-contiguous A and B (the weight gradients dW =
    // dG^T X without time-shifted rows: with the three shift forms of B's staging the build spilled
    // 10-57 VGPRs, so the time-shifted dW_hh keeps VAR 0).  An image is [64 k][256 m] (512-byte k-rows), so
    // its contiguous halves are k-halves (32 k-rows = 16 pieces), and a phase multiplies one k-half
    // of one 64-row sub: P1 (kh 0, sub 0) reads A 4 + B 4 fragments, P2 (kh 0, sub 1) A 4, P3 (kh 1,
    // sub 1) A 4 + B 4, P4 (kh 1, sub 0) A 4 (16 MFMAs each; fragments by ds_read_b64_tr_b16).
    // Last reads per K-tile: B kh0 P1, A kh0 P2, B kh1 P3, A kh1 P4; first reads: kh0 P1, kh1 P3.
    // Staging slots (phase: buffer half, K-tile): 2: b0 Bk0 t+2, 3: b0 Ak0 t+2, 4: b0 Bk1 t+2,
    // 5: b0 Ak1 t+2, 6: b1 Bk0 t+3, 7: b1 Ak0 t+3, 8: b1 Bk1 t+3, 1: b1 Ak1 t+1 -- each >= 1 phase
    // after its half's last read and >= 3 phases before its first (VAR 16's waits and barriers).
    static_assert(!AKC && !BKC, "VAR 18: m/n-contiguous operands");
    const int wv = __builtin_amdgcn_readfirstlane(wave);
    const int grpw = wv >> 2;
    // [operand][buffer]: the two buffers of an operand 32 KB apart, inside a ds_read's immediate
    // offset, so one set of lane addresses serves both
    auto img = [&](int buf, int ab) -> short* { return lds + (ab * 2 + buf) * IMG; };
    // this wave's two pieces of k-half h are pieces 16 h + 2 wave + j: k-half 0's lane offsets
    // serve both (k-half 1 = 32 k-rows further: the column swizzle repeats every 16 rows)
    McLanes<2> lA, lB;
    lA.init(2 * wv, lane, g.lda, m0, g.M);
    lB.init(2 * wv, lane, g.ldb, n0, g.N);
    auto stage_half = [&](int buf, int ab, int h, int kt) {
      const int k0 = kbeg + kt * TBK + 32 * h;
      const int ke = kt < nk ? kend : k0;  // K-tiles past the end: every row out of range (zeros)
      if (ab == 0) lA.stage<0, true>(img(buf, 0) + 16 * h * 512, ra, rwa, g.lda, k0, ke, 0, 0, 2 * wv);
      else lB.stage<0, true>(img(buf, 1) + 16 * h * 512, rb, rwb, g.ldb, k0, ke, 0, 0, 2 * wv);
    };
    bf16x8 afr[4], bfr[4];
    auto read_a = [&](const short* As, int sa, int kh) {
#pragma unroll
      for (int i = 0; i < 4; ++i) afr[i] = frag<false>(As, wm * 128 + sa * 64 + i * 16, kh * 32, lane);
    };
    auto read_b = [&](const short* Bs, int kh) {
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = frag<false>(Bs, wn * 64 + j * 16, kh * 32, lane);
    };
    auto phase_tail = [&](int buf, int ab, int h, int kt, int sa) {
      stage_half(buf, ab, h, kt);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[4 * sa + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], afr[i], acc[4 * sa + i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
    };
    // prologue: K-tile 0 whole (buffer 0); K-tile 1's halves but A kh1 (slot 1 of the loop)
    stage_half(0, 0, 0, 0); stage_half(0, 0, 1, 0); stage_half(0, 1, 0, 0); stage_half(0, 1, 1, 0);
    stage_half(1, 1, 0, 1); stage_half(1, 0, 0, 1); stage_half(1, 1, 1, 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (grpw == 1) __builtin_amdgcn_s_barrier();  // group 1 runs one barrier behind
    const int niter = (nk + 1) / 2;
    for (int itr = 0; itr < niter; ++itr) {
      const int t = 2 * itr;
#pragma unroll
      for (int b = 0; b < 2; ++b) {  // K-tile t + b in buffer b
        const short* As = img(b, 0);
        const short* Bs = img(b, 1);
        read_b(Bs, 0);
        read_a(As, 0, 0);
        if (b == 0) phase_tail(1, 0, 1, t + 1, 0);   // phase 1: b1 Ak1 (t+1)
        else phase_tail(0, 0, 1, t + 2, 0);          // phase 5: b0 Ak1 (t+2)
        read_a(As, 1, 0);
        if (b == 0) phase_tail(0, 1, 0, t + 2, 1);   // phase 2: b0 Bk0 (t+2)
        else phase_tail(1, 1, 0, t + 3, 1);          // phase 6: b1 Bk0 (t+3)
        read_b(Bs, 1);
        read_a(As, 1, 1);
        if (b == 0) phase_tail(0, 0, 0, t + 2, 1);   // phase 3: b0 Ak0 (t+2)
        else phase_tail(1, 0, 0, t + 3, 1);          // phase 7: b1 Ak0 (t+3)
        read_a(As, 0, 1);
        if (b == 0) phase_tail(0, 1, 1, t + 2, 0);   // phase 4: b0 Bk1 (t+2)
        else phase_tail(1, 1, 1, t + 3, 0);          // phase 8: b1 Bk1 (t+3)
      }
    }
    if (grpw == 0) __builtin_amdgcn_s_barrier();  // both groups pass the same number of barriers
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the zero-fill stages past the end land
    __syncthreads();                                   // before the epilogue reuses the LDS
  } else if constexpr (VAR == 9) {
    static_assert(!AKC && !BKC, "VAR 9: fp8 operands stored m/n-contiguous");
    auto stage_both = [&](int buf, int k0) {
      stage8_mc(lds + (buf * 2 + 0) * IMG, ra, rwa, g.lda, m0, g.M, k0, kend, 0, 0, wave, lane);
      stage8_mc(lds + (buf * 2 + 1) * IMG, rb, rwb, g.ldb, n0, g.N, k0, kend, g.kshiftT, sh, wave, lane);
    };
    if (nk > 0) {
      stage_both(0, kbeg);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
    for (int it = 0; it < nk; ++it) {
      const int cur = it & 1;
      if (it + 1 < nk) stage_both(cur ^ 1, kbeg + (it + 1) * SBK);
      const short* As = lds + (cur * 2 + 0) * IMG;
      const short* Bs = lds + (cur * 2 + 1) * IMG;
      i32x8 af[8], bfr[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = frag8_mc(Bs, wn * 64 + j * 16, lane);
#pragma unroll
      for (int i = 0; i < 8; ++i) af[i] = frag8_mc(As, wm * 128 + i * 16, lane);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(bfr[j], af[i], acc[i][j], 0, 0, 0, 127,
                                                                       0, 127);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  } else if constexpr (VAR == 8) {
    static_assert(AKC && BKC, "fp8 operands are k-contiguous");
    auto stage_both = [&](int buf, int k0) {
      stage<true>(lds + (buf * 2 + 0) * IMG, ra, rwa, g.lda, m0, g.M, k0, kend, 0, 0, wave, lane);
      stage<true>(lds + (buf * 2 + 1) * IMG, rb, rwb, g.ldb, n0, g.N, k0, kend, 0, 0, wave, lane);
    };
    if (nk > 0) {
      stage_both(0, kbeg);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
    for (int it = 0; it < nk; ++it) {
      const int cur = it & 1;
      if (it + 1 < nk) stage_both(cur ^ 1, kbeg + (it + 1) * TBK);
      const short* As = lds + (cur * 2 + 0) * IMG;
      const short* Bs = lds + (cur * 2 + 1) * IMG;
      i32x8 af[8], bfr[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = frag8(Bs, wn * 64 + j * 16, lane);
#pragma unroll
      for (int i = 0; i < 8; ++i) af[i] = frag8(As, wm * 128 + i * 16, lane);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(bfr[j], af[i], acc[i][j], 0, 0, 0, 127,
                                                                       0, 127);
      __builtin_amdgcn_s_setprio(0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  } else {
  McLanes<4> mla, mlb;
  const int pbw = __builtin_amdgcn_readfirstlane(wave) * 4;  // this wave's first piece (wave-uniform)
  if constexpr (!AKC) mla.init(pbw, lane, g.lda, m0, g.M);
  if constexpr (!BKC) mlb.init(pbw, lane, g.ldb, n0, g.N);
  auto stage_both = [&](int buf, int k0) {
    if constexpr (AKC)
      stage<AKC, ADMA>(lds + (buf * 2 + 0) * IMG, ra, rwa, g.lda, m0, g.M, k0, kend, 0, 0, wave, lane);
    else
      mla.stage<0, ADMA>(lds + (buf * 2 + 0) * IMG, ra, rwa, g.lda, k0, kend, 0, 0, pbw);
    if constexpr (BKC)
      stage<BKC, ADMA>(lds + (buf * 2 + 1) * IMG, rb, rwb, g.ldb, n0, g.N, k0, kend, g.kshiftT, sh, wave, lane);
    else
      mlb.stage_any<ADMA>(lds + (buf * 2 + 1) * IMG, rb, rwb, g.ldb, k0, kend, g.kshiftT, sh, pbw, TBK);
  };
  if (nk > 0) {
    stage_both(0, kbeg);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  for (int it = 0; it < nk; ++it) {
    const int cur = it & 1;
    if (it + 1 < nk && !(VAR == 6 && (g.abl & 2))) stage_both(cur ^ 1, kbeg + (it + 1) * TBK);
    const short* As = lds + (cur * 2 + 0) * IMG;
    const short* Bs = lds + (cur * 2 + 1) * IMG;
#pragma unroll
    for (int kk = 0; kk < TBK; kk += 32) {
      bf16x8 af[8], bfr[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = frag<BKC>(Bs, wn * 64 + j * 16, kk, lane);
#pragma unroll
      for (int i = 0; i < 8; ++i) af[i] = frag<AKC>(As, wm * 128 + i * 16, kk, lane);
      if (VAR == 6 && (g.abl & 1)) {  // ablation build (VAR 6): fragments read, no MFMA
#pragma unroll
        for (int i = 0; i < 8; ++i) asm volatile("" ::"v"(af[i]));
#pragma unroll
        for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(bfr[j]));
        continue;
      }
      // operands swapped (D = B^T A^T): a lane's 4 results are 4 consecutive columns of one
      // row, so the epilogue stores 16 B per lane (s_setprio(1) around these MFMAs measured
      // 7-8 % slower on the weight gradients: profiles/r02_gemm_wgrad_var_ab.txt)
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // tile it+1 has landed (this wave's pieces)
    __syncthreads();                                 // ... everyone's; buffer cur is free
  }
  }

  if (g.abl & 8) return;  // timing ablation: no epilogue at all
  if (g.alpha) {  // fp8 operand scales
    const float al = *g.alpha;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] *= al;
  }
  // epilogue: lane holds C[m0 + wm*128 + i*16 + (lane&15)][n0 + wn*64 + j*16 + 4*(lane>>4) + r]
  const bool split = g.splits > 1;
  const unsigned long long dkey = drop_key(g.dseed);
  float* Cb = g.c16 ? reinterpret_cast<float*>(reinterpret_cast<unsigned short*>(g.C) + bz * g.c_bs)
                    : g.C + bz * g.c_bs;
  float* wsz = split ? g.ws + ((size_t)bz * g.splits + kz) * (size_t)g.M * g.N : nullptr;
  const bool vec = (g.ldc % 4) == 0 && (((uintptr_t)Cb) % 16) == 0;
  // Row-contiguous epilogue through the (now free) LDS: four passes of 64 tile rows; every
  // store instruction then writes one whole 1 KB row segment instead of 16 rows x 64 B
  // (fp32 output, no beta; split partial slabs too).  c2 skinny projection: 88 -> 56 us.
  const bool bias_vec = ((uintptr_t)g.bias1 % 16) == 0 && ((uintptr_t)g.bias2 % 16) == 0;
  if ((g.N % 4) == 0 && g.beta == 0.f && !(g.abl & 4) &&  // (ablation bit 4: the direct stores)
      (split || (vec && bias_vec && (g.epi == EPI_NONE || g.epi == EPI_DROPOUT || g.epi == EPI_LRELU)))) {
    constexpr int LSR = TBN + 4;  // staged row stride (floats)
    float* st = reinterpret_cast<float*>(smem);  // [64][LSR] = 66.5 KB of the 128 KB
    float* dst = split ? wsz : Cb;
    const int ldd = split ? g.N : g.ldc;
    // the bias columns of this thread, loaded before the first store: a load issued behind the
    // stores would wait for them (vmcnt counts in issue order)
    const int c4 = tid & 63, col = n0 + 4 * c4;
    // 16-bit C: a lane stores 8 columns (16 B) -- half the store instructions of 4-column lanes
    // (the tile's store burst is issue-bound: cdna_hip_programming.md T21)
    const bool w8 = !split && g.c16 && (g.N % 8) == 0 && (g.ldc % 8) == 0 && ((uintptr_t)Cb % 16) == 0 &&
                    !(g.abl & 64);
    const int c8 = tid & 31, col8 = n0 + 8 * c8;
    f32x4 b = {0.f, 0.f, 0.f, 0.f}, b2 = {0.f, 0.f, 0.f, 0.f};
    if (w8) {
      if (col8 < g.N) {
        if (g.bias1) {
          b += *reinterpret_cast<const f32x4*>(g.bias1 + col8);
          b2 += *reinterpret_cast<const f32x4*>(g.bias1 + col8 + 4);
        }
        if (g.bias2) {
          b += *reinterpret_cast<const f32x4*>(g.bias2 + col8);
          b2 += *reinterpret_cast<const f32x4*>(g.bias2 + col8 + 4);
        }
      }
    } else if (!split && col < g.N) {
      if (g.bias1) b += *reinterpret_cast<const f32x4*>(g.bias1 + col);
      if (g.bias2) b += *reinterpret_cast<const f32x4*>(g.bias2 + col);
    }
#pragma unroll
    for (int pass = 0; pass < 4; ++pass) {
#pragma unroll
      for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int lr = wm * 32 + ii * 16 + (lane & 15);
          *reinterpret_cast<f32x4*>(st + lr * LSR + wn * 64 + j * 16 + 4 * (lane >> 4)) =
              acc[2 * pass + ii][j];
        }
      lds_barrier();
      if (w8) {
#pragma unroll 2
        for (int q = 0; q < 4; ++q) {
          const int lr = q * 16 + (tid >> 5);  // 16 staged rows per round, 32 lanes per row
          const int row = m0 + (lr >> 5) * 128 + (2 * pass + ((lr >> 4) & 1)) * 16 + (lr & 15);
          if (row >= g.M || col8 >= g.N) continue;
          f32x4 v = *reinterpret_cast<const f32x4*>(st + lr * LSR + 8 * c8) + b;
          f32x4 v2 = *reinterpret_cast<const f32x4*>(st + lr * LSR + 8 * c8 + 4) + b2;
          if (g.epi == EPI_DROPOUT) {
            const unsigned long long rq = drop_quad(dkey, (g.doff + (size_t)row * g.ldc + col8) >> 2);
            const unsigned long long rq2 = drop_quad(dkey, ((g.doff + (size_t)row * g.ldc + col8) >> 2) + 1);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              v[r] *= drop_elem_scale(rq, r, g.dkeep, g.dscale);
              v2[r] *= drop_elem_scale(rq2, r, g.dkeep, g.dscale);
            }
          }
          if (g.epi == EPI_LRELU) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              v[r] = lrelu(v[r]);
              v2[r] = lrelu(v2[r]);
            }
          }
          u32x2 lo, hi;
          if (g.c16 == 2) {
            lo = u32x2{(unsigned)(unsigned short)f2bf(v[0]) | ((unsigned)(unsigned short)f2bf(v[1]) << 16),
                       (unsigned)(unsigned short)f2bf(v[2]) | ((unsigned)(unsigned short)f2bf(v[3]) << 16)};
            hi = u32x2{(unsigned)(unsigned short)f2bf(v2[0]) | ((unsigned)(unsigned short)f2bf(v2[1]) << 16),
                       (unsigned)(unsigned short)f2bf(v2[2]) | ((unsigned)(unsigned short)f2bf(v2[3]) << 16)};
          } else {
            lo = f2h4(v);
            hi = f2h4(v2);
          }
          *reinterpret_cast<u32x4*>(reinterpret_cast<unsigned short*>(Cb) + (size_t)row * g.ldc + col8) =
              u32x4{lo[0], lo[1], hi[0], hi[1]};
        }
        lds_barrier();
        continue;
      }
#pragma unroll 2  // (fully unrolled, the four passes outgrew the unroller: acc went to scratch)
      for (int q = 0; q < 8; ++q) {
        const int lr = q * 8 + (tid >> 6);  // wave w stores staged rows w, w + 8, ...
        const int row = m0 + (lr >> 5) * 128 + (2 * pass + ((lr >> 4) & 1)) * 16 + (lr & 15);
        if (row >= g.M || col >= g.N) continue;
        f32x4 v = *reinterpret_cast<const f32x4*>(st + lr * LSR + 4 * c4) + b;
        if (!split && g.epi == EPI_DROPOUT) {  // one mask quad per 4 aligned columns
          const unsigned long long rq = drop_quad(dkey, (g.doff + (size_t)row * g.ldc + col) >> 2);
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] *= drop_elem_scale(rq, r, g.dkeep, g.dscale);
        }
        if (!split && g.epi == EPI_LRELU) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = lrelu(v[r]);
        }
        if (!split && g.c16 == 2)
          *reinterpret_cast<u32x2*>(reinterpret_cast<unsigned short*>(Cb) + (size_t)row * ldd + col) =
              u32x2{(unsigned)(unsigned short)f2bf(v[0]) | ((unsigned)(unsigned short)f2bf(v[1]) << 16),
                    (unsigned)(unsigned short)f2bf(v[2]) | ((unsigned)(unsigned short)f2bf(v[3]) << 16)};
        else if (!split && g.c16)
          *reinterpret_cast<u32x2*>(reinterpret_cast<unsigned short*>(Cb) + (size_t)row * ldd + col) = f2h4(v);
        else
          *reinterpret_cast<f32x4*>(dst + (size_t)row * ldd + col) = v;
      }
      lds_barrier();  // the staging rows are rewritten by the next pass
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = n0 + wn * 64 + j * 16 + 4 * (lane >> 4);
    if (col >= g.N) continue;
    f32x4 b = {0.f, 0.f, 0.f, 0.f};
    if (!split) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (col + r < g.N) {
          if (g.bias1) b[r] += g.bias1[col + r];
          if (g.bias2) b[r] += g.bias2[col + r];
        }
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = m0 + wm * 128 + i * 16 + (lane & 15);
      if (row >= g.M) continue;
      if (split) {  // N % 4 == 0 whenever split (checked on the host)
        *reinterpret_cast<f32x4*>(wsz + (size_t)row * g.N + col) = acc[i][j];
        continue;
      }
      if (g.c16) {  // (reached with ablation bit 4 only: 16-bit C always takes the staged path)
        f32x4 v = acc[i][j] + b;
        if (g.epi == EPI_DROPOUT) {
          const unsigned long long rq = drop_quad(dkey, (g.doff + (size_t)row * g.ldc + col) >> 2);
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] *= drop_elem_scale(rq, r, g.dkeep, g.dscale);
        }
        if (g.epi == EPI_LRELU) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = lrelu(v[r]);
        }
        unsigned short* cp16 = reinterpret_cast<unsigned short*>(Cb) + (size_t)row * g.ldc + col;
        if (g.c16 == 2)
          *reinterpret_cast<u32x2*>(cp16) =
              u32x2{(unsigned)(unsigned short)f2bf(v[0]) | ((unsigned)(unsigned short)f2bf(v[1]) << 16),
                    (unsigned)(unsigned short)f2bf(v[2]) | ((unsigned)(unsigned short)f2bf(v[3]) << 16)};
        else
          *reinterpret_cast<u32x2*>(cp16) = f2h4(v);
        continue;
      }
      float* cp = Cb + (size_t)row * g.ldc + col;
      if (vec && col + 3 < g.N && g.beta == 0.f && g.epi == EPI_NONE) {
        *reinterpret_cast<f32x4*>(cp) = acc[i][j] + b;
      } else if (vec && col + 3 < g.N && g.beta == 0.f && g.epi == EPI_DROPOUT) {
        // the 4 columns are one aligned mask quad (row*ldc + col is a multiple of 4): one
        // hash gives all four, as dropout_scale() does element by element
        const unsigned long long rq = drop_quad(dkey, (g.doff + (size_t)row * g.ldc + col) >> 2);
        f32x4 v = acc[i][j] + b;
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] *= drop_elem_scale(rq, r, g.dkeep, g.dscale);
        *reinterpret_cast<f32x4*>(cp) = v;
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (col + r < g.N) cp[r] = epi_apply(g, acc[i][j][r] + b[r], row, col + r, cp + r);
      }
    }
  }
}


__global__ __launch_bounds__(256) void splitk_reduce_fast(GFArgs g) {
  const size_t MN = (size_t)g.M * g.N;
  const int bz = blockIdx.y;
  const float* ws = g.ws + (size_t)bz * g.splits * MN;
  float* Cb = g.c16 ? reinterpret_cast<float*>(reinterpret_cast<unsigned short*>(g.C) + bz * g.c_bs)
                    : g.C + bz * g.c_bs;
  for (size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x; idx < MN; idx += (size_t)gridDim.x * 256) {
    float s = 0.f;
#pragma unroll 8  // loads in flight; the adds keep their order
    for (int z = 0; z < g.splits; ++z) s += ws[z * MN + idx];
    const int row = (int)(idx / g.N), col = (int)(idx % g.N);
    if (g.bias1) s += g.bias1[col];
    if (g.bias2) s += g.bias2[col];
    if (g.c16) {  // beta == 0, epi NONE / DROPOUT (fp16) or NONE / LRELU / DROPOUT (bf16) (checked on the host)
      if (g.epi == EPI_DROPOUT) s *= dropout_scale(g.dseed, g.doff + (size_t)row * g.ldc + col, g.dkeep, g.dscale);
      if (g.epi == EPI_LRELU) s = lrelu(s);
      reinterpret_cast<unsigned short*>(Cb)[(size_t)row * g.ldc + col] =
          g.c16 == 2 ? (unsigned short)f2bf(s) : f2h(s);
      continue;
    }
    float* cp = Cb + (size_t)row * g.ldc + col;
    *cp = epi_apply(g, s, row, col, cp);
  }
}

template <bool AKC, bool BKC, int VAR>
int launch_fast_v(const GFArgs& g, dim3 grid, hipStream_t s) {
  auto k = gemm256_kernel<AKC, BKC, VAR>;
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)FAST_LDS) != hipSuccess) {
      mlvae_set_error("gemm_bf16: cannot reserve %zu B LDS", FAST_LDS);
      return 2;
    }
    attr = true;
  }
  k<<<grid, 512, FAST_LDS, s>>>(g);
  return 0;
}

int gemm_cus() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        n <= 0)
      n = 256;
  }
  return n;
}

template <bool AKC, bool BKC>
int launch_fast(const GFArgs& g, dim3 grid, hipStream_t s, int var) {
  switch (var) {
    case 4:
      if constexpr (AKC && BKC) return launch_fast_v<true, true, 4>(g, grid, s);
      return launch_fast_v<AKC, BKC, 0>(g, grid, s);
    case 5: return launch_fast_v<AKC, BKC, 0>(g, grid, s);  // the previous default (A/B)
    case 6: return launch_fast_v<AKC, BKC, 6>(g, grid, s);  // VAR 0 with the MLVAE_GEMM_ABL switches
    case 12: return launch_fast_v<AKC, BKC, 12>(g, grid, s);
    case 18:  // the same for m/n-contiguous A and B (weight gradients without time-shifted rows)
      if constexpr (!AKC && !BKC)
        if (g.kshift == 0 && g.kshift_bstep == 0) return launch_fast_v<false, false, 18>(g, grid, s);
      if constexpr (AKC && BKC) return launch_fast_v<true, true, 16>(g, grid, s);
      if constexpr (AKC) return launch_fast_v<true, BKC, 12>(g, grid, s);
      return launch_fast_v<AKC, BKC, 0>(g, grid, s);
    case 16:  // eight phases over two 64-deep K-tiles (k-contiguous A and B; else the default)
      if constexpr (AKC && BKC) return launch_fast_v<true, true, 16>(g, grid, s);
      if constexpr (AKC) return launch_fast_v<true, BKC, 12>(g, grid, s);
      return launch_fast_v<AKC, BKC, 0>(g, grid, s);
    case 13:  // VAR 12 with the timing ablations (k-contiguous operands only)
      if constexpr (AKC && BKC) return launch_fast_v<true, true, 13>(g, grid, s);
      return 1;
    case 8:
      if constexpr (AKC && BKC) return launch_fast_v<true, true, 8>(g, grid, s);
      return 1;
    default:
      // k-contiguous A and B (projection, dgrad against W^T, the heads' products): the eight-phase
      // loop (round 6, profiles/ab/r06_gemm_var16.txt: same process, c3 shapes, projection
      // 1,305 -> 1,271 us, dgrad (W^T) 1,139 -> 1,082, 4096^3 1,185 -> 1,280 TF/s; in the c3 step
      // projection 1.06 -> 1.01 ms, dgrad 0.96 -> 0.865, step 9.78 -> 9.60 ms).  k-contiguous A with
      // m/n-contiguous B: the ping-pong ring (against VAR 4: projection 1.328 -> 1.287 ms, dgrad
      // 1.134 -> 1.098 (W^T) / 1.361 -> 1.252 (W)); m-contiguous A (weight gradients): VAR 0
      // m/n-contiguous A and B without time-shifted rows (dW_ih, the heads' dW1): VAR 18 (c3, in
      // the step: dW_ih_l1 0.936 -> 0.82 ms, profiles/ab/r06_gemm_var18.txt); time-shifted (dW_hh):
      // VAR 0
      if constexpr (AKC && BKC) return launch_fast_v<true, true, 16>(g, grid, s);
      if constexpr (AKC) return launch_fast_v<true, BKC, 12>(g, grid, s);
      if constexpr (!AKC && !BKC)
        if (g.kshift == 0 && g.kshift_bstep == 0) return launch_fast_v<false, false, 18>(g, grid, s);
      return launch_fast_v<AKC, BKC, 0>(g, grid, s);
  }
}

// split-K: long-K products (weight gradients over B*T frames) with fewer tiles than half the
// CUs, until ~1 workgroup per CU, keeping >= 8 K-steps per split (at >= 128 tiles the extra
// partial-slab round trip costs more than the idle CUs: dgrad 252 tiles, 224 vs 196 us)
// split-K workgroup target (~256 = one per CU).  mlvae_gemm_bf16_set_split_target() lowers it
// for weight gradients that overlap a recurrence: fewer workgroups leave CUs and memory
// bandwidth to the latency-bound hand-off chain (c2: 256 -> 128 takes 0.15 ms off the step).
int g_split_target = 256;
int split_target() { return g_split_target; }

// main-loop variant (gemm256_kernel VAR; 0 = the default per operand layout): MLVAE_GEMM_VAR or
// mlvae_gemm_bf16_set_variant() select another for same-process A/B timing
int g_variant = -1;
int gemm_variant() {
  if (g_variant < 0) {
    const char* e = getenv("MLVAE_GEMM_VAR");
    g_variant = e ? atoi(e) : 0;
  }
  return g_variant;
}

void fast_plan(int M, int N, int K, int batch, int* splits, int* kchunk) {
  const long tiles = (long)((M + TBM - 1) / TBM) * ((N + TBN - 1) / TBN) * batch;
  int s = 1;
  if (tiles < 128 && K >= TBK * 16) {
    s = (int)((split_target() + tiles - 1) / tiles);
    const int maxs = K / (TBK * 8);
    if (s > maxs) s = maxs;
    if (s > 32) s = 32;
    if (s < 1) s = 1;
  }
  int kc = (K + s - 1) / s;
  kc = (kc + TBK - 1) / TBK * TBK;
  s = kc > 0 ? (K + kc - 1) / kc : 1;
  *splits = s < 1 ? 1 : s;
  *kchunk = kc > 0 ? kc : TBK;
}

}  // namespace

extern "C" int mlvae_gemm_bf16_set_split_target(int workgroups) {
  const int prev = g_split_target;
  if (workgroups >= 1) g_split_target = workgroups;
  return prev;
}

extern "C" int mlvae_gemm_bf16_set_variant(int var) {
  const int prev = gemm_variant();
  if (var >= 0) g_variant = var;
  return prev;
}

extern "C" size_t mlvae_gemm_bf16_workspace_size(int M, int N, int K, int batch) {
  int s, kc;
  fast_plan(M, N, K, batch < 1 ? 1 : batch, &s, &kc);
  return s > 1 ? (size_t)s * M * N * (batch < 1 ? 1 : batch) * sizeof(float) : 0;
}

extern "C" int mlvae_gemm_bf16(int trans_a, int trans_b, int M, int N, int K, int batch,
                               const void* A, int lda, long long a_bstride, const void* B, int ldb,
                               long long b_bstride, float* C, int ldc, long long c_bstride,
                               float beta, const float* bias1, const float* bias2, int epi,
                               const float* aux, int ldaux, int kshift_T, int kshift,
                               int kshift_bstep, unsigned long long drop_seed,
                               unsigned long long drop_offset, float drop_p,
                               float* ws, size_t ws_bytes, void* stream) {
  if (M < 0 || N < 0 || K < 0 || batch < 1 || !C || (K > 0 && (!A || !B))) {
    mlvae_set_error("mlvae_gemm_bf16: bad shape/ptr");
    return 1;
  }
  if (M == 0 || N == 0) return 0;
  const int c16 = (epi & EPI_OUT_BF16) ? 2 : ((epi & EPI_OUT_F16) ? 1 : 0);
  epi &= ~(EPI_OUT_F16 | EPI_OUT_BF16);
  if (c16 && (beta != 0.f || (c16 == 1 && epi != EPI_NONE && epi != EPI_DROPOUT) ||
              (c16 == 2 && epi != EPI_NONE && epi != EPI_LRELU && epi != EPI_DROPOUT) || N % 4 || ldc % 4 ||
              ((uintptr_t)C % 16) || (c_bstride % 8) || ((uintptr_t)bias1 % 16) || ((uintptr_t)bias2 % 16))) {
    mlvae_set_error("mlvae_gemm_bf16: 16-bit C needs beta 0, epilogue none/dropout (fp16) or none/lrelu/dropout (bf16), "
                    "N and ldc %% 4, aligned C/bias");
    return 1;
  }
  if (epi < EPI_NONE || epi > EPI_DROPOUT) { mlvae_set_error("mlvae_gemm_bf16: bad epilogue %d", epi); return 1; }
  if (epi == EPI_DLRELU && !aux) { mlvae_set_error("mlvae_gemm_bf16: DLRELU needs aux"); return 1; }
  if (epi == EPI_DROPOUT && !(drop_p >= 0.f && drop_p < 1.f)) {
    mlvae_set_error("mlvae_gemm_bf16: dropout p=%f out of range", drop_p);
    return 1;
  }
  if ((kshift != 0 || kshift_bstep != 0) && (trans_b || kshift_T <= 0)) {
    mlvae_set_error("mlvae_gemm_bf16: kshift needs trans_b = 0, T > 0");
    return 1;
  }
  // 16-byte chunks along the contiguous dimension: aligned bases, ld and extent multiples of 8
  const bool akc = !trans_a, bkc = trans_b;
  const int acont = akc ? K : M, bcont = bkc ? K : N;
  if (((uintptr_t)A % 16) || ((uintptr_t)B % 16) || (lda % 8) || (ldb % 8) || (acont % 8) ||
      (bcont % 8) || (a_bstride % 8) || (b_bstride % 8)) {
    mlvae_set_error("mlvae_gemm_bf16: operands need 16-byte chunks (ld, contiguous extent %% 8)");
    return 1;
  }
  // every in-range byte offset must stay below the descriptor's 2^31 range (each batch entry has
  // its own descriptor at A + z a_bstride, so the strides -- negative ones too -- do not count)
  const size_t a_rows = akc ? (size_t)M : (size_t)K, b_rows = bkc ? (size_t)N : (size_t)K;
  if (a_rows * lda * 2 >= OOB || b_rows * ldb * 2 >= OOB) {
    mlvae_set_error("mlvae_gemm_bf16: operand larger than 2 GB");
    return 1;
  }
  GFArgs g;
  g.M = M; g.N = N; g.K = K;
  g.A = static_cast<const short*>(A); g.lda = lda; g.a_bs = a_bstride;
  g.B = static_cast<const short*>(B); g.ldb = ldb; g.b_bs = b_bstride;
  g.C = C; g.ldc = ldc; g.c_bs = c_bstride; g.beta = beta;
  g.bias1 = bias1; g.bias2 = bias2; g.epi = epi; g.aux = aux; g.ldaux = ldaux;
  g.kshiftT = kshift_T; g.kshift = kshift; g.kshift_bstep = kshift_bstep;
  g.dseed = drop_seed; g.doff = drop_offset; g.dkeep = 1.f - drop_p; g.dscale = 1.f / (1.f - drop_p);
  g.ws = ws;
  g.alpha = nullptr;
  static const int abl = [] {
    const char* e = getenv("MLVAE_GEMM_ABL");
    return e ? atoi(e) : 0;
  }();
  g.abl = abl;
  int s, kc;
  fast_plan(M, N, K, batch, &s, &kc);
  if (s > 1 && (N % 4 != 0 || !ws || ws_bytes < (size_t)s * M * N * batch * sizeof(float))) {
    s = 1;
    kc = ((K + TBK - 1) / TBK) * TBK;
  }
  if (K == 0) { s = 1; kc = TBK; }
  g.splits = s; g.kchunk = kc;
  // tile order: groups of 8 M-panels walked column-major (projection at c2: plain row-major
  // runs 189 -> 173 us with groups of 4; groups of 8 at c3, same box, alternating: projection
  // 1.098 -> 1.069 ms per launch, profiles/ab/r04_gemm_group.txt);
  // MLVAE_GEMM_GROUP_M overrides (0/1 = plain row-major runs)
  static const int group_m = [] {
    const char* e = getenv("MLVAE_GEMM_GROUP_M");
    return e ? atoi(e) : 8;
  }();
  g.group_m = group_m;
  g.c16 = c16;
  hipStream_t st = (hipStream_t)stream;
  dim3 grid(((N + TBN - 1) / TBN) * ((M + TBM - 1) / TBM), batch, s);
  int rc;
  // main-loop variant (gemm256_kernel VAR): MLVAE_GEMM_VAR / set_variant override (A/B timing).
  // Measured and dropped: a BK-32 four-buffer loop without ping-pong (proj 1359 vs 1324 us, wgrad
  // 1469 vs 1236), the same with register-double-buffered fragments (proj 1.38 vs 1.31 ms), the
  // staging pieces spread one per 8 MFMAs (+-1 %)
  const int var = gemm_variant();
  if (akc && bkc) rc = launch_fast<true, true>(g, grid, st, var);
  else if (akc) rc = launch_fast<true, false>(g, grid, st, var);
  else if (bkc) rc = launch_fast<false, true>(g, grid, st, var);
  else rc = launch_fast<false, false>(g, grid, st, var);
  if (rc) return rc;
  MLVAE_CHECK_LAUNCH();
  if (s > 1) {
    const size_t MN = (size_t)M * N;
    int blocks = (int)((MN + 255) / 256);
    if (blocks > 2048) blocks = 2048;
    splitk_reduce_fast<<<dim3(blocks, batch), 256, 0, st>>>(g);
    MLVAE_CHECK_LAUNCH();
  }
  return 0;
}

// C[M,N] (fp32) = (*alpha) * A^T B over fp8 e4m3 (OCP) operands stored [K][M] and [K][N] (m- and
// n-contiguous: the weight gradient dW = dG^T X over K frames), deterministic split-K through the
// workspace (mlvae_gemm_fp8_tn_workspace_size).  gemm256_kernel VAR 9.
static void fp8_tn_plan(int M, int N, int K, int batch, int* splits, int* kchunk) {
  const long tiles = (long)((M + TBM - 1) / TBM) * ((N + TBN - 1) / TBN) * batch;
  int s = 1;
  if (tiles < 128 && K >= 128 * 16) {
    s = (int)((split_target() + tiles - 1) / tiles);
    const int maxs = K / (128 * 8);
    if (s > maxs) s = maxs;
    if (s > 32) s = 32;
    if (s < 1) s = 1;
  }
  int kc = (K + s - 1) / s;
  kc = (kc + 127) / 128 * 128;
  if (kc < 128) kc = 128;
  *splits = (K + kc - 1) / kc < 1 ? 1 : (K + kc - 1) / kc;
  *kchunk = kc;
}

extern "C" size_t mlvae_gemm_fp8_tn_ex_workspace_size(int M, int N, int K, int batch) {
  if (M <= 0 || N <= 0 || K <= 0 || batch < 1) return 0;
  int s, kc;
  fp8_tn_plan(M, N, K, batch, &s, &kc);
  return s > 1 ? (size_t)s * M * N * batch * sizeof(float) : 0;
}

extern "C" size_t mlvae_gemm_fp8_tn_workspace_size(int M, int N, int K) {
  return mlvae_gemm_fp8_tn_ex_workspace_size(M, N, K, 1);
}

// batched, with time-shifted B rows: C_z = (*alpha) A_z^T B_z~ (z < batch; A_z = A + z a_bstride,
// B_z = B + z b_bstride bytes, C_z = C + z c_bstride floats) where B_z~ row k is B_z row k + sh_z,
// sh_z = kshift + z kshift_bstep, for 0 <= k % kshift_T + sh_z < kshift_T, else zeros -- the
// recurrent weight gradient dW_hh of both directions, sum_t dG_t^T h_{t -/+ 1}, on e4m3 operands
// (as mlvae_gemm_bf16's kshift arguments)
extern "C" int mlvae_gemm_fp8_tn_ex(int M, int N, int K, int batch, const void* A, int lda, long long a_bstride,
                                    const void* B, int ldb, long long b_bstride, float* C, int ldc,
                                    long long c_bstride, const float* alpha, int kshift_T, int kshift,
                                    int kshift_bstep, float* ws, size_t ws_bytes, void* stream) {
  if (M < 0 || N < 0 || K < 0 || batch < 1 || !C || !alpha || (K > 0 && (!A || !B))) {
    mlvae_set_error("mlvae_gemm_fp8_tn: bad shape/ptr");
    return 1;
  }
  if (M == 0 || N == 0) return 0;
  if (((uintptr_t)A % 16) || ((uintptr_t)B % 16) || (lda % 16) || (ldb % 16) || (M % 16) || (N % 16) ||
      lda < M || ldb < N || N % 4 || ldc % 4 || ((uintptr_t)C % 16) || ldc < N || (a_bstride % 16) ||
      (b_bstride % 16) || (c_bstride % 4) || a_bstride < 0 || b_bstride < 0 || c_bstride < 0) {
    mlvae_set_error("mlvae_gemm_fp8_tn: M, N, lda, ldb %% 16, aligned operands and batch strides, ldc %% 4, aligned C");
    return 1;
  }
  const bool shifted = kshift != 0 || kshift_bstep != 0;
  const int shmax = std::max(std::abs(kshift), std::abs(kshift + (batch - 1) * kshift_bstep));
  if (shifted && (kshift_T <= 0 || K % kshift_T || shmax >= kshift_T)) {
    mlvae_set_error("mlvae_gemm_fp8_tn: time-shifted rows need K %% kshift_T == 0 and |shift| < kshift_T");
    return 1;
  }
  if ((size_t)K * lda + (size_t)(batch - 1) * a_bstride >= OOB ||
      (size_t)K * ldb + (size_t)(batch - 1) * b_bstride >= OOB) {
    mlvae_set_error("mlvae_gemm_fp8_tn: operand larger than 2 GB");
    return 1;
  }
  int s, kc;
  fp8_tn_plan(M, N, K, batch, &s, &kc);
  if (s > 1 && (!ws || ws_bytes < (size_t)s * M * N * batch * sizeof(float))) {
    mlvae_set_error("mlvae_gemm_fp8_tn: workspace too small (%zu B)", ws_bytes);
    return 1;
  }
  GFArgs g;
  g.M = M; g.N = N; g.K = K;
  // byte units (VAR 9); the batch strides in the kernel's 2-byte pointer units
  g.A = static_cast<const short*>(A); g.lda = lda; g.a_bs = a_bstride / 2;
  g.B = static_cast<const short*>(B); g.ldb = ldb; g.b_bs = b_bstride / 2;
  g.C = C; g.ldc = ldc; g.c_bs = c_bstride; g.beta = 0.f;
  g.bias1 = nullptr; g.bias2 = nullptr; g.epi = EPI_NONE; g.aux = nullptr; g.ldaux = 0;
  g.kshiftT = shifted ? kshift_T : 0; g.kshift = kshift; g.kshift_bstep = kshift_bstep;
  g.dseed = 0; g.doff = 0; g.dkeep = 1.f; g.dscale = 1.f;
  g.ws = ws; g.alpha = alpha; g.abl = 0;
  g.splits = s; g.kchunk = kc;
  g.group_m = 1;
  g.c16 = 0;
  hipStream_t st = (hipStream_t)stream;
  dim3 grid(((N + TBN - 1) / TBN) * ((M + TBM - 1) / TBM), batch, s);
  const int rc = launch_fast_v<false, false, 9>(g, grid, st);
  if (rc) return rc;
  MLVAE_CHECK_LAUNCH();
  if (s > 1) {
    const size_t MN = (size_t)M * N;
    int blocks = (int)((MN + 255) / 256);
    if (blocks > 2048) blocks = 2048;
    splitk_reduce_fast<<<dim3(blocks, batch), 256, 0, st>>>(g);
    MLVAE_CHECK_LAUNCH();
  }
  return 0;
}

extern "C" int mlvae_gemm_fp8_tn(int M, int N, int K, const void* A, int lda, const void* B, int ldb, float* C,
                                 int ldc, const float* alpha, float* ws, size_t ws_bytes, void* stream) {
  return mlvae_gemm_fp8_tn_ex(M, N, K, 1, A, lda, 0, B, ldb, 0, C, ldc, 0, alpha, 0, 0, 0, ws, ws_bytes, stream);
}

// C[M,N] (fp32, or fp16 with EPI_OUT_F16) = (*alpha) * A . B^T + bias1 + bias2 over fp8 e4m3 (OCP)
// operands A [M][K], B [N][K] (k-contiguous, leading dims in elements).  gemm256_kernel VAR 8.
extern "C" int mlvae_gemm_fp8_ex(int M, int N, int K, const void* A, int lda, const void* B, int ldb, void* C,
                                 int ldc, const float* alpha, const float* bias1, const float* bias2, int epi,
                                 unsigned long long drop_seed, unsigned long long drop_offset, float drop_p,
                                 void* stream);

extern "C" int mlvae_gemm_fp8(int M, int N, int K, const void* A, int lda, const void* B, int ldb, void* C, int ldc,
                              const float* alpha, const float* bias1, const float* bias2, int epi, void* stream) {
  return mlvae_gemm_fp8_ex(M, N, K, A, lda, B, ldb, C, ldc, alpha, bias1, bias2, epi, 0ull, 0ull, 0.f, stream);
}

// epi: EPI_NONE or EPI_DROPOUT (the inter-layer dropout's backward: C *= mask of element
// drop_offset + row * ldc + col, the Philox mask of the forward), optionally | EPI_OUT_F16 (with
// NONE) or | EPI_OUT_BF16
extern "C" int mlvae_gemm_fp8_ex(int M, int N, int K, const void* A, int lda, const void* B, int ldb, void* C,
                                 int ldc, const float* alpha, const float* bias1, const float* bias2, int epi,
                                 unsigned long long drop_seed, unsigned long long drop_offset, float drop_p,
                                 void* stream) {
  if (M < 0 || N < 0 || K < 0 || !C || (K > 0 && (!A || !B))) {
    mlvae_set_error("mlvae_gemm_fp8: bad shape/ptr");
    return 1;
  }
  if (M == 0 || N == 0) return 0;
  const int c16 = (epi & EPI_OUT_BF16) ? 2 : ((epi & EPI_OUT_F16) ? 1 : 0);
  epi &= ~(EPI_OUT_F16 | EPI_OUT_BF16);
  if ((epi != EPI_NONE && epi != EPI_DROPOUT) || N % 4 || ldc % 4 || ((uintptr_t)C % 16) ||
      ((uintptr_t)bias1 % 16) || ((uintptr_t)bias2 % 16) ||
      (epi == EPI_DROPOUT && (c16 == 1 || !(drop_p >= 0.f && drop_p < 1.f)))) {
    mlvae_set_error("mlvae_gemm_fp8: epilogue none (+ fp16 / bf16 C) or dropout (fp32 / bf16 C), N and ldc %% 4, "
                    "aligned C / bias");
    return 1;
  }
  if (((uintptr_t)A % 16) || ((uintptr_t)B % 16) || (lda % 16) || (ldb % 16) || (K % 16)) {
    mlvae_set_error("mlvae_gemm_fp8: operands need 16-byte chunks (K, lda, ldb %% 16, aligned)");
    return 1;
  }
  if ((size_t)M * lda >= OOB || (size_t)N * ldb >= OOB) {
    mlvae_set_error("mlvae_gemm_fp8: operand larger than 2 GB");
    return 1;
  }
  // the staging works in 2-byte units: an fp8 row of K elements is K / 2 "shorts"
  GFArgs g;
  g.M = M; g.N = N; g.K = K / 2;
  g.A = static_cast<const short*>(A); g.lda = lda / 2; g.a_bs = 0;
  g.B = static_cast<const short*>(B); g.ldb = ldb / 2; g.b_bs = 0;
  g.C = static_cast<float*>(C); g.ldc = ldc; g.c_bs = 0; g.beta = 0.f;
  g.bias1 = bias1; g.bias2 = bias2; g.epi = epi; g.aux = nullptr; g.ldaux = 0;
  g.kshiftT = 0; g.kshift = 0; g.kshift_bstep = 0;
  g.dseed = drop_seed; g.doff = drop_offset; g.dkeep = 1.f - drop_p;
  g.dscale = drop_p < 1.f ? 1.f / (1.f - drop_p) : 0.f;
  g.ws = nullptr; g.alpha = alpha; g.abl = 0;
  g.splits = 1; g.kchunk = ((g.K + TBK - 1) / TBK) * TBK;
  if (g.K == 0) g.kchunk = TBK;
  static const int group_m = [] {
    const char* e = getenv("MLVAE_GEMM_GROUP_M");
    return e ? atoi(e) : 8;
  }();
  g.group_m = group_m;
  g.c16 = c16;
  dim3 grid(((N + TBN - 1) / TBN) * ((M + TBM - 1) / TBM), 1, 1);
  const int rc = launch_fast<true, true>(g, grid, (hipStream_t)stream, 8);
  if (rc) return rc;
  MLVAE_CHECK_LAUNCH();
  return 0;
}
