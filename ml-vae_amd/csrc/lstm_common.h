// Shared pieces of the persistent LSTM recurrences (lstm.hip: the batch-group kernels;
// lstm_wide.hip: the wide-batch kernels): launch arguments, the tagged-granule hand-off
// (MI355X_MICROARCH.md "Valid forms" R2) and diagnostics stamps.
#pragma once
#include "common.h"
#include <type_traits>

// Diagnostics -- phase / realtime stamps and the debug-mode timing variants of the recurrences'
// step loops -- compile in only with -DMLVAE_DIAG=1 (python -m mlvae_hip.build --diag ->
// libmlvae_diag.so, which tools/lstm_stamps.py and friends load through MLVAE_LIB_PATH): the
// shipped kernels carry no runtime debug branch.  Host-side launch choices (mlvae_lstm_set_debug_mode
// bits read by the launchers, e.g. 4096 / 256 in the tests) stay runtime in both builds.
#ifndef MLVAE_DIAG
#define MLVAE_DIAG 0
#endif
#define DMODE(a) (MLVAE_DIAG ? (a).dbg_mode : 0)
#define DPTR(a) (MLVAE_DIAG ? (a).dbg : (unsigned long long*)nullptr)

namespace {

constexpr int BG = 16;             // utterances per batch group (= MFMA N/M tile)
constexpr int NSLOT = 4;           // exchange slots (step mod 4)
constexpr unsigned SPIN_LIMIT = 1u << 20;
constexpr int MIN_LDS = 82 * 1024; // > half of 160 KiB: one workgroup per CU (residency)

struct LstmArgs {
  int B, T, H;        // B = utterances handled by this launch (<= NB*16)
  int NB, NJ, HJ;     // batch groups, hidden slices per group, hidden units per slice
  int ndir;           // directions: 2 (bidirectional, gates [N,8H], h [N,2H]) or 1 ([N,4H], [N,H])
  int Kp;             // H padded (pow2 >= 128): fwd exchange row stride / MFMA K
  int K4p;            // 4H padded (pow2 >= 128): bwd exchange row stride / MFMA K
  const float* W0;    // W_hh forward dir  [4H, H]
  const float* W1;    // W_hh reverse dir  [4H, H]
  float* G;           // [B*T, 8H] fwd: in x-proj(+biases) out activated gates; bwd: in gates, out dG
  float* Cs;          // [B*T, 2H] cell states (fwd writes, bwd reads)
  float* Y;           // [B*T, 2H] fwd: out h; bwd: in dY (grad wrt layer output)
  void* xbuf;         // exchange buffer [2 dirs][NB][NSLOT][16][Kp or K4p]
  int* err;
  unsigned long long* dbg;  // optional per-step phase stamps of workgroup 0 (diagnostics)
  int dbg_mode;             // diagnostics: bit0 = skip saved-activation stores (timing only)
  int xcd_local;            // group g = blocks b with b % 8 == g (one XCD each, when the
                            // dispatcher deals round-robin); others exit at once
  unsigned* xtab;           // [ngroups][NJ] XCC id + 1 of every member (zeroed per launch)
  unsigned short* Yb;       // optional bf16 copy of h [B*T, 2H] (fwd; GEMM operand)
  unsigned short* dGb;      // optional: bwd writes dG as bf16 [B*T, 8H] here instead of into G
  float* dbias;             // wide bwd, optional: per batch group sums of dG over (utterance, t),
                            // [ceil(B/16)][8H] fp32 -- the bias gradients before the group sum
  // wide-batch forward only: bf16 dropout(h) [B*T, 2H] for the next layer (Philox mask of
  // element doff + row*2H + col, keep prob dkeep, scale dscale; NULL = none)
  unsigned short* Ydb;
  unsigned long long dseed, doff;
  float dkeep, dscale;
  // fp8 mode (configs[4]), wide kernels, optional: the forward's e4m3 copy of dropout(h) scaled
  // by x8scale (the next layer's fp8 projection operand); the BPTT's e4m3 copy of dG scaled by
  // *g8scale (delayed scaling: from the previous step's amax) and this launch's max |dG|
  // atomically max-ed into *g8amax as float bits (g8amax alone: amax only)
  unsigned char* Y8;
  float x8scale;
  unsigned char* dG8;
  const float* g8scale;
  unsigned* g8amax;
  const unsigned short* dYb;  // wide BPTT, optional: dY as bf16 [B*T, 2H] instead of Y (fp32)
  // wide forward, optional (ZP): the layer input z (bf16 [B*T rows, ldz], 32 wide) whose
  // projection z W_ih^T + b_ih + b_hh the kernel computes itself -- G then only receives the
  // activated gates (no 8H-wide fp16 projection written and read back)
  const unsigned short* Zb;
  int ldz;
  const float* Wz0;           // W_ih forward / reverse [4H, 32]
  const float* Wz1;
  const float* bz[4];         // b_ih, b_hh forward; b_ih, b_hh reverse [4H]
  // wide forward, optional: Yb row t receives the h ENTERING step t (h_{t-1} forward, h_{t+1}
  // reverse; zeros at each utterance's first step) -- dW_hh's time-shifted operand pre-shifted,
  // when no other reader takes Yb (the layer below a dropout)
  int yb_prev;
};

// XCC (XCD) id of the executing workgroup: s_getreg_b32 HW_REG_XCC_ID (id 20, bits [3:0])
__device__ __forceinline__ unsigned xcc_id() {
  return __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 0xf;
}

// One-time placement check of an XCD-local group: every member publishes its XCC id, then
// reads all members' ids.  Returns true (uniformly across the group: all read the same
// table) iff the whole group runs on one XCD -- then hand-off stores may be plain (the line
// stays in that XCD's L2, which every member's sc1 loads read); otherwise they stay
// write-through sc1, which is correct at any placement.  Bounded spin; false on timeout.
__device__ bool group_on_one_xcd(unsigned* tab, int members, int me, int* scratch) {
  const int tid = threadIdx.x;
  const unsigned mine = xcc_id() + 1;
  if (tid == 0) { *scratch = 0; st_flag(tab + me, mine); }
  __syncthreads();
  if (tid < members) {
    unsigned v = 0, spins = 0;
    while ((v = ld_flag(tab + tid)) == 0 && ++spins < (1u << 16)) __builtin_amdgcn_s_sleep(2);
    if (v != mine) atomicOr(scratch, 1);
  }
  __syncthreads();
  return *scratch == 0;
}

// Phase stamps (s_memtime) of workgroup 0, thread 0: dbg[s*16 + phase].  The LDS-buffered and
// realtime stamps below compile only into the kernels' DBG instances (template flag), which the
// host launches only while a stamp buffer is set (mlvae_lstm_set_debug): production instances
// carry no stamp code (it cost the forward 35 spilled SGPRs).
#define STAMP(ph)                                                              \
  do {                                                                         \
    if (DPTR(a) && blockIdx.x == 0 && threadIdx.x == 0)                          \
      a.dbg[(size_t)s * 16 + (ph)] = __builtin_amdgcn_s_memtime();             \
  } while (0)
// per-wave stamp (lane 0 of every wave of workgroup 0): dbg[s*16 + slot + wave]
#define WSTAMP(slot)                                                           \
  do {                                                                         \
    if (DPTR(a) && blockIdx.x == 0 && (threadIdx.x & 63) == 0)                   \
      a.dbg[(size_t)s * 16 + (slot) + (threadIdx.x >> 6)] = __builtin_amdgcn_s_memtime(); \
  } while (0)

// debug bit 4 (wide forward): wave 4 (an io wave) of workgroup 0 stamps its own phases into
// slots 8 + k instead of the per-wave poll-completion stamps
#define IOSTAMP(k)                                                             \
  do {                                                                         \
    if (DBG && DPTR(a) && (DMODE(a) & 16) && blockIdx.x == 0 && threadIdx.x == 256 && \
        (unsigned)(s - STW0) < (unsigned)STWN)                                 \
      stamp_lds[(s - STW0) * 16 + 8 + (k)] = __builtin_amdgcn_s_memtime();     \
  } while (0)
// LDS-buffered stamps (wide kernels): thread 0 of workgroup 0 records s_memtime at the phase
// points of steps [STW0, STW0 + STWN) in LDS and writes them to dbg[s*16 + phase] once, after
// the step loop -- no global store inside the loop, so no vmcnt wait ever queues behind one
constexpr int STW0 = 64, STWN = 32;
#define LSTAMP_DECL                                                            \
  __shared__ unsigned long long stamp_lds[DBG ? STWN * 16 : 1];                \
  if (DBG && DPTR(a) && blockIdx.x == 0 && threadIdx.x == 0)                     \
    for (int i_ = 0; i_ < STWN * 16; ++i_) stamp_lds[i_] = 0
#define LSTAMP(ph)                                                             \
  do {                                                                         \
    if (DBG && DPTR(a) && blockIdx.x == 0 && threadIdx.x == 0 &&                        \
        (unsigned)(s - STW0) < (unsigned)STWN)                                 \
      stamp_lds[(s - STW0) * 16 + (ph)] = __builtin_amdgcn_s_memtime();        \
  } while (0)
// per-wave stamp (lane 0 of every wave of workgroup 0) into slot 8 + wave
#define LWSTAMP()                                                              \
  do {                                                                         \
    if (DBG && DPTR(a) && !(DMODE(a) & 16) && blockIdx.x == 0 && (threadIdx.x & 63) == 0 && \
        (unsigned)(s - STW0) < (unsigned)STWN)                                 \
      stamp_lds[(s - STW0) * 16 + 8 + (threadIdx.x >> 6)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#define LSTAMP_FLUSH()                                                         \
  do {                                                                         \
    if (DBG) __syncthreads();                                                  \
    if (DBG && DPTR(a) && blockIdx.x == 0 && threadIdx.x == 0)                   \
      for (int i_ = 0; i_ < STWN * 16; ++i_)                                   \
        a.dbg[(size_t)STW0 * 16 + i_] = stamp_lds[i_];                         \
  } while (0)

// Realtime stamps of EVERY workgroup (debug bit 3; s_memrealtime, the chip-wide 100 MHz clock, so
// a producer's publish and its consumer's poll completion compare across CUs): per wave w its
// publish of step s (slot w) and, for the polling waves, the poll completion of step s (slot
// 8 + w), steps [STW0, STW0 + STWN); written after the step loop to
// dbg[T * 16 + blockIdx * STWN * 16 + (s - STW0) * 16 + slot].
#define RTS_DECL                                                               \
  __shared__ unsigned long long rts_lds[DBG ? STWN * 16 : 1];                  \
  const bool rts_on = DBG && DPTR(a) && (DMODE(a) & 8);                        \
  if (rts_on)                                                                  \
    for (int i_ = threadIdx.x; i_ < STWN * 16; i_ += blockDim.x) rts_lds[i_] = 0
#define RTS(slot)                                                              \
  do {                                                                         \
    if (rts_on && (threadIdx.x & 63) == 0 && (unsigned)(s - STW0) < (unsigned)STWN) \
      rts_lds[(s - STW0) * 16 + (slot)] = __builtin_amdgcn_s_memrealtime();    \
  } while (0)
#define RTS_FLUSH()                                                            \
  do {                                                                         \
    if (DBG) __syncthreads();                                                  \
    if (rts_on)                                                                \
      for (int i_ = threadIdx.x; i_ < STWN * 16; i_ += blockDim.x)             \
        a.dbg[(size_t)a.T * 16 + (size_t)blockIdx.x * STWN * 16 + i_] = rts_lds[i_]; \
  } while (0)

// Debug bit 29 (A/B): phase-stagger the independent recurrence chains.  Every group (one batch
// group of one direction) runs in lock step with its own members only, yet all groups start
// together and so issue their saved-activation stores / next-step loads in the same chip-wide
// bursts.  Groups with ((gid ^ gid >> 3) & 1) start ((mode >> 5) & 7) x 1024 cycles late.
__device__ __forceinline__ void stagger_start(int gid, int mode) {
  if (!(mode & (1 << 29)) || !((gid ^ (gid >> 3)) & 1)) return;
  for (int i = 0; i < ((mode >> 5) & 7); ++i) __builtin_amdgcn_s_sleep(16);
}

template <int PREC> struct Elt;
template <> struct Elt<PREC_F32> { typedef float T; static constexpr int GE = 2; };   // per granule
template <> struct Elt<PREC_BF16> { typedef short T; static constexpr int GE = 4; };

__device__ __forceinline__ unsigned step_tag(int s) { return (unsigned)(((s >> 2) + 1) & 1); }
// the same over 2^lg slots (the wide kernels)
__device__ __forceinline__ unsigned step_tag_lg(int s, int lg) { return (unsigned)(((s >> lg) + 1) & 1); }

// Granule packing: value 0 carries the tag in its least significant bit.
__device__ __forceinline__ unsigned long long pack_bf16(float v0, float v1, float v2, float v3,
                                                        unsigned tag) {
  const unsigned e0 = ((unsigned)(unsigned short)f2bf(v0) & ~1u) | tag;
  const unsigned lo = e0 | ((unsigned)(unsigned short)f2bf(v1) << 16);
  const unsigned hi = (unsigned)(unsigned short)f2bf(v2) | ((unsigned)(unsigned short)f2bf(v3) << 16);
  return ((unsigned long long)hi << 32) | lo;
}
__device__ __forceinline__ unsigned long long pack_f32(float v0, float v1, unsigned tag) {
  const unsigned e0 = (__float_as_uint(v0) & ~1u) | tag;
  return ((unsigned long long)__float_as_uint(v1) << 32) | e0;
}
// one 8-byte write-through store per granule (buffer_store_dwordx2 ... sc1)
__device__ __forceinline__ void st_granule(__amdgpu_buffer_rsrc_t r, unsigned byte_off,
                                           unsigned long long v) {
  u32x2 w = {(unsigned)v, (unsigned)(v >> 32)};
  __builtin_amdgcn_raw_buffer_store_b64(w, r, byte_off, 0, 16 /*sc1*/);
}
// a 16-byte load holds two granules; their tags sit in dwords 0 and 2
__device__ __forceinline__ bool tags_ok(u32x4 v, unsigned tag, bool g0, bool g1) {
  return (!g0 || (v[0] & 1u) == tag) && (!g1 || (v[2] & 1u) == tag);
}

}  // namespace

// Wide-batch recurrences (lstm_wide.hip): one launch covers every utterance of a layer when
// the batch-group kernels would need several chunks.  Return -1 when the shape is not
// supported (the caller then falls back to chunked batch-group launches), else a status.
struct WideFp8 {  // the fp8 mode's fused outputs of the wide kernels (LstmArgs fields)
  unsigned char* y8 = nullptr;
  float x8scale = 0.f;
  unsigned char* dg8 = nullptr;
  const float* g8scale = nullptr;
  unsigned* g8amax = nullptr;
};
struct WideZ {  // the wide forward's fused layer-0 input projection (LstmArgs Zb ... bz)
  const unsigned short* zb = nullptr;
  int ldz = 0;
  const float* w0 = nullptr;
  const float* w1 = nullptr;
  const float* b[4] = {nullptr, nullptr, nullptr, nullptr};
  int yb_prev = 0;  // LstmArgs::yb_prev
};
int lstm_wide_run(bool fwd, int B, int T, int H, const float* W0, const float* W1, float* G,
                  float* Cs, float* Y, void* xbuf, size_t xbytes, int* err, hipStream_t st,
                  unsigned short* yb, unsigned short* dgb, float* dbias, unsigned short* ydb,
                  unsigned long long dseed, unsigned long long doff, float dp,
                  unsigned long long* dbg, int dbg_mode, const WideFp8& f8 = WideFp8(),
                  const unsigned short* dyb = nullptr, const WideZ& wz = WideZ());
// exchange bytes the wide kernels need at (B, H), or 0 when they do not apply
size_t lstm_wide_xbytes(int B, int H, bool fwd);
// the wide kernels address one batch group's rows through 32-bit buffer offsets: T bound
bool lstm_wide_t_ok(int T, int H);
// workgroups of the wide launch at (B, H), or 0 when it does not apply
int lstm_wide_workgroups(int B, int H, bool fwd);
