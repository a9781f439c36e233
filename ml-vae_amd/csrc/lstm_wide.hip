// Wide-batch persistent BiLSTM recurrence (bf16 MFMA operands, fp32 state), forward + BPTT.
//
// Reference op: nn.LSTM(z, H, L, bidirectional=True, batch_first=True) at
// ref:src/modules/decoder.py:14-15,22 (gate order i,f,g,o; h0 = c0 = 0; no packing).
//
// lstm.hip's batch-group kernels give every workgroup 16 utterances x 16 hidden units, so a
// layer needs 2 dirs x B/16 groups x H/16 slices workgroups; past 64 utterances at H = 512 that
// exceeds the 256 CUs and the batch is run in sequential chunks (4 launches per layer at the
// metric's B = 256).  Here a workgroup owns 16 utterances x HJ = 32*TPW units (TPW = 1, 2), so
// one co-resident launch of 2 x B/16 x H/HJ <= 256 workgroups covers B = 128 (HJ 32) or
// B = 256 (HJ 64): the per-step MFMA work of a workgroup grows 2-4x while the serial hand-off
// chain -- the recurrence's real bound -- is paid once per layer instead of once per chunk.
//
// Workgroup = 8 waves (512 threads, one per CU: the VGPR file is full).
//   forward:  gates^T[4HJ x 16] = W_hh[rows of my units] . h_{t-1}^T.  Wave w owns TPW M-tiles
//             (16 gate rows = 4 units x i,f,g,o) as resident A-fragments for all of K = H;
//             lane (utt, q) ends with the 4 gates of one unit -> in-register cell update.
//             Waves 0-3 poll h_{t-1} (tagged granules, a quarter of K each) into an LDS image
//             every wave reads its B-fragments from; waves 4-7 move the step's HBM traffic
//             (input projection two steps ahead, saved activations one step behind) through
//             LDS rings with coalesced 16-byte accesses, so the pollers' memory queues hold
//             nothing but the hand-off (lstm.hip's io-wave finding, 2.74 -> 2.18 us/step).
//   backward: reduce-scatter form.  Wave w multiplies the workgroup's own dG_t slice
//             [16 x 4HJ] (LDS) by resident W_hh row fragments [4HJ x 64 units] and publishes
//             the partial dh_{t-1} of those 64 units to the consumer workgroup(s) owning them;
//             each workgroup sums its NJ producers' partials with a DPP reduce-scatter.
// Hand-off protocol, slots and tags: lstm_common.h / lstm.hip header.
#include "lstm_common.h"
#include <stdlib.h>
#include <type_traits>

namespace {

constexpr int WW = 8;  // waves per workgroup
// forward: k-chunks whose A-fragments (W_hh) live in LDS instead of registers.  4 (was 2) frees
// the VGPRs that let each wave read a quarter of its B-fragments (h) ahead of the MFMAs that
// consume them (the 2-chunk build read one fragment, waited for it and issued its two MFMAs, so
// every k-chunk exposed an LDS round trip)
constexpr int FWD_KLF = 4;
// BPTT: the wave's tiles are multiplied and published in this many groups (below): halves
// (single tiles at TPW 2, the A-fragments then read 4 times: c3 BPTT 1.27 -> 1.35 ms per launch)
template <int TPW> constexpr int bptt_groups() { return 2; }
#ifndef NT_AUX
#define NT_AUX 2  // cache policy of the read-once activation streams (2 = nt)
#endif

// Publish one 8-byte granule: a plain store when the whole group was verified to run on one
// XCD (the line stays in that XCD's L2, where the members' sc1 loads read it), else a
// write-through sc1 store (correct at any placement).
__device__ __forceinline__ void publish(__amdgpu_buffer_rsrc_t r, unsigned byte_off,
                                        unsigned long long v, bool plain) {
  if (plain) {
    u32x2 w = {(unsigned)v, (unsigned)(v >> 32)};
    __builtin_amdgcn_raw_buffer_store_b64(w, r, byte_off, 0, 0);
  } else {
    st_granule(r, byte_off, v);
  }
}

// 16-byte slot of row `utt` in an XOR-swizzled LDS image (conflict-free B/A-fragment reads)
__device__ __forceinline__ int swz(int utt, int slot) { return slot ^ (utt & 15); }

// ---------------------------------------------------------------------------------------
// forward
// ---------------------------------------------------------------------------------------
// OCC = minimum waves per SIMD (2: one 512-thread workgroup per CU)
// Exchange layout [slot][H / 8][utt][8]: the 8 units of one wave (TPW 2: both tiles, one
// 16-byte store per utterance; TPW 1: two waves' 8-byte halves) for 8 utterances fill one
// 128-byte line, written by one store instruction.  (The earlier [slot][utt][H] layout
// assembled each line from 16 granule stores of 8 waves: same box, B = 256 / 64 / 32 forward
// 3.45 / 2.24 / 2.21 -> 3.22 / 1.99 / 1.95 us per step, profiles/ab/r04_fwd_variants.txt.)
// AS: asymmetric tile split (TPW 1).  The io waves (4-7) issue the step's HBM traffic, whose
// issue stalls for ~1,000 ticks behind the chip-wide bursts, so with equal tile shares they
// published their units last (realtime stamps, tools/lstm_handoff.py: the last producer wave of
// every hand-off was an io wave, 500-850 ns behind the pollers).  With AS the pollers own both
// tiles of each SIMD and the io waves only move data: their DMA and stores right behind the
// barrier, inside the pollers' MFMA / cell phase.  Same box, in the step: forward per launch
// c2 0.954 -> 0.863, c5 (B = 64) 0.979 -> 0.872, c4 3.95 -> 3.49 ms (profiles/ab/r04_as.txt);
// the only form at TPW 1 since round 6.  At TPW 2 the pollers' 3 tiles spilled 46 VGPRs.
// ZP: the layer-0 input projection fused (a.Zb): io wave 4 DMAs the step's 16 z rows (64 B each)
// into the gx ring's space and each tile's gate inputs are one v_mfma_f32_16x16x32_bf16 of the
// resident W_ih fragment (K = 32 = the latent width) onto the tile's b_ih + b_hh -- instead of
// reading 8 KB of fp16 projection per utterance and step that a separate kernel wrote.
// NT: N-tiles (16 utterances each) per workgroup.  NT = 2 (the asymmetric TPW-1 split only): a
// workgroup owns 32 utterances x 32 units, the pollers 2 M-tiles x 2 N-tiles each (every W_hh
// A-fragment feeds two MFMAs), and the io waves own no tile at every batch size -- at B = 256
// that replaces TPW 2 (16 utterances x 64 units, every wave owning tiles), whose io waves reached
// the step barrier ~1,400 ticks after the pollers, waiting for the saved-activation stores they
// had issued behind their own publish (profiles/r06_lstm_stamps.txt).  Tile-less io waves issue
// those stores right behind the barrier instead, a whole step ahead of the wait.  Groups have
// 16 members (H / 32), two groups per XCD.
// W12: 12 waves (768 threads, three per SIMD).  Waves 0-7 each own ONE M-tile (4 units) across
// the NT N-tiles -- its W_hh A-fragments all in registers (64 VGPRs, under the 168 a wave gets at
// three per SIMD) -- and all eight poll; waves 8-11 only move data.  Every SIMD keeps two MFMA
// waves (one's cell overlaps the other's MFMAs) beside a tile-less io wave.
template <int TPW, int NKC, int OCC, bool DBG = false, bool AS = false, bool ZP = false, int NT = 1,
          bool W12 = false>
__global__ __launch_bounds__(W12 ? 768 : 512, W12 ? 1 : OCC) void lstm_fwd_wide_kernel(LstmArgs a) {
  static_assert(NT == 1 || (NT == 2 && AS && TPW == 1), "two N-tiles: the asymmetric TPW-1 split");
  static_assert(!W12 || (AS && TPW == 1), "12 waves: the asymmetric TPW-1 split");
  constexpr int NWV = W12 ? 12 : 8;           // waves per workgroup
  constexpr int NPOLL = W12 ? 8 : 4;          // polling waves (0 .. NPOLL-1)
  constexpr int IO0 = NWV - 4;                // first io wave
  constexpr int BGW = BG * NT;                // utterances per workgroup
  constexpr int HJ = WW * TPW * 4;
  constexpr int H = NKC * 32;
  constexpr int PL = NKC / NPOLL;             // poll loads (k-chunks) per lane and N-tile
  constexpr int ROWB = H * 2;                 // bytes of one h-image row (bf16)
  constexpr int HIMG = BGW * ROWB;
  constexpr int GXU = 4 * HJ + 8;             // gx ring halfs per utterance: [gate][unit] + 16 B
  // out ring bytes per utterance: gates fp16 [i f g o][HJ] | c fp32 [HJ] | h fp32 [HJ] | 16 B
  constexpr int OUB = 4 * HJ * 2 + 2 * HJ * 4 + 16;
  constexpr int NC8 = BGW * HJ / 8;           // 8-unit chunks of h per step
  // k-chunks whose A-fragments live in LDS (VGPR budget; at TPW 1 one tile's 16 fit in registers)
  constexpr int KLF = ((TPW == 1 && !AS) || W12) ? 0 : FWD_KLF;
  constexpr int KR = NKC - KLF;               // ... and in registers
  constexpr int HB = 4;                       // B-fragments (h) read ahead per batch
  constexpr int NQ = 16 * 4 * HJ / 4;         // 16-byte quads of gx / gates per step
  constexpr int QPT = NQ / 256;               // quads per io thread
  static_assert(NQ % 256 == 0, "io split");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  LSTAMP_DECL;
  RTS_DECL;
  char* himg = smem;                                        // [2][BGW][ROWB], swizzled slots
  unsigned short* gxr = reinterpret_cast<unsigned short*>(smem + 2 * HIMG);  // [2][BGW][GXU] fp16
  char* outr = reinterpret_cast<char*>(gxr + 2 * BGW * GXU);                // [2][BGW][OUB]
  bf16x8* wlds = reinterpret_cast<bf16x8*>(outr + 2 * BGW * OUB);  // [wave][TPW][KLF][lane]
  unsigned* dbl = reinterpret_cast<unsigned*>(wlds + 8 * TPW * KLF * 64);  // [2][NC8] keep bits
  __shared__ int abort_flag;

  // group slots padded to a multiple of 8 (idle slots exit at once): members gid + k * gstride
  // then share one XCD under round-robin dispatch at every batch size (B = 32: 4 groups)
  const int ngroups = 2 * a.NB, gstride = (ngroups + 7) & ~7;
  const int gid = blockIdx.x % gstride, js = blockIdx.x / gstride;
  if (gid >= ngroups) return;
  const int dir = gid / a.NB, grp = gid % a.NB;
  const int T = a.T, j0 = js * HJ;
  const int tid = threadIdx.x, lane = tid & 63;
  // exchange slots in use: 2 (every member of a group is producer and consumer of every other,
  // so a slot is rewritten only after all its readers have loaded it); bit 24: all NSLOT
  const int nlg = (DMODE(a) & (1 << 24)) ? 2 : 1, nmask = (1 << nlg) - 1;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: role branches stay scalar
  const float* W = dir ? a.W1 : a.W0;
  const int bi = lane & 15, q = lane >> 4;
  bool valid[NT];  // utterance 16 n + bi of the workgroup exists
#pragma unroll
  for (int n = 0; n < NT; ++n) valid[n] = grp * BGW + 16 * n + bi < a.B;

  // tiles per poller / io wave (AS) and a wave's first tile
  // (TPW 2 as 3 + 1 spilled 46 VGPRs: the split applies to TPW 1 only)
  static_assert(!AS || TPW == 1, "asymmetric split: TPW 1 only");
  constexpr int TPP = W12 ? 1 : AS ? 2 : TPW;
  constexpr int TPI = AS ? 0 : TPW;
  static_assert(NPOLL * TPP + 4 * TPI == WW * TPW, "every tile owned once");
  // resident A-fragments: tile m, row r = bi -> unit 4m + (r >> 2), gate r & 3; k-chunks
  // [0, KR) in registers, [KR, NKC) in LDS (lane-linear, conflict-free 16-B reads)
  auto load_w = [&](auto* wreg, int m0, int mt) {
    for (int t = 0; t < mt; ++t) {
      const int m = m0 + t;
      const float* wrow = W + (size_t)((bi & 3) * H + j0 + 4 * m + (bi >> 2)) * H;
#pragma unroll
      for (int kc = 0; kc < NKC; ++kc) {
        const f32x4 w0 = *reinterpret_cast<const f32x4*>(wrow + kc * 32 + 8 * q);
        const f32x4 w1 = *reinterpret_cast<const f32x4*>(wrow + kc * 32 + 8 * q + 4);
        bf16x8 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) { v[e] = f2bf(w0[e]); v[4 + e] = f2bf(w1[e]); }
        if (kc < KR) wreg[t][kc < KR ? kc : 0] = v;
        else wlds[(m * KLF + (kc - KR)) * 64 + lane] = v;
      }
    }
  };
  // group members are blocks gid + k * gstride: one XCD under round-robin dispatch; verified
  // at run time, never assumed (lstm_common.h group_on_one_xcd)
  __shared__ int placement;
  const bool same_xcd = group_on_one_xcd(a.xtab + gid * a.NJ, a.NJ, js, &placement) &&
                        !(DMODE(a) & 32768);  // bit 15: force write-through hand-offs
  if (tid == 0) abort_flag = 0;

  const size_t xslot = (size_t)BGW * H;  // elements per exchange slot: [H / 8][BGW][8]
  short* xb = reinterpret_cast<short*>(a.xbuf) + (size_t)(dir * a.NB + grp) * NSLOT * xslot;
  auto xr = make_rsrc(xb, (unsigned)(NSLOT * xslot * sizeof(short)));

  // ---- io role (waves 4-7).  G is fp16 in the wide path.  The input projection of a step goes
  // HBM -> LDS by LDS-DMA (buffer_load ... lds: one utterance's 4 gates x HJ units = 8 HJ bytes
  // per wave-instruction, no registers); the saved activations go LDS -> registers -> 16-byte
  // stores: gates (fp16), c (fp32), h (bf16 GEMM operand), the next layer's dropout(h) (bf16,
  // Philox mask: replaces a separate dropout pass) and -- only when asked -- h in fp32.
  const int iot = tid - 64 * IO0;
  const bool io = wave >= IO0;
  const int iow = wave - IO0;  // io wave index (0 .. 3)
  typedef __attribute__((address_space(3))) void* lds_ptr_t;
  unsigned short* G16 = reinterpret_cast<unsigned short*>(a.G);
  const auto rgx = make_rsrc(G16 + (size_t)grp * BGW * T * 8 * H, 0xffffffffu);
  // debug bit 10 (timing probe only, outputs wrong): the saved activations and the gx loads
  // addressed time-major (row t * B + b) -- one step's rows of all utterances contiguous in HBM
  const bool tmaj = (DMODE(a) & 1024) != 0;
  auto rowof = [&](int b_, int t_) -> size_t { return tmaj ? (size_t)t_ * a.B + b_ : (size_t)b_ * T + t_; };
  // (the probe's absolute descriptor: range-checked to the gate buffer, at most 4 GB)
  const auto rgx_abs = make_rsrc(G16, (unsigned)min((size_t)a.B * T * 8 * H * 2, (size_t)0xffffffffu));
  // ZP: z rows [16 utt][32] bf16 per ring slot, lane-linear (lane 4 u + c: 16 B chunk c of utt u)
  unsigned short* zr = gxr;
  const auto rz = make_rsrc(a.Zb, (unsigned)min((size_t)a.B * T * a.ldz * 2, (size_t)0x7fffffff));
  auto io_load = [&](int s_) {  // input projection of step s_ into gx ring slot s_ & 1
    if (s_ >= T || (s_ > 0 && (DMODE(a) & 8192))) return;  // bit 13: timing without the loads
    const int t_ = dir ? T - 1 - s_ : s_;
    if constexpr (ZP) {
      if (iow < NT) {  // io wave n: the z rows of N-tile n
        const int u = iow * 16 + (lane >> 2), b = grp * BGW + u;
        const unsigned off = b < a.B ? (unsigned)((((size_t)b * T + t_) * a.ldz + 8 * (lane & 3)) * 2) : 0x80000000u;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rz, (lds_ptr_t)(zr + ((s_ & 1) * BGW + iow * 16) * 32), 16,
                                                 off, 0, 0, NT_AUX);
      }
      return;
    }
    constexpr int UPW = BGW / 4;  // utterances per io wave
    // one descriptor over the group's 16 utterances (per-utterance descriptors spilled SGPRs
    // into the io waves' MFMA phase); the host keeps 16 T 8H halfs under 4 GB
#pragma unroll
    for (int i = 0; i < UPW; ++i) {
      const int u = iow * UPW + i, b = grp * BGW + u;
      if (b >= a.B) continue;
      // lane l < HJ/2 -> gate l / (HJ/8), units 8 (l % (HJ/8)) .. + 7
      const int g = lane / (HJ / 8), uu = (lane % (HJ / 8)) * 8;
      const unsigned off = tmaj ? (unsigned)((((size_t)t_ * a.B + b) * 8 * H + dir * 4 * H + g * H + j0 + uu) * 2)
                                : (unsigned)((((size_t)u * T + t_) * 8 * H + dir * 4 * H + g * H + j0 + uu) * 2);
      const auto rs = tmaj ? rgx_abs : rgx;
      unsigned short* dst = gxr + (s_ & 1) * BGW * GXU + u * GXU;
      // nt: read-once stream, kept from displacing the hand-off lines in L2
      if (lane < HJ / 2) __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)dst, 16, off, 0, 0, NT_AUX);
    }
  };
  // dropout keep bits (bit e = element e) of h chunk c8 (8 units) at step s_: one mask quad per
  // 4 aligned elements, as dropout_scale in common.h
  auto drop_bits = [&](int s_, int c8) -> unsigned {
    const int u = c8 / (HJ / 8), uu = (c8 % (HJ / 8)) * 8;
    const int t_ = dir ? T - 1 - s_ : s_;
    const size_t o = ((size_t)(grp * BGW + u) * T + t_) * 2 * H + dir * H + j0 + uu;
    const unsigned long long k = drop_key(a.dseed);
    const unsigned long long r0 = drop_quad(k, (a.doff + o) >> 2), r1 = drop_quad(k, (a.doff + o + 4) >> 2);
    unsigned bits = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      bits |= (drop_elem_scale(r0, e, a.dkeep, 1.f) != 0.f ? 1u : 0u) << e;
      bits |= (drop_elem_scale(r1, e, a.dkeep, 1.f) != 0.f ? 1u : 0u) << (4 + e);
    }
    return bits;
  };
  auto io_store = [&](int s_) {  // saved activations of step s_ from out ring slot s_ & 1
    if (s_ < 0 || s_ >= T || (DMODE(a) & 1)) return;
    const int t_ = dir ? T - 1 - s_ : s_;
    const char* src = outr + (s_ & 1) * BGW * OUB;
    // activated gates (fp16 in the ring already): BGW utt x 4 gates x HJ/8 chunks, LDS -> HBM
    constexpr int NG8 = BGW * 4 * HJ / 8;
    for (int ci = iot; ci < NG8; ci += 256) {
      const int row = ci / (HJ / 8), uu = (ci % (HJ / 8)) * 8;
      const int u = row >> 2, g = row & 3, b = grp * BGW + u;
      if (b >= a.B) continue;
      *reinterpret_cast<u32x4*>(G16 + rowof(b, t_) * 8 * H + dir * 4 * H + g * H + j0 + uu) =
          *reinterpret_cast<const u32x4*>(src + u * OUB + (g * HJ + uu) * 2);
    }
    // c (fp32) and, when asked, h (fp32): 16 x HJ/4 quads
    constexpr int NQ2 = BGW * HJ / 4;
    for (int qi = iot; qi < NQ2; qi += 256) {
      const int u = qi / (HJ / 4), uu = (qi % (HJ / 4)) * 4, b = grp * BGW + u;
      if (b >= a.B) continue;
      const size_t o = rowof(b, t_) * 2 * H + dir * H + j0 + uu;
      const float* cf = reinterpret_cast<const float*>(src + u * OUB + 8 * HJ);
      *reinterpret_cast<f32x4*>(a.Cs + o) = *reinterpret_cast<const f32x4*>(cf + uu);
      if (a.Y) *reinterpret_cast<f32x4*>(a.Y + o) = *reinterpret_cast<const f32x4*>(cf + HJ + uu);
    }
    // h (bf16) by io threads [0, NC8), dropout(h) (bf16) by the next NC8: chunks of 8 units
    static_assert(2 * NC8 <= 256, "one h chunk per io thread");
    const bool drop8 = iot >= NC8;
    const int ci8 = drop8 ? iot - NC8 : iot;
    if (ci8 < NC8 && (drop8 ? (a.Ydb != nullptr || a.Y8 != nullptr) : a.Yb != nullptr)) {
      const int u = ci8 / (HJ / 8), uu = (ci8 % (HJ / 8)) * 8, b = grp * BGW + u;
      if (b < a.B) {
        const float* hf = reinterpret_cast<const float*>(src + u * OUB + 8 * HJ) + HJ;
        f32x4 v0 = *reinterpret_cast<const f32x4*>(hf + uu);
        f32x4 v1 = *reinterpret_cast<const f32x4*>(hf + uu + 4);
        size_t o = rowof(b, t_) * 2 * H + dir * H + j0 + uu;
        // (the fused-z layer-0 instances only: mlvae_lstm_fwd_z2 -- in the others the branch cost
        // the TPW-2 forward 8 spilled SGPRs and ~5 % per launch)
        if (ZP && !drop8 && a.yb_prev) {  // h_t enters step s_ + 1: row t + 1 (forward) / t - 1 (reverse)
          if (s_ == 0)  // nothing enters the first step
            *reinterpret_cast<bf16x8*>(a.Yb + o) = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
          const int tn = dir ? t_ - 1 : t_ + 1;
          if (tn < 0 || tn >= T) return;
          o = rowof(b, tn) * 2 * H + dir * H + j0 + uu;
        }
        if (drop8) {  // keep bits drawn by the pollers at the end of step s_
          const unsigned bits = dbl[(s_ & 1) * NC8 + ci8];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v0[e] = (bits >> e) & 1 ? v0[e] * a.dscale : 0.f;
            v1[e] = (bits >> (4 + e)) & 1 ? v1[e] * a.dscale : 0.f;
          }
        }
        if (!drop8 || a.Ydb)  // (fp8 mode may ask for the e4m3 dropout(h) alone)
          *reinterpret_cast<bf16x8*>((drop8 ? a.Ydb : a.Yb) + o) =
              bf16x8{f2bf(v0[0]), f2bf(v0[1]), f2bf(v0[2]), f2bf(v0[3]),
                     f2bf(v1[0]), f2bf(v1[1]), f2bf(v1[2]), f2bf(v1[3])};
        if (drop8 && a.Y8) {  // fp8 mode: the next layer's e4m3 projection operand, fixed scale
          const float xs = a.x8scale;
          *reinterpret_cast<u32x2*>(a.Y8 + o) =
              u32x2{pack4_fp8(v0[0] * xs, v0[1] * xs, v0[2] * xs, v0[3] * xs),
                    pack4_fp8(v1[0] * xs, v1[1] * xs, v1[2] * xs, v1[3] * xs)};
        }
      }
    }
  };
  // The step loop, instantiated once per role (IO: waves 4-7 move the step's HBM traffic;
  // else waves 0-3 poll the hand-off): each instance keeps only its own role's state live,
  // and both pass the same barriers.
  const bool want_drop = a.Ydb || a.Y8;  // a dropout(h) output (bf16 and / or e4m3)
  const bool late_bits = want_drop && !(DMODE(a) & (1 << 27));
  const bool late_dma_s = (2 * a.NB * a.NJ <= 64) != ((DMODE(a) & (1 << 17)) != 0);
  auto run = [&](auto io_tag) {
    constexpr bool IO = decltype(io_tag)::value;
    constexpr int MT = IO ? TPI : TPP;         // this wave's tiles
    constexpr int MTA = MT > 0 ? MT : 1;       // (array extent)
    const int m0 = IO ? NPOLL * TPP + iow * TPI : wave * TPP;
    bf16x8 wreg[MTA][KR];
    load_w(wreg, m0, MT);
    // ZP: the tiles' W_ih fragments (row bi: gate bi & 3, unit 4 m + (bi >> 2); k = 8 q .. 8 q + 7)
    // and b_ih + b_hh in the accumulator layout (element g: gate g of unit 4 m + q)
    bf16x8 wz[ZP ? MTA : 1];
    f32x4 bz4[ZP ? MTA : 1];
    if constexpr (ZP) {
      const float* Wz = dir ? a.Wz1 : a.Wz0;
      const float* bih = a.bz[2 * dir];
      const float* bhh = a.bz[2 * dir + 1];
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const int m = m0 + t;
        const float* wrow = Wz + (size_t)((bi & 3) * H + j0 + 4 * m + (bi >> 2)) * 32 + 8 * q;
        const f32x4 w0 = *reinterpret_cast<const f32x4*>(wrow);
        const f32x4 w1 = *reinterpret_cast<const f32x4*>(wrow + 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) { wz[t][e] = f2bf(w0[e]); wz[t][4 + e] = f2bf(w1[e]); }
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) bz4[t][g4] = bih[g4 * H + j0 + 4 * m + q] + bhh[g4 * H + j0 + 4 * m + q];
      }
    }
    // AS with tile-less io waves: their DMA and stores right behind the barrier
    constexpr bool PURE_IO = IO && MT == 0;
    if (IO) {
      io_load(0);
      io_load(1);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    float c[MTA][NT];
#pragma unroll
    for (int t = 0; t < MTA; ++t)
#pragma unroll
      for (int n = 0; n < NT; ++n) c[t][n] = 0.f;
    stagger_start(gid, DMODE(a));
    for (int s = 0; s < T; ++s) {
      LSTAMP(0);
      IOSTAMP(0);
      f32x4 acc[MTA][NT];
#pragma unroll
      for (int t = 0; t < MTA; ++t)
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[t][n] = f32x4{0.f, 0.f, 0.f, 0.f};
      char* hb = himg + (s & 1) * HIMG;
      // this step's input projection (fp16, LDS ring): read before the MFMAs, so the LDS
      // latency is not exposed between the last MFMA and the cell update
      // gate inputs: ZP's fp32 z-projection results, else the fp16 ring words (converted in the
      // cell, behind the padded end of the MFMA chain -- see there)
      float gxv[MTA][NT][4];
      unsigned short gxh[MTA][NT][4];
      auto read_gx = [&]() {
        if constexpr (ZP) {
          if constexpr (MT > 0) {
#pragma unroll
            for (int n = 0; n < NT; ++n) {
              const bf16x8 zf = *reinterpret_cast<const bf16x8*>(zr + ((s & 1) * BGW + 16 * n + bi) * 32 + 8 * q);
#pragma unroll
              for (int t = 0; t < MT; ++t) {
                const f32x4 r = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wz[t], zf, bz4[t], 0, 0, 0);
#pragma unroll
                for (int g4 = 0; g4 < 4; ++g4) gxv[t][n][g4] = r[g4];
              }
            }
          }
          return;
        }
#pragma unroll
        for (int n = 0; n < NT; ++n) {
          const unsigned short* gx = gxr + ((s & 1) * BGW + 16 * n + bi) * GXU;
#pragma unroll
          for (int t = 0; t < MT; ++t) {
            const int u = 4 * (m0 + t) + q;
#pragma unroll
            for (int g4 = 0; g4 < 4; ++g4) gxh[t][n][g4] = gx[g4 * HJ + u];
          }
        }
      };
      if (s == 0) read_gx();
      if (s > 0) {
        if (IO) {
          if (!(DMODE(a) & 16384))  // bit 14: timing without the wait
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's gx(s) LDS-DMA has landed
          IOSTAMP(1);
        } else {
          // poll = load: this wave's quarter of h_{t-1} (PL k-chunks), retried until every
          // granule carries step s-1's tag; then into the swizzled LDS image
          const unsigned tag = step_tag_lg(s - 1, nlg);
          // load (i, n): units u = 32 (wave PL + i) + 8 q = chunk u / 8 of utterance 16 n + bi
          const unsigned xbase = (unsigned)(((s - 1) & nmask) * xslot) + (((wave * PL * 32 + 8 * q) >> 3) * BGW + bi) * 8;
          auto poll_off = [&](int i) -> unsigned {
            return xbase + (unsigned)((i / NT) * (32 / 8) * BGW + (i % NT) * 16) * 8;
          };
          constexpr int PLN = PL * NT;  // loads per lane: PL chunks x NT utterances
          u32x4 hv[PLN];
          unsigned spins = 0;
          // When the grid fills the chip, retries re-load only the chunks whose tags were stale,
          // with a shorter back-off (s_sleep 2 instead of 6): less L2 poll traffic per retry and
          // a finer retry period (same box, alternating: c3 12.15 -> 11.77 and 12.19 -> 11.98
          // ms/step; at c2's 128 workgroups full sweeps with s_sleep 6 stay 1 % faster).  A/B
          // bit 28: full re-loads with s_sleep 6 at every size; bit 30: s_sleep 1
          const bool partial = (int)gridDim.x >= 256 && !(DMODE(a) & (1 << 28));
#pragma unroll
          for (int i = 0; i < PLN; ++i) hv[i] = u32x4{tag ^ 1u, 0u, tag ^ 1u, 0u};  // stale: first sweep loads all
          while (true) {
#pragma unroll
            for (int i = 0; i < PLN; ++i)
              if (!partial || !tags_ok(hv[i], tag, true, true)) hv[i] = ld_sc1_b128(xr, poll_off(i) * sizeof(short));
            // step s-1's dropout keep bits, drawn while the first poll's loads are in flight
            // (drawn before them, at the end of step s-1, they delayed the poll's issue; with the
            // io-first MFMAs: c3 12.06 -> 11.92, c2 4.95 -> 4.72 ms/step).  A/B bit 27: the old place
            if (late_bits && spins == 0 && tid < NC8) dbl[((s - 1) & 1) * NC8 + tid] = drop_bits(s - 1, tid);
            bool ok = true;
#pragma unroll
            for (int i = 0; i < PLN; ++i) ok &= tags_ok(hv[i], tag, true, true);
            if (__all(ok)) break;
            if (++spins > SPIN_LIMIT) {
              if (lane == 0) { atomicExch(a.err, 1); abort_flag = 1; }
              break;
            }
            // a longer back-off thins the L2 poll traffic (3.27 -> 3.20 us/step at B = 256);
            // bit 18: the previous s_sleep(2)
            if (partial && (DMODE(a) & (1 << 30))) __builtin_amdgcn_s_sleep(1);
            else if (partial || (DMODE(a) & 262144)) __builtin_amdgcn_s_sleep(2);
            else __builtin_amdgcn_s_sleep(6);
          }
          LSTAMP(1);
          RTS(8 + wave);
#pragma unroll
          for (int i = 0; i < PLN; ++i)
            *reinterpret_cast<u32x4*>(hb + (16 * (i % NT) + bi) * ROWB + swz(bi, (wave * PL + i / NT) * 4 + q) * 16) = hv[i];
        }
        if (wave < 8) LWSTAMP();  // (stamp slots 8 .. 15)
        __syncthreads();  // h image of step s complete; gx ring slot s & 1 landed
        LSTAMP(2);
        if (abort_flag) break;
        // gx of step s+1 right behind the barrier (it lands before barrier s+1)
        IOSTAMP(2);
        // gx of step s+1: right behind the barrier, or behind the io wave's publish of step s,
        // off its barrier -> publish path (the DMA issue stalls ~1,000 ticks there) but in the
        // pollers' window.  Same box, in the step: at 64 active workgroups (c2) the late DMA
        // takes the forward 1.004 -> 0.962 ms per launch, at 128 (c5) and 256 (c3) it costs
        // (1.016 -> 1.030, 1.266 -> 1.482): by grid size; bit 17 flips the choice (A/B)
        if (IO && (PURE_IO || !late_dma_s)) io_load(s + 1);
        if (PURE_IO && s > 0) io_store(s - 1);  // (out ring slot s-1 & 1 complete at barrier s)
        IOSTAMP(3);
        if constexpr (!ZP || MT == 0) read_gx();  // (ZP: inside the first k-batch below)
        // The io waves' MFMAs at priority 1: the io wave of each SIMD finishes its MFMAs first
        // and its cell update (VALU / transcendental) overlaps the poller's MFMAs, instead of both
        // waves' cells following both MFMA streams (same box, alternating: c3 12.06 -> 11.99,
        // c2 4.95 -> 4.79 ms/step).  A/B bits: 25 off; 26 the pollers first instead (no gain)
        // (AS: the pollers, owning most tiles, go first)
        const bool first = AS ? !IO : IO ? !(DMODE(a) & (1 << 25)) : (DMODE(a) & (1 << 26)) != 0;
        if (first) __builtin_amdgcn_s_setprio(1);
        // k-chunks in the order KR .. NKC-1, 0 .. KR-1: the chunks whose A-fragments live in LDS
        // first, their fragment reads (and ZP's z-row read) issued with the first batch's h
        // reads right behind the barrier, where one LDS round trip is exposed anyway -- read
        // inside the chain they had one or two MFMAs of cover each
        constexpr int KLA = KLF > 0 ? KLF : 1;
        bf16x8 wl[MTA][KLA];
        bf16x8 zf[NT];
#pragma unroll
        for (int k0 = 0; k0 < NKC; k0 += HB) {
          bf16x8 hfrag[HB][NT];
#pragma unroll
          for (int i = 0; i < HB; ++i)
#pragma unroll
            for (int n = 0; n < NT; ++n)
              hfrag[i][n] = *reinterpret_cast<const bf16x8*>(hb + (16 * n + bi) * ROWB + swz(bi, ((k0 + i + KR) % NKC) * 4 + q) * 16);
          if (k0 == 0) {
#pragma unroll
            for (int t = 0; t < MT; ++t)
#pragma unroll
              for (int j = 0; j < KLF; ++j) wl[t][j] = wlds[((m0 + t) * KLF + j) * 64 + lane];
            if constexpr (ZP) {
#pragma unroll
              for (int n = 0; n < NT; ++n)
                zf[n] = *reinterpret_cast<const bf16x8*>(zr + ((s & 1) * BGW + 16 * n + bi) * 32 + 8 * q);
            }
          }
          __builtin_amdgcn_sched_barrier(0);  // the batch's reads issue before its MFMAs
          if constexpr (ZP) {
            if (k0 == 0) {
#pragma unroll
              for (int t = 0; t < MT; ++t)
#pragma unroll
                for (int n = 0; n < NT; ++n) {
                  const f32x4 r = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wz[t], zf[n], bz4[t], 0, 0, 0);
#pragma unroll
                  for (int g4 = 0; g4 < 4; ++g4) gxv[t][n][g4] = r[g4];
                }
            }
          }
#pragma unroll
          for (int i = 0; i < HB; ++i) {
            const int kc = (k0 + i + KR) % NKC;
#pragma unroll
            for (int t = 0; t < MT; ++t) {
              const bf16x8 wf = kc < KR ? wreg[t][kc < KR ? kc : 0] : wl[t][kc >= KR ? kc - KR : 0];
#pragma unroll
              for (int n = 0; n < NT; ++n)
                acc[t][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, hfrag[i][n], acc[t][n], 0, 0, 0);
            }
          }
        }
        // The cell reads the accumulators right behind the chain.  With one M-tile per wave (the
        // 12-wave form at NT = 1, and the retired equal-shares TPW-1 form) hipcc (ROCm 7.2) put the
        // gx conversions INSIDE the chain -- writing the B-fragment registers of the MFMA just
        // issued -- and read the last MFMA's accumulator 3 wait states after it: a share of the
        // lanes lost their gx term (tools/dbg_fwd_err.py: the wrong pre-activations equal h W^T
        // exactly).  The chain now ends here, padded, and the fp16 gx words are converted only in
        // the cell, behind this barrier.
        __builtin_amdgcn_sched_barrier(0);
        if (MT > 0) asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        if (first) __builtin_amdgcn_s_setprio(0);
        LSTAMP(3);
        IOSTAMP(4);
      }
      // cell update: lane (utt bi, q) owns unit 4m + q of each of its tiles
      float hvals[MTA][NT], gates[MTA][NT][4];
#pragma unroll
      for (int n = 0; n < NT; ++n)
#pragma unroll
        for (int t = 0; t < MT; ++t) {
          float gi[4];
#pragma unroll
          for (int g4 = 0; g4 < 4; ++g4) gi[g4] = ZP ? gxv[t][n][g4] : h2f(gxh[t][n][g4]);
          const float ig = sigmoid_fast(acc[t][n][0] + gi[0]);
          const float fg = sigmoid_fast(acc[t][n][1] + gi[1]);
          const float gg = tanh_fast(acc[t][n][2] + gi[2]);
          const float og = sigmoid_fast(acc[t][n][3] + gi[3]);
          c[t][n] = valid[n] ? fg * c[t][n] + ig * gg : 0.f;
          hvals[t][n] = valid[n] ? og * tanh_fast(c[t][n]) : 0.f;
          gates[t][n][0] = ig; gates[t][n][1] = fg; gates[t][n][2] = gg; gates[t][n][3] = og;
        }
      if (DBG && !(DMODE(a) & (1 << 23))) {  // diagnostics: cell math done (slot 5)
        __builtin_amdgcn_sched_barrier(0);
        LSTAMP(5);
        __builtin_amdgcn_sched_barrier(0);
      }
      if (s + 1 < T) {
        // publish h_t: granule = 4 consecutive units (lanes q = 0..3) of one utterance
        const unsigned tag = step_tag_lg(s, nlg);
        unsigned long long gr[MTA][NT];
#pragma unroll
        for (int n = 0; n < NT; ++n)
#pragma unroll
          for (int t = 0; t < MT; ++t) {
            // units 4m+1..3 of lane (bi, 0) sit in lanes bi + 16, 32, 48: VALU permlane swaps
            // (lane row 0 of each result) instead of three LDS-routed ds_bpermute round trips
            const unsigned hu = __float_as_uint(hvals[t][n]);
            const unsigned x1 = __builtin_amdgcn_permlane16_swap(hu, hu, false, false)[1];  // row0 <- row1
            const unsigned x2 = __builtin_amdgcn_permlane32_swap(hu, hu, false, false)[1];  // row0 <- row2
            const unsigned x3 = __builtin_amdgcn_permlane32_swap(x1, x1, false, false)[1];  // row0 <- row3
            const float h1 = __uint_as_float(x1), h2 = __uint_as_float(x2), h3 = __uint_as_float(x3);
            gr[t][n] = pack_bf16(hvals[t][n], h1, h2, h3, tag);
          }
        if (AS && q == 0) {
          if constexpr (MT == 2) {
            // the poller's two tiles are units 8 w .. 8 w + 7: adjacent granules, one 16-byte store
            // per utterance (consecutive publish stores reach the consumers ~120 ns apart: see the
            // BPTT's publish)
            const int u0 = j0 + 4 * m0;
#pragma unroll
            for (int n = 0; n < NT; ++n) {
              const u32x4 v = {(unsigned)gr[0][n], (unsigned)(gr[0][n] >> 32), (unsigned)gr[1][n], (unsigned)(gr[1][n] >> 32)};
              const unsigned cell = (unsigned)((s & nmask) * xslot) + ((u0 >> 3) * BGW + 16 * n + bi) * 8 + (u0 & 7);
              if (same_xcd) __builtin_amdgcn_raw_buffer_store_b128(v, xr, cell * sizeof(short), 0, 0);
              else st_sc1_b128(xr, cell * sizeof(short), v);
            }
          } else {  // one 8-byte granule per tile
#pragma unroll
            for (int n = 0; n < NT; ++n)
#pragma unroll
              for (int t = 0; t < MT; ++t) {
                const int u0 = j0 + 4 * (m0 + t);
                publish(xr, ((unsigned)((s & nmask) * xslot) + ((u0 >> 3) * BGW + 16 * n + bi) * 8 + (u0 & 7)) * sizeof(short),
                        gr[t][n], same_xcd);
              }
          }
        } else if (q == 0) {
          // (equal shares: NT = 1, static_assert at the top)
          const int u0 = j0 + 4 * TPW * wave;  // the wave's first unit
          const unsigned cell = (unsigned)((s & nmask) * xslot) + ((u0 >> 3) * 16 + bi) * 8 + (u0 & 7);
          if constexpr (TPW == 2) {
            const u32x4 v = {(unsigned)gr[0][0], (unsigned)(gr[0][0] >> 32), (unsigned)gr[1][0], (unsigned)(gr[1][0] >> 32)};
            if (same_xcd) __builtin_amdgcn_raw_buffer_store_b128(v, xr, cell * sizeof(short), 0, 0);
            else st_sc1_b128(xr, cell * sizeof(short), v);
          } else {
            publish(xr, cell * sizeof(short), gr[0][0], same_xcd);
          }
        }
      }
      LSTAMP(4);
      RTS(wave);
      IOSTAMP(5);
      if (!IO && (DMODE(a) & (1 << 23))) {  // diagnostics: the publish stores' ack latency
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        LSTAMP(5);
      }
      // Behind the publish, off the hand-off's path: the io waves store step s-1's saved
      // activations (right after the barrier they delayed the io waves' own publish: 4.2 vs
      // 3.7 us/step at B = 256; round 4, same box: behind every wave's publish 3.19 vs 3.19,
      // from registers right after the barrier 3.35 vs 3.19 us/step); every wave puts step s's
      // into the out ring (gates as fp16).
      if (IO && !PURE_IO && late_dma_s) io_load(s + 1);  // (slot s+1 & 1 was last read before barrier s)
      if (IO && !PURE_IO && s > 0) io_store(s - 1);
      IOSTAMP(6);
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        char* ob = outr + ((s & 1) * BGW + 16 * n + bi) * OUB;
        unsigned short* og = reinterpret_cast<unsigned short*>(ob);
        float* of = reinterpret_cast<float*>(ob + 8 * HJ);
#pragma unroll
        for (int t = 0; t < MT; ++t) {
          const int u = 4 * (m0 + t) + q;
          og[u] = f2h(gates[t][n][0]); og[HJ + u] = f2h(gates[t][n][1]);
          og[2 * HJ + u] = f2h(gates[t][n][2]); og[3 * HJ + u] = f2h(gates[t][n][3]);
          of[u] = c[t][n]; of[HJ + u] = hvals[t][n];
        }
      }
      LSTAMP(6);
      // the pollers draw step s's dropout keep bits before polling for step s+1 (drawn by io
      // waves 4-5 instead, they held the barrier: 1.38 vs 1.33 ms per forward launch at c3;
      // spread over all four poller waves, one Philox call each: no change, 11.82 vs 11.73 ms
      // per step).  Tried and reverted as well (same box, c3 12.60-12.73 -> 12.78-12.92 ms):
      // io waves waiting for their gx LDS-DMA alone by a counted vmcnt (their stores left in
      // flight across the barrier), and the BPTT's dG stores moved behind the next poll.
      if (!IO && want_drop && tid < NC8 && (!late_bits || s + 1 == T)) dbl[(s & 1) * NC8 + tid] = drop_bits(s, tid);
      LSTAMP(7);
    }
    __syncthreads();
    if (IO) io_store(T - 1);
  };
  if (io) run(std::true_type{});
  else run(std::false_type{});
  LSTAMP_FLUSH();
  RTS_FLUSH();
}

// ---------------------------------------------------------------------------------------
// backward (BPTT), reduce-scatter form
// ---------------------------------------------------------------------------------------
// F8: the fp8 mode's e4m3 dG copy + amax (a separate instantiation: the bf16 path's registers
// stay as they are)
// DYB: dY (the layer output's gradient) arrives as bf16 (a.dYb) instead of fp32 (a.Y): half the
// bytes in the cell-input stream (and in the producers' epilogues)
template <int TPW, int NKC, int OCC, bool F8 = false, bool DYB = false, bool DBG = false>  // HJ = 32 * TPW, H = 32 * NKC
__global__ __launch_bounds__(512, OCC) void lstm_bwd_wide_kernel(LstmArgs a) {
  constexpr int HJ = 32 * TPW;
  constexpr int H = NKC * 32;
  constexpr int NJ = H / HJ;                  // workgroups per (dir, group) = producers = consumers
  constexpr int NTW = NKC / 4;                // N-tiles (16 units) per wave: 8 waves cover H
  constexpr int KC = 4 * HJ / 32;             // k-chunks of the own-dG operand (K = 4 HJ)
  // k-chunks whose B-fragments live in LDS (VGPR budget at TPW 2; TPW 1 keeps all of them in
  // registers).  The <2,16> build reloads ~11 spilled dwords once, in the prologue (not in the
  // step loop: checked in the ISA)
  constexpr int KLB = TPW == 1 ? 0 : KC / 4;
  constexpr int KR = KC - KLB;
  // k-chunks per batch of fragment reads: all 4 at TPW 1 (c2 BPTT 0.999 -> 0.966 ms, c5 1.10 ->
  // 1.04); at TPW 2 one per batch, the compiler's own order (4: c3 1.230 -> 1.249 ms)
  constexpr int BKB = TPW == 1 ? 4 : 1;
  constexpr int ROWB = 4 * HJ * 2;            // bytes of one A-image row
  constexpr int AIMG = 16 * ROWB;
  constexpr int NPL = NJ / 8;                 // producers per lane in the reduce-scatter
  constexpr int CPG = 2 * HJ / 64;            // (unit, utterance-half) combos per 8-lane group
  static_assert(NPL >= 1 && CPG >= 1 && NPL * CPG == 2, "two 16-byte partial loads per lane");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  LSTAMP_DECL;
  RTS_DECL;
  char* aimg = smem;  // [2][16][4HJ] bf16 own dG, gate-major k = g*HJ + u, swizzled slots
  bf16x8* wlds = reinterpret_cast<bf16x8*>(smem + 2 * AIMG);  // [wave][NTW][KLB][lane]
  // cell inputs of a step, staged: [2][16 utt][ gates fp16 4*HJ (+16 B) | c_{t-1} HJ | dy HJ (fp32, +32 B) ]
  constexpr int CG_B = 4 * HJ * 2 + 16;       // gate row bytes (padded: 8 utterances -> 32 banks)
  constexpr int CF_B = HJ * 4 + 32;           // c / dy row bytes (padded likewise)
  // dy row bytes: bf16 rows padded so a row of the staged block is an odd multiple of 4 dwords
  // past a bank period (HJ 32: 528 B, HJ 64: 976 B) -- 8 utterances' reads of one unit hit 8
  // distinct banks (16 B of padding left HJ 32 at 512 B per row: 8-way conflicts, c2 +6 %)
  constexpr int CD_B = DYB ? HJ * 2 + 32 : CF_B;
  static_assert(((CG_B + CF_B + CD_B) / 4) % 8 == 4 || ((CG_B + CF_B + CD_B) / 4) % 64 == 20,
                "conflict-free staged rows");
  constexpr int CUTT = CG_B + CF_B + CD_B;    // bytes per utterance
  char* cst = smem + 2 * AIMG + (size_t)8 * NTW * KLB * 64 * 16;  // [2][16][CUTT]
  __shared__ int abort_flag;

  // group slots padded to a multiple of 8 (idle slots exit at once): members gid + k * gstride
  // then share one XCD under round-robin dispatch at every batch size (B = 32: 4 groups)
  const int ngroups = 2 * a.NB, gstride = (ngroups + 7) & ~7;
  const int gid = blockIdx.x % gstride, js = blockIdx.x / gstride;
  if (gid >= ngroups) return;
  const int dir = gid / a.NB, grp = gid % a.NB;
  const int T = a.T, j0 = js * HJ;
  const int tid = threadIdx.x, lane = tid & 63;
  // exchange slots in use: 2 (every member of a group is producer and consumer of every other,
  // so a slot is rewritten only after all its readers have loaded it); bit 24: all NSLOT
  const int nlg = (DMODE(a) & (1 << 24)) ? 2 : 1, nmask = (1 << nlg) - 1;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: role branches stay scalar
  const float* W = dir ? a.W1 : a.W0;
  const int bi = lane & 15, q = lane >> 4;

  // resident B-fragments: tile nt -> global units n = (wave*NTW + nt)*16 + col;
  // B[k][n] = W_hh[g*H + j0 + u][n], k = g*HJ + u
  bf16x8 wreg[NTW][KR];
  static_assert(KLB > 0 || KR == KC, "");
#pragma unroll
  for (int nt = 0; nt < NTW; ++nt) {
    const int n = (wave * NTW + nt) * 16 + bi;
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      bf16x8 v;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int k = kc * 32 + 8 * q + e;
        v[e] = f2bf(W[(size_t)((k / HJ) * H + j0 + (k % HJ)) * H + n]);
      }
      if (kc < KR) wreg[nt][kc < KR ? kc : 0] = v;
      else wlds[((wave * NTW + nt) * KLB + (kc - KR)) * 64 + lane] = v;
    }
  }
  __shared__ int placement;
  const bool same_xcd = group_on_one_xcd(a.xtab + gid * NJ, NJ, js, &placement) &&
                        !(DMODE(a) & 32768);  // bit 15: force write-through hand-offs
  if (tid == 0) abort_flag = 0;
  if (DBG && DPTR(a) && (DMODE(a) & 8) && tid == 0) a.dbg[blockIdx.x] = same_xcd ? 1 : 2;  // (placement)
  __syncthreads();

  // exchange: [slot][consumer][producer][HJ units][16 utterances] bf16
  const size_t xslot = (size_t)NJ * NJ * HJ * 16;
  short* xb = reinterpret_cast<short*>(a.xbuf) + (size_t)(dir * a.NB + grp) * NSLOT * xslot;
  auto xr = make_rsrc(xb, (unsigned)(NSLOT * xslot * sizeof(short)));

  // reduce-scatter / cell role: 8-lane group gq, lane pg; combo cb -> (unit uc, half);
  // after the reduce lane pg holds utterance half*8 + pg
  // The reduce-scatter needs no selects: every lane keeps its low register slots and adds the
  // partner's high ones (half-row mirror, then xor 2, xor 1), so lane pg of a group must hold the
  // partial of utterance e in slot e ^ rs_perm(pg).  The producer arranges that for free: its
  // A-image row of utterance u is row u ^ rs_perm(js / NPL), so the MFMA writes the partials of the
  // consumer lane that loads them in that lane's order.  After the reduce lane pg holds utterance
  // half * 8 + rs_perm(pg).
  auto rs_perm = [](int g) { return g ^ ((g & 4) ? 3 : 0); };
  const int arow = rs_perm(js / NPL);  // A-image row of utterance u: u ^ arow
  const int gq = tid >> 3, pg = lane & 7;
  int uc[CPG], cu[CPG];
  bool bv[CPG];
#pragma unroll
  for (int ci = 0; ci < CPG; ++ci) {
    const int cb = gq * CPG + ci;
    uc[ci] = cb >> 1;
    cu[ci] = (cb & 1) * 8 + rs_perm(pg);
    bv[ci] = grp * BG + cu[ci] < a.B;
  }
  // Cell inputs (gates, c_{t-1}, dy) of step s_ in 16-byte row chunks -- whole 128-byte lines
  // per wave instruction instead of each lane's scattered words -- into registers, two steps
  // ahead; staged to LDS one step ahead (cst slot s_ & 1).  Chunks: 16 x 4 x HJ/8 gate chunks
  // (8 fp16 units), 16 x HJ/4 c chunks, 16 x HJ/4 dy chunks (4 fp32 units).
  // dy chunks: fp32 4 units or bf16 8 units; chunks past NCH (bf16 dy) are dummies -- loaded from a
  // valid address (unconditional loads, below) and never staged
  constexpr int NGC = 16 * 4 * HJ / 8, NFC = 16 * HJ / 4, NDC = DYB ? 16 * HJ / 8 : NFC;
  constexpr int NCH = NGC + NFC + NDC;
  constexpr int CPT = (NCH + 511) / 512;      // chunks per thread
  static_assert(DYB || NCH % 512 == 0, "whole chunks per thread");
  static_assert(NGC % 64 == 0 && NFC % 64 == 0 && NDC % 64 == 0, "chunk kinds change at whole waves");
  const size_t gbase = (size_t)grp * BG * T;  // first row (utterance grp*16, t = 0) of the group
  const auto rG = make_rsrc(reinterpret_cast<const unsigned short*>(a.G) + gbase * 8 * H, 0xffffffffu);
  const auto rC = make_rsrc(a.Cs + gbase * 2 * H, 0xffffffffu);
  const auto rY = DYB ? make_rsrc(a.dYb + gbase * 2 * H, 0xffffffffu) : make_rsrc(a.Y + gbase * 2 * H, 0xffffffffu);
  u32x4 creg[CPT];
  auto chunk_lds = [&](int c) -> int {  // LDS byte offset of chunk c within a slot
    if (c < NGC) {
      const int u = c / (4 * HJ / 8), k = c % (4 * HJ / 8);
      return u * CUTT + k * 16;
    }
    const int f = c - NGC;
    if (f < NFC) {
      const int u = f / (HJ / 4), k = f % (HJ / 4);
      return u * CUTT + CG_B + k * 16;
    }
    const int r = f - NFC, upr = DYB ? HJ / 8 : HJ / 4;  // dy chunks per utterance row
    return (r / upr) * CUTT + CG_B + CF_B + (r % upr) * 16;
  };
  // Unconditional loads (steps past the end and padded utterances read a clamped valid row and
  // are never consumed): a conditional load would make the compiler merge the register values
  // and wait for the loads right here, an HBM round trip on the hand-off's path.  The chunk
  // kind changes at multiples of 64 chunks, so it -- and the buffer resource -- is wave-uniform.
  const int ulast = a.B - 1 - grp * BG;  // last valid utterance of the group (>= 0)
  auto load_cell = [&](int s_) {
    const int sc = s_ < T ? s_ : T - 1;
    const int t_ = dir ? sc : T - 1 - sc;
    const int tp_ = dir ? t_ + 1 : t_ - 1;
    const int tpc = tp_ < 0 ? 0 : (tp_ >= T ? T - 1 : tp_);
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int cw0 = wave * 64 + 512 * i;  // first chunk of this wave (uniform)
      const int cw = cw0 < NCH ? cw0 : 0;   // dummy chunks (bf16 dy) re-load chunk 0's row
      const int c = cw + lane;
      const bool isg = cw < NGC, ydy = cw - NGC >= NFC;  // uniform: gates, c, dy chunks
      const int r = c - NGC - (ydy ? NFC : 0);
      const int ug = c / (4 * HJ / 8), k = c % (4 * HJ / 8), g = k / (HJ / 8), ugu = (k % (HJ / 8)) * 8;
      const int upr = (ydy && DYB) ? HJ / 8 : HJ / 4, epr = (ydy && DYB) ? 8 : 4;  // chunks / units
      const int uf = r / upr, ufu = (r % upr) * epr;
      const int u = min(isg ? ug : uf, ulast);
      const unsigned og = ((unsigned)(u * T + t_) * 8 * H + dir * 4 * H + g * H + j0 + ugu) * 2u;
      const unsigned of = ((unsigned)(u * T + (ydy ? t_ : tpc)) * 2 * H + dir * H + j0 + ufu) *
                          ((ydy && DYB) ? 2u : 4u);
      creg[i] = __builtin_bit_cast(
          u32x4, __builtin_amdgcn_raw_buffer_load_b128(isg ? rG : (ydy ? rY : rC), isg ? og : of, 0, NT_AUX));
    }
  };
  auto stage_cell = [&](int s_) {  // registers -> LDS slot s_ & 1 (visible after the next barrier)
    char* dst = cst + (s_ & 1) * 16 * CUTT;
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      if (wave * 64 + 512 * i < NCH)  // (uniform) dummies are not staged
        *reinterpret_cast<u32x4*>(dst + chunk_lds(wave * 64 + 512 * i + lane)) = creg[i];
    }
  };
  float dc[CPG], cc[CPG], bsum[CPG][4];
#pragma unroll
  for (int ci = 0; ci < CPG; ++ci) {
    dc[ci] = 0.f;
    cc[ci] = 0.f;
    bsum[ci][0] = bsum[ci][1] = bsum[ci][2] = bsum[ci][3] = 0.f;
    if (bv[ci]) {
      const int t0 = dir ? 0 : T - 1;
      cc[ci] = a.Cs[((size_t)(grp * BG + cu[ci]) * T + t0) * 2 * H + dir * H + j0 + uc[ci]];
    }
  }
#pragma unroll
  for (int i = 0; i < CPT; ++i) creg[i] = u32x4{0u, 0u, 0u, 0u};
  load_cell(0);
  stage_cell(0);   // (waits for the loads: prologue only)
  load_cell(1);
  __syncthreads();
  float g8max = 0.f;                                        // fp8 mode: running max |dG|
  const float g8s = (F8 && a.dG8) ? *a.g8scale : 0.f;       // fp8 mode: this step's dG scale

  auto step = [&](int s) -> bool {
    LSTAMP(0);
    // this step's cell inputs (staged in LDS last step) into registers before the poll, so
    // the LDS latency hides behind the hand-off wait
    float xi[CPG], xf[CPG], xgg[CPG], xo[CPG], xcp[CPG], xdy[CPG];
#pragma unroll
    for (int ci = 0; ci < CPG; ++ci) {
      const char* cu_row = cst + (s & 1) * 16 * CUTT + cu[ci] * CUTT;
      const unsigned short* xg = reinterpret_cast<const unsigned short*>(cu_row) + uc[ci];
      xi[ci] = h2f(xg[0]); xf[ci] = h2f(xg[HJ]); xgg[ci] = h2f(xg[2 * HJ]); xo[ci] = h2f(xg[3 * HJ]);
      xcp[ci] = reinterpret_cast<const float*>(cu_row + CG_B)[uc[ci]];
      if constexpr (DYB)
        xdy[ci] = __uint_as_float((unsigned)reinterpret_cast<const unsigned short*>(cu_row + CG_B + CF_B)[uc[ci]] << 16);
      else
        xdy[ci] = reinterpret_cast<const float*>(cu_row + CG_B + CF_B)[uc[ci]];
    }
    float dh[CPG];
#pragma unroll
    for (int ci = 0; ci < CPG; ++ci) dh[ci] = 0.f;
    // The cell's factors that do not depend on the incoming dh (everything but three FMAs and
    // four products per cell) are formed while the first poll's loads are in flight, off the
    // hand-off's critical path:  dcs = dc + dht * fA,  dG = dcs * (f0, f1, f2) and dht * f3,
    // dc' = dcs * fF  (padded utterances: all zero, so their dG and dc stay 0)
    float fA[CPG], fF[CPG], f0[CPG], f1[CPG], f2[CPG], f3[CPG];
    auto factors = [&]() {
#pragma unroll
      for (int ci = 0; ci < CPG; ++ci) {
        const float cpv = s + 1 < T ? xcp[ci] : 0.f;  // c_{t-1}; none at the sequence start
        const float tc = tanh_fast(cc[ci]);
        const bool v = bv[ci];
        fA[ci] = v ? xo[ci] * (1.f - tc * tc) : 0.f;
        fF[ci] = v ? xf[ci] : 0.f;
        f0[ci] = v ? xgg[ci] * xi[ci] * (1.f - xi[ci]) : 0.f;
        f1[ci] = v ? cpv * xf[ci] * (1.f - xf[ci]) : 0.f;
        f2[ci] = v ? xi[ci] * (1.f - xgg[ci] * xgg[ci]) : 0.f;
        f3[ci] = v ? tc * xo[ci] * (1.f - xo[ci]) : 0.f;
        cc[ci] = xcp[ci];  // c_{t-1} is the next step's c_t
      }
    };
    u32x4 pv[CPG][NPL];
    // Step s+1's cell inputs are staged to LDS while the first poll's loads are in flight
    // instead of after the poll (same box, c3: BPTT 1.292 / 1.283 -> 1.269 / 1.260 ms per
    // launch; bit 19 restores the old place).  (The pollers at priority 2 while they poll, so a
    // wave still polling gets the issue slots before its SIMD partner's post-poll work: 1.337 /
    // 1.304, dropped.)
    const bool early_stage = !(DMODE(a) & (1 << 19)) && s > 0;
    if (s > 0) {
      const unsigned tag = step_tag_lg(s - 1, nlg);
      const size_t sb = (size_t)((s - 1) & nmask) * xslot + (size_t)js * NJ * HJ * 16;
      unsigned spins = 0;
      auto sweep = [&]() {
#pragma unroll
        for (int ci = 0; ci < CPG; ++ci)
#pragma unroll
          for (int i = 0; i < NPL; ++i) {
            const int p = pg * NPL + i;
            const size_t off = sb + ((size_t)p * HJ + uc[ci]) * 16 + (cu[ci] >> 3) * 8;
            pv[ci][i] = ld_sc1_b128(xr, (unsigned)(off * sizeof(short)));
          }
      };
      // (re-loading only the stale partial tiles measured no faster here: full sweeps)
      sweep();
      factors();
      if (early_stage) stage_cell(s + 1);
      while (true) {
        bool ok = true;
#pragma unroll
        for (int ci = 0; ci < CPG; ++ci)
#pragma unroll
          for (int i = 0; i < NPL; ++i) ok &= tags_ok(pv[ci][i], tag, true, true);
        if (__all(ok)) break;
        if (++spins > SPIN_LIMIT) {
          if (lane == 0) { atomicExch(a.err, 1); abort_flag = 1; }
          break;
        }
        // BPTT: a shorter back-off (3.03 -> 2.97 us/step at B = 256); bit 18: s_sleep(2)
        if (DMODE(a) & 262144) __builtin_amdgcn_s_sleep(2);
        else __builtin_amdgcn_s_sleep(1);
        sweep();
      }
    } else {
      factors();
    }
    LSTAMP(1);
    // per-wave stamps (slots 8 + wave): poll done, or (debug bit 21) reduce done, (bit 22) the
    // cell's A-image writes issued, just before the step barrier
    if (!(DMODE(a) & (3 << 21))) LWSTAMP();
    RTS(8 + wave);
    // step s+1's inputs (landed: the poll waited for every earlier load) to LDS, and step
    // s+2's loads issued right behind this step's hand-off -- one program point per step, so
    // the loaded registers need no merge (and no wait for the loads)
    if (!early_stage) stage_cell(s + 1);
    LSTAMP(5);
    // At full-chip grids the prefetch is issued after the barrier, so no wave's HBM loads sit in
    // the CU's memory queue ahead of a later wave's poll loads (same box: c3 12.11 -> 11.99
    // ms/step; at c2's 128 workgroups right after the poll stays 2 % faster).  A/B bit 16:
    // right after the poll at every size.  (The io waves' stores issued before their MFMAs
    // instead of behind their publish, in the forward: c3 12.11 -> 12.48, c2 4.97 -> 5.62.)
    const bool late_pf = (int)gridDim.x >= 256 && !(DMODE(a) & (1 << 16));
    if (!late_pf) load_cell(s + 2);
    LSTAMP(6);
    if (s > 0) {
#pragma unroll
      for (int ci = 0; ci < CPG; ++ci) {
        float v[8];
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          v[2 * d] = __uint_as_float(pv[ci][0][d] << 16);
          v[2 * d + 1] = __uint_as_float(pv[ci][0][d] & 0xffff0000u);
        }
#pragma unroll
        for (int i = 1; i < NPL; ++i)
#pragma unroll
          for (int d = 0; d < 4; ++d) {
            v[2 * d] += __uint_as_float(pv[ci][i][d] << 16);
            v[2 * d + 1] += __uint_as_float(pv[ci][i][d] & 0xffff0000u);
          }
        // reduce-scatter over the 8 lanes: DPP row_half_mirror, quad_perm xor 2, quad_perm xor 1
        float w4[4], w2[2];
#pragma unroll
        for (int k = 0; k < 4; ++k) w4[k] = v[k] + dpp_f<0x141>(v[k + 4]);
#pragma unroll
        for (int k = 0; k < 2; ++k) w2[k] = w4[k] + dpp_f<0x4E>(w4[k + 2]);
        dh[ci] = w2[0] + dpp_f<0xB1>(w2[1]);
      }
    }
    LSTAMP(2);
    if (DMODE(a) & (1 << 21)) LWSTAMP();
    // cell BPTT -> dG of (utterance cu, unit uc), into the A-image of this step
    char* ab = aimg + (s & 1) * AIMG;
#pragma unroll
    for (int ci = 0; ci < CPG; ++ci) {
      const float dht = xdy[ci] + dh[ci];
      const float dcs = __builtin_fmaf(dht, fA[ci], dc[ci]);
      dc[ci] = dcs * fF[ci];
      const float dg[4] = {dcs * f0[ci], dcs * f1[ci], dcs * f2[ci], dht * f3[ci]};
      const int u = uc[ci], r = cu[ci] ^ arow;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int k = g * HJ + u;
        *reinterpret_cast<short*>(ab + r * ROWB + swz(r, k >> 3) * 16 + (k & 7) * 2) = f2bf(dg[g]);
      }
#pragma unroll
      for (int g = 0; g < 4; ++g) bsum[ci][g] += dg[g];
    }
    if (DMODE(a) & (1 << 22)) LWSTAMP();
    __syncthreads();  // double-buffered A-image: one barrier per step
    LSTAMP(7);
    // (issued before the barrier instead, by each wave as it arrives: c3 BPTT 1.13 -> 1.23 ms)
    if (late_pf) load_cell(s + 2);
    LSTAMP(3);
    if (abort_flag) return false;
    if (s + 1 < T) {
      const unsigned tag = step_tag_lg(s, nlg);
      const size_t sb = (size_t)(s & nmask) * xslot;
      // The wave's NTW tiles in halves, each half's products then its publish: the first half's
      // stores go out while the second half's MFMAs run, so the last tile's store no longer
      // queues behind all the others (consecutive publish stores of a wave become visible ~120 ns
      // apart: realtime stamps, tools/lstm_handoff.py --bwd; the step barrier waits for the
      // consumer wave whose tile landed last).  The A-fragments are read once per half.
      constexpr int NGRP = bptt_groups<TPW>();
      static_assert(NTW % NGRP == 0 && (TPW != 1 || (NTW / NGRP) % 2 == 0), "tile groups");
      constexpr int TPH = NTW / NGRP;
      // TPW 1 (one batch of BKB = KC k-chunks): the step's A-fragments are read once, for both
      // tile groups (the VGPRs are there at TPW 1), instead of once per group
      constexpr bool AONCE = BKB == KC && NGRP > 1;
      bf16x8 afr_all[AONCE ? KC : 1];
      if constexpr (AONCE) {
#pragma unroll
        for (int i = 0; i < KC; ++i)
          afr_all[i] = *reinterpret_cast<const bf16x8*>(ab + bi * ROWB + swz(bi, i * 4 + q) * 16);
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int hf = 0; hf < NGRP; ++hf) {
        f32x4 acc[TPH];
#pragma unroll
        for (int t = 0; t < TPH; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
        // The A-fragments of a batch of BKB k-chunks are read before its MFMAs: left to itself the
        // compiler issued each read one k-chunk ahead and waited for it (5 exposed LDS round trips
        // per step at TPW 1).  (Round 5, measured and dropped: per-wave LDS flags instead of this
        // barrier, each wave multiplying the k-chunks whose cell outputs were ready -- BPTT 1.36 ->
        // 1.72 ms per launch at c3, 0.97 -> 1.19 at c2; profiles/r05_bptt_flags_stamps.txt)
#pragma unroll
        for (int k0 = 0; k0 < KC; k0 += BKB) {
          bf16x8 afr[BKB];
          if constexpr (AONCE) {
#pragma unroll
            for (int i = 0; i < BKB; ++i) afr[i] = afr_all[k0 + i];
          } else {
#pragma unroll
            for (int i = 0; i < BKB; ++i)
              afr[i] = *reinterpret_cast<const bf16x8*>(ab + bi * ROWB + swz(bi, (k0 + i) * 4 + q) * 16);
            __builtin_amdgcn_sched_barrier(0);  // the batch's reads issue before its MFMAs
          }
#pragma unroll
          for (int i = 0; i < BKB; ++i) {
            const int kc = k0 + i;
#pragma unroll
            for (int t = 0; t < TPH; ++t) {
              const int nt = hf * TPH + t;
              const bf16x8 wf = kc < KR ? wreg[nt][kc < KR ? kc : 0] : wlds[((wave * NTW + nt) * KLB + (kc - KR)) * 64 + lane];
              acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[i], wf, acc[t], 0, 0, 0);
            }
          }
        }
        // TPW 1: two tiles per 16-byte store.  acc[t] gives lane (bi, q) utterances 4q .. 4q+3 of
        // unit nt*16 + bi; a row swap (v_permlane16_swap, q <-> q^1) of tiles A, B leaves lanes of
        // even q with A's utterances 8(q>>1) .. +7 and odd q with B's -- the consumer's 16-byte
        // chunk of one unit, so the exchange layout and the polls are unchanged.  Same box,
        // alternating (profiles/ab/r05_bwd_pair_publish.txt): c2 BPTT 0.968 -> 0.940 ms per
        // launch; at TPW 2 (c3) 1.312 -> 1.33 (the pair still lands 160 ns apart): one store per tile.
        if constexpr (TPW != 1) {
#pragma unroll
          for (int t = 0; t < TPH; ++t) {
            // acc[t][r]: partial dh of utterance 4q + r, unit n
            const int n = (wave * NTW + hf * TPH + t) * 16 + bi;
            const int cons = n / HJ, un = n % HJ;
            const size_t off = sb + (((size_t)cons * NJ + js) * HJ + un) * 16 + 4 * q;
            publish(xr, (unsigned)(off * sizeof(short)),
                    pack_bf16(acc[t][0], acc[t][1], acc[t][2], acc[t][3], tag), same_xcd);
          }
        } else {
#pragma unroll
          for (int pr = 0; pr < TPH / 2; ++pr) {
            const int ta = 2 * pr, tb = 2 * pr + 1;
            const unsigned long long ga = pack_bf16(acc[ta][0], acc[ta][1], acc[ta][2], acc[ta][3], tag);
            const unsigned long long gb = pack_bf16(acc[tb][0], acc[tb][1], acc[tb][2], acc[tb][3], tag);
            const auto lo = __builtin_amdgcn_permlane16_swap((unsigned)ga, (unsigned)gb, false, false);
            const auto hi = __builtin_amdgcn_permlane16_swap((unsigned)(ga >> 32), (unsigned)(gb >> 32), false, false);
            const u32x4 v = {lo[0], hi[0], lo[1], hi[1]};
            const int n = (wave * NTW + hf * TPH + ((q & 1) ? tb : ta)) * 16 + bi;
            const int cons = n / HJ, un = n % HJ;
            const size_t off = sb + (((size_t)cons * NJ + js) * HJ + un) * 16 + 8 * (q >> 1);
            if (same_xcd) __builtin_amdgcn_raw_buffer_store_b128(v, xr, (unsigned)(off * sizeof(short)), 0, 0);
            else st_sc1_b128(xr, (unsigned)(off * sizeof(short)), v);
          }
        }
      }
    }
    LSTAMP(4);
    RTS(wave);
    // dG of this step for the weight-gradient GEMMs: 16-byte rows out of the A-image
    // (fp8 mode: also the e4m3 copy for the fp8 dgrad, and the running max |dG|)
    if (!(DMODE(a) & 1)) {
      constexpr int NSL = 16 * 4 * HJ / 8;  // 16-byte slots
      const int t = dir ? s : T - 1 - s;
      for (int sl = tid; sl < NSL; sl += 512) {
        const int r = sl / (4 * HJ / 8), kslot = sl % (4 * HJ / 8);
        const int b = grp * BG + (r ^ arow);
        if (b >= a.B) continue;
        const int k = kslot * 8, g = k / HJ, u = k % HJ;
        const u32x4 v = *reinterpret_cast<const u32x4*>(ab + r * ROWB + swz(r, kslot) * 16);
        const size_t o = ((size_t)b * T + t) * 8 * H + dir * 4 * H + g * H + j0 + u;
        // G is fp16 here: dG goes to dGb (NULL in fp8 mode when every reader takes the e4m3 copy)
        if (!F8 || a.dGb) *reinterpret_cast<u32x4*>(a.dGb + o) = v;
        if constexpr (F8) {
          float f[8];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            f[2 * e] = __uint_as_float(v[e] << 16);
            f[2 * e + 1] = __uint_as_float(v[e] & 0xffff0000u);
          }
#pragma unroll
          for (int e = 0; e < 8; ++e) g8max = fmaxf(g8max, fabsf(f[e]));
          if (a.dG8)
            *reinterpret_cast<u32x2*>(a.dG8 + o) =
                u32x2{pack4_fp8(f[0] * g8s, f[1] * g8s, f[2] * g8s, f[3] * g8s),
                      pack4_fp8(f[4] * g8s, f[5] * g8s, f[6] * g8s, f[7] * g8s)};
        }
      }
    }
    return true;
  };
  stagger_start(gid, DMODE(a));
  for (int s = 0; s < T; ++s)
    if (!step(s)) break;
  LSTAMP_FLUSH();
  RTS_FLUSH();
  if constexpr (F8) {  // this launch's max |dG| (the next step's fp8 scale): one atomic per wave
    float m = g8max;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    if (lane == 0) atomicMax(a.g8amax, __float_as_uint(m));  // |x| >= 0: float order = uint order
  }
  // bias gradients of this workgroup's units: the lane sums over its steps, then over the
  // group's 16 utterances (8 lanes x CPG halves; fixed order), one row per batch group
  if (a.dbias) {
    float bs[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      float v = bsum[0][g];
#pragma unroll
      for (int ci = 1; ci < CPG; ++ci) v += bsum[ci][g];  // CPG 2: both halves share the unit
      v += __shfl_xor(v, 1, 64);
      v += __shfl_xor(v, 2, 64);
      v += __shfl_xor(v, 4, 64);
      if (CPG == 1) v += __shfl_xor(v, 8, 64);  // CPG 1: the two halves are adjacent groups
      bs[g] = v;
    }
    if (pg == 0 && (CPG == 2 || (gq & 1) == 0)) {
#pragma unroll
      for (int g = 0; g < 4; ++g)
        a.dbias[(size_t)grp * 8 * H + dir * 4 * H + g * H + j0 + uc[0]] = bs[g];
    }
  }
}

// ---------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------
struct WidePlan {
  int tpw, nkc, NB, NJ, HJ;
  int nt;    // forward: N-tiles (16 utterances each) per workgroup
  bool w12;  // forward: the 12-wave form (lstm_fwd_wide_kernel W12)
  size_t lds, xbytes, xtab_off;
  bool ok;
};

int wide_cus() {
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    cus = 256;
  return cus;
}

size_t wide_lds(int H, int hj, bool fwd, int nt = 1) {
  const size_t bgw = (size_t)BG * nt;
  if (fwd)
    return 2 * bgw * H * 2 + 2 * bgw * (4 * hj + 8) * 2 +  // h image, gx ring
           2 * bgw * (4 * hj * 2 + 2 * hj * 4 + 16) +      // out ring
           (size_t)8 * (hj / 32) * FWD_KLF * 64 * 16 +     // + the LDS-resident A-fragments
           2 * (bgw * hj / 8) * 4;                         // + dropout keep bits
  return (size_t)2 * 16 * 4 * hj * 2 +
         (size_t)8 * (H / 128) * (hj == 32 ? 0 : hj / 32) * 64 * 16 +  // + LDS B-fragments (KLB)
         (size_t)2 * 16 * ((4 * hj * 2 + 16) + 2 * (hj * 4 + 32));  // + staged cell inputs
}

// mode bits (mlvae_lstm_set_debug_mode, A/B): 9 -- past B = 64 the forward takes the 32-utterance
// form (NT = 2) instead of TPW 2 (16 utterances x 64 units per workgroup); 11 -- the TPW-1 forward
// in 8 waves (4 pollers with two M-tiles each + 4 io waves) instead of 12.
// Same box, in the step (profiles/ab/r06_fwd_w12.txt): c2 forward 0.84 -> 0.74 ms per launch with
// 12 waves (step 4.10 -> 3.90 ms); at c3 NT = 2 runs 1.25 ms in 12 waves, 1.48 in 8, against TPW 2's
// 1.17 -- its h image is twice as large, and every MFMA wave reads all of it (256 vs 192 KB of LDS
// reads per CU per step)
WidePlan wide_plan(int B, int H, bool fwd, int mode = 0) {
  WidePlan p{};
  p.ok = false;
  p.nt = 1;
  p.w12 = false;
  if (H != 512) return p;  // the decoder's H (c2-c5); other H run the batch-group kernels
  p.nkc = H / 32;
  p.NB = (B + BG - 1) / BG;
  const int cus = wide_cus();
  // forward past one HJ = 32 launch of 16-utterance groups (B > 64): 32 utterances x 32 units per
  // workgroup, tile-less io waves (lstm_fwd_wide_kernel NT = 2)
  if (fwd && (mode & 512) && 2 * p.NB * (H / 32) > cus) {
    const int nb2 = (B + 2 * BG - 1) / (2 * BG);
    if (2 * nb2 * (H / 32) <= cus) {
      p.nt = 2; p.tpw = 1; p.HJ = 32; p.NJ = H / 32; p.NB = nb2; p.ok = true;
    }
  }
  if (!p.ok)
  // HJ = 32 units per workgroup where the grid fits the chip (it beat HJ = 64 at every shard,
  // round 2: 7.94 vs 8.02, 5.58 vs 6.34, 4.72 vs 5.68 ms/step); HJ = 64 at B = 256
  for (int tpw = 1; tpw <= 2; ++tpw) {
    if (fwd && tpw * p.nkc * 4 > 128) break;   // resident A-fragments <= 128 VGPRs
    p.NB = (B + BG - 1) / BG;
    const int hj = 32 * tpw, nj = H / hj;
    if (!fwd && (nj < 8 || nj % 8)) continue;   // reduce-scatter: NJ multiple of 8
    // one workgroup per CU.  (Two co-resident HJ = 32 workgroups per CU at B = 256, whose step
    // chains could overlap each other's hand-off waits, measured slower: forward 1.70 vs 1.33 ms,
    // BPTT 1.93 vs 1.38 ms per launch -- 16 producers per consumer and twice the pollers per CU
    // lengthened the hand-off, 2,896 -> 4,320 ticks)
    if (2 * p.NB * nj <= cus) {
      p.tpw = tpw; p.HJ = hj; p.NJ = nj; p.ok = true;
      break;
    }
  }
  if (!p.ok) return p;
  // (TPW 2 in 12 waves -- 2 M-tiles per MFMA wave -- spills 65-117 VGPRs past the 168 a wave has
  // at three per SIMD: W_hh's resident 12 k-chunks alone take 96, and LDS has room for no more.
  // The BPTT in 12 waves at TPW 1 -- 8 compute waves, 4 io waves staging the cell inputs and
  // storing dG -- measured slower, 0.86 -> 0.97 ms per launch at c2 with the io traffic right
  // behind the step barrier (it queued ahead of the compute waves' publish), 1.0 ms with it held
  // until every compute wave had polled (the barrier then waited for the io waves).)
  if (fwd && p.tpw == 1) p.w12 = !(mode & 2048);
  p.lds = wide_lds(H, p.HJ, fwd, p.nt);
  if (fwd) p.xbytes = (size_t)2 * p.NB * NSLOT * BG * p.nt * H * 2;
  else p.xbytes = (size_t)2 * p.NB * NSLOT * p.NJ * p.NJ * p.HJ * 16 * 2;
  if (p.lds < (size_t)MIN_LDS) p.lds = MIN_LDS;  // one recurrence workgroup per CU (residency)
  p.xtab_off = p.xbytes;                          // + [groups][NJ] XCC ids (placement check)
  p.xbytes += (size_t)2 * p.NB * p.NJ * sizeof(unsigned);
  return p;
}

template <int TPW, int NKC, int OCC>
int launch_wide(bool fwd, const LstmArgs& a, const WidePlan& p, hipStream_t s) {
  // DBG instances (phase stamps) only while a stamp buffer is set; the BPTT's only for the bf16
  // train step's form (bf16 dY, no fp8 copy)
  const bool dbg = a.dbg != nullptr;
  // the forward at TPW 1 always takes the asymmetric split (the equal-shares form, debug bit 8
  // through round 5, was retired in round 6); TPW 2 keeps equal shares
  constexpr bool AS1 = TPW == 1;
  const bool zp = a.Zb != nullptr;          // fused layer-0 projection (checked: no DBG with it)
  auto k = (fwd && p.w12)
               ? (p.nt == 2 ? (dbg ? lstm_fwd_wide_kernel<1, NKC, OCC, true, true, false, 2, true>
                                   : zp ? lstm_fwd_wide_kernel<1, NKC, OCC, false, true, true, 2, true>
                                        : lstm_fwd_wide_kernel<1, NKC, OCC, false, true, false, 2, true>)
                            : (dbg ? lstm_fwd_wide_kernel<1, NKC, OCC, true, true, false, 1, true>
                                   : zp ? lstm_fwd_wide_kernel<1, NKC, OCC, false, true, true, 1, true>
                                        : lstm_fwd_wide_kernel<1, NKC, OCC, false, true, false, 1, true>))
         : (fwd && p.nt == 2)
               ? (dbg ? lstm_fwd_wide_kernel<1, NKC, OCC, true, true, false, 2>
                      : zp ? lstm_fwd_wide_kernel<1, NKC, OCC, false, true, true, 2>
                           : lstm_fwd_wide_kernel<1, NKC, OCC, false, true, false, 2>)
         : fwd ? (dbg ? lstm_fwd_wide_kernel<TPW, NKC, OCC, true, AS1>
                      : zp ? lstm_fwd_wide_kernel<TPW, NKC, OCC, false, AS1, true>
                           : lstm_fwd_wide_kernel<TPW, NKC, OCC, false, AS1>)
               : (a.g8amax ? (a.dYb ? lstm_bwd_wide_kernel<TPW, NKC, OCC, true, true>
                                    : lstm_bwd_wide_kernel<TPW, NKC, OCC, true, false>)
                           : (a.dYb ? (dbg ? lstm_bwd_wide_kernel<TPW, NKC, OCC, false, true, true>
                                           : lstm_bwd_wide_kernel<TPW, NKC, OCC, false, true>)
                                    : (dbg ? lstm_bwd_wide_kernel<TPW, NKC, OCC, false, false, true>
                                           : lstm_bwd_wide_kernel<TPW, NKC, OCC, false>)));
  if (hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)p.lds) != hipSuccess) {
    mlvae_set_error("lstm_wide: cannot reserve %zu B LDS", p.lds);
    return 2;
  }
  k<<<dim3(((2 * p.NB + 7) & ~7) * p.NJ), (fwd && p.w12) ? 768 : 512, p.lds, s>>>(a);
  MLVAE_CHECK_LAUNCH();
  return 0;
}

}  // namespace

// (the forward's 32-utterance groups: one descriptor spans 2 BG utterances' rows)
bool lstm_wide_t_ok(int T, int H) {
  return (size_t)2 * BG * T * 8 * H * 2 <= 0xffffffffull && (size_t)2 * BG * T * 2 * H * 4 <= 0xffffffffull;
}

int lstm_wide_workgroups(int B, int H, bool fwd) {
  WidePlan p = wide_plan(B, H, fwd);
  if (!p.ok) return 0;
  return 2 * p.NB * p.NJ;
}

size_t lstm_wide_xbytes(int B, int H, bool fwd) {
  WidePlan p = wide_plan(B, H, fwd), q = wide_plan(B, H, fwd, 512);  // either form past B = 64
  if (!p.ok) return 0;
  return p.xbytes > q.xbytes ? p.xbytes : q.xbytes;
}

int lstm_wide_run(bool fwd, int B, int T, int H, const float* W0, const float* W1, float* G,
                  float* Cs, float* Y, void* xbuf, size_t xbytes, int* err, hipStream_t st,
                  unsigned short* yb, unsigned short* dgb, float* dbias, unsigned short* ydb,
                  unsigned long long dseed, unsigned long long doff, float dp,
                  unsigned long long* dbg, int dbg_mode, const WideFp8& f8, const unsigned short* dyb,
                  const WideZ& wz) {
  WidePlan p = wide_plan(B, H, fwd, dbg_mode);
  if (!p.ok) return -1;
  // the kernels address a batch group's rows through one buffer descriptor (32-bit offsets)
  if (!lstm_wide_t_ok(T, H)) {
    mlvae_set_error("lstm_wide: T=%d too long for the wide kernels' 32-bit batch-group addressing at H=%d "
                    "(mlvae_lstm_gates_fp16_t(B, T, H, prec) = 0: pass fp32 gates)", T, H);
    return 1;
  }
  if (!xbuf || xbytes < p.xbytes || !err) {
    mlvae_set_error("lstm_wide: exchange workspace too small (need %zu B)", p.xbytes);
    return 1;
  }
  LstmArgs a{};
  a.ndir = 2;
  a.B = B; a.T = T; a.H = H; a.NB = p.NB; a.NJ = p.NJ; a.HJ = p.HJ; a.Kp = H; a.K4p = 4 * H;
  a.W0 = W0; a.W1 = W1; a.G = G; a.Cs = Cs; a.Y = Y; a.xbuf = xbuf; a.err = err;
  a.dbg = dbg; a.dbg_mode = dbg_mode; a.xcd_local = 0; a.Yb = yb; a.dGb = dgb;
  a.dbias = dbias; a.Ydb = ydb; a.dseed = dseed; a.doff = doff; a.dkeep = 1.f - dp;
  a.Y8 = f8.y8; a.x8scale = f8.x8scale; a.dG8 = f8.dg8; a.g8scale = f8.g8scale; a.g8amax = f8.g8amax;
  a.dYb = fwd ? nullptr : dyb;
  if (wz.zb && dbg) a.dbg = dbg = nullptr;  // (no stamp instance of the fused-z forward: run it unstamped)
  if (wz.zb) {
    if (!fwd || !wz.w0 || !wz.w1 || !wz.b[0] || !wz.b[1] || !wz.b[2] || !wz.b[3] ||
        wz.ldz < 32 || wz.ldz % 8 || ((uintptr_t)wz.zb % 16)) {
      mlvae_set_error("lstm_wide: the fused z projection needs the forward, "
                      "both W_ih and all four biases, a 16-byte aligned z with ldz >= 32, ldz %% 8 == 0");
      return 1;
    }
    a.Zb = wz.zb; a.ldz = wz.ldz; a.Wz0 = wz.w0; a.Wz1 = wz.w1; a.yb_prev = wz.yb_prev;
    for (int i = 0; i < 4; ++i) a.bz[i] = wz.b[i];
  }
  if (a.Y8 && (!fwd || !(a.x8scale > 0.f) || !(dp >= 0.f && dp < 1.f))) {
    mlvae_set_error("lstm_wide: the e4m3 dropout(h) output needs the forward, a positive scale and 0 <= p < 1");
    return 1;
  }
  if (a.dG8 && (!a.g8scale || !a.g8amax)) {
    mlvae_set_error("lstm_wide: the fp8 dG copy needs its scale and amax words");
    return 1;
  }
  a.dscale = dp < 1.f ? 1.f / (1.f - dp) : 0.f;
  a.xtab = reinterpret_cast<unsigned*>(static_cast<char*>(xbuf) + p.xtab_off);
  // zero fill = a stale tag in every granule (and an empty placement table)
  if (hipMemsetAsync(xbuf, 0, p.xbytes, st) != hipSuccess) {
    mlvae_set_error("lstm_wide: memset failed");
    return 2;
  }
  return p.tpw == 2 ? launch_wide<2, 16, 2>(fwd, a, p, st) : launch_wide<1, 16, 2>(fwd, a, p, st);
}
