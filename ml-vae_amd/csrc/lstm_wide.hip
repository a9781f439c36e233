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

namespace {

constexpr int WW = 8;  // waves per workgroup

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
template <int TPW, int NKC>  // M-tiles per wave (HJ = 32 * TPW), k-chunks of 32 (H = 32 * NKC)
__global__ __launch_bounds__(512) void lstm_fwd_wide_kernel(LstmArgs a) {
  constexpr int HJ = WW * TPW * 4;
  constexpr int H = NKC * 32;
  constexpr int PL = NKC / 4;                 // poll loads (k-chunks) per lane, waves 0-3
  constexpr int ROWB = H * 2;                 // bytes of one h-image row (bf16)
  constexpr int HIMG = 16 * ROWB;
  constexpr int GXU = 4 * HJ + 4;             // gx ring floats per utterance: [gate][unit] + 16 B
  constexpr int OUU = 6 * HJ + 4;             // out ring floats per utterance: [i f g o c h][unit]
  constexpr int KLF = 2;                      // k-chunks whose A-fragments live in LDS (VGPR budget)
  constexpr int KR = NKC - KLF;               // ... and in registers
  constexpr int NQ = 16 * 4 * HJ / 4;         // 16-byte quads of gx / gates per step
  constexpr int QPT = NQ / 256;               // quads per io thread
  static_assert(NQ % 256 == 0, "io split");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* himg = smem;                                        // [2][16][ROWB], swizzled slots
  float* gxr = reinterpret_cast<float*>(smem + 2 * HIMG);   // [2][16][GXU]
  float* outr = gxr + 2 * 16 * GXU;                          // [2][16][OUU]
  bf16x8* wlds = reinterpret_cast<bf16x8*>(outr + 2 * 16 * OUU);  // [wave][TPW][KLF][lane]
  __shared__ int abort_flag;

  const int ngroups = 2 * a.NB;
  const int gid = blockIdx.x % ngroups, js = blockIdx.x / ngroups;
  const int dir = gid / a.NB, grp = gid % a.NB;
  const int T = a.T, j0 = js * HJ;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float* W = dir ? a.W1 : a.W0;
  const int bi = lane & 15, q = lane >> 4;
  const int bglob = grp * BG + bi;
  const bool valid = bglob < a.B;

  // resident A-fragments: tile m = wave*TPW + t, row r = bi -> unit 4m + (r >> 2), gate r & 3;
  // k-chunks [0, KR) in registers, [KR, NKC) in LDS (lane-linear, conflict-free 16-B reads)
  bf16x8 wreg[TPW][KR];
#pragma unroll
  for (int t = 0; t < TPW; ++t) {
    const int m = wave * TPW + t;
    const float* wrow = W + (size_t)((bi & 3) * H + j0 + 4 * m + (bi >> 2)) * H;
#pragma unroll
    for (int kc = 0; kc < NKC; ++kc) {
      const f32x4 w0 = *reinterpret_cast<const f32x4*>(wrow + kc * 32 + 8 * q);
      const f32x4 w1 = *reinterpret_cast<const f32x4*>(wrow + kc * 32 + 8 * q + 4);
      bf16x8 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) { v[e] = f2bf(w0[e]); v[4 + e] = f2bf(w1[e]); }
      if (kc < KR) wreg[t][kc < KR ? kc : 0] = v;
      else wlds[((wave * TPW + t) * KLF + (kc - KR)) * 64 + lane] = v;
    }
  }
  // group members are blocks gid + k * ngroups: one XCD under round-robin dispatch whenever
  // ngroups % 8 == 0; verified at run time, never assumed (lstm_common.h group_on_one_xcd)
  __shared__ int placement;
  const bool same_xcd = group_on_one_xcd(a.xtab + gid * a.NJ, a.NJ, js, &placement) &&
                        !(a.dbg_mode & 32768);  // bit 15: force write-through hand-offs
  if (tid == 0) abort_flag = 0;

  const size_t xslot = (size_t)BG * H;  // elements per exchange slot
  short* xb = reinterpret_cast<short*>(a.xbuf) + (size_t)(dir * a.NB + grp) * NSLOT * xslot;
  auto xr = make_rsrc(xb, (unsigned)(NSLOT * xslot * sizeof(short)));

  // ---- io role (waves 4-7).  The input projection of a step goes HBM -> LDS by LDS-DMA
  // (buffer_load ... lds: 1 KB per wave-instruction = one utterance's 4 gates x 64 units, no
  // registers); the saved activations go LDS -> registers -> 16-byte stores.
  const int iot = tid - 256;
  const bool io = wave >= 4;
  typedef __attribute__((address_space(3))) void* lds_ptr_t;
  auto io_load = [&](int s_) {  // input projection of step s_ into gx ring slot s_ & 1
    if (s_ >= T || (s_ > 0 && (a.dbg_mode & 8192))) return;  // bit 13: timing without the loads
    const int t_ = dir ? T - 1 - s_ : s_;
    constexpr int UPW = 16 / 4;  // utterances per io wave
#pragma unroll
    for (int i = 0; i < UPW; ++i) {
      const int u = (wave - 4) * UPW + i, b = grp * BG + u;
      if (b >= a.B) continue;
      // lane l < HJ -> gate l / (HJ/4), units 4 (l % (HJ/4)) .. + 3: 4 gates x HJ units in one
      // instruction (HJ = 64: all lanes; HJ = 32: lanes 0-31)
      const float* base = a.G + (size_t)b * T * 8 * H;
      const auto rs = make_rsrc(base, (unsigned)((size_t)T * 8 * H * sizeof(float)));
      const int g = lane / (HJ / 4), uu = (lane % (HJ / 4)) * 4;
      const unsigned off = (unsigned)((((size_t)t_ * 8 * H + dir * 4 * H + g * H + j0 + uu)) * sizeof(float));
      float* dst = gxr + (s_ & 1) * 16 * GXU + u * GXU;
      if (lane < HJ) __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)dst, 16, off, 0, 0, 0);
    }
  };
  auto io_store = [&](int s_) {  // saved activations of step s_ from out ring slot s_ & 1
    if (s_ < 0 || s_ >= T || (a.dbg_mode & 1)) return;
    const int t_ = dir ? T - 1 - s_ : s_;
    const float* src = outr + (s_ & 1) * 16 * OUU;
    // activated gates: NQ quads
#pragma unroll
    for (int i = 0; i < QPT; ++i) {
      const int qi = iot + 256 * i, row = qi / (HJ / 4), uu = (qi % (HJ / 4)) * 4;
      const int u = row >> 2, g = row & 3, b = grp * BG + u;
      if (b < a.B)
        *reinterpret_cast<f32x4*>(a.G + ((size_t)b * T + t_) * 8 * H + dir * 4 * H + g * H + j0 + uu) =
            *reinterpret_cast<const f32x4*>(src + u * OUU + g * HJ + uu);
    }
    // c, h (fp32) and h (bf16): 16 x HJ each
    constexpr int NQ2 = 16 * HJ / 4;
    for (int qi = iot; qi < NQ2; qi += 256) {
      const int u = qi / (HJ / 4), uu = (qi % (HJ / 4)) * 4, b = grp * BG + u;
      if (b >= a.B) continue;
      const size_t o = ((size_t)b * T + t_) * 2 * H + dir * H + j0 + uu;
      const f32x4 cv = *reinterpret_cast<const f32x4*>(src + u * OUU + 4 * HJ + uu);
      const f32x4 hv = *reinterpret_cast<const f32x4*>(src + u * OUU + 5 * HJ + uu);
      *reinterpret_cast<f32x4*>(a.Cs + o) = cv;
      *reinterpret_cast<f32x4*>(a.Y + o) = hv;
      if (a.Yb)
        *reinterpret_cast<bf16x4*>(a.Yb + o) = bf16x4{f2bf(hv[0]), f2bf(hv[1]), f2bf(hv[2]), f2bf(hv[3])};
    }
  };
  if (io) {
    io_load(0);
    io_load(1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();

  float c[TPW];
#pragma unroll
  for (int t = 0; t < TPW; ++t) c[t] = 0.f;
  for (int s = 0; s < T; ++s) {
    STAMP(0);
    f32x4 acc[TPW];
#pragma unroll
    for (int t = 0; t < TPW; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    char* hb = himg + (s & 1) * HIMG;
    if (s > 0) {
      if (io) {
        if (!(a.dbg_mode & 16384))  // bit 14: timing without the wait
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's gx(s) LDS-DMA has landed
      } else {
        // poll = load: this wave's quarter of h_{t-1} (PL k-chunks), retried until every
        // granule carries step s-1's tag; then into the swizzled LDS image
        const unsigned tag = step_tag(s - 1);
        const unsigned ebase = (unsigned)(((s - 1) & (NSLOT - 1)) * xslot) + bi * H + wave * PL * 32 + 8 * q;
        u32x4 hv[PL];
        unsigned spins = 0;
        while (true) {
#pragma unroll
          for (int i = 0; i < PL; ++i) hv[i] = ld_sc1_b128(xr, (ebase + i * 32) * sizeof(short));
          bool ok = true;
#pragma unroll
          for (int i = 0; i < PL; ++i) ok &= tags_ok(hv[i], tag, true, true);
          if (__all(ok)) break;
          if (++spins > SPIN_LIMIT) {
            if (lane == 0) { atomicExch(a.err, 1); abort_flag = 1; }
            break;
          }
          __builtin_amdgcn_s_sleep(2);
        }
        STAMP(1);
#pragma unroll
        for (int i = 0; i < PL; ++i)
          *reinterpret_cast<u32x4*>(hb + bi * ROWB + swz(bi, (wave * PL + i) * 4 + q) * 16) = hv[i];
      }
      __syncthreads();  // h image of step s complete; gx ring slot s & 1 landed
      STAMP(2);
      if (abort_flag) break;
      if (io) {
        // the step's HBM traffic right behind the barrier, while the pollers run MFMAs: it
        // drains before their next poll (issued behind the publish it delayed the hand-off:
        // 4.3 vs 3.x us/step at B = 256).  gx of step s+1 lands before barrier s+1.
        io_load(s + 1);
        io_store(s - 1);
      }
#pragma unroll
      for (int kc = 0; kc < NKC; ++kc) {
        const bf16x8 hfrag = *reinterpret_cast<const bf16x8*>(hb + bi * ROWB + swz(bi, kc * 4 + q) * 16);
#pragma unroll
        for (int t = 0; t < TPW; ++t) {
          const bf16x8 wf = kc < KR ? wreg[t][kc < KR ? kc : 0]
                                    : wlds[((wave * TPW + t) * KLF + (kc - KR)) * 64 + lane];
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, hfrag, acc[t], 0, 0, 0);
        }
      }
      STAMP(3);
    }
    // cell update: lane (utt bi, q) owns unit 4m + q of each of its tiles
    const float* gx = gxr + (s & 1) * 16 * GXU + bi * GXU;
    float* ob = outr + (s & 1) * 16 * OUU + bi * OUU;
    float hvals[TPW];
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
      const int u = 4 * (wave * TPW + t) + q;
      const float ig = sigmoid_fast(acc[t][0] + gx[u]);
      const float fg = sigmoid_fast(acc[t][1] + gx[HJ + u]);
      const float gg = tanh_fast(acc[t][2] + gx[2 * HJ + u]);
      const float og = sigmoid_fast(acc[t][3] + gx[3 * HJ + u]);
      c[t] = valid ? fg * c[t] + ig * gg : 0.f;
      const float h = valid ? og * tanh_fast(c[t]) : 0.f;
      hvals[t] = h;
      ob[u] = ig; ob[HJ + u] = fg; ob[2 * HJ + u] = gg; ob[3 * HJ + u] = og;
      ob[4 * HJ + u] = c[t]; ob[5 * HJ + u] = h;
    }
    if (s + 1 < T) {
      // publish h_t: granule = 4 consecutive units (lanes q = 0..3) of one utterance
      const unsigned tag = step_tag(s);
      const size_t row = (size_t)(s & (NSLOT - 1)) * xslot + (size_t)bi * H + j0;
#pragma unroll
      for (int t = 0; t < TPW; ++t) {
        const float h1 = __shfl(hvals[t], lane + 16, 64);
        const float h2 = __shfl(hvals[t], lane + 32, 64);
        const float h3 = __shfl(hvals[t], lane + 48, 64);
        if (q == 0)
          publish(xr, (unsigned)((row + 4 * (wave * TPW + t)) * sizeof(short)),
                  pack_bf16(hvals[t], h1, h2, h3, tag), same_xcd);
      }
    }
    STAMP(4);
  }
  __syncthreads();
  if (io) io_store(T - 1);
}

// ---------------------------------------------------------------------------------------
// backward (BPTT), reduce-scatter form
// ---------------------------------------------------------------------------------------
template <int TPW, int NKC>  // HJ = 32 * TPW units per workgroup, H = 32 * NKC
__global__ __launch_bounds__(512) void lstm_bwd_wide_kernel(LstmArgs a) {
  constexpr int HJ = 32 * TPW;
  constexpr int H = NKC * 32;
  constexpr int NJ = H / HJ;                  // workgroups per (dir, group) = producers = consumers
  constexpr int NTW = NKC / 4;                // N-tiles (16 units) per wave: 8 waves cover H
  constexpr int KC = 4 * HJ / 32;             // k-chunks of the own-dG operand (K = 4 HJ)
  constexpr int KLB = KC / 4;                 // k-chunks whose B-fragments live in LDS (VGPR budget)
  constexpr int KR = KC - KLB;
  constexpr int ROWB = 4 * HJ * 2;            // bytes of one A-image row
  constexpr int AIMG = 16 * ROWB;
  constexpr int NPL = NJ / 8;                 // producers per lane in the reduce-scatter
  constexpr int CPG = 2 * HJ / 64;            // (unit, utterance-half) combos per 8-lane group
  static_assert(NPL >= 1 && CPG >= 1 && NPL * CPG == 2, "two 16-byte partial loads per lane");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* aimg = smem;  // [2][16][4HJ] bf16 own dG, gate-major k = g*HJ + u, swizzled slots
  bf16x8* wlds = reinterpret_cast<bf16x8*>(smem + 2 * AIMG);  // [wave][NTW][KLB][lane]
  __shared__ int abort_flag;

  const int ngroups = 2 * a.NB;
  const int gid = blockIdx.x % ngroups, js = blockIdx.x / ngroups;
  const int dir = gid / a.NB, grp = gid % a.NB;
  const int T = a.T, j0 = js * HJ;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float* W = dir ? a.W1 : a.W0;
  const int bi = lane & 15, q = lane >> 4;

  // resident B-fragments: tile nt -> global units n = (wave*NTW + nt)*16 + col;
  // B[k][n] = W_hh[g*H + j0 + u][n], k = g*HJ + u
  bf16x8 wreg[NTW][KR];
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
                        !(a.dbg_mode & 32768);  // bit 15: force write-through hand-offs
  if (tid == 0) abort_flag = 0;
  __syncthreads();

  // exchange: [slot][consumer][producer][HJ units][16 utterances] bf16
  const size_t xslot = (size_t)NJ * NJ * HJ * 16;
  short* xb = reinterpret_cast<short*>(a.xbuf) + (size_t)(dir * a.NB + grp) * NSLOT * xslot;
  auto xr = make_rsrc(xb, (unsigned)(NSLOT * xslot * sizeof(short)));

  // reduce-scatter / cell role: 8-lane group gq, lane pg; combo cb -> (unit uc, half);
  // after the reduce lane pg holds utterance half*8 + pg
  const int gq = tid >> 3, pg = lane & 7;
  int uc[CPG], cu[CPG];
  bool bv[CPG];
#pragma unroll
  for (int ci = 0; ci < CPG; ++ci) {
    const int cb = gq * CPG + ci;
    uc[ci] = cb >> 1;
    cu[ci] = (cb & 1) * 8 + pg;
    bv[ci] = grp * BG + cu[ci] < a.B;
  }
  struct CellIn { float gi, gf, gg, go, cp, dy; };
  // cell inputs through buffer loads: one 32-bit offset per cell (the group's rows are within
  // 4 GB of its base), the four gates at scalar offsets 0, H, 2H, 3H
  const size_t gbase = (size_t)grp * BG * T;  // first row (utterance grp*16, t = 0) of the group
  const auto rG = make_rsrc(a.G + gbase * 8 * H, 0xffffffffu);
  const auto rC = make_rsrc(a.Cs + gbase * 2 * H, 0xffffffffu);
  const auto rY = make_rsrc(a.Y + gbase * 2 * H, 0xffffffffu);
  auto load_cell = [&](int s_, CellIn (&c)[CPG]) {
    if (s_ >= T || (s_ > 1 && (a.dbg_mode & 2048))) return;  // bit 11: timing without the loads
    const int t_ = dir ? s_ : T - 1 - s_;
    const int tp_ = dir ? t_ + 1 : t_ - 1;
    const int tpc = tp_ < 0 ? 0 : (tp_ >= T ? T - 1 : tp_);
#pragma unroll
    for (int ci = 0; ci < CPG; ++ci) {
      if (!bv[ci]) continue;
      const unsigned r = (unsigned)(cu[ci] * T + t_), rp = (unsigned)(cu[ci] * T + tpc);
      const unsigned og = (r * 8 * H + dir * 4 * H + j0 + uc[ci]) * 4u;
      c[ci].gi = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rG, og, 0, 0));
      c[ci].gf = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rG, og, 4 * H, 0));
      c[ci].gg = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rG, og, 8 * H, 0));
      c[ci].go = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rG, og, 12 * H, 0));
      const unsigned oc = (dir * H + j0 + uc[ci]) * 4u;
      c[ci].cp = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rC, rp * 2 * H * 4 + oc, 0, 0));
      c[ci].dy = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rY, r * 2 * H * 4 + oc, 0, 0));
    }
  };
  float dc[CPG], cc[CPG];
#pragma unroll
  for (int ci = 0; ci < CPG; ++ci) {
    dc[ci] = 0.f;
    cc[ci] = 0.f;
    if (bv[ci]) {
      const int t0 = dir ? 0 : T - 1;
      cc[ci] = a.Cs[((size_t)(grp * BG + cu[ci]) * T + t0) * 2 * H + dir * H + j0 + uc[ci]];
    }
  }
  CellIn cin[2][CPG];
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int ci = 0; ci < CPG; ++ci) cin[r][ci] = CellIn{0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  load_cell(0, cin[0]);

  auto step = [&](int s, CellIn (&cur)[CPG], CellIn (&fill)[CPG]) -> bool {
    STAMP(0);
    float dh[CPG];
#pragma unroll
    for (int ci = 0; ci < CPG; ++ci) dh[ci] = 0.f;
    if (s == 0) load_cell(1, fill);
    if (s > 0) {
      const unsigned tag = step_tag(s - 1);
      const size_t sb = (size_t)((s - 1) & (NSLOT - 1)) * xslot + (size_t)js * NJ * HJ * 16;
      u32x4 pv[CPG][NPL];
      unsigned spins = 0;
      while (true) {
#pragma unroll
        for (int ci = 0; ci < CPG; ++ci)
#pragma unroll
          for (int i = 0; i < NPL; ++i) {
            const int p = pg * NPL + i;
            const size_t off = sb + ((size_t)p * HJ + uc[ci]) * 16 + (cu[ci] >> 3) * 8;
            pv[ci][i] = ld_sc1_b128(xr, (unsigned)(off * sizeof(short)));
          }
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
        __builtin_amdgcn_s_sleep(2);
      }
      STAMP(1);
      load_cell(s + 1, fill);  // next step's cell inputs, right behind this step's hand-off
      const bool b2 = pg & 4, b1 = pg & 2, b0 = pg & 1;
#pragma unroll
      for (int ci = 0; ci < CPG; ++ci) {
        float v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = 0.f;
#pragma unroll
        for (int i = 0; i < NPL; ++i)
#pragma unroll
          for (int d = 0; d < 4; ++d) {
            v[2 * d] += __uint_as_float(pv[ci][i][d] << 16);
            v[2 * d + 1] += __uint_as_float(pv[ci][i][d] & 0xffff0000u);
          }
        // reduce-scatter over the 8 lanes (DPP row_shr/shl:4, quad_perm xor 2 / xor 1)
        float w4[4], w2[2];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float send = b2 ? v[k] : v[k + 4], keep = b2 ? v[k + 4] : v[k];
          const float from_lo = dpp_f<0x114>(send);
          const float from_hi = dpp_f<0x104>(send);
          w4[k] = keep + (b2 ? from_lo : from_hi);
        }
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const float send = b1 ? w4[k] : w4[k + 2], keep = b1 ? w4[k + 2] : w4[k];
          w2[k] = keep + dpp_f<0x4E>(send);
        }
        const float send = b0 ? w2[0] : w2[1], keep = b0 ? w2[1] : w2[0];
        dh[ci] = keep + dpp_f<0xB1>(send);
      }
    }
    STAMP(2);
    // cell BPTT -> dG of (utterance cu, unit uc), into the A-image of this step
    char* ab = aimg + (s & 1) * AIMG;
#pragma unroll
    for (int ci = 0; ci < CPG; ++ci) {
      float d0 = 0.f, d1 = 0.f, d2 = 0.f, d3 = 0.f;
      const CellIn& x = cur[ci];
      const float cpv = s + 1 < T ? x.cp : 0.f;  // c_{t-1}; none at the sequence start
      if (bv[ci]) {
        const float dht = x.dy + dh[ci];
        const float tc = tanh_fast(cc[ci]);
        const float d_o = dht * tc;
        const float dcs = dc[ci] + dht * x.go * (1.f - tc * tc);
        dc[ci] = dcs * x.gf;
        d0 = dcs * x.gg * x.gi * (1.f - x.gi);
        d1 = dcs * cpv * x.gf * (1.f - x.gf);
        d2 = dcs * x.gi * (1.f - x.gg * x.gg);
        d3 = d_o * x.go * (1.f - x.go);
      }
      cc[ci] = x.cp;  // c_{t-1} is the next step's c_t
      const int u = uc[ci], r = cu[ci];
      const float dg[4] = {d0, d1, d2, d3};
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int k = g * HJ + u;
        *reinterpret_cast<short*>(ab + r * ROWB + swz(r, k >> 3) * 16 + (k & 7) * 2) = f2bf(dg[g]);
      }
    }
    __syncthreads();  // double-buffered A-image: one barrier per step
    STAMP(3);
    if (abort_flag) return false;
    if (s + 1 < T) {
      f32x4 acc[NTW];
#pragma unroll
      for (int nt = 0; nt < NTW; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) {
        const bf16x8 af = *reinterpret_cast<const bf16x8*>(ab + bi * ROWB + swz(bi, kc * 4 + q) * 16);
#pragma unroll
        for (int nt = 0; nt < NTW; ++nt) {
          const bf16x8 wf = kc < KR ? wreg[nt][kc < KR ? kc : 0]
                                    : wlds[((wave * NTW + nt) * KLB + (kc - KR)) * 64 + lane];
          acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, wf, acc[nt], 0, 0, 0);
        }
      }
      const unsigned tag = step_tag(s);
      const size_t sb = (size_t)(s & (NSLOT - 1)) * xslot;
#pragma unroll
      for (int nt = 0; nt < NTW; ++nt) {
        // acc[nt][r]: partial dh of utterance 4q + r, unit n
        const int n = (wave * NTW + nt) * 16 + bi;
        const int cons = n / HJ, un = n % HJ;
        const size_t off = sb + (((size_t)cons * NJ + js) * HJ + un) * 16 + 4 * q;
        publish(xr, (unsigned)(off * sizeof(short)),
                pack_bf16(acc[nt][0], acc[nt][1], acc[nt][2], acc[nt][3], tag), same_xcd);
      }
    }
    STAMP(4);
    // dG of this step for the weight-gradient GEMMs: 16-byte rows out of the A-image
    if (!(a.dbg_mode & 1)) {
      constexpr int NSL = 16 * 4 * HJ / 8;  // 16-byte slots
      const int t = dir ? s : T - 1 - s;
      for (int sl = tid; sl < NSL; sl += 512) {
        const int r = sl / (4 * HJ / 8), kslot = sl % (4 * HJ / 8);
        const int b = grp * BG + r;
        if (b >= a.B) continue;
        const int k = kslot * 8, g = k / HJ, u = k % HJ;
        const u32x4 v = *reinterpret_cast<const u32x4*>(ab + r * ROWB + swz(r, kslot) * 16);
        const size_t o = ((size_t)b * T + t) * 8 * H + dir * 4 * H + g * H + j0 + u;
        if (a.dGb) {
          *reinterpret_cast<u32x4*>(a.dGb + o) = v;
        } else {
          float* gp = a.G + o;
#pragma unroll
          for (int d = 0; d < 4; ++d) {
            gp[2 * d] = __uint_as_float(v[d] << 16);
            gp[2 * d + 1] = __uint_as_float(v[d] & 0xffff0000u);
          }
        }
      }
    }
    return true;
  };
  for (int s = 0; s < T; s += 2) {
    if (!step(s, cin[0], cin[1])) break;
    if (s + 1 < T && !step(s + 1, cin[1], cin[0])) break;
  }
}

// ---------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------
struct WidePlan {
  int tpw, nkc, NB, NJ, HJ;
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

WidePlan wide_plan(int B, int H, bool fwd) {
  WidePlan p{};
  p.ok = false;
  if (H != 512) return p;  // the decoder's H (c2-c5); other H run the batch-group kernels
  p.nkc = H / 32;
  p.NB = (B + BG - 1) / BG;
  const int cus = wide_cus();
  for (int tpw = 1; tpw <= 2; ++tpw) {
    if (fwd && tpw * p.nkc * 4 > 128) break;   // resident A-fragments <= 128 VGPRs
    const int hj = 32 * tpw, nj = H / hj;
    if (!fwd && (nj < 8 || nj % 8)) continue;   // reduce-scatter: NJ multiple of 8
    if (2 * p.NB * nj <= cus) {
      p.tpw = tpw; p.HJ = hj; p.NJ = nj; p.ok = true;
      break;
    }
  }
  if (!p.ok) return p;
  if (fwd) {
    p.lds = (size_t)2 * 16 * H * 2 + (size_t)2 * 16 * (4 * p.HJ + 4) * 4 + (size_t)2 * 16 * (6 * p.HJ + 4) * 4 +
            (size_t)8 * p.tpw * 2 * 64 * 16;  // + the LDS-resident A-fragments (KLF = 2)
    p.xbytes = (size_t)2 * p.NB * NSLOT * BG * H * 2;
  } else {
    p.lds = (size_t)2 * 16 * 4 * p.HJ * 2 +
            (size_t)8 * (H / 128) * (p.HJ / 32) * 64 * 16;  // + LDS-resident B-fragments (KLB = KC/4)
    p.xbytes = (size_t)2 * p.NB * NSLOT * p.NJ * p.NJ * p.HJ * 16 * 2;
  }
  if (p.lds < (size_t)MIN_LDS) p.lds = MIN_LDS;  // one recurrence workgroup per CU
  p.xtab_off = p.xbytes;                          // + [groups][NJ] XCC ids (placement check)
  p.xbytes += (size_t)2 * p.NB * p.NJ * sizeof(unsigned);
  return p;
}

template <int TPW, int NKC>
int launch_wide(bool fwd, const LstmArgs& a, const WidePlan& p, hipStream_t s) {
  auto k = fwd ? lstm_fwd_wide_kernel<TPW, NKC> : lstm_bwd_wide_kernel<TPW, NKC>;
  if (hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)p.lds) != hipSuccess) {
    mlvae_set_error("lstm_wide: cannot reserve %zu B LDS", p.lds);
    return 2;
  }
  k<<<dim3(2 * p.NB * p.NJ), 512, p.lds, s>>>(a);
  MLVAE_CHECK_LAUNCH();
  return 0;
}

}  // namespace

int lstm_wide_workgroups(int B, int H, bool fwd) {
  WidePlan p = wide_plan(B, H, fwd);
  return p.ok ? 2 * p.NB * p.NJ : 0;
}

size_t lstm_wide_xbytes(int B, int H, bool fwd) {
  WidePlan p = wide_plan(B, H, fwd);
  return p.ok ? p.xbytes : 0;
}

int lstm_wide_run(bool fwd, int B, int T, int H, const float* W0, const float* W1, float* G,
                  float* Cs, float* Y, void* xbuf, size_t xbytes, int* err, hipStream_t st,
                  unsigned short* yb, unsigned short* dgb, unsigned long long* dbg, int dbg_mode) {
  WidePlan p = wide_plan(B, H, fwd);
  if (!p.ok) return -1;
  if (!xbuf || xbytes < p.xbytes || !err) {
    mlvae_set_error("lstm_wide: exchange workspace too small (need %zu B)", p.xbytes);
    return 1;
  }
  LstmArgs a{};
  a.B = B; a.T = T; a.H = H; a.NB = p.NB; a.NJ = p.NJ; a.HJ = p.HJ; a.Kp = H; a.K4p = 4 * H;
  a.W0 = W0; a.W1 = W1; a.G = G; a.Cs = Cs; a.Y = Y; a.xbuf = xbuf; a.err = err;
  a.dbg = dbg; a.dbg_mode = dbg_mode; a.xcd_local = 0; a.Yb = yb; a.dGb = dgb;
  a.xtab = reinterpret_cast<unsigned*>(static_cast<char*>(xbuf) + p.xtab_off);
  // zero fill = a stale tag in every granule (and an empty placement table)
  if (hipMemsetAsync(xbuf, 0, p.xbytes, st) != hipSuccess) {
    mlvae_set_error("lstm_wide: memset failed");
    return 2;
  }
  return p.tpw == 2 ? launch_wide<2, 16>(fwd, a, p, st) : launch_wide<1, 16>(fwd, a, p, st);
}
