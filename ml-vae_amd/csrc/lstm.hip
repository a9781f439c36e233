// Persistent bidirectional-LSTM recurrence (forward and BPTT backward) for gfx950.
//
// Reference op: nn.LSTM(z, H, L, bidirectional=True, batch_first=True), called at
// ref:src/modules/decoder.py:14-15,22 -- gate order i,f,g,o; h0 = c0 = 0; no packing
// (the reverse direction starts at the padded tail t = T-1).
//
// The input projection x W_ih^T + b_ih + b_hh is a batched MFMA GEMM (gemm.hip) done
// beforehand into G[B*T, 8H] (cols [0,4H) forward dir, [4H,8H) reverse dir).  What is left
// here is the serial part: per step, gates = G[:,t] + h_{t-1} W_hh^T, then the cell update.
//
// Decomposition (one launch per layer, both directions):
//   workgroup = (dir, batch group of 16 utterances, hidden slice of HJ units)
//   its W_hh rows (4*HJ gate rows, interleaved  r = jj*4 + q  so one MFMA lane ends up
//   holding i,f,g,o of one (unit, utterance)) stay resident in LDS for all T steps;
//   the cell state c lives in a register of that lane.
//
// Hand-off (per step, between the workgroups of one (dir, batch group)): the data IS the
// flag.  Every 8-byte granule of the exchange buffer (4 bf16 or 2 fp32 values) is written by
// ONE write-through (sc1) 8-byte store and carries a one-bit step tag in the least significant
// mantissa bit of its first value; a consumer issues all its operand loads (sc1, straight into
// MFMA operand registers), checks every granule's tag and re-issues until all match.  Four
// slots (step mod 4) with tag = ((step >> 2) + 1) & 1 make a stale granule (4 steps old, or
// the zero fill) always fail the check; no consumer can lag a producer by 4 steps because
// every step needs every producer's previous step (MI355X_MICROARCH.md "Valid forms": R2
// granules, one workgroup per CU, hipMalloc memory).  There is no flag, no drain before a
// publish and no workgroup barrier on the forward step's critical path.
// The backward pass all-gathers the pre-activation gate gradients dG_t the same way and forms
// dh_{t-1} = dG_t W_hh for its own hidden slice from a resident W_hh^T column slice.
#include "common.h"
#include <stdlib.h>
#include <type_traits>

#include "lstm_common.h"

namespace {


// ---------------------------------------------------------------------------------------
// forward recurrence
// ---------------------------------------------------------------------------------------
// K is split over the 4 waves (each polls/loads a quarter of h_{t-1}: 4x less hand-off
// traffic than every wave reading all of it) and partials are reduced through LDS:
// double-buffered for bf16 (one barrier per step); single-buffered for fp32, whose
// resident weights leave no room for a second buffer (two barriers).
template <int PREC, int HJ, int NL>
__global__ __launch_bounds__(320) void lstm_fwd_kernel(LstmArgs a) {
  typedef typename Elt<PREC>::T ET;
  constexpr int ROWS = 4 * HJ, MT = ROWS / 16;       // gate rows, 16-row MFMA tiles
  constexpr int KS = 4;
  constexpr int NRED = PREC == PREC_F32 ? 1 : 2;     // reduction buffers
  constexpr int KSTEP = PREC == PREC_F32 ? 16 : 32;  // k consumed per 16-byte operand load
  constexpr int EPL = PREC == PREC_F32 ? 4 : 8;      // elements per 16-byte load
  constexpr int GE = Elt<PREC>::GE;
  // bf16, 16 units per workgroup: a fifth "io" wave moves the step's HBM traffic through two
  // LDS rings -- the input projection two steps ahead, the saved activations two steps behind
  // -- so the four polling waves' memory queues hold nothing but the hand-off (an HBM load
  // queued ahead of a poll delays it: 2.74 -> 2.14 us/step with the loads taken out)
  constexpr bool IOW = PREC == PREC_BF16 && HJ == 16;
  constexpr int GXS = 16 * 4 + 4, OUS = 16 * 8 + 4;  // padded per-utterance strides (floats)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  f32x4* red0 = reinterpret_cast<f32x4*>(smem);  // [NRED][4][MT][64] partials
  float* gxr = reinterpret_cast<float*>(smem + NRED * 4 * MT * 64 * 16);  // [2][16 utt][16 unit][4 gate]
  float* outr = gxr + 2 * 16 * GXS;                                        // [2][16 utt][16 unit][8]
  __shared__ int abort_flag;
  __shared__ volatile int poll_seq;  // last step whose hand-off wave 0 has received

  const int ngroups = a.ndir * a.NB;
  int gid, js;
  if (a.xcd_local) {
    gid = blockIdx.x & 7; js = blockIdx.x >> 3;
    if (gid >= ngroups) return;  // the whole workgroup leaves before any barrier
  } else {
    gid = blockIdx.x % ngroups; js = blockIdx.x / ngroups;
  }
  const int dir = gid / a.NB, grp = gid % a.NB;
  const int GLD = 4 * a.H * a.ndir, YLD = a.H * a.ndir;  // row strides of G and of c / h
  const int H = a.H, T = a.T, j0 = js * HJ;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float* W = dir ? a.W1 : a.W0;
  __shared__ int placement;

  // wave w owns M-tile w: lane (bi, q) holds gates i,f,g,o of unit 4w+q, utterance bi.
  // Every wave computes partials of all MT tiles over its quarter of K.
  const int bi = lane & 15, q = lane >> 4;
  const bool owner = wave < MT;
  const int jj = wave * 4 + q;
  const int bglob = grp * BG + bi;
  const bool valid = owner && bglob < a.B;
  const int kb = wave * (a.Kp / 4);
  const bool loader = true;

  // The resident weight slice lives in registers as ready MFMA A-fragments:
  // tile m row r = jj*4 + q  <-  W_hh[q*H + j0 + jj][k], zero padded to Kp.
  typedef typename std::conditional<PREC == PREC_F32, f32x4, bf16x8>::type WFrag;
  WFrag wreg[NL][MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int r = m * 16 + bi;
    const float* wrow = W + (size_t)((r & 3) * H + j0 + (r >> 2)) * H;
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int k0 = kb + i * KSTEP + EPL * q;
#pragma unroll
      for (int e = 0; e < EPL; ++e) {  // clamped, unconditional loads: no per-element branch
        const float ld = wrow[min(k0 + e, H - 1)];
        const float v = k0 + e < H ? ld : 0.f;
        if constexpr (PREC == PREC_F32) wreg[i][m][e] = v; else wreg[i][m][e] = f2bf(v);
      }
    }
  }
  const bool plain_st = a.xcd_local && group_on_one_xcd(a.xtab + gid * a.NJ, a.NJ, js, &placement);
  if (DPTR(a) && blockIdx.x == 0 && tid == 0) a.dbg[7] = (plain_st ? 1 : 0) | (a.xcd_local ? 2 : 0);
  if (tid == 0) { abort_flag = 0; poll_seq = 0; }

  // ---- io wave (IOW): lane (b = lane >> 2, g = lane & 3) moves the 64-byte row segment of
  // utterance b, gate g, 16 units; lanes (b, kind) of the c / h / h-bf16 rows likewise
  const int iob = lane >> 2, iog = lane & 3, iobg = grp * BG + iob;
  const bool iobv = iobg < a.B;
  f32x4 ld0[4], ld1[4];  // input-projection segments in flight (even / odd steps)
#pragma unroll
  for (int i = 0; i < 4; ++i) ld0[i] = ld1[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto io_gload = [&](int s_, f32x4 (&v)[4]) {
    if (iobv && s_ < T) {
      const int t_ = dir ? T - 1 - s_ : s_;
      const float* p = a.G + ((size_t)iobg * T + t_) * GLD + dir * 4 * H + iog * H + j0;
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = *reinterpret_cast<const f32x4*>(p + 4 * i);
    }
  };
  auto io_gwrite = [&](int s_, const f32x4 (&v)[4]) {
    float* d = gxr + ((s_ & 1) * 16 + iob) * GXS + iog;
#pragma unroll
    for (int u = 0; u < 16; ++u) d[u * 4] = v[u >> 2][u & 3];
  };
  auto io_store = [&](int s_) {
    if (s_ < 0 || s_ >= T || (DMODE(a) & 1)) return;
    const int t_ = dir ? T - 1 - s_ : s_;
    const float* src = outr + (s_ & 1) * 16 * OUS;
    if (iobv) {  // activated gates of (b, g)
      float v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = src[iob * OUS + u * 8 + iog];
      float* gp = a.G + ((size_t)iobg * T + t_) * GLD + dir * 4 * H + iog * H + j0;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        *reinterpret_cast<f32x4*>(gp + 4 * i) = f32x4{v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]};
    }
    const int b2 = lane & 15, kind = lane >> 4, bg2 = grp * BG + b2;
    if (kind < 3 && bg2 < a.B) {  // kind 0: c, 1: h, 2: h as bf16
      float v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = src[b2 * OUS + u * 8 + (kind == 0 ? 4 : 5)];
      const size_t o = ((size_t)bg2 * T + t_) * YLD + dir * H + j0;
      if (kind < 2) {
        float* dp = (kind == 0 ? a.Cs : a.Y) + o;
#pragma unroll
        for (int i = 0; i < 4; ++i)
          *reinterpret_cast<f32x4*>(dp + 4 * i) = f32x4{v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]};
      } else if (a.Yb) {
        bf16x8 h0, h1;
#pragma unroll
        for (int u = 0; u < 8; ++u) { h0[u] = f2bf(v[u]); h1[u] = f2bf(v[8 + u]); }
        *reinterpret_cast<bf16x8*>(a.Yb + o) = h0;
        *reinterpret_cast<bf16x8*>(a.Yb + o + 8) = h1;
      }
    }
  };
  if (IOW && wave == 4) {
    io_gload(0, ld0);
    io_gload(1, ld1);
    io_gwrite(0, ld0);
    io_gload(2, ld0);
  }
  __syncthreads();

  const size_t xslot = (size_t)BG * a.Kp;  // elements per slot
  ET* xb = reinterpret_cast<ET*>(a.xbuf) + (size_t)(dir * a.NB + grp) * NSLOT * xslot;
  auto xr = make_rsrc(xb, (unsigned)(NSLOT * xslot * sizeof(ET)));

  // input projection of step s, loaded one step ahead (issued before the previous step's
  // plain stores, so the compiler never has to drain those stores to order an aliasing load)
  float gx[4] = {0.f, 0.f, 0.f, 0.f};
  auto load_gx = [&](int s_) {
    if (valid && s_ < T && !(s_ > 0 && (DMODE(a) & 2048))) {  // bit 11: timing without prefetch
      const int t_ = dir ? T - 1 - s_ : s_;
      const float* gp = a.G + ((size_t)bglob * T + t_) * GLD + dir * 4 * H + j0 + jj;
#pragma unroll
      for (int g = 0; g < 4; ++g) gx[g] = gp[g * H];
    }
  };
  if constexpr (!IOW) load_gx(0);
  float c = 0.f;
  if (!IOW || wave < 4) {
  for (int s = 0; s < T; ++s) {
    STAMP(0);
    const int t = dir ? T - 1 - s : s;
    const size_t n = (size_t)bglob * T + t;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    f32x4* red = red0 + (NRED == 2 ? (s & 1) * 4 * MT * 64 : 0);
    if (s > 0) {
      if (loader) {
        // poll = load: issue every operand load, check every granule's tag, retry until fresh
        const unsigned tag = step_tag(s - 1);
        const unsigned ebase = (unsigned)(((s - 1) & (NSLOT - 1)) * xslot) + bi * a.Kp + kb + EPL * q;
        u32x4 hv[NL];
        unsigned spins = 0;
        for (int d = (DMODE(a) >> 5) & 63; d > 0; --d) __builtin_amdgcn_s_sleep(1);  // diag: delayed first sweep
        unsigned long long t_issue = 0;
        while (true) {
          if (DPTR(a)) t_issue = __builtin_amdgcn_s_memtime();
#pragma unroll
          for (int i = 0; i < NL; ++i) hv[i] = ld_sc1_b128(xr, (ebase + i * KSTEP) * sizeof(ET));
          bool ok = true;
#pragma unroll
          for (int i = 0; i < NL; ++i) {
            const int k0 = kb + i * KSTEP + EPL * q;
            ok &= tags_ok(hv[i], tag, k0 < H, k0 + GE < H);
          }
          if (__all(ok)) break;
          if (++spins > SPIN_LIMIT) {
            if (lane == 0) { atomicExch(a.err, 1); abort_flag = 1; }
            break;
          }
          if (DMODE(a) & 16) __builtin_amdgcn_s_sleep(1); else __builtin_amdgcn_s_sleep(4);
        }
        STAMP(1);
        if (tid == 0) poll_seq = s;  // the io wave issues its HBM traffic behind this poll
        if (DPTR(a) && blockIdx.x == 0 && threadIdx.x == 0) {
          a.dbg[(size_t)s * 16 + 5] = t_issue;
          a.dbg[(size_t)s * 16 + 6] = spins;
        }
        f32x4 part[MT];
#pragma unroll
        for (int m = 0; m < MT; ++m) part[m] = acc;
#pragma unroll
        for (int i = 0; i < NL; ++i) {
#pragma unroll
          for (int m = 0; m < MT; ++m) {
            if constexpr (PREC == PREC_F32) {
#pragma unroll
              for (int e = 0; e < 4; ++e)
                part[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(wreg[i][m][e], __uint_as_float(hv[i][e]), part[m], 0, 0, 0);
            } else {
              bf16x8 hb = *reinterpret_cast<bf16x8*>(&hv[i]);
              part[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wreg[i][m], hb, part[m], 0, 0, 0);
            }
          }
        }
        if constexpr (KS == 1) {
          acc = part[0];
        } else {
#pragma unroll
          for (int m = 0; m < MT; ++m) red[(wave * MT + m) * 64 + lane] = part[m];
        }
      }
      STAMP(2);
      if constexpr (KS > 1) {
        __syncthreads();
        if (owner) {
#pragma unroll
          for (int w = 0; w < 4; ++w) acc += red[(w * MT + wave) * 64 + lane];
        }
        if (NRED == 1) __syncthreads();  // red is reused next step
      } else {
        if (abort_flag) break;
      }
      if (KS > 1 && abort_flag) break;
      STAMP(3);
    }
    if constexpr (IOW) {  // this step's input projection, staged by the io wave
      if (owner) {
        const f32x4 g4 = *reinterpret_cast<const f32x4*>(gxr + ((s & 1) * 16 + bi) * GXS + jj * 4);
        gx[0] = g4[0]; gx[1] = g4[1]; gx[2] = g4[2]; gx[3] = g4[3];
      }
    }
    float ig = 0.f, fg = 0.f, gg = 0.f, og = 0.f, hv = 0.f;
    if (owner) {
      if (valid) {
        // acc[q'] = recurrent part of gate q' for unit jj, utterance bi
        ig = sigmoid_p<PREC>(acc[0] + gx[0]);
        fg = sigmoid_p<PREC>(acc[1] + gx[1]);
        gg = tanh_p<PREC>(acc[2] + gx[2]);
        og = sigmoid_p<PREC>(acc[3] + gx[3]);
        c = fg * c + ig * gg;
        hv = og * tanh_p<PREC>(c);
      }
      if (s + 1 < T) {
        // gather 4 (bf16) / 2 (fp32) consecutive units of one utterance into one granule;
        // padded utterances publish zeros so every granule a consumer checks gets written
        const unsigned tag = step_tag(s);
        const size_t row = (size_t)(s & (NSLOT - 1)) * xslot + (size_t)bi * a.Kp + j0 + wave * 4;
        if constexpr (PREC == PREC_F32) {
          const float h1 = __shfl(hv, lane + 16, 64);
          if ((q & 1) == 0) st_granule(xr, (unsigned)((row + q) * sizeof(ET)), pack_f32(hv, h1, tag));
        } else {
          const float h1 = __shfl(hv, lane + 16, 64);
          const float h2 = __shfl(hv, lane + 32, 64);
          const float h3 = __shfl(hv, lane + 48, 64);
          if (q == 0) {
            const unsigned long long gv = pack_bf16(hv, h1, h2, h3, tag);
            if (plain_st) {  // same-XCD group: the line stays in the shared L2
              u32x2 w2 = {(unsigned)gv, (unsigned)(gv >> 32)};
              __builtin_amdgcn_raw_buffer_store_b64(w2, xr, (unsigned)(row * sizeof(ET)), 0, 0);
            } else {
              st_granule(xr, (unsigned)(row * sizeof(ET)), gv);
            }
          }
        }
      }
    }
    STAMP(4);
    if constexpr (IOW) {  // saved activations into the out ring; the io wave stores them
      if (owner) {
        float* o = outr + ((s & 1) * 16 + bi) * OUS + jj * 8;
        *reinterpret_cast<f32x4*>(o) = f32x4{ig, fg, gg, og};
        o[4] = c;
        o[5] = hv;
      }
    } else {
      load_gx(s + 1);
      if (valid && !(DMODE(a) & 1)) {  // saved activations: plain stores, off the critical path
        float* gp = a.G + n * GLD + dir * 4 * H + j0 + jj;
        gp[0] = ig; gp[H] = fg; gp[2 * H] = gg; gp[3 * H] = og;
        a.Cs[n * YLD + dir * H + j0 + jj] = c;
        a.Y[n * YLD + dir * H + j0 + jj] = hv;
        if (a.Yb) a.Yb[n * YLD + dir * H + j0 + jj] = (unsigned short)f2bf(hv);
      }
    }
  }
  } else if constexpr (IOW) {
    // io wave: one barrier per step s >= 1 like the polling waves.  Before barrier s: the
    // input projection of step s into ring slot s & 1 (loaded two steps ago), the load of
    // step s + 2, and the stores of step s - 2's activations (written before barrier s - 1)
    auto io_step = [&](int s_, f32x4 (&v)[4]) -> bool {
      io_gwrite(s_, v);
      // issue the HBM traffic only once step s_'s hand-off has arrived, so that it has drained
      // before the next poll is issued (measured 2.34 -> 2.18 us/step)
      for (unsigned sp = 0; poll_seq < s_ && sp < SPIN_LIMIT; ++sp) __builtin_amdgcn_s_sleep(1);
      io_gload(s_ + 2, v);
      io_store(s_ - 2);
      __syncthreads();
      return !abort_flag;
    };
    for (int s = 1; s < T; s += 2) {
      if (!io_step(s, ld1)) break;
      if (s + 1 < T && !io_step(s + 1, ld0)) break;
    }
  }
  if constexpr (IOW) {
    __syncthreads();  // the last step's activations are in the ring
    if (wave == 4) {
      io_store(T - 2);
      io_store(T - 1);
    }
  }
}

// ---------------------------------------------------------------------------------------
// backward recurrence (BPTT)
// ---------------------------------------------------------------------------------------
// HJ units per workgroup: HJ <= 16 -> one 16-wide MFMA N-tile (padded), one unit per thread;
// HJ = 32 -> two N-tiles and two units per thread.  Larger HJ = fewer workgroups per group,
// and the all-gather volume (every workgroup reads the group's whole dG_t) scales with that
// count, so the backward prefers HJ = 32.
template <int PREC, int HJ, int NL>
__global__ __launch_bounds__(256) void lstm_bwd_kernel(LstmArgs a) {
  typedef typename Elt<PREC>::T ET;
  constexpr int KSTEP = PREC == PREC_F32 ? 16 : 32;
  constexpr int EPL = PREC == PREC_F32 ? 4 : 8;
  constexpr int GE = Elt<PREC>::GE;
  constexpr int NT = HJ > 16 ? HJ / 16 : 1;   // MFMA N-tiles (units)
  constexpr int UPT = NT;                      // units per thread in the cell phase
  constexpr int RW = 16 * NT;                  // reduction row width (units)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* red = reinterpret_cast<float*>(smem);  // [2][4 waves][16 utterances][RW] partials
  __shared__ int abort_flag;

  const int ngroups = a.ndir * a.NB;
  const int gid = blockIdx.x % ngroups, js = blockIdx.x / ngroups;
  const int dir = gid / a.NB, grp = gid % a.NB;
  const int GLD = 4 * a.H * a.ndir, YLD = a.H * a.ndir;  // row strides of G and of c / h
  const int H = a.H, T = a.T, j0 = js * HJ, G4 = 4 * H;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float* W = dir ? a.W1 : a.W0;

  // MFMA roles: A = dG (rows = utterances), B = W_hh^T slice (cols = units), K = 4H over 4 waves
  const int bi = lane & 15, q = lane >> 4;
  const int kb = wave * (a.K4p / 4);
  // cell roles: thread -> (utterance cb, units cj + 16u); a wave holds 4 utterances
  const int cb = tid >> 4, cj = tid & 15;
  const int bglob = grp * BG + cb;
  const bool bvalid = bglob < a.B;

  // resident W_hh^T column slice as ready MFMA B-fragments: tile nt, column bi = unit nt*16+bi
  typedef typename std::conditional<PREC == PREC_F32, f32x4, bf16x8>::type WFrag;
  WFrag wreg[NL][NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int u = nt * 16 + bi;
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int g0 = kb + i * KSTEP + EPL * q;
#pragma unroll
      for (int e = 0; e < EPL; ++e) {  // clamped, unconditional loads: no per-element branch
        const float ld = W[(size_t)min(g0 + e, G4 - 1) * H + j0 + min(u, HJ - 1)];
        const float v = (u < HJ && g0 + e < G4) ? ld : 0.f;
        if constexpr (PREC == PREC_F32) wreg[i][nt][e] = v; else wreg[i][nt][e] = f2bf(v);
      }
    }
  }
  if (tid == 0) abort_flag = 0;
  __syncthreads();

  const size_t xslot = (size_t)BG * a.K4p;
  ET* xb = reinterpret_cast<ET*>(a.xbuf) + (size_t)(dir * a.NB + grp) * NSLOT * xslot;
  auto xr = make_rsrc(xb, (unsigned)(NSLOT * xslot * sizeof(ET)));

  // cell inputs of step s (saved gates, c_t, c_{t-1}, dY) per owned unit, loaded one step
  // ahead and issued before the previous step's dG stores (no store drain on aliasing loads)
  float gi[UPT], gf[UPT], gg[UPT], go[UPT], cc[UPT], cp[UPT], dy[UPT], dc[UPT];
#pragma unroll
  for (int u = 0; u < UPT; ++u) { gi[u] = gf[u] = gg[u] = go[u] = cc[u] = cp[u] = dy[u] = dc[u] = 0.f; }
  auto load_cell = [&](int s_) {
    if (bvalid && s_ < T) {
      const int t_ = dir ? s_ : T - 1 - s_;
      const int tp_ = dir ? t_ + 1 : t_ - 1;
      const bool has_prev = tp_ >= 0 && tp_ < T;
      const size_t n_ = (size_t)bglob * T + t_;
      const size_t np_ = (size_t)bglob * T + min(max(tp_, 0), T - 1);
#pragma unroll
      for (int u = 0; u < UPT; ++u) {
        const int uu = cj + 16 * u;
        if (uu < HJ) {
          const int j = j0 + uu;
          const float* gp = a.G + n_ * GLD + dir * 4 * H + j;
          gi[u] = gp[0]; gf[u] = gp[H]; gg[u] = gp[2 * H]; go[u] = gp[3 * H];
          cc[u] = a.Cs[n_ * YLD + dir * H + j];
          const float cpl = a.Cs[np_ * YLD + dir * H + j];
          cp[u] = has_prev ? cpl : 0.f;
          dy[u] = a.Y[n_ * YLD + dir * H + j];
        }
      }
    }
  };
  load_cell(0);
  for (int s = 0; s < T; ++s) {
    STAMP(0);
    const int t = dir ? s : T - 1 - s;          // reverse of the forward processing order
    const size_t n = (size_t)bglob * T + t;
    float* rb = red + (s & 1) * 4 * 16 * RW;
    float dhrec[UPT];
#pragma unroll
    for (int u = 0; u < UPT; ++u) dhrec[u] = 0.f;
    if (s > 0) {
      const unsigned tag = step_tag(s - 1);
      const unsigned ebase = (unsigned)(((s - 1) & (NSLOT - 1)) * xslot) + bi * a.K4p + kb + EPL * q;
      u32x4 gv[NL];
      unsigned spins = 0;
      unsigned long long t_issue = 0;
      while (true) {
        if (DPTR(a)) t_issue = __builtin_amdgcn_s_memtime();
#pragma unroll
        for (int i = 0; i < NL; ++i) gv[i] = ld_sc1_b128(xr, (ebase + i * KSTEP) * sizeof(ET));
        bool ok = true;
#pragma unroll
        for (int i = 0; i < NL; ++i) {
          const int g0 = kb + i * KSTEP + EPL * q;
          ok &= tags_ok(gv[i], tag, g0 < G4, g0 + GE < G4);
        }
        if (__all(ok)) break;
        if (++spins > SPIN_LIMIT) {
          if (lane == 0) { atomicExch(a.err, 1); abort_flag = 1; }
          break;
        }
        if (DMODE(a) & 16) __builtin_amdgcn_s_sleep(1); else __builtin_amdgcn_s_sleep(4);
      }
      STAMP(1);
      if (DPTR(a) && blockIdx.x == 0 && threadIdx.x == 0) {
        a.dbg[(size_t)s * 16 + 5] = t_issue;
        a.dbg[(size_t)s * 16 + 6] = spins;
      }
      f32x4 acc[NT];
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < NL; ++i) {
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          if constexpr (PREC == PREC_F32) {
#pragma unroll
            for (int e = 0; e < 4; ++e)
              acc[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(gv[i][e]), wreg[i][nt][e], acc[nt], 0, 0, 0);
          } else {
            bf16x8 gb = *reinterpret_cast<bf16x8*>(&gv[i]);
            acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(gb, wreg[i][nt], acc[nt], 0, 0, 0);
          }
        }
      }
      // C layout: col = lane&15 = unit (of tile nt), row = 4*(lane>>4)+r = utterance
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int r = 0; r < 4; ++r) rb[(wave * 16 + 4 * q + r) * RW + nt * 16 + bi] = acc[nt][r];
      STAMP(2);
      __syncthreads();  // double-buffered red: one barrier per step
      STAMP(3);
      if (abort_flag) break;
#pragma unroll
      for (int u = 0; u < UPT; ++u) {
        const int uu = cj + 16 * u;
        dhrec[u] = rb[(0 * 16 + cb) * RW + uu] + rb[(1 * 16 + cb) * RW + uu] +
                   rb[(2 * 16 + cb) * RW + uu] + rb[(3 * 16 + cb) * RW + uu];
      }
    }
    float dG[UPT][4];
    float sgi[UPT], sgf[UPT], sgg[UPT], sgo[UPT], scc[UPT], scp[UPT], sdy[UPT];
#pragma unroll
    for (int u = 0; u < UPT; ++u) {
      sgi[u] = gi[u]; sgf[u] = gf[u]; sgg[u] = gg[u]; sgo[u] = go[u];
      scc[u] = cc[u]; scp[u] = cp[u]; sdy[u] = dy[u];
    }
    load_cell(s + 1);
#pragma unroll
    for (int u = 0; u < UPT; ++u) {
      dG[u][0] = dG[u][1] = dG[u][2] = dG[u][3] = 0.f;
      if (bvalid && cj + 16 * u < HJ) {
        const float dh = sdy[u] + dhrec[u];
        const float tc = tanh_p<PREC>(scc[u]);
        const float d_o = dh * tc;
        const float dcs = dc[u] + dh * sgo[u] * (1.f - tc * tc);
        const float di = dcs * sgg[u], dgg = dcs * sgi[u], df = dcs * scp[u];
        dc[u] = dcs * sgf[u];
        dG[u][0] = di * sgi[u] * (1.f - sgi[u]);
        dG[u][1] = df * sgf[u] * (1.f - sgf[u]);
        dG[u][2] = dgg * (1.f - sgg[u] * sgg[u]);
        dG[u][3] = d_o * sgo[u] * (1.f - sgo[u]);
      }
    }
    if (s + 1 < T) {
      // granules of 4 (bf16) / 2 (fp32) consecutive units of one gate and utterance; the
      // lanes of consecutive units are adjacent (cj = tid & 15); padded utterances publish 0
      const unsigned tag = step_tag(s);
#pragma unroll
      for (int u = 0; u < UPT; ++u) {
        const int uu = cj + 16 * u;
        const size_t row = (size_t)(s & (NSLOT - 1)) * xslot + (size_t)cb * a.K4p + j0 + uu;
        if constexpr (PREC == PREC_F32) {
          float v1[4];
#pragma unroll
          for (int g = 0; g < 4; ++g) v1[g] = __shfl(dG[u][g], lane + 1, 64);
          if (uu < HJ && (cj & 1) == 0) {
#pragma unroll
            for (int g = 0; g < 4; ++g)
              st_granule(xr, (unsigned)((row + (size_t)g * H) * sizeof(ET)), pack_f32(dG[u][g], v1[g], tag));
          }
        } else {
          float v1[4], v2[4], v3[4];
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            v1[g] = __shfl(dG[u][g], lane + 1, 64);
            v2[g] = __shfl(dG[u][g], lane + 2, 64);
            v3[g] = __shfl(dG[u][g], lane + 3, 64);
          }
          if (uu < HJ && (cj & 3) == 0) {
#pragma unroll
            for (int g = 0; g < 4; ++g)
              st_granule(xr, (unsigned)((row + (size_t)g * H) * sizeof(ET)),
                         pack_bf16(dG[u][g], v1[g], v2[g], v3[g], tag));
          }
        }
      }
    }
    STAMP(4);
    if (bvalid) {  // dG for the weight-gradient GEMMs: plain stores after the hand-off
#pragma unroll
      for (int u = 0; u < UPT; ++u) {
        const int uu = cj + 16 * u;
        if (uu < HJ) {
          const size_t o = n * GLD + dir * 4 * H + j0 + uu;
          if (a.dGb) {
            unsigned short* gb = a.dGb + o;
            gb[0] = (unsigned short)f2bf(dG[u][0]); gb[H] = (unsigned short)f2bf(dG[u][1]);
            gb[2 * H] = (unsigned short)f2bf(dG[u][2]); gb[3 * H] = (unsigned short)f2bf(dG[u][3]);
          } else {
            float* gp = a.G + o;
            gp[0] = dG[u][0]; gp[H] = dG[u][1]; gp[2 * H] = dG[u][2]; gp[3 * H] = dG[u][3];
          }
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// backward recurrence, reduce-scatter form (bf16; H in {128, 256, 512, 1024})
// ---------------------------------------------------------------------------------------
// dh_{t-1}[:, J'] = sum_J dG_t[:, gates of J] W_hh[gates of J, J'].  The gather form above has
// every workgroup read the group's whole dG_t (16 x 4H bf16 = 64 KB at H = 512) to multiply it
// by its W_hh column slice.  Here workgroup J multiplies ITS OWN dG slice [16 x 64] by its
// W_hh row slice [64 x H] and publishes the [16 x H] partial product cut into one [16 x 16]
// tile per consumer; workgroup J' reads only the NJ tiles addressed to it (16 KB at H = 512)
// and sums them in a fixed order.  4x less hand-off traffic per consumer, and the operand of
// the step's MFMA is the workgroup's own data (one LDS hop, no cross-wave K reduction).
template <int NTW>
__global__ __launch_bounds__(256) void lstm_bwd_rs_kernel(LstmArgs a) {
  constexpr int NJ = NTW * 4;     // workgroups per (dir, batch group) = producers = consumers
  constexpr int NPL = NJ / 8;     // partial-tile loads per lane
  constexpr int AST = 72;         // LDS row stride of the own-dG tile (bf16: 64 + 8 pad)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  short* abuf = reinterpret_cast<short*>(smem);  // [2][16 utterances][AST]
  __shared__ int abort_flag, placement;

  const int ngroups = a.ndir * a.NB;
  int gid, js;
  if (a.xcd_local) {
    gid = blockIdx.x & 7; js = blockIdx.x >> 3;
    if (gid >= ngroups) return;  // the whole workgroup leaves before any barrier
  } else {
    gid = blockIdx.x % ngroups; js = blockIdx.x / ngroups;
  }
  const int dir = gid / a.NB, grp = gid % a.NB;
  const int GLD = 4 * a.H * a.ndir, YLD = a.H * a.ndir;  // row strides of G and of c / h
  const int H = a.H, T = a.T, j0 = js * 16;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float* W = dir ? a.W1 : a.W0;

  // reduction + cell role: the 8 contiguous lanes pg = 0..7 of one (unit uc, utterance half)
  // each load NPL producers' partials of 8 utterances, then reduce-scatter so that lane pg
  // ends with utterance half*8 + pg
  const int combo = wave * 8 + (lane >> 3);
  const int uc = combo >> 1, half = combo & 1, pg = lane & 7;
  const int cu = half * 8 + pg;
  const int bglob = grp * BG + cu;
  const bool bvalid = bglob < a.B;
  // MFMA role (16x16x32 bf16): A row / B column = lane & 15, k octet = lane >> 4
  const int bi = lane & 15, q = lane >> 4;

  // resident W_hh row slice as MFMA B fragments: tile t = consumer nt = wave*NTW + t,
  // k chunk kc: B[k][n] = W_hh[g*H + j0 + jj][nt*16 + n] with k = jj*4 + g
  bf16x8 wreg[NTW][2];
#pragma unroll
  for (int t = 0; t < NTW; ++t) {
    const int col = (wave * NTW + t) * 16 + bi;
#pragma unroll
    for (int kc = 0; kc < 2; ++kc)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int k = kc * 32 + q * 8 + e;
        wreg[t][kc][e] = f2bf(W[(size_t)((k & 3) * H + j0 + (k >> 2)) * H + col]);
      }
  }
  const bool plain_st = a.xcd_local && group_on_one_xcd(a.xtab + gid * NJ, NJ, js, &placement);
  if (DPTR(a) && blockIdx.x == 0 && tid == 0) a.dbg[7] = (plain_st ? 1 : 0) | (a.xcd_local ? 2 : 0);
  if (tid == 0) abort_flag = 0;
  __syncthreads();

  // exchange: [slot][consumer][producer][16 units][16 utterances] bf16
  const size_t xslot = (size_t)NJ * NJ * 256;
  short* xb = reinterpret_cast<short*>(a.xbuf) + (size_t)(dir * a.NB + grp) * NSLOT * xslot;
  auto xr = make_rsrc(xb, (unsigned)(NSLOT * xslot * sizeof(short)));

  // Cell inputs of one step, prefetched a step ahead into one of two explicit buffers (the
  // loop is unrolled by two so no register copy -- and no wait on the prefetch -- sits at the
  // loop latch).  c_{t-1} is loaded clamped and masked at use: a select right after the load
  // would make the compiler wait for it on the spot.
  struct CellIn { float gi, gf, gg, go, cc, cp, dy; };
  const int j = j0 + uc;
  auto load_cell = [&](int s_, CellIn& c) {
    if (bvalid && s_ < T && !(s_ > 0 && (DMODE(a) & 2048))) {  // bit 11: timing without prefetch
      const int t_ = dir ? s_ : T - 1 - s_;
      const int tp_ = dir ? t_ + 1 : t_ - 1;
      const size_t n_ = (size_t)bglob * T + t_;
      const size_t np_ = (size_t)bglob * T + min(max(tp_, 0), T - 1);
      const float* gp = a.G + n_ * GLD + dir * 4 * H + j;
      c.gi = gp[0]; c.gf = gp[H]; c.gg = gp[2 * H]; c.go = gp[3 * H];
      c.cc = a.Cs[n_ * YLD + dir * H + j];
      c.cp = a.Cs[np_ * YLD + dir * H + j];
      c.dy = a.Y[n_ * YLD + dir * H + j];
    }
  };
  float dc = 0.f;
  // one BPTT step; false = abort (spin limit).  The cell inputs of step s + 2 are loaded right
  // behind step s's hand-off (three rotating buffers): a full step before the next poll is
  // issued, so that poll does not queue behind HBM loads in this wave's memory queue
  auto step = [&](int s, const CellIn& cur, CellIn& fill) -> bool {
    STAMP(0);
    const int t = dir ? s : T - 1 - s;
    const size_t n = (size_t)bglob * T + t;
    float dhrec = 0.f;
    if (s == 0) load_cell(2, fill);
    if (s > 0) {
      const unsigned tag = step_tag(s - 1);
      const unsigned ebase = (unsigned)(((s - 1) & (NSLOT - 1)) * xslot + (size_t)js * NJ * 256 +
                                        uc * 16 + half * 8);
      u32x4 pv[NPL];
      unsigned spins = 0;
      for (int d = (DMODE(a) >> 5) & 63; d > 0; --d) __builtin_amdgcn_s_sleep(1);  // diag: delayed first sweep
      unsigned long long t_issue = 0;
      while (true) {
        if (DPTR(a)) t_issue = __builtin_amdgcn_s_memtime();
#pragma unroll
        for (int i = 0; i < NPL; ++i)
          pv[i] = ld_sc1_b128(xr, (ebase + (unsigned)(pg * NPL + i) * 256u) * sizeof(short));
        bool ok = true;
#pragma unroll
        for (int i = 0; i < NPL; ++i) ok &= tags_ok(pv[i], tag, true, true);
        if (__all(ok)) break;
        if (++spins > SPIN_LIMIT) {
          if (lane == 0) { atomicExch(a.err, 1); abort_flag = 1; }
          break;
        }
        if (DMODE(a) & 16) __builtin_amdgcn_s_sleep(1); else __builtin_amdgcn_s_sleep(4);
      }
      STAMP(1);
      WSTAMP(8);
      load_cell(s + 2, fill);
      if (DPTR(a) && blockIdx.x == 0 && threadIdx.x == 0) {
        a.dbg[(size_t)s * 16 + 5] = t_issue;
        a.dbg[(size_t)s * 16 + 6] = spins;
      }
      // sum this lane's producers (utterances half*8 + 0..7), then reduce-scatter over pg
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = 0.f;
#pragma unroll
      for (int i = 0; i < NPL; ++i)
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          v[2 * d] += __uint_as_float(pv[i][d] << 16);
          v[2 * d + 1] += __uint_as_float(pv[i][d] & 0xffff0000u);
        }
      // reduce-scatter over the 8 lanes with DPP moves (row_shl/shr:4, quad_perm xor 2 / 1)
      const bool b2 = pg & 4, b1 = pg & 2, b0 = pg & 1;
      float w4[4], w2[2];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float send = b2 ? v[k] : v[k + 4], keep = b2 ? v[k + 4] : v[k];
        const float from_lo = dpp_f<0x114>(send);   // row_shr:4 (lane - 4)
        const float from_hi = dpp_f<0x104>(send);   // row_shl:4 (lane + 4)
        w4[k] = keep + (b2 ? from_lo : from_hi);
      }
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const float send = b1 ? w4[k] : w4[k + 2], keep = b1 ? w4[k + 2] : w4[k];
        w2[k] = keep + dpp_f<0x4E>(send);           // quad_perm [2,3,0,1]: lane ^ 2
      }
      {
        const float send = b0 ? w2[0] : w2[1], keep = b0 ? w2[1] : w2[0];
        dhrec = keep + dpp_f<0xB1>(send);           // quad_perm [1,0,3,2]: lane ^ 1
      }
    }
    STAMP(2);
    float dG0 = 0.f, dG1 = 0.f, dG2 = 0.f, dG3 = 0.f;
    if (bvalid) {
      const float cpv = s + 1 < T ? cur.cp : 0.f;  // c_{t-1}; none at the sequence start
      const float dh = cur.dy + dhrec;
      const float tc = tanh_fast(cur.cc);
      const float d_o = dh * tc;
      const float dcs = dc + dh * cur.go * (1.f - tc * tc);
      dc = dcs * cur.gf;
      dG0 = dcs * cur.gg * cur.gi * (1.f - cur.gi);
      dG1 = dcs * cpv * cur.gf * (1.f - cur.gf);
      dG2 = dcs * cur.gi * (1.f - cur.gg * cur.gg);
      dG3 = d_o * cur.go * (1.f - cur.go);
    }
    if (s + 1 < T) {
      short* A = abuf + (s & 1) * 16 * AST;
      bf16x4 pk = {f2bf(dG0), f2bf(dG1), f2bf(dG2), f2bf(dG3)};
      *reinterpret_cast<bf16x4*>(A + cu * AST + uc * 4) = pk;
      WSTAMP(12);
      __syncthreads();  // double-buffered A: one barrier per step
      STAMP(3);
      if (abort_flag) return false;
      const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(A + bi * AST + q * 8);
      const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(A + bi * AST + 32 + q * 8);
      const unsigned tag = step_tag(s);
      const size_t sbase = (size_t)(s & (NSLOT - 1)) * xslot + (size_t)js * 256 + bi * 16 + 4 * q;
      unsigned long long gr[NTW];
#pragma unroll
      for (int t2 = 0; t2 < NTW; ++t2) {
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, wreg[t2][0], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, wreg[t2][1], acc, 0, 0, 0);
        // acc[r]: partial dh of utterance 4q + r, unit (consumer nt) column bi
        gr[t2] = pack_bf16(acc[0], acc[1], acc[2], acc[3], tag);
      }
      if (plain_st) {  // same-XCD group: keep the lines in the shared L2
#pragma unroll
        for (int t2 = 0; t2 < NTW; ++t2) {
          const unsigned off = (unsigned)((sbase + (size_t)(wave * NTW + t2) * NJ * 256) * sizeof(short));
          u32x2 w = {(unsigned)gr[t2], (unsigned)(gr[t2] >> 32)};
          __builtin_amdgcn_raw_buffer_store_b64(w, xr, off, 0, 0);
        }
      } else {
#pragma unroll
        for (int t2 = 0; t2 < NTW; ++t2)
          st_granule(xr, (unsigned)((sbase + (size_t)(wave * NTW + t2) * NJ * 256) * sizeof(short)), gr[t2]);
      }
    }
    STAMP(4);
    if (bvalid && !(DMODE(a) & 1)) {  // dG for the weight-gradient GEMMs: plain stores
      const size_t o = n * GLD + dir * 4 * H + j;
      if (a.dGb) {
        unsigned short* gb = a.dGb + o;
        gb[0] = (unsigned short)f2bf(dG0); gb[H] = (unsigned short)f2bf(dG1);
        gb[2 * H] = (unsigned short)f2bf(dG2); gb[3 * H] = (unsigned short)f2bf(dG3);
      } else {
        float* gp = a.G + o;
        gp[0] = dG0; gp[H] = dG1; gp[2 * H] = dG2; gp[3 * H] = dG3;
      }
    }
    return true;
  };
  CellIn c0 = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, c1 = c0, c2 = c0;
  load_cell(0, c0);
  load_cell(1, c1);
  for (int s = 0; s < T; s += 3) {
    if (!step(s, c0, c2)) break;
    if (s + 1 < T && !step(s + 1, c1, c0)) break;
    if (s + 2 < T && !step(s + 2, c2, c1)) break;
  }
}

// ---------------------------------------------------------------------------------------
// fp32 BPTT past the persistent kernels' register budget (the gather form holds a quarter of
// the 4H-wide dG operand per wave in registers: H <= 512 in fp32).  The parity mode has no
// such limit in nn.LSTM (ref:src/modules/decoder.py:14-15), so larger H run one launch per
// step: the launch boundary is the hand-off.  Block = (64 units, 16 utterances, direction),
// 256 threads = 64 units x 4 k-quarters; dG of the previously processed step is staged through
// LDS in 256-wide k chunks and multiplied by coalesced W_hh rows.  dG overwrites the gates in
// place (as the persistent kernels do); dc, the cell gradient carried between steps, lives in
// the caller's workspace.
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void lstm_bwd_step_f32(int B, int T, int H, int ndir, int s,
                                                         const float* W0, const float* W1, float* G,
                                                         const float* Cs, const float* Y, float* dcbuf,
                                                         unsigned short* dGb) {
  __shared__ float dgp[16][257];
  __shared__ float red[4][16][65];
  const int dir = blockIdx.z, b0 = blockIdx.y * 16, j0 = blockIdx.x * 64;
  const int tid = threadIdx.x, jl = tid & 63, kq = tid >> 6;
  const int j = j0 + jl, K4 = 4 * H;
  const float* W = dir ? W1 : W0;
  const int t = dir ? s : T - 1 - s;
  const int tq = dir ? t - 1 : t + 1;  // the step processed before this one
  const size_t gld = (size_t)K4 * ndir, yld = (size_t)H * ndir;
  float acc[16];
#pragma unroll
  for (int bl = 0; bl < 16; ++bl) acc[bl] = 0.f;
  if (s > 0) {
    for (int k0 = 0; k0 < K4; k0 += 256) {
      for (int e = tid; e < 16 * 256; e += 256) {
        const int bl = e >> 8, kk = e & 255, b = b0 + bl;
        dgp[bl][kk] = (b < B && k0 + kk < K4) ? G[((size_t)b * T + tq) * gld + (size_t)dir * K4 + k0 + kk] : 0.f;
      }
      __syncthreads();
      if (j < H) {
        const int kend = min(64, K4 - k0 - kq * 64);
        for (int kk = 0; kk < kend; ++kk) {
          const float w = W[(size_t)(k0 + kq * 64 + kk) * H + j];
#pragma unroll
          for (int bl = 0; bl < 16; ++bl) acc[bl] += dgp[bl][kq * 64 + kk] * w;
        }
      }
      __syncthreads();
    }
  }
#pragma unroll
  for (int bl = 0; bl < 16; ++bl) red[kq][bl][jl] = acc[bl];
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int idx = tid + 256 * r, bl = idx >> 6, ju = idx & 63;
    const int b = b0 + bl, jj = j0 + ju;
    if (b >= B || jj >= H) continue;
    const float dhrec = red[0][bl][ju] + red[1][bl][ju] + red[2][bl][ju] + red[3][bl][ju];
    const size_t n = (size_t)b * T + t;
    float* gp = G + n * gld + (size_t)dir * K4 + jj;
    const float gi = gp[0], gf = gp[H], gg = gp[2 * H], go = gp[3 * H];
    const float cc = Cs[n * yld + (size_t)dir * H + jj];
    const int tp = dir ? t + 1 : t - 1;  // the cell's previous step in forward time
    const float cp = (tp >= 0 && tp < T) ? Cs[((size_t)b * T + tp) * yld + (size_t)dir * H + jj] : 0.f;
    float* dcp = dcbuf + ((size_t)dir * B + b) * H + jj;
    const float dcv = s > 0 ? *dcp : 0.f;
    const float dh = Y[n * yld + (size_t)dir * H + jj] + dhrec;
    const float tc = tanhf(cc);
    const float d_o = dh * tc;
    const float dcs = dcv + dh * go * (1.f - tc * tc);
    *dcp = dcs * gf;
    const float dgi = dcs * gg * gi * (1.f - gi), dgf = dcs * cp * gf * (1.f - gf);
    const float dgg = dcs * gi * (1.f - gg * gg), dgo = d_o * go * (1.f - go);
    gp[0] = dgi; gp[H] = dgf; gp[2 * H] = dgg; gp[3 * H] = dgo;
    if (dGb) {
      unsigned short* gb = dGb + n * gld + (size_t)dir * K4 + jj;
      gb[0] = (unsigned short)f2bf(dgi); gb[H] = (unsigned short)f2bf(dgf);
      gb[2 * H] = (unsigned short)f2bf(dgg); gb[3 * H] = (unsigned short)f2bf(dgo);
    }
  }
}

// fp32 gather-form BPTT holds 4H / (4 x 16) operand loads per wave: more than 32 -> stepwise
bool use_stepwise_bwd(int H, int prec) { return prec == PREC_F32 && H > 512; }

int run_bwd_stepwise(int B, int T, int H, int ndir, const float* W0, const float* W1, float* G,
                     const float* Cs, const float* Y, void* xbuf, size_t xbytes, unsigned short* dgb,
                     hipStream_t st) {
  const size_t need = (size_t)ndir * B * H * sizeof(float);
  if (!xbuf || xbytes < need) {
    mlvae_set_error("lstm: exchange workspace too small (need %zu B)", need);
    return 1;
  }
  float* dc = static_cast<float*>(xbuf);
  const dim3 grid((H + 63) / 64, (B + 15) / 16, ndir);
  for (int s = 0; s < T; ++s) {
    lstm_bwd_step_f32<<<grid, 256, 0, st>>>(B, T, H, ndir, s, W0, W1, G, Cs, Y, dc, dgb);
    MLVAE_CHECK_LAUNCH();
  }
  return 0;
}

unsigned long long* g_dbg = nullptr;
// debug / A-B bits of the recurrence kernels (mlvae_lstm_set_debug_mode); MLVAE_LSTM_DBG sets
// the initial value so a whole bench run can be timed under one variant
int g_dbg_mode = [] {
  const char* e = getenv("MLVAE_LSTM_DBG");
  return e ? (int)strtol(e, nullptr, 0) : 0;
}();

struct Plan {
  int NB, NJ, HJ, Kp, K4p;   // NJ/HJ of the launch being planned (fwd or bwd)
  bool rs;                   // backward in reduce-scatter form (lstm_bwd_rs_kernel)
  bool xcd;                  // XCD-local groups (grid 8*NJ, group g on blocks b%8 == g)
  size_t lds, xbytes_fwd, xbytes_bwd;
};

// reduce-scatter backward: bf16, 16 units per workgroup, NJ = H/16 in {8, 16, 32, 64}
bool use_rs(int H, int prec) {
  return prec == PREC_BF16 && (H == 128 || H == 256 || H == 512 || H == 1024);
}

int pow2_at_least(int v) { int p = 1; while (p < v) p <<= 1; return p; }

int pick_hj(int H, bool fwd, int prec) {
  // HJ = 32 halves the backward's all-gather traffic but measured slower at c2 (5.6 vs
  // 5.0 us/step: per-workgroup load latency, not aggregate bandwidth, bounds the step);
  // kept selectable for larger H.
  if (!fwd && use_rs(H, prec)) return 16;
  if (!fwd && prec == PREC_BF16 && H % 32 == 0 && H >= 2048) return 32;
  return H % 16 == 0 ? 16 : (H % 8 == 0 ? 8 : (H % 4 == 0 ? 4 : 0));
}

Plan make_plan(int B, int H, int prec, bool fwd) {
  Plan p;
  p.HJ = pick_hj(H, fwd, prec);
  p.NJ = p.HJ ? H / p.HJ : 0;
  p.NB = (B + BG - 1) / BG;
  p.Kp = pow2_at_least(H < 128 ? 128 : H);
  p.K4p = pow2_at_least(4 * H < 128 ? 128 : 4 * H);
  const size_t esz = prec == PREC_F32 ? 4 : 2;
  const int hjt = p.HJ > 16 ? p.HJ : 16;
  p.lds = fwd ? (size_t)(prec == PREC_F32 ? 1 : 2) * 4 * (p.HJ / 4) * 64 * 16
              : (size_t)2 * 4 * 16 * hjt * 4;
  if (fwd && prec == PREC_BF16 && p.HJ == 16) p.lds += (size_t)2 * 16 * (68 + 132) * 4;  // io rings
  // > half of the CU's LDS keeps a second recurrence workgroup off the CU; bit 3 of the
  // diagnostics mode reserves enough to keep a 74 KB GEMM workgroup off it too
  const size_t min_lds = (g_dbg_mode & 8) ? (size_t)100 * 1024 : (size_t)MIN_LDS;
  if (p.lds < min_lds) p.lds = min_lds;
  p.xbytes_fwd = (size_t)2 * p.NB * NSLOT * BG * p.Kp * esz + (size_t)2 * p.NB * p.NJ * sizeof(unsigned);
  p.rs = !fwd && use_rs(H, prec);
  p.xcd = (p.rs || (fwd && prec == PREC_BF16 && p.HJ == 16)) && p.NJ <= 32 && 2 * p.NB <= 8;
  p.xbytes_bwd = p.rs ? (size_t)2 * p.NB * NSLOT * p.NJ * p.NJ * 256 * sizeof(short) +
                            (size_t)2 * p.NB * p.NJ * sizeof(unsigned)
                      : (size_t)2 * p.NB * NSLOT * BG * p.K4p * esz;
  return p;
}

int device_cus() {
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    cus = 256;
  return cus;
}

int max_batch_per_launch(int H, bool fwd, int prec) {
  const int cus = device_cus();
  int hj = pick_hj(H, fwd, prec);
  int nj = hj ? H / hj : 1;
  int nb = cus / (2 * nj);
  return nb * BG;
}

template <int PREC, int HJ, int NL>
int launch_nl(bool fwd, const LstmArgs& a, const Plan& p, hipStream_t s) {
  dim3 grid(a.xcd_local ? 8 * a.NJ : a.ndir * a.NB * a.NJ);
  auto k = fwd ? lstm_fwd_kernel<PREC, HJ, NL> : lstm_bwd_kernel<PREC, HJ, NL>;
  const size_t lds = p.lds;
  if (hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) {
    mlvae_set_error("lstm: cannot reserve %zu B LDS", lds);
    return 2;
  }
  const int nthr = (fwd && PREC == PREC_BF16 && HJ == 16) ? 320 : 256;  // + the io wave
  k<<<grid, nthr, lds, s>>>(a);
  MLVAE_CHECK_LAUNCH();
  return 0;
}

template <int PREC, int HJ>
int launch(bool fwd, const LstmArgs& a, const Plan& p, hipStream_t s) {
  constexpr int KSTEP = PREC == PREC_F32 ? 16 : 32;
  constexpr int KSF = 4;  // forward K split (see lstm_fwd_kernel)
  const int nl = fwd ? a.Kp / (KSF * KSTEP) : a.K4p / (4 * KSTEP);
  switch (nl) {
    case 1: return launch_nl<PREC, HJ, 1>(fwd, a, p, s);
    case 2: return launch_nl<PREC, HJ, 2>(fwd, a, p, s);
    case 4: return launch_nl<PREC, HJ, 4>(fwd, a, p, s);
    case 8: return launch_nl<PREC, HJ, 8>(fwd, a, p, s);
    case 16: return launch_nl<PREC, HJ, 16>(fwd, a, p, s);
    case 32: return launch_nl<PREC, HJ, 32>(fwd, a, p, s);
    default:
      mlvae_set_error("lstm: H=%d needs %d operand loads per wave (max 32)", a.H, nl);
      return 1;
  }
}

template <int NTW>
int launch_rs(const LstmArgs& a, const Plan& p, hipStream_t s) {
  dim3 grid(a.xcd_local ? 8 * a.NJ : a.ndir * a.NB * a.NJ);
  auto k = lstm_bwd_rs_kernel<NTW>;
  if (hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)p.lds) != hipSuccess) {
    mlvae_set_error("lstm: cannot reserve %zu B LDS", p.lds);
    return 2;
  }
  k<<<grid, 256, p.lds, s>>>(a);
  MLVAE_CHECK_LAUNCH();
  return 0;
}

// bf16 past one batch-group launch's batch: one wide-batch launch per direction pair
// (lstm_wide.hip) instead of sequential batch chunks, forward AND backward (they share the
// fp16 gate buffer); debug mode bit 12 forces it at any batch (A/B timing)
bool use_wide(int B, int H, int prec) {
  if (prec != PREC_BF16 || H <= 0 || H % 4) return false;
  const int bf = max_batch_per_launch(H, true, prec), bb = max_batch_per_launch(H, false, prec);
  // the wide kernels at every batch size they support (c2 B=32: 5.79 -> 4.83 ms/step, c4 T=2000:
  // 31.2 -> 23.4, the c5 shard 7.6 -> 5.7); bit 20 keeps the batch-group kernels (A/B timing)
  (void)bf; (void)bb;
  if (g_dbg_mode & (1 << 20)) return false;
  return lstm_wide_workgroups(B, H, true) > 0 && lstm_wide_workgroups(B, H, false) > 0;
}

struct WideExtra {  // outputs only the wide kernels write
  unsigned short* ydb = nullptr;  // forward: bf16 dropout(h)
  float* dbias = nullptr;         // backward: per batch group bias-gradient rows
  unsigned long long seed = 0, off = 0;
  float p = 0.f;
  WideFp8 f8;                     // fp8 mode: e4m3 dropout(h) / dG copies, dG amax
  const unsigned short* dyb = nullptr;  // backward: dY as bf16 (Y unused)
  WideZ wz;                             // forward: fused layer-0 input projection
};

int run(bool fwd, int prec, int B, int T, int H, const float* W0, const float* W1, float* G,
        float* Cs, float* Y, void* xbuf, size_t xbytes, int* err, hipStream_t st,
        unsigned short* yb = nullptr, unsigned short* dgb = nullptr, int gates_fp16 = 0,
        const WideExtra& ex = WideExtra(), int ndir = 2) {
  if (B <= 0 || T <= 0) return 0;
  if (H <= 0 || H % 4 != 0) { mlvae_set_error("lstm: H=%d must be a positive multiple of 4", H); return 1; }
  if (prec != PREC_F32 && prec != PREC_BF16) { mlvae_set_error("lstm: bad prec %d", prec); return 1; }
  // fp16 gates select the wide-batch kernels; fp32 gates the batch-group kernels (chunked)
  const bool wide = gates_fp16 != 0;
  if (ndir != 1 && ndir != 2) { mlvae_set_error("lstm: %d directions", ndir); return 1; }
  if (wide && ndir != 2) { mlvae_set_error("lstm: fp16 gates are bidirectional only"); return 1; }
  if (wide && !use_wide(B, H, prec)) {
    mlvae_set_error("lstm: B=%d H=%d prec=%d: fp16 gates only where mlvae_lstm_gates_fp16() = 1", B, H, prec);
    return 1;
  }
  if (wide) {
    if (!fwd && !dgb && !ex.f8.dg8) {
      mlvae_set_error("lstm: the wide-batch backward writes dG to dg_bf16 or (fp8 mode) dg_fp8 (both NULL)");
      return 1;
    }
    if (ex.ydb && !(ex.p >= 0.f && ex.p < 1.f)) { mlvae_set_error("lstm: dropout p=%g", ex.p); return 1; }
    return lstm_wide_run(fwd, B, T, H, W0, W1, G, Cs, Y, xbuf, xbytes, err, st, yb, dgb, ex.dbias, ex.ydb,
                         ex.seed, ex.off, ex.p, g_dbg, g_dbg_mode, ex.f8, ex.dyb, ex.wz);
  }
  if (ex.dyb) { mlvae_set_error("lstm: bf16 dY only on the wide-batch path (fp16 gates)"); return 1; }
  if (ex.ydb || ex.dbias || !Y) {
    mlvae_set_error("lstm: fused dropout / bias-gradient outputs, Y = NULL only on the wide-batch path");
    return 1;
  }
  if (!fwd && use_stepwise_bwd(H, prec)) return run_bwd_stepwise(B, T, H, ndir, W0, W1, G, Cs, Y, xbuf, xbytes, dgb, st);
  const int bmax = max_batch_per_launch(H, fwd, prec);
  if (bmax < BG) { mlvae_set_error("lstm: H=%d too large for one resident launch", H); return 1; }
  Plan full = make_plan(bmax < B ? bmax : B, H, prec, fwd);
  const size_t need_x = fwd ? full.xbytes_fwd : full.xbytes_bwd;
  if (!xbuf || xbytes < need_x || !err) {
    mlvae_set_error("lstm: exchange workspace too small (need %zu B)", need_x);
    return 1;
  }
  // batch chunks of <= bmax utterances (rows are independent)
  for (int b0 = 0; b0 < B; b0 += bmax) {
    const int bc = B - b0 < bmax ? B - b0 : bmax;
    Plan p = make_plan(bc, H, prec, fwd);
    LstmArgs a{};
    a.B = bc; a.T = T; a.H = H; a.NB = p.NB; a.NJ = p.NJ; a.HJ = p.HJ; a.Kp = p.Kp; a.K4p = p.K4p;
    a.W0 = W0; a.W1 = W1;
    const size_t gld = (size_t)4 * H * ndir, yld = (size_t)H * ndir;  // row strides
    a.ndir = ndir;
    a.G = G + (size_t)b0 * T * gld;
    a.Cs = Cs + (size_t)b0 * T * yld;
    a.Y = Y + (size_t)b0 * T * yld;
    a.xbuf = xbuf; a.err = err; a.dbg = g_dbg; a.dbg_mode = g_dbg_mode;
    a.Yb = yb ? yb + (size_t)b0 * T * yld : nullptr;
    a.dGb = dgb ? dgb + (size_t)b0 * T * gld : nullptr;
    // XCD-local groups: on by default for the forward (measured 2.67 vs 2.73 us/step at c2;
    // bit 2 turns it off), opt-in for the backward (bit 1: no gain inside a training step,
    // where the side-stream weight-gradient GEMMs want those XCDs)
    a.xcd_local = p.xcd && device_cus() == 256 && (fwd ? !(g_dbg_mode & 4) : (g_dbg_mode & 2));
    a.xtab = reinterpret_cast<unsigned*>(
        static_cast<char*>(xbuf) + (p.rs ? (size_t)2 * p.NB * NSLOT * p.NJ * p.NJ * 256 * sizeof(short)
                                         : (size_t)2 * p.NB * NSLOT * BG * p.Kp * (prec == PREC_F32 ? 4 : 2)));
    // re-initialise the exchange every call: zero fill = stale tag, zero padding
    if (hipMemsetAsync(xbuf, 0, fwd ? p.xbytes_fwd : p.xbytes_bwd, st) != hipSuccess) {
      mlvae_set_error("lstm: memset failed");
      return 2;
    }
    int rc;
    if (p.rs) {
      rc = p.NJ == 8 ? launch_rs<2>(a, p, st) : p.NJ == 16 ? launch_rs<4>(a, p, st)
         : p.NJ == 32 ? launch_rs<8>(a, p, st) : launch_rs<16>(a, p, st);
    } else if (prec == PREC_F32) {
      rc = p.HJ == 16 ? launch<PREC_F32, 16>(fwd, a, p, st)
         : p.HJ == 8 ? launch<PREC_F32, 8>(fwd, a, p, st) : launch<PREC_F32, 4>(fwd, a, p, st);
    } else {
      rc = p.HJ == 32 ? launch<PREC_BF16, 32>(fwd, a, p, st)
         : p.HJ == 16 ? launch<PREC_BF16, 16>(fwd, a, p, st)
         : p.HJ == 8 ? launch<PREC_BF16, 8>(fwd, a, p, st) : launch<PREC_BF16, 4>(fwd, a, p, st);
    }
    if (rc) return rc;
  }
  return 0;
}

}  // namespace

extern "C" int mlvae_lstm_workspace_size(int B, int H, int prec, size_t* xbytes) {
  if (H <= 0 || H % 4 != 0) { mlvae_set_error("lstm: H=%d must be a positive multiple of 4", H); return 1; }
  const int bf = max_batch_per_launch(H, true, prec), bb = max_batch_per_launch(H, false, prec);
  Plan pf = make_plan(bf < B ? bf : B, H, prec, true);
  Plan pb = make_plan(bb < B ? bb : B, H, prec, false);
  *xbytes = pf.xbytes_fwd > pb.xbytes_bwd ? pf.xbytes_fwd : pb.xbytes_bwd;
  if (use_stepwise_bwd(H, prec) && (size_t)2 * B * H * sizeof(float) > *xbytes)
    *xbytes = (size_t)2 * B * H * sizeof(float);  // the stepwise BPTT's dc state
  if (prec == PREC_BF16) {  // the wide-batch kernels' exchange (used past one launch's batch)
    const size_t wf = lstm_wide_xbytes(B, H, true), wb = lstm_wide_xbytes(B, H, false);
    if (wf > *xbytes) *xbytes = wf;
    if (wb > *xbytes) *xbytes = wb;
  }
  return 0;
}

// Workgroups one recurrence launch of this shape occupies (one per CU, all co-resident): the
// engine keeps side-stream GEMMs away from recurrences that fill the chip.
extern "C" int mlvae_lstm_launch_workgroups(int B, int H, int prec, int fwd) {
  if (B <= 0 || H <= 0 || H % 4) return 0;
  const int bmax = max_batch_per_launch(H, fwd != 0, prec);
  if (use_wide(B, H, prec)) return lstm_wide_workgroups(B, H, fwd != 0);  // with fp16 gates
  Plan p = make_plan(bmax < B ? bmax : B, H, prec, fwd != 0);
  return 2 * p.NB * p.NJ;
}

// 1 when this shape can run the wide-batch kernels (one launch for the whole batch), whose
// gate buffer is fp16 [B*T, 8H]: the caller then passes fp16 gates to the _ex2 entry points.
// fp32 gates (every other entry point) always run the batch-group kernels, batch-chunked.
extern "C" int mlvae_lstm_gates_fp16(int B, int H, int prec) { return use_wide(B, H, prec) ? 1 : 0; }
// the same for a sequence length T: 0 also where T exceeds the wide kernels' addressing
extern "C" int mlvae_lstm_gates_fp16_t(int B, int T, int H, int prec) {
  return use_wide(B, H, prec) && lstm_wide_t_ok(T, H) ? 1 : 0;
}

extern "C" int mlvae_lstm_fwd_ex2(int prec, int B, int T, int H, const float* w_hh_fwd,
                                  const float* w_hh_rev, void* gates, int gates_fp16, float* cells,
                                  float* y, void* y_bf16, void* y_drop_bf16,
                                  unsigned long long drop_seed, unsigned long long drop_offset,
                                  float drop_p, void* xbuf, size_t xbytes, int* err, void* stream) {
  WideExtra ex;
  ex.ydb = static_cast<unsigned short*>(y_drop_bf16);
  ex.seed = drop_seed; ex.off = drop_offset; ex.p = drop_p;
  return run(true, prec, B, T, H, w_hh_fwd, w_hh_rev, static_cast<float*>(gates), cells, y, xbuf,
             xbytes, err, (hipStream_t)stream, static_cast<unsigned short*>(y_bf16), nullptr,
             gates_fp16, ex);
}

// fp8 mode (configs[4]) of the wide kernels: the forward also writes dropout(h) * x8_scale as
// e4m3 (the next layer's fp8 projection operand; y_drop_bf16 NULL: the e4m3 copy alone, when no
// bf16 GEMM reads dropout(h) this step); the backward also writes dG * (*dg8_scale) as
// e4m3 (the fp8 dgrad's operand; NULL: amax only) and max-es max |dG| into *dg_amax (float bits)
extern "C" int mlvae_lstm_fwd_fp8(int B, int T, int H, const float* w_hh_fwd, const float* w_hh_rev,
                                  void* gates, float* cells, void* y_bf16, void* y_drop_bf16,
                                  void* y_drop_fp8, float x8_scale, unsigned long long drop_seed,
                                  unsigned long long drop_offset, float drop_p, void* xbuf,
                                  size_t xbytes, int* err, void* stream) {
  if (!use_wide(B, H, PREC_BF16) || !y_drop_fp8 || !(x8_scale > 0.f)) {
    mlvae_set_error("lstm_fwd_fp8: wide-batch shapes with an e4m3 dropout output and a positive scale only");
    return 1;
  }
  WideExtra ex;
  ex.ydb = static_cast<unsigned short*>(y_drop_bf16);
  ex.seed = drop_seed; ex.off = drop_offset; ex.p = drop_p;
  ex.f8.y8 = static_cast<unsigned char*>(y_drop_fp8);
  ex.f8.x8scale = x8_scale;
  return run(true, PREC_BF16, B, T, H, w_hh_fwd, w_hh_rev, static_cast<float*>(gates), cells, nullptr,
             xbuf, xbytes, err, (hipStream_t)stream, static_cast<unsigned short*>(y_bf16), nullptr, 1, ex);
}
// Wide forward of layer 0 with its input projection fused: G = z W_ih^T + b_ih + b_hh is never
// written -- each step's gate inputs come from the 32-wide bf16 layer input z [B*T rows, ldz]
// inside the recurrence (one MFMA per tile); gates receives the activated gates as from
// mlvae_lstm_fwd_ex2.  y (fp32 h), y_drop_bf16 and y_drop_fp8 (with x8_scale) are optional.
// y_bf16_prev = 1: y_bf16 row t receives the h entering step t (h_{t-1} forward, h_{t+1} reverse,
// zeros at each utterance's first step) -- dW_hh_l0's time-shifted operand pre-shifted.
extern "C" int mlvae_lstm_fwd_z2(int B, int T, int H, const float* w_hh_fwd, const float* w_hh_rev,
                                 const void* z_bf16, int ldz, int Z, const float* w_ih_fwd,
                                 const float* w_ih_rev, const float* b_ih_fwd, const float* b_hh_fwd,
                                 const float* b_ih_rev, const float* b_hh_rev, void* gates, float* cells,
                                 float* y, void* y_bf16, int y_bf16_prev, void* y_drop_bf16, void* y_drop_fp8,
                                 float x8_scale, unsigned long long drop_seed, unsigned long long drop_offset,
                                 float drop_p, void* xbuf, size_t xbytes, int* err, void* stream) {
  if (Z != 32 || !z_bf16 || !use_wide(B, H, PREC_BF16) || (y_drop_fp8 && !(x8_scale > 0.f))) {
    mlvae_set_error("lstm_fwd_z: Z = 32 on wide-batch shapes; an e4m3 dropout output needs a scale");
    return 1;
  }
  WideExtra ex;
  ex.ydb = static_cast<unsigned short*>(y_drop_bf16);
  ex.seed = drop_seed; ex.off = drop_offset; ex.p = drop_p;
  ex.f8.y8 = static_cast<unsigned char*>(y_drop_fp8);
  ex.f8.x8scale = x8_scale;
  ex.wz.zb = static_cast<const unsigned short*>(z_bf16);
  ex.wz.ldz = ldz;
  ex.wz.w0 = w_ih_fwd; ex.wz.w1 = w_ih_rev;
  ex.wz.b[0] = b_ih_fwd; ex.wz.b[1] = b_hh_fwd; ex.wz.b[2] = b_ih_rev; ex.wz.b[3] = b_hh_rev;
  ex.wz.yb_prev = y_bf16 && y_bf16_prev ? 1 : 0;
  return run(true, PREC_BF16, B, T, H, w_hh_fwd, w_hh_rev, static_cast<float*>(gates), cells, y, xbuf, xbytes,
             err, (hipStream_t)stream, static_cast<unsigned short*>(y_bf16), nullptr, 1, ex);
}
extern "C" int mlvae_lstm_fwd_z(int B, int T, int H, const float* w_hh_fwd, const float* w_hh_rev,
                                const void* z_bf16, int ldz, int Z, const float* w_ih_fwd,
                                const float* w_ih_rev, const float* b_ih_fwd, const float* b_hh_fwd,
                                const float* b_ih_rev, const float* b_hh_rev, void* gates, float* cells,
                                float* y, void* y_bf16, void* y_drop_bf16, void* y_drop_fp8, float x8_scale,
                                unsigned long long drop_seed, unsigned long long drop_offset, float drop_p,
                                void* xbuf, size_t xbytes, int* err, void* stream) {
  return mlvae_lstm_fwd_z2(B, T, H, w_hh_fwd, w_hh_rev, z_bf16, ldz, Z, w_ih_fwd, w_ih_rev, b_ih_fwd, b_hh_fwd,
                           b_ih_rev, b_hh_rev, gates, cells, y, y_bf16, 0, y_drop_bf16, y_drop_fp8, x8_scale,
                           drop_seed, drop_offset, drop_p, xbuf, xbytes, err, stream);
}
extern "C" int mlvae_lstm_bwd_fp8_ex(int B, int T, int H, const float* w_hh_fwd, const float* w_hh_rev,
                                     void* gates, const float* cells, const void* dy, int dy_bf16,
                                     void* dg_bf16, float* dbias_rows, void* dg_fp8,
                                     const float* dg8_scale, unsigned* dg_amax, void* xbuf,
                                     size_t xbytes, int* err, void* stream) {
  if (!use_wide(B, H, PREC_BF16) || !dg_amax || (dg_fp8 && !dg8_scale)) {
    mlvae_set_error("lstm_bwd_fp8: wide-batch shapes; the amax word, and a scale with the fp8 copy");
    return 1;
  }
  WideExtra ex;
  ex.dbias = dbias_rows;
  ex.f8.dg8 = static_cast<unsigned char*>(dg_fp8);
  ex.f8.g8scale = dg8_scale;
  ex.f8.g8amax = dg_amax;
  if (dy_bf16) ex.dyb = static_cast<const unsigned short*>(dy);
  return run(false, PREC_BF16, B, T, H, w_hh_fwd, w_hh_rev, static_cast<float*>(gates),
             const_cast<float*>(cells), dy_bf16 ? nullptr : static_cast<float*>(const_cast<void*>(dy)), xbuf,
             xbytes, err, (hipStream_t)stream, nullptr, static_cast<unsigned short*>(dg_bf16), 1, ex);
}
extern "C" int mlvae_lstm_bwd_fp8(int B, int T, int H, const float* w_hh_fwd, const float* w_hh_rev,
                                  void* gates, const float* cells, const float* dy, void* dg_bf16,
                                  float* dbias_rows, void* dg_fp8, const float* dg8_scale,
                                  unsigned* dg_amax, void* xbuf, size_t xbytes, int* err, void* stream) {
  return mlvae_lstm_bwd_fp8_ex(B, T, H, w_hh_fwd, w_hh_rev, gates, cells, dy, 0, dg_bf16, dbias_rows, dg_fp8,
                               dg8_scale, dg_amax, xbuf, xbytes, err, stream);
}

extern "C" int mlvae_lstm_bwd_ex2(int prec, int B, int T, int H, const float* w_hh_fwd,
                                  const float* w_hh_rev, void* gates, int gates_fp16,
                                  const float* cells, const float* dy, void* dg_bf16,
                                  float* dbias_rows, void* xbuf, size_t xbytes, int* err,
                                  void* stream) {
  WideExtra ex;
  ex.dbias = dbias_rows;
  return run(false, prec, B, T, H, w_hh_fwd, w_hh_rev, static_cast<float*>(gates),
             const_cast<float*>(cells), const_cast<float*>(dy), xbuf, xbytes, err,
             (hipStream_t)stream, nullptr, static_cast<unsigned short*>(dg_bf16), gates_fp16, ex);
}

// The wide-batch BPTT with dY as bf16 [B*T, 2H] (dy_bf16 = 1; the fused engine's heads and dgrad
// write it so): half the dY bytes of mlvae_lstm_bwd_ex2.  dy_bf16 = 0 is mlvae_lstm_bwd_ex2.
extern "C" int mlvae_lstm_bwd_ex3(int prec, int B, int T, int H, const float* w_hh_fwd,
                                  const float* w_hh_rev, void* gates, int gates_fp16,
                                  const float* cells, const void* dy, int dy_bf16, void* dg_bf16,
                                  float* dbias_rows, void* xbuf, size_t xbytes, int* err,
                                  void* stream) {
  if (dy_bf16 && !gates_fp16) {
    mlvae_set_error("lstm_bwd_ex3: bf16 dY needs the wide-batch path (fp16 gates)");
    return 1;
  }
  WideExtra ex;
  ex.dbias = dbias_rows;
  if (dy_bf16) ex.dyb = static_cast<const unsigned short*>(dy);
  return run(false, prec, B, T, H, w_hh_fwd, w_hh_rev, static_cast<float*>(gates),
             const_cast<float*>(cells), dy_bf16 ? nullptr : static_cast<float*>(const_cast<void*>(dy)), xbuf,
             xbytes, err, (hipStream_t)stream, nullptr, static_cast<unsigned short*>(dg_bf16), gates_fp16, ex);
}

// Unidirectional layer (nn.LSTM(bidirectional=False)): gates [B*T, 4H] fp32 (in: x W_ih^T + b;
// out: activated i,f,g,o), cells / y [B*T, H]; batch-group kernels with one direction's groups.
extern "C" int mlvae_lstm1_fwd(int prec, int B, int T, int H, const float* w_hh, float* gates,
                               float* cells, float* y, void* y_bf16, void* xbuf, size_t xbytes,
                               int* err, void* stream) {
  return run(true, prec, B, T, H, w_hh, w_hh, gates, cells, y, xbuf, xbytes, err,
             (hipStream_t)stream, static_cast<unsigned short*>(y_bf16), nullptr, 0, WideExtra(), 1);
}

extern "C" int mlvae_lstm1_bwd(int prec, int B, int T, int H, const float* w_hh, float* gates,
                               const float* cells, const float* dy, void* dg_bf16, void* xbuf,
                               size_t xbytes, int* err, void* stream) {
  return run(false, prec, B, T, H, w_hh, w_hh, gates, const_cast<float*>(cells),
             const_cast<float*>(dy), xbuf, xbytes, err, (hipStream_t)stream, nullptr,
             static_cast<unsigned short*>(dg_bf16), 0, WideExtra(), 1);
}

extern "C" int mlvae_lstm_fwd_ex(int prec, int B, int T, int H, const float* w_hh_fwd,
                                 const float* w_hh_rev, float* gates, float* cells, float* y,
                                 void* y_bf16, void* xbuf, size_t xbytes, int* err, void* stream) {
  return run(true, prec, B, T, H, w_hh_fwd, w_hh_rev, gates, cells, y, xbuf, xbytes, err,
             (hipStream_t)stream, static_cast<unsigned short*>(y_bf16), nullptr);
}

extern "C" int mlvae_lstm_fwd(int prec, int B, int T, int H, const float* w_hh_fwd,
                              const float* w_hh_rev, float* gates, float* cells, float* y,
                              void* xbuf, size_t xbytes, int* err, void* stream) {
  return mlvae_lstm_fwd_ex(prec, B, T, H, w_hh_fwd, w_hh_rev, gates, cells, y, nullptr, xbuf,
                           xbytes, err, stream);
}

extern "C" int mlvae_lstm_bwd_ex(int prec, int B, int T, int H, const float* w_hh_fwd,
                                 const float* w_hh_rev, float* gates, const float* cells,
                                 const float* dy, void* dg_bf16, void* xbuf, size_t xbytes,
                                 int* err, void* stream) {
  return run(false, prec, B, T, H, w_hh_fwd, w_hh_rev, gates, const_cast<float*>(cells),
             const_cast<float*>(dy), xbuf, xbytes, err, (hipStream_t)stream, nullptr,
             static_cast<unsigned short*>(dg_bf16));
}

extern "C" int mlvae_lstm_bwd(int prec, int B, int T, int H, const float* w_hh_fwd,
                              const float* w_hh_rev, float* gates, const float* cells,
                              const float* dy, void* xbuf, size_t xbytes, int* err, void* stream) {
  return mlvae_lstm_bwd_ex(prec, B, T, H, w_hh_fwd, w_hh_rev, gates, cells, dy, nullptr, xbuf,
                           xbytes, err, stream);
}

// Diagnostics: when set, the next recurrence launches record per-step phase stamps of
// workgroup 0 into buf[T*8] (s_memtime ticks).  Pass NULL to disable.
// Needs the diagnostics build (MLVAE_DIAG, lstm_common.h): the shipped library refuses a buffer.
extern "C" int mlvae_lstm_set_debug(void* buf) {
  if (buf && !MLVAE_DIAG) {
    mlvae_set_error("lstm stamps need the diagnostics build (python -m mlvae_hip.build --diag, MLVAE_LIB_PATH)");
    return 1;
  }
  g_dbg = reinterpret_cast<unsigned long long*>(buf);
  return 0;
}

// Diagnostics only (timing experiments; the bits read inside the kernels act in the MLVAE_DIAG
// build only, the launchers' bits -- 12, and 8 of the wide forward -- in both): bit0 skips the forward's saved-activation stores,
// bit1 enables XCD-local group placement of the reduce-scatter backward (measured at c2: poll
// round trip 980 vs 1376 cycles, the same step time, and 3 % slower training steps -- the
// groups take whole XCDs from the side-stream GEMMs), bit2 disables it for the forward,
// bit3 reserves 100 KB LDS per recurrence workgroup, bit4 polls with s_sleep 1 instead of 4,
// bits 5-10 delay the first poll sweep of every step by that many s_sleep 1, bit 11 times the
// batch-group kernels without their prefetch, bit 12 runs the wide-batch kernels at any batch,
// bit 23 stamps the forward pollers' publish acknowledgement, bit 24 makes the wide kernels
// cycle through all NSLOT exchange slots instead of 2 (A/B: 2 slots keep the BPTT's partial
// tiles in L2 -- PMC 5.34 -> 3.45 GB per launch at c3, 1.53 -> 1.46 ms standalone).
extern "C" int mlvae_lstm_set_debug_mode(int mode) {
  g_dbg_mode = mode;
  return 0;
}
