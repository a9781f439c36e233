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
// Per step the workgroups of one (dir, group) all-gather h_{t-1} through a small exchange
// buffer: payload stored write-through (sc1), every storing wave drains vmcnt, one lane
// raises the slice's step flag (relaxed agent store), consumers poll the group's flags with
// one wave, barrier, then read the payload with sc1 loads straight into MFMA operands
// (MI355X_MICROARCH.md "Valid forms", row 1: one workgroup per CU, hipMalloc memory).
// The backward pass all-gathers the pre-activation gate gradients dG_t instead and
// forms dh_{t-1} = dG_t W_hh for its own hidden slice from a resident W_hh^T column slice.
#include "common.h"

namespace {

constexpr int BG = 16;             // utterances per batch group (= MFMA N/M tile)
constexpr int MAX_NJ = 64;         // hidden slices per group (flag stride)
constexpr unsigned SPIN_LIMIT = 1u << 22;
constexpr int MIN_LDS = 82 * 1024; // > half of 160 KiB: one workgroup per CU (residency)

struct LstmArgs {
  int B, T, H;        // B = utterances handled by this launch (<= NB*16)
  int NB, NJ, HJ;     // batch groups, hidden slices per group, hidden units per slice
  int Kp;             // H rounded up to 128 (fwd exchange row stride / MFMA K)
  int K4p;            // 4H rounded up to 128 (bwd exchange row stride / MFMA K)
  const float* W0;    // W_hh forward dir  [4H, H]
  const float* W1;    // W_hh reverse dir  [4H, H]
  float* G;           // [B*T, 8H] fwd: in x-proj(+biases) out activated gates; bwd: in gates, out dG
  float* Cs;          // [B*T, 2H] cell states (fwd writes, bwd reads)
  float* Y;           // [B*T, 2H] fwd: out h; bwd: in dY (grad wrt layer output)
  void* xbuf;         // exchange buffer [2 dirs][NB][2 slots][16][Kp or K4p]
  unsigned* flags;    // [2][NB][MAX_NJ]
  int* err;
};

template <int PREC> struct Elt;
template <> struct Elt<PREC_F32> { typedef float T; };
template <> struct Elt<PREC_BF16> { typedef short T; };

__device__ __forceinline__ bool wait_group(const unsigned* flags, int NJ, unsigned target,
                                           int lane, int* err) {
  unsigned spins = 0;
  while (true) {
    unsigned f = lane < NJ ? ld_flag(flags + lane) : 0xffffffffu;
    if (__all(f >= target)) return true;
    if (++spins > SPIN_LIMIT) {
      if (lane == 0) atomicExch(err, 1);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

__device__ __forceinline__ void drain_and_publish(unsigned* flag, unsigned value) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
  __syncthreads();
  if (threadIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    st_flag(flag, value);
  }
}

// ---------------------------------------------------------------------------------------
// forward recurrence
// ---------------------------------------------------------------------------------------
template <int PREC, int HJ>
__global__ __launch_bounds__(256) void lstm_fwd_kernel(LstmArgs a) {
  typedef typename Elt<PREC>::T ET;
  constexpr int ROWS = 4 * HJ, MT = ROWS / 16, KS = MT >= 4 ? 1 : 4 / MT;
  constexpr int KSTEP = PREC == PREC_F32 ? 16 : 32;  // k consumed per operand load
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int LDW = a.Kp + (PREC == PREC_F32 ? 4 : 8);
  ET* Wl = reinterpret_cast<ET*>(smem);
  float* red = reinterpret_cast<float*>(smem + (size_t)ROWS * LDW * sizeof(ET));
  __shared__ int abort_flag;

  const int ngroups = 2 * a.NB;
  const int gid = blockIdx.x % ngroups, js = blockIdx.x / ngroups;
  const int dir = gid / a.NB, grp = gid % a.NB;
  const int H = a.H, T = a.T, j0 = js * HJ;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float* W = dir ? a.W1 : a.W0;

  // resident weight slice: row r = jj*4 + q  <-  W_hh[q*H + j0 + jj][:], zero padded to Kp
  for (int idx = tid; idx < ROWS * a.Kp; idx += 256) {
    int r = idx / a.Kp, k = idx % a.Kp;
    int jj = r >> 2, q = r & 3;
    float v = k < H ? W[(size_t)(q * H + j0 + jj) * H + k] : 0.f;
    if constexpr (PREC == PREC_F32) Wl[r * LDW + k] = v; else Wl[r * LDW + k] = f2bf(v);
  }
  if (tid == 0) abort_flag = 0;
  __syncthreads();

  const int mt = wave % MT, ks = wave / MT;
  const bool active = ks < KS && wave < MT * KS;
  const bool owner = active && ks == 0;  // lanes that own (unit, utterance) cells
  const int bi = lane & 15, q = lane >> 4;
  const int jj = mt * 4 + q;             // owned unit (owner lanes)
  const int bglob = grp * BG + bi;
  const bool valid = owner && bglob < a.B;
  const int kper = a.Kp / KS, kb = ks * kper;

  const size_t xstride = (size_t)BG * a.Kp;  // one slot
  ET* xb = reinterpret_cast<ET*>(a.xbuf) + (size_t)(dir * a.NB + grp) * 2 * xstride;
  const unsigned xbytes = (unsigned)(2 * xstride * sizeof(ET));
  auto xr = make_rsrc(xb, xbytes);
  unsigned* gflags = a.flags + (size_t)(dir * a.NB + grp) * MAX_NJ;

  float c = 0.f;
  for (int s = 0; s < T; ++s) {
    const int t = dir ? T - 1 - s : s;
    const size_t n = (size_t)bglob * T + t;
    float gx[4] = {0.f, 0.f, 0.f, 0.f};
    if (valid) {
      const float* gp = a.G + n * 8 * H + dir * 4 * H + j0 + jj;
#pragma unroll
      for (int g = 0; g < 4; ++g) gx[g] = gp[g * H];
    }
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    if (s > 0) {
      if (wave == 0 && !wait_group(gflags, a.NJ, (unsigned)s, lane, a.err)) abort_flag = 1;
      __syncthreads();
      if (abort_flag) break;
      if (active) {
        const unsigned slot_off = (unsigned)(((s - 1) & 1) * xstride);
        const ET* wrow = Wl + (mt * 16 + bi) * LDW;
        for (int kk = kb; kk < kb + kper; kk += KSTEP) {
          if constexpr (PREC == PREC_F32) {
            u32x4 hv = ld_sc1_b128(xr, (slot_off + bi * a.Kp + kk + 4 * q) * 4);
            f32x4 wv = *reinterpret_cast<const f32x4*>(wrow + kk + 4 * q);
#pragma unroll
            for (int e = 0; e < 4; ++e)
              acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wv[e], __uint_as_float(hv[e]), acc, 0, 0, 0);
          } else {
            u32x4 hv = ld_sc1_b128(xr, (slot_off + bi * a.Kp + kk + 8 * q) * 2);
            bf16x8 wv = *reinterpret_cast<const bf16x8*>(wrow + kk + 8 * q);
            bf16x8 hb = *reinterpret_cast<bf16x8*>(&hv);
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wv, hb, acc, 0, 0, 0);
          }
        }
      }
      if constexpr (KS > 1) {
        if (active && ks > 0) *reinterpret_cast<f32x4*>(red + (((ks - 1) * MT + mt) * 64 + lane) * 4) = acc;
        __syncthreads();
        if (owner) {
#pragma unroll
          for (int p = 1; p < KS; ++p) {
            f32x4 o = *reinterpret_cast<const f32x4*>(red + (((p - 1) * MT + mt) * 64 + lane) * 4);
            acc += o;
          }
        }
      }
    }
    if (valid) {
      // acc[q'] = recurrent part of gate q' for unit jj, utterance bi
      float ig = sigmoidf_(acc[0] + gx[0]);
      float fg = sigmoidf_(acc[1] + gx[1]);
      float gg = tanhf(acc[2] + gx[2]);
      float og = sigmoidf_(acc[3] + gx[3]);
      c = fg * c + ig * gg;
      float hv = og * tanhf(c);
      float* gp = a.G + n * 8 * H + dir * 4 * H + j0 + jj;
      gp[0] = ig; gp[H] = fg; gp[2 * H] = gg; gp[3 * H] = og;
      a.Cs[n * 2 * H + dir * H + j0 + jj] = c;
      a.Y[n * 2 * H + dir * H + j0 + jj] = hv;
      const unsigned off = (unsigned)((s & 1) * xstride + bi * a.Kp + j0 + jj);
      if constexpr (PREC == PREC_F32) st_sc1_b32(xr, off * 4, __float_as_uint(hv));
      else st_sc1_b16(xr, off * 2, (unsigned short)f2bf(hv));
    }
    if (s + 1 < T) drain_and_publish(gflags + js, (unsigned)(s + 1));
  }
}

// ---------------------------------------------------------------------------------------
// backward recurrence (BPTT)
// ---------------------------------------------------------------------------------------
template <int PREC, int HJ>
__global__ __launch_bounds__(256) void lstm_bwd_kernel(LstmArgs a) {
  typedef typename Elt<PREC>::T ET;
  constexpr int KSTEP = PREC == PREC_F32 ? 16 : 32;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int LDW = a.K4p + (PREC == PREC_F32 ? 4 : 8);
  ET* Wt = reinterpret_cast<ET*>(smem);  // [16 cols (unit jj)][K4p] : W_hh[g][j0+jj]
  float* red = reinterpret_cast<float*>(smem + (size_t)16 * LDW * sizeof(ET));  // [4][16][16]
  __shared__ int abort_flag;

  const int ngroups = 2 * a.NB;
  const int gid = blockIdx.x % ngroups, js = blockIdx.x / ngroups;
  const int dir = gid / a.NB, grp = gid % a.NB;
  const int H = a.H, T = a.T, j0 = js * HJ, G4 = 4 * H;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float* W = dir ? a.W1 : a.W0;

  for (int idx = tid; idx < 16 * a.K4p; idx += 256) {
    int jj = idx / a.K4p, g = idx % a.K4p;
    float v = (jj < HJ && g < G4) ? W[(size_t)g * H + j0 + jj] : 0.f;
    if constexpr (PREC == PREC_F32) Wt[jj * LDW + g] = v; else Wt[jj * LDW + g] = f2bf(v);
  }
  if (tid == 0) abort_flag = 0;
  __syncthreads();

  // MFMA roles: A = dG (rows = utterances), B = W_hh^T slice (cols = units), K = 4H over 4 waves
  const int bi = lane & 15, q = lane >> 4;
  const int kper = a.K4p / 4, kb = wave * kper;
  // cell roles: thread -> (utterance cb, unit cj)
  const int cb = tid >> 4, cj = tid & 15;
  const int bglob = grp * BG + cb;
  const bool valid = cj < HJ && bglob < a.B;
  const int j = j0 + cj;

  const size_t xstride = (size_t)BG * a.K4p;
  ET* xb = reinterpret_cast<ET*>(a.xbuf) + (size_t)(dir * a.NB + grp) * 2 * xstride;
  auto xr = make_rsrc(xb, (unsigned)(2 * xstride * sizeof(ET)));
  unsigned* gflags = a.flags + (size_t)(dir * a.NB + grp) * MAX_NJ;
  const int grp_b0 = grp * BG;

  float dc = 0.f;
  for (int s = 0; s < T; ++s) {
    const int t = dir ? s : T - 1 - s;          // reverse of the forward processing order
    const int tprev = dir ? t + 1 : t - 1;       // the forward's previous step
    const size_t n = (size_t)bglob * T + t;
    // prefetch this step's cell inputs
    float gi = 0.f, gf = 0.f, gg = 0.f, go = 0.f, cc = 0.f, cp = 0.f, dy = 0.f;
    if (valid) {
      const float* gp = a.G + n * 8 * H + dir * 4 * H + j;
      gi = gp[0]; gf = gp[H]; gg = gp[2 * H]; go = gp[3 * H];
      cc = a.Cs[n * 2 * H + dir * H + j];
      if (tprev >= 0 && tprev < T) cp = a.Cs[((size_t)bglob * T + tprev) * 2 * H + dir * H + j];
      dy = a.Y[n * 2 * H + dir * H + j];
    }
    float dhrec = 0.f;
    if (s > 0) {
      if (wave == 0 && !wait_group(gflags, a.NJ, (unsigned)s, lane, a.err)) abort_flag = 1;
      __syncthreads();
      if (abort_flag) break;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      const unsigned slot_off = (unsigned)(((s - 1) & 1) * xstride);
      const ET* wcol = Wt + bi * LDW;  // B operand column = unit bi
      for (int kk = kb; kk < kb + kper; kk += KSTEP) {
        if constexpr (PREC == PREC_F32) {
          u32x4 gv = ld_sc1_b128(xr, (slot_off + bi * a.K4p + kk + 4 * q) * 4);
          f32x4 wv = *reinterpret_cast<const f32x4*>(wcol + kk + 4 * q);
#pragma unroll
          for (int e = 0; e < 4; ++e)
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(gv[e]), wv[e], acc, 0, 0, 0);
        } else {
          u32x4 gv = ld_sc1_b128(xr, (slot_off + bi * a.K4p + kk + 8 * q) * 2);
          bf16x8 gb = *reinterpret_cast<bf16x8*>(&gv);
          bf16x8 wv = *reinterpret_cast<const bf16x8*>(wcol + kk + 8 * q);
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(gb, wv, acc, 0, 0, 0);
        }
      }
      // C layout: col = lane&15 = unit, row = 4*(lane>>4)+r = utterance
#pragma unroll
      for (int r = 0; r < 4; ++r) red[(wave * 16 + 4 * q + r) * 16 + bi] = acc[r];
      __syncthreads();
      dhrec = red[(0 * 16 + cb) * 16 + cj] + red[(1 * 16 + cb) * 16 + cj] +
              red[(2 * 16 + cb) * 16 + cj] + red[(3 * 16 + cb) * 16 + cj];
    }
    if (valid) {
      const float dh = dy + dhrec;
      const float tc = tanhf(cc);
      const float d_o = dh * tc;
      const float dcs = dc + dh * go * (1.f - tc * tc);
      const float di = dcs * gg, dgg = dcs * gi, df = dcs * cp;
      dc = dcs * gf;
      const float dai = di * gi * (1.f - gi);
      const float daf = df * gf * (1.f - gf);
      const float dag = dgg * (1.f - gg * gg);
      const float dao = d_o * go * (1.f - go);
      float* gp = a.G + n * 8 * H + dir * 4 * H + j;
      gp[0] = dai; gp[H] = daf; gp[2 * H] = dag; gp[3 * H] = dao;
      const unsigned off = (unsigned)((s & 1) * xstride + cb * a.K4p + j);
      if constexpr (PREC == PREC_F32) {
        st_sc1_b32(xr, (off + 0 * H) * 4, __float_as_uint(dai));
        st_sc1_b32(xr, (off + 1 * H) * 4, __float_as_uint(daf));
        st_sc1_b32(xr, (off + 2 * H) * 4, __float_as_uint(dag));
        st_sc1_b32(xr, (off + 3 * H) * 4, __float_as_uint(dao));
      } else {
        st_sc1_b16(xr, (off + 0 * H) * 2, (unsigned short)f2bf(dai));
        st_sc1_b16(xr, (off + 1 * H) * 2, (unsigned short)f2bf(daf));
        st_sc1_b16(xr, (off + 2 * H) * 2, (unsigned short)f2bf(dag));
        st_sc1_b16(xr, (off + 3 * H) * 2, (unsigned short)f2bf(dao));
      }
    }
    (void)grp_b0;
    if (s + 1 < T) drain_and_publish(gflags + js, (unsigned)(s + 1));
  }
}

struct Plan {
  int NB, NJ, HJ, Kp, K4p;
  size_t lds_fwd, lds_bwd, xbytes_fwd, xbytes_bwd;
};

int pick_hj(int H) { return H % 16 == 0 ? 16 : (H % 8 == 0 ? 8 : (H % 4 == 0 ? 4 : 0)); }

Plan make_plan(int B, int H, int prec) {
  Plan p;
  p.HJ = pick_hj(H);
  p.NJ = p.HJ ? H / p.HJ : 0;
  p.NB = (B + BG - 1) / BG;
  p.Kp = (H + 127) / 128 * 128;
  p.K4p = (4 * H + 127) / 128 * 128;
  const size_t esz = prec == PREC_F32 ? 4 : 2;
  const int pad = prec == PREC_F32 ? 4 : 8;
  p.lds_fwd = (size_t)4 * p.HJ * (p.Kp + pad) * esz + 3 * 64 * 4 * 4 * 4;
  p.lds_bwd = (size_t)16 * (p.K4p + pad) * esz + 4 * 16 * 16 * 4;
  if (p.lds_fwd < MIN_LDS) p.lds_fwd = MIN_LDS;
  if (p.lds_bwd < MIN_LDS) p.lds_bwd = MIN_LDS;
  p.xbytes_fwd = (size_t)2 * p.NB * 2 * BG * p.Kp * esz;
  p.xbytes_bwd = (size_t)2 * p.NB * 2 * BG * p.K4p * esz;
  return p;
}

int max_batch_per_launch(int H) {
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    cus = 256;
  int hj = pick_hj(H);
  int nj = hj ? H / hj : 1;
  int nb = cus / (2 * nj);
  return nb * BG;
}

template <int PREC, int HJ>
int launch(bool fwd, const LstmArgs& a, const Plan& p, hipStream_t s) {
  dim3 grid(2 * a.NB * a.NJ);
  if (fwd) {
    auto k = lstm_fwd_kernel<PREC, HJ>;
    if (hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)p.lds_fwd) != hipSuccess) {
      mlvae_set_error("lstm: cannot reserve %zu B LDS", p.lds_fwd);
      return 2;
    }
    k<<<grid, 256, p.lds_fwd, s>>>(a);
  } else {
    auto k = lstm_bwd_kernel<PREC, HJ>;
    if (hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)p.lds_bwd) != hipSuccess) {
      mlvae_set_error("lstm: cannot reserve %zu B LDS", p.lds_bwd);
      return 2;
    }
    k<<<grid, 256, p.lds_bwd, s>>>(a);
  }
  MLVAE_CHECK_LAUNCH();
  return 0;
}

int run(bool fwd, int prec, int B, int T, int H, const float* W0, const float* W1, float* G,
        float* Cs, float* Y, void* xbuf, size_t xbytes, unsigned* flags, size_t fbytes, int* err,
        hipStream_t st) {
  if (B <= 0 || T <= 0) return 0;
  if (H <= 0 || H % 4 != 0) { mlvae_set_error("lstm: H=%d must be a positive multiple of 4", H); return 1; }
  if (prec != PREC_F32 && prec != PREC_BF16) { mlvae_set_error("lstm: bad prec %d", prec); return 1; }
  const int bmax = max_batch_per_launch(H);
  if (bmax < BG) { mlvae_set_error("lstm: H=%d too large for one resident launch", H); return 1; }
  Plan full = make_plan(bmax < B ? bmax : B, H, prec);
  if (full.NJ > MAX_NJ) { mlvae_set_error("lstm: H=%d needs %d slices > %d", H, full.NJ, MAX_NJ); return 1; }
  const size_t need_x = fwd ? full.xbytes_fwd : full.xbytes_bwd;
  const size_t need_f = (size_t)2 * full.NB * MAX_NJ * sizeof(unsigned);
  if (!xbuf || xbytes < need_x || !flags || fbytes < need_f || !err) {
    mlvae_set_error("lstm: workspace too small (need x=%zu flags=%zu)", need_x, need_f);
    return 1;
  }
  // batch chunks of <= bmax utterances (rows are independent)
  for (int b0 = 0; b0 < B; b0 += bmax) {
    const int bc = B - b0 < bmax ? B - b0 : bmax;
    Plan p = make_plan(bc, H, prec);
    LstmArgs a;
    a.B = bc; a.T = T; a.H = H; a.NB = p.NB; a.NJ = p.NJ; a.HJ = p.HJ; a.Kp = p.Kp; a.K4p = p.K4p;
    a.W0 = W0; a.W1 = W1;
    a.G = G + (size_t)b0 * T * 8 * H;
    a.Cs = Cs + (size_t)b0 * T * 2 * H;
    a.Y = Y + (size_t)b0 * T * 2 * H;
    a.xbuf = xbuf; a.flags = flags; a.err = err;
    // re-initialise every polled word and the zero padding of the exchange rows
    if (hipMemsetAsync(flags, 0, need_f, st) != hipSuccess ||
        hipMemsetAsync(xbuf, 0, fwd ? p.xbytes_fwd : p.xbytes_bwd, st) != hipSuccess) {
      mlvae_set_error("lstm: memset failed");
      return 2;
    }
    int rc;
    if (prec == PREC_F32) {
      rc = p.HJ == 16 ? launch<PREC_F32, 16>(fwd, a, p, st)
         : p.HJ == 8 ? launch<PREC_F32, 8>(fwd, a, p, st) : launch<PREC_F32, 4>(fwd, a, p, st);
    } else {
      rc = p.HJ == 16 ? launch<PREC_BF16, 16>(fwd, a, p, st)
         : p.HJ == 8 ? launch<PREC_BF16, 8>(fwd, a, p, st) : launch<PREC_BF16, 4>(fwd, a, p, st);
    }
    if (rc) return rc;
  }
  return 0;
}

}  // namespace

extern "C" int mlvae_lstm_workspace_size(int B, int H, int prec, size_t* xbytes, size_t* fbytes) {
  if (H <= 0 || H % 4 != 0) { mlvae_set_error("lstm: H=%d must be a positive multiple of 4", H); return 1; }
  const int bmax = max_batch_per_launch(H);
  Plan p = make_plan(bmax < B ? bmax : B, H, prec);
  *xbytes = p.xbytes_fwd > p.xbytes_bwd ? p.xbytes_fwd : p.xbytes_bwd;
  *fbytes = (size_t)2 * p.NB * MAX_NJ * sizeof(unsigned);
  return 0;
}

extern "C" int mlvae_lstm_fwd(int prec, int B, int T, int H, const float* w_hh_fwd,
                              const float* w_hh_rev, float* gates, float* cells, float* y,
                              void* xbuf, size_t xbytes, unsigned* flags, size_t fbytes, int* err,
                              void* stream) {
  return run(true, prec, B, T, H, w_hh_fwd, w_hh_rev, gates, cells, y, xbuf, xbytes, flags, fbytes,
             err, (hipStream_t)stream);
}

extern "C" int mlvae_lstm_bwd(int prec, int B, int T, int H, const float* w_hh_fwd,
                              const float* w_hh_rev, float* gates, const float* cells,
                              const float* dy, void* xbuf, size_t xbytes, unsigned* flags,
                              size_t fbytes, int* err, void* stream) {
  return run(false, prec, B, T, H, w_hh_fwd, w_hh_rev, gates, const_cast<float*>(cells),
             const_cast<float*>(dy), xbuf, xbytes, flags, fbytes, err, (hipStream_t)stream);
}
