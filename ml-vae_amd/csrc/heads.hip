// Fused decoder heads of the VAE train step (bf16 mode): both FCBlock heads forward, the
// reconstruction loss with its masked partial sums and gradient, both heads backward and the
// gradient wrt the BiLSTM output, in ONE launch over 64-frame row tiles.
//
//   mean_fc / log_var_fc = FCBlock([2H, C, C, F])    ref:src/modules/decoder.py:16-17,24-25
//     P1 = lrelu(Y W1^T + b1)      (the two heads' first layers stacked: W1 [2C, 2H])
//     P2 = lrelu(P1_h W2_h^T + b2_h)                 ref:src/modules/fc_block.py:9-16
//     OUT_h = P2_h W3_h^T + b3_h   (mean, log_var)
//   compute_recon_loss                               ref:src/modules/decoder.py:37-53
//     likelihood: 0.5 (log 2pi + lv + (x - mu)^2 / (e^lv + 1e-5));  mse: (x - mu)^2
//   apply_lens_to_loss mask / count (gradient scale w_rec / (count * F))
//                                                    ref:src/utils/data_utils.py:67-104
//   backward: dOUT -> dP2 = (dOUT W3) * lrelu'(P2) -> dP1 = (dP2 W2) * lrelu'(P1) -> dY = dP1 W1
//
// It replaces 12-14 dependent launches (GEMMs of 13-40 us each at M = B*T, N <= 128, plus the
// recon kernel) on the step's critical path between the last forward recurrence and the first
// BPTT.  Every product is v_mfma_f32_16x16x32_bf16 with fp32 accumulation; operands swapped
// (D^T = B^T A^T) so a lane's four results are four consecutive columns of one row (16-byte
// stores, 8-byte LDS writes).
//
// Workgroup = 64 rows, 4 waves; wave w owns rows 16w .. 16w+15 through every stage, so the
// per-row LDS images are private to a wave and only the shared weight images and the staged
// W1 / W1^T chunks need workgroup barriers.  Weight images are built per workgroup from the
// fp32 parameters (two row-major, two transposed; bf16, padded rows: conflict-free 16-lane
// ds_read_b128).  Saved tensors for the weight-gradient GEMMs (side stream) are written fp32.
#include "common.h"
#include <stdlib.h>

namespace {

constexpr float LOG_2PI_H = 1.8378770351409912f;  // fp32(log(2 pi)), ref:src/modules/decoder.py:42
constexpr int RT = 64;                             // rows per workgroup

struct HeadArgs {
  int B, T, N, H2, loss_type, train;
  const unsigned short* Y;    // [N, H2] bf16
  const unsigned short* W1;   // [2C, H2] bf16
  const unsigned short* W1t;  // [H2, 2C] bf16 (train)
  const float* b1;            // [2C]
  const float* W2[2]; const float* b2[2]; const float* W3[2]; const float* b3[2];
  const float* x; const float* lens; const int* count; float rec_scale;
  float* P1; float* P2[2]; float* OUT[2]; float* dOUT[2]; float* dP2[2]; float* dP1; float* dY;
  float* partials;
  int sbf;         // the saved intermediates (P1, P2, dOUT, dP2, dP1) are bf16 (packed rows)
  float* bias_ws;  // train, optional: per-workgroup column sums [gridDim.x][NBS] of dOUT_m | dOUT_v |
                   // dP2_m | dP2_v | dP1 (the five bias gradients before the workgroup sum)
  float* wg_ws;    // split form, optional: per-workgroup partial dW3 / dW2 slabs (heads_mid_kernel<.., true>)
};

// bias-gradient column sums per workgroup: [dOUT_m F | dOUT_v F | dP2_m C | dP2_v C | dP1 2C]
template <int C, int F> constexpr int nbs() { return 2 * F + 2 * C + 2 * C; }

// sum of a lane's 4 columns over the 16 rows (lanes l15) of its wave; lanes l15 == 0 add the
// result into this wave's slot of the LDS column sums (fixed order: deterministic)
__device__ __forceinline__ void rows16_to_lds(f32x4 v, float* dst, int lane) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float x = v[r];
    x += __shfl_xor(x, 1, 64);
    x += __shfl_xor(x, 2, 64);
    x += __shfl_xor(x, 4, 64);
    x += __shfl_xor(x, 8, 64);
    v[r] = x;
  }
  if ((lane & 15) == 0) *reinterpret_cast<f32x4*>(dst + 4 * (lane >> 4)) = v;
}

__device__ __forceinline__ bf16x8 lds8(const short* p) { return *reinterpret_cast<const bf16x8*>(p); }
typedef __attribute__((address_space(3))) bf16x4* lds_b4h_p;
// MFMA operand fragment (m or n = base + (lane & 15), k = kk + 8 (lane >> 4) + e) of an LDS image
// stored [k rows][ld], read transposed by ds_read_b64_tr_b16: the weight gradients below take
// the frame rows as K
__device__ __forceinline__ bf16x8 trk(const short* img, int ld, int base, int kk, int lane) {
  const int g = lane >> 4, i4 = lane & 15, qq = i4 >> 2, pp = i4 & 3;
  const int r1 = kk + 8 * g + qq, r2 = r1 + 4;
  const bf16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_b4h_p)(img + r1 * ld + base + 4 * pp));
  const bf16x4 v2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_b4h_p)(img + r2 * ld + base + 4 * pp));
  return bf16x8{v1[0], v1[1], v1[2], v1[3], v2[0], v2[1], v2[2], v2[3]};
}
// weight-gradient tiles (16 x 16) of the fused form: dW3 of both heads [F x C], then dW2 [C x C]
template <int C, int F> constexpr int nt3() { return 2 * (F / 16) * (C / 16); }
template <int C, int F> constexpr int nt2() { return 2 * (C / 16) * (C / 16); }
// floats of one workgroup's slab (fragment order: ((tile * 64 + lane) * 4 + r))
template <int C, int F> constexpr int wg_slab() { return (nt3<C, F>() + nt2<C, F>()) * 256; }
__device__ __forceinline__ void st4bf(short* p, f32x4 v) {
  *reinterpret_cast<bf16x4*>(p) = bf16x4{f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3])};
}
// a lane's 4 consecutive values of a saved intermediate: fp32, or bf16 (the weight-gradient
// GEMMs read bf16 operands either way: same rounding, half the bytes)
__device__ __forceinline__ void st_saved(float* base, size_t idx, f32x4 v, int sbf) {
  if (sbf) st4bf(reinterpret_cast<short*>(base) + idx, v);
  else *reinterpret_cast<f32x4*>(base + idx) = v;
}
__device__ __forceinline__ bf16x8 gld8(const unsigned short* p) {
  return *reinterpret_cast<const bf16x8*>(p);
}
__device__ __forceinline__ f32x4 mfma(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

template <int C, int F>
__global__ __launch_bounds__(256) void heads_kernel(HeadArgs a) {
  constexpr int C2 = 2 * C, FK = (F + 31) / 32 * 32;
  constexpr int LC = C + 8, LF = FK + 8, L2C = C2 + 8, LS1 = 64 + 8;
  constexpr int NC = C / 16, NF = F / 16, NC2 = C2 / 16;
  // LDS image offsets (shorts)
  constexpr int O_W2I = 0, O_W2T = O_W2I + 2 * C * LC, O_W3I = O_W2T + 2 * C * LC;
  constexpr int O_W3T = O_W3I + 2 * F * LC, O_P1 = O_W3T + 2 * C * LF;
  constexpr int O_P2 = O_P1 + RT * L2C, O_DO = O_P2 + 2 * RT * LC, O_END = O_DO + 2 * RT * LF;
  constexpr int O_S1 = O_P2;   // stage-1 W1 chunks (2 x [2C][72]) alias P2 + dOUT images
  constexpr int O_S7 = O_W3I;  // stage-7 W1^T chunk ([128][L2C]) aliases the W3 images
  static_assert(O_S1 + 2 * C2 * LS1 <= O_END, "stage-1 staging overlaps");
  static_assert(O_S7 + 128 * L2C <= O_P1, "stage-7 staging overlaps");
  static_assert(O_END * 2 <= 160 * 1024, "LDS budget");
  extern __shared__ __attribute__((aligned(16))) short sm[];
  __shared__ float red[4];
  constexpr int NBS = nbs<C, F>();
  __shared__ __attribute__((aligned(16))) float bred[4][NBS];  // per-wave bias column sums
  const bool bsum = a.train && a.bias_ws != nullptr;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l15 = lane & 15, q = lane >> 4;
  const int r0 = blockIdx.x * RT;
  const int lrow = 16 * wave + l15;          // this lane's row within the tile (operand / result)
  const int grow = r0 + lrow;                // global frame row
  const bool rv = grow < a.N;
  const int H2 = a.H2;

  // ---- stage 0: weight images (bf16) from the fp32 parameters
  for (int idx = tid; idx < 2 * C * (C / 4); idx += 256) {
    const int h = idx / (C * C / 4), rem = idx % (C * C / 4), n = rem / (C / 4), k = (rem % (C / 4)) * 4;
    const f32x4 v = *reinterpret_cast<const f32x4*>(a.W2[h] + n * C + k);
    st4bf(sm + O_W2I + h * C * LC + n * LC + k, v);
#pragma unroll
    for (int i = 0; i < 4; ++i) sm[O_W2T + h * C * LC + (k + i) * LC + n] = f2bf(v[i]);
  }
  for (int idx = tid; idx < 2 * F * (C / 4); idx += 256) {
    const int h = idx / (F * C / 4), rem = idx % (F * C / 4), f = rem / (C / 4), k = (rem % (C / 4)) * 4;
    const f32x4 v = *reinterpret_cast<const f32x4*>(a.W3[h] + f * C + k);
    st4bf(sm + O_W3I + h * F * LC + f * LC + k, v);
#pragma unroll
    for (int i = 0; i < 4; ++i) sm[O_W3T + h * C * LF + (k + i) * LF + f] = f2bf(v[i]);
  }
  if constexpr (FK > F) {  // zero K padding of W3^T
    for (int idx = tid; idx < 2 * C * (FK - F); idx += 256) {
      const int h = idx / (C * (FK - F)), rem = idx % (C * (FK - F));
      sm[O_W3T + h * C * LF + (rem / (FK - F)) * LF + F + rem % (FK - F)] = 0;
    }
  }

  // ---- stage 1: P1 = lrelu(Y W1^T + b1) over K = 2H in 64-wide chunks
  f32x4 acc1[NC2];
#pragma unroll
  for (int j = 0; j < NC2; ++j) acc1[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  {
    constexpr int WPT = C2 * 8 / 256;  // 16-byte pieces of a W1 chunk per thread
    u32x4 wr[WPT];
    auto wload = [&](int k0) {
#pragma unroll
      for (int i = 0; i < WPT; ++i) {
        const int idx = tid + 256 * i, row = idx >> 3, c8 = idx & 7;
        wr[i] = *reinterpret_cast<const u32x4*>(a.W1 + (size_t)row * H2 + k0 + 8 * c8);
      }
    };
    auto wstore = [&](int buf) {
#pragma unroll
      for (int i = 0; i < WPT; ++i) {
        const int idx = tid + 256 * i, row = idx >> 3, c8 = idx & 7;
        *reinterpret_cast<u32x4*>(sm + O_S1 + buf * C2 * LS1 + row * LS1 + 8 * c8) = wr[i];
      }
    };
    const unsigned short* yrow = a.Y + (size_t)(rv ? grow : 0) * H2;
    bf16x8 ac[2], an[2];
    const bf16x8 z8 = {0, 0, 0, 0, 0, 0, 0, 0};
    auto aload = [&](int k0, bf16x8* d) {
#pragma unroll
      for (int s = 0; s < 2; ++s) d[s] = rv ? gld8(yrow + k0 + 32 * s + 8 * q) : z8;
    };
    const int nk = H2 / 64;
    wload(0);
    aload(0, ac);
    wstore(0);
    __syncthreads();
    for (int kc = 0; kc < nk; ++kc) {
      if (kc + 1 < nk) { wload((kc + 1) * 64); aload((kc + 1) * 64, an); }
      const short* Wb = sm + O_S1 + (kc & 1) * C2 * LS1;
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int j = 0; j < NC2; ++j)
          acc1[j] = mfma(lds8(Wb + (16 * j + l15) * LS1 + 32 * s + 8 * q), ac[s], acc1[j]);
      if (kc + 1 < nk) wstore((kc + 1) & 1);
      __syncthreads();
      ac[0] = an[0]; ac[1] = an[1];
    }
  }
  // lane: P1[lrow][16j + 4q + r]
#pragma unroll
  for (int j = 0; j < NC2; ++j) {
    const int col = 16 * j + 4 * q;
#pragma unroll
    for (int r = 0; r < 4; ++r) acc1[j][r] = lrelu(acc1[j][r] + a.b1[col + r]);
    st4bf(sm + O_P1 + lrow * L2C + col, acc1[j]);
    if (rv && a.train) st_saved(a.P1, (size_t)grow * C2 + col, acc1[j], a.sbf);
  }

  // ---- stages 2-3 per head: P2 = lrelu(P1_h W2^T + b2), OUT = P2 W3^T + b3
  f32x4 acc2[2][NC], acc3[2][NF];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int j = 0; j < NC; ++j) acc2[h][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < C; kk += 32) {
      const bf16x8 av = lds8(sm + O_P1 + lrow * L2C + h * C + kk + 8 * q);
#pragma unroll
      for (int j = 0; j < NC; ++j)
        acc2[h][j] = mfma(lds8(sm + O_W2I + h * C * LC + (16 * j + l15) * LC + kk + 8 * q), av, acc2[h][j]);
    }
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      const int col = 16 * j + 4 * q;
#pragma unroll
      for (int r = 0; r < 4; ++r) acc2[h][j][r] = lrelu(acc2[h][j][r] + a.b2[h][col + r]);
      st4bf(sm + O_P2 + h * RT * LC + lrow * LC + col, acc2[h][j]);
      if (rv && a.train) st_saved(a.P2[h], (size_t)grow * C + col, acc2[h][j], a.sbf);
    }
#pragma unroll
    for (int j = 0; j < NF; ++j) acc3[h][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < C; kk += 32) {
      const bf16x8 av = lds8(sm + O_P2 + h * RT * LC + lrow * LC + kk + 8 * q);
#pragma unroll
      for (int j = 0; j < NF; ++j)
        acc3[h][j] = mfma(lds8(sm + O_W3I + h * F * LC + (16 * j + l15) * LC + kk + 8 * q), av, acc3[h][j]);
    }
#pragma unroll
    for (int j = 0; j < NF; ++j) {
      const int col = 16 * j + 4 * q;
#pragma unroll
      for (int r = 0; r < 4; ++r) acc3[h][j][r] += a.b3[h][col + r];
      if (rv) *reinterpret_cast<f32x4*>(a.OUT[h] + (size_t)grow * F + col) = acc3[h][j];
    }
  }

  // ---- stage 4: reconstruction loss, masked partial sum, gradient wrt (mu, log_var)
  __shared__ float inv_cnt;
  __shared__ int cnt_sh;
  {
    const int c = block_frames(a.lens, a.B, a.T, a.count, &cnt_sh);
    if (tid == 0) inv_cnt = c > 0 ? 1.f / ((float)c * (float)F) : 0.f;
  }
  __syncthreads();  // also: all waves are past stage 1 (the staging aliases P2 / dOUT images)
  const bool lik = a.loss_type == 0;
  bool m = false;
  if (rv) {
    const int b = grow / a.T, t = grow % a.T;
    m = t < valid_frames(a.lens[b], a.T);
  }
  const float s = m ? a.rec_scale * inv_cnt : 0.f;
  float lsum = 0.f;
#pragma unroll
  for (int j = 0; j < NF; ++j) {
    const int col = 16 * j + 4 * q;
    f32x4 xv = {0.f, 0.f, 0.f, 0.f};
    if (rv) xv = *reinterpret_cast<const f32x4*>(a.x + (size_t)grow * F + col);
    f32x4 gm, gv;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float mu = acc3[0][j][r], d = xv[r] - mu;
      float rr, gmu, glv = 0.f;
      if (lik) {
        const float lv = acc3[1][j][r];
        const float elv = expf(lv), ev = elv + 1e-5f;
        rr = 0.5f * (LOG_2PI_H + lv + d * d / ev);
        gmu = -d / ev;
        glv = 0.5f * (1.f - d * d * elv / (ev * ev));
      } else {
        rr = d * d;
        gmu = -2.f * d;
      }
      if (m) lsum += rr;
      gm[r] = s * gmu;
      gv[r] = s * glv;
    }
    if (bsum) {
      rows16_to_lds(gm, &bred[wave][16 * j], lane);
      rows16_to_lds(gv, &bred[wave][F + 16 * j], lane);
    }
    if (a.train) {
      st4bf(sm + O_DO + lrow * LF + col, gm);
      st4bf(sm + O_DO + RT * LF + lrow * LF + col, gv);
      if (rv) {
        st_saved(a.dOUT[0], (size_t)grow * F + col, gm, a.sbf);
        if (lik) st_saved(a.dOUT[1], (size_t)grow * F + col, gv, a.sbf);
      }
    }
  }
  lsum = wave_sum(lsum);
  if (lane == 0) red[wave] = lsum;
  if constexpr (FK > F) {
    if (a.train) {  // zero the K padding of this wave's dOUT rows
      for (int idx = lane; idx < 2 * 16 * (FK - F); idx += 64) {
        const int h = idx / (16 * (FK - F)), rem = idx % (16 * (FK - F));
        sm[O_DO + h * RT * LF + (16 * wave + rem / (FK - F)) * LF + F + rem % (FK - F)] = 0;
      }
    }
  }
  __syncthreads();
  if (tid == 0) a.partials[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
  if (!a.train) return;

  // ---- stages 5-6 per head: dP2 = (dOUT W3) * lrelu'(P2), dP1_h = (dP2 W2) * lrelu'(P1_h)
  const int nh = lik ? 2 : 1;  // mse: log_var gets no gradient (torch leaves its grads None)
  for (int h = 0; h < 2; ++h) {
    f32x4 acc5[NC];
#pragma unroll
    for (int j = 0; j < NC; ++j) acc5[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (h < nh) {
#pragma unroll
      for (int kk = 0; kk < FK; kk += 32) {
        const bf16x8 av = lds8(sm + O_DO + h * RT * LF + lrow * LF + kk + 8 * q);
#pragma unroll
        for (int j = 0; j < NC; ++j)
          acc5[j] = mfma(lds8(sm + O_W3T + h * C * LF + (16 * j + l15) * LF + kk + 8 * q), av, acc5[j]);
      }
    }
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      const int col = 16 * j + 4 * q;
#pragma unroll
      for (int r = 0; r < 4; ++r) acc5[j][r] *= lrelu_d(acc2[h][j][r]);
      if (bsum) rows16_to_lds(acc5[j], &bred[wave][2 * F + h * C + 16 * j], lane);
      // dP2 image reuses this head's P2 image (P2 itself is dead after stage 3)
      st4bf(sm + O_P2 + h * RT * LC + lrow * LC + col, acc5[j]);
      if (rv && h < nh) st_saved(a.dP2[h], (size_t)grow * C + col, acc5[j], a.sbf);
    }
    f32x4 acc6[NC];
#pragma unroll
    for (int j = 0; j < NC; ++j) acc6[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (h < nh) {
#pragma unroll
      for (int kk = 0; kk < C; kk += 32) {
        const bf16x8 av = lds8(sm + O_P2 + h * RT * LC + lrow * LC + kk + 8 * q);
#pragma unroll
        for (int j = 0; j < NC; ++j)
          acc6[j] = mfma(lds8(sm + O_W2T + h * C * LC + (16 * j + l15) * LC + kk + 8 * q), av, acc6[j]);
      }
    }
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      const int col = h * C + 16 * j + 4 * q;
#pragma unroll
      for (int r = 0; r < 4; ++r) acc6[j][r] *= lrelu_d(acc1[h * NC + j][r]);
      if (bsum) rows16_to_lds(acc6[j], &bred[wave][2 * F + 2 * C + h * C + 16 * j], lane);
      st4bf(sm + O_P1 + lrow * L2C + col, acc6[j]);  // dP1 image reuses the P1 image
      if (rv) st_saved(a.dP1, (size_t)grow * C2 + col, acc6[j], a.sbf);
    }
  }

  // ---- stage 7: dY = dP1 W1 (K = 2C), 128 output columns per staged W1^T chunk
  bf16x8 af[C2 / 32];
#pragma unroll
  for (int s7 = 0; s7 < C2 / 32; ++s7) af[s7] = lds8(sm + O_P1 + lrow * L2C + 32 * s7 + 8 * q);
  float* dyrow = a.dY + (size_t)grow * H2;
  for (int n0 = 0; n0 < H2; n0 += 128) {
    __syncthreads();  // previous chunk consumed (first pass: every wave is past stage 5)
    if (bsum && n0 == 0) {  // this workgroup's bias column sums, the four waves in a fixed order
      for (int c = tid; c < NBS; c += 256)
        a.bias_ws[(size_t)blockIdx.x * NBS + c] = (bred[0][c] + bred[1][c]) + (bred[2][c] + bred[3][c]);
    }
    constexpr int PPT = 128 * C2 / 8 / 256;  // 16-byte pieces per thread
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      const int idx = tid + 256 * i, row = idx / (C2 / 8), c8 = idx % (C2 / 8);
      *reinterpret_cast<u32x4*>(sm + O_S7 + row * L2C + 8 * c8) =
          *reinterpret_cast<const u32x4*>(a.W1t + (size_t)(n0 + row) * C2 + 8 * c8);
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s7 = 0; s7 < C2 / 32; ++s7)
        acc = mfma(lds8(sm + O_S7 + (16 * j + l15) * L2C + 32 * s7 + 8 * q), af[s7], acc);
      if (rv) *reinterpret_cast<f32x4*>(dyrow + n0 + 16 * j + 4 * q) = acc;
    }
  }
}

// ---------------------------------------------------------------------------------------
// Split form (train, bf16 saved intermediates): the two wide products leave the fused kernel,
// whose per-tile W1 / W1^T streaming (16 + 8 dependent L2 round trips per 64-row tile at one
// workgroup per CU) made it latency-bound (1.7 TB/s):
//   1. P1 = lrelu(Y W1^T + b1)  bf16       gemm256 (bias + LReLU + bf16 staged epilogue)
//   2. heads_mid_kernel: stages 2-6 below over P1 -- persistent workgroups build the four small
//      weight images once and walk 64-row tiles, the next tile's P1 rows and x prefetched into
//      registers while the current one computes
//   3. dY = dP1 W1             fp32       gemm256 (k-contiguous dP1 and W1^T)
// The partial sums and bias column sums keep the fused kernel's per-tile layout.
// WG: the four small weight gradients (dW3 = dOUT^T P2, dW2 = dP2^T P1 per head) accumulated here
// over the workgroup's tiles, K = the 64 frame rows of a tile read transposed from the LDS images
// the stages already hold -- instead of four split-K GEMM launches (+ their reduces) re-reading
// the saved P2 / dOUT / dP2 from HBM, which are then not written at all.  Each wave owns a quarter
// of the 16 x 16 output tiles; per-workgroup slabs, reduced in a fixed order (heads_wg_reduce*).
// SPL (split-bf16 forward, the accurate-ELBO step): stages 2-3 run as P1 (W2_hi + W2_lo)^T and
// P2_hi (W3_hi + W3_lo)^T + P2_lo W3_hi^T (P2 split in registers, its lo fragment in the encoder's
// permuted k order, W3_hi read in that order by two 8-byte LDS reads), so mu_x / log_var_x carry
// the bf16 rounding of no weight (tools/elbo_budget.py: the heads' W2 / W3 rounding is the largest
// single term of the bf16 step's ELBO error).  The lo images take the room of the transposed
// W2^T / W3^T images, whose backward fragments are then read transposed from the row-major ones
// (ds_read_b64_tr_b16); W3's image then has FK zero-padded rows per head.  The backward stages
// stay bf16.
template <int C, int F, bool WG, bool SPL>
__global__ __launch_bounds__(256) void heads_mid_kernel(HeadArgs a) {
  constexpr int C2 = 2 * C, FK = (F + 31) / 32 * 32;
  constexpr int LC = C + 8, LF = FK + 8, L2C = C2 + 8;
  constexpr int NC = C / 16, NF = F / 16, NC2 = C2 / 16;
  constexpr int W3R = SPL ? FK : F;  // rows per head of the W3 image
  constexpr int O_W2I = 0, O_W2T = O_W2I + 2 * C * LC, O_W3I = O_W2T + 2 * C * LC;
  constexpr int O_W3T = O_W3I + 2 * W3R * LC, O_P1 = O_W3T + 2 * C * LF;  // SPL: W2T = W2 lo, W3T = W3 lo
  constexpr int O_P2 = O_P1 + RT * L2C, O_DO = O_P2 + 2 * RT * LC, O_END = O_DO + 2 * RT * LF;
  static_assert(!SPL || 2 * F * LC <= 2 * C * LF, "W3 lo image fits the W3^T room");
  static_assert(O_END * 2 <= 160 * 1024, "LDS budget");
  static_assert(C2 == 128, "P1 row = 16 lanes x 16 bytes");
  extern __shared__ __attribute__((aligned(16))) short sm[];
  __shared__ float red[4];
  constexpr int NBS = nbs<C, F>();
  __shared__ __attribute__((aligned(16))) float bred[4][NBS];
  __shared__ float inv_cnt;
  // b2 | b3 of both heads, staged once: read from global memory inside the tile loop, every bias
  // quad's vmcnt wait also waited for the next tile's prefetch and this tile's stores
  __shared__ __attribute__((aligned(16))) float sbias[2 * C + 2 * F];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l15 = lane & 15, q = lane >> 4;
  const int ntiles = (a.N + RT - 1) / RT;
  const bool lik = a.loss_type == 0;
  const int nh = lik ? 2 : 1;

  // ---- weight images (bf16) from the fp32 parameters, once per workgroup
  for (int idx = tid; idx < 2 * C * (C / 4); idx += 256) {
    const int h = idx / (C * C / 4), rem = idx % (C * C / 4), n = rem / (C / 4), k = (rem % (C / 4)) * 4;
    const f32x4 v = *reinterpret_cast<const f32x4*>(a.W2[h] + n * C + k);
    st4bf(sm + O_W2I + h * C * LC + n * LC + k, v);
    if constexpr (SPL) {
      *reinterpret_cast<bf16x4*>(sm + O_W2T + h * C * LC + n * LC + k) =
          bf16x4{f2bf_lo(v[0]), f2bf_lo(v[1]), f2bf_lo(v[2]), f2bf_lo(v[3])};
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) sm[O_W2T + h * C * LC + (k + i) * LC + n] = f2bf(v[i]);
    }
  }
  for (int idx = tid; idx < 2 * F * (C / 4); idx += 256) {
    const int h = idx / (F * C / 4), rem = idx % (F * C / 4), f = rem / (C / 4), k = (rem % (C / 4)) * 4;
    const f32x4 v = *reinterpret_cast<const f32x4*>(a.W3[h] + f * C + k);
    st4bf(sm + O_W3I + h * W3R * LC + f * LC + k, v);
    if constexpr (SPL) {
      *reinterpret_cast<bf16x4*>(sm + O_W3T + h * F * LC + f * LC + k) =
          bf16x4{f2bf_lo(v[0]), f2bf_lo(v[1]), f2bf_lo(v[2]), f2bf_lo(v[3])};
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) sm[O_W3T + h * C * LF + (k + i) * LF + f] = f2bf(v[i]);
    }
  }
  if constexpr (FK > F) {  // zero K padding of W3^T and of the dOUT images (never rewritten)
    if constexpr (SPL) {   // (SPL: the padding rows F..FK-1 of each head's W3 image)
      for (int idx = tid; idx < 2 * (FK - F) * LC; idx += 256)
        sm[O_W3I + (idx / ((FK - F) * LC)) * W3R * LC + F * LC + idx % ((FK - F) * LC)] = 0;
    } else {
      for (int idx = tid; idx < 2 * C * (FK - F); idx += 256) {
        const int h = idx / (C * (FK - F)), rem = idx % (C * (FK - F));
        sm[O_W3T + h * C * LF + (rem / (FK - F)) * LF + F + rem % (FK - F)] = 0;
      }
    }
    for (int idx = tid; idx < 2 * RT * (FK - F); idx += 256) {
      const int h = idx / (RT * (FK - F)), rem = idx % (RT * (FK - F));
      sm[O_DO + h * RT * LF + (rem / (FK - F)) * LF + F + rem % (FK - F)] = 0;
    }
  }
  {
    __shared__ int cnt_sh;
    const int c = block_frames(a.lens, a.B, a.T, a.count, &cnt_sh);
    if (tid == 0) inv_cnt = c > 0 ? 1.f / ((float)c * (float)F) : 0.f;
  }

  // a lane's share of its wave's 16 P1 rows (row l15 + 16 wave... as 4 x 16-byte chunks: chunk
  // q + 4 i of row l15) and its x values (row l15, columns 16 j + 4 q), prefetched a tile ahead
  const unsigned short* P1b = reinterpret_cast<const unsigned short*>(a.P1);
  u32x4 pn[4];
  f32x4 xn[NF];
  float lnn;  // ... and the row's utterance length (read in stage 4: with the tile's own loads its
              // wait would include the next tile's prefetch)
  auto prefetch = [&](int tile) {
    const int grow = tile * RT + 16 * wave + l15;
    const bool rv = tile < ntiles && grow < a.N;
    lnn = rv ? a.lens[grow / a.T] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      pn[i] = rv ? *reinterpret_cast<const u32x4*>(P1b + (size_t)grow * C2 + 8 * (q + 4 * i)) : u32x4{0u, 0u, 0u, 0u};
#pragma unroll
    for (int j = 0; j < NF; ++j)
      xn[j] = rv ? *reinterpret_cast<const f32x4*>(a.x + (size_t)grow * F + 16 * j + 4 * q) : f32x4{0.f, 0.f, 0.f, 0.f};
  };
  prefetch(blockIdx.x);
  for (int i = tid; i < 2 * C; i += 256) sbias[i] = a.b2[i / C] ? a.b2[i / C][i % C] : 0.f;
  for (int i = tid; i < 2 * F; i += 256) sbias[2 * C + i] = a.b3[i / F] ? a.b3[i / F][i % F] : 0.f;
  __syncthreads();

  const int lrow = 16 * wave + l15;
  constexpr int NT3W = nt3<C, F>() / 4, NT2W = nt2<C, F>() / 4;  // tiles per wave
  static_assert(nt3<C, F>() % 4 == 0 && nt2<C, F>() % 4 == 0, "tiles split over 4 waves");
  f32x4 aw3[WG ? NT3W : 1], aw2[WG ? NT2W : 1];
  if constexpr (WG) {
#pragma unroll
    for (int i = 0; i < NT3W; ++i) aw3[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < NT2W; ++i) aw2[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  constexpr bool SAVE = !WG;  // P2 / dOUT / dP2 have no other reader than the weight gradients
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int grow = tile * RT + lrow;
    const bool rv = grow < a.N;
    const float lenb = lnn;
    // this tile's P1 rows into the wave's P1 image; the next tile's loads go out behind them
#pragma unroll
    for (int i = 0; i < 4; ++i) *reinterpret_cast<u32x4*>(sm + O_P1 + lrow * L2C + 8 * (q + 4 * i)) = pn[i];
    f32x4 xv[NF];
#pragma unroll
    for (int j = 0; j < NF; ++j) xv[j] = xn[j];
    prefetch(tile + gridDim.x);
    // P1 in the result layout (lane: row lrow, columns 16 j + 4 q .. + 3) for lrelu' in stage 6
    f32x4 p1r[NC2];
#pragma unroll
    for (int j = 0; j < NC2; ++j) {
      const bf16x4 v = *reinterpret_cast<const bf16x4*>(sm + O_P1 + lrow * L2C + 16 * j + 4 * q);
#pragma unroll
      for (int r = 0; r < 4; ++r) p1r[j][r] = bf2f(v[r]);
    }

    // ---- stages 2-3 per head: P2 = lrelu(P1_h W2^T + b2), OUT = P2 W3^T + b3
    f32x4 acc2[2][NC], acc3[2][NF];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
      for (int j = 0; j < NC; ++j) acc2[h][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < C; kk += 32) {
        const bf16x8 av = lds8(sm + O_P1 + lrow * L2C + h * C + kk + 8 * q);
#pragma unroll
        for (int j = 0; j < NC; ++j) {
          acc2[h][j] = mfma(lds8(sm + O_W2I + h * C * LC + (16 * j + l15) * LC + kk + 8 * q), av, acc2[h][j]);
          if constexpr (SPL)
            acc2[h][j] = mfma(lds8(sm + O_W2T + h * C * LC + (16 * j + l15) * LC + kk + 8 * q), av, acc2[h][j]);
        }
      }
#pragma unroll
      for (int j = 0; j < NC; ++j) {
        const int col = 16 * j + 4 * q;
        const f32x4 bb = *reinterpret_cast<const f32x4*>(sbias + h * C + col);
#pragma unroll
        for (int r = 0; r < 4; ++r) acc2[h][j][r] = lrelu(acc2[h][j][r] + bb[r]);
        st4bf(sm + O_P2 + h * RT * LC + lrow * LC + col, acc2[h][j]);
        if (SAVE && rv) st_saved(a.P2[h], (size_t)grow * C + col, acc2[h][j], 1);
      }
#pragma unroll
      for (int j = 0; j < NF; ++j) acc3[h][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < C; kk += 32) {
        const bf16x8 av = lds8(sm + O_P2 + h * RT * LC + lrow * LC + kk + 8 * q);
#pragma unroll
        for (int j = 0; j < NF; ++j) {
          const short* wr = sm + O_W3I + h * W3R * LC + (16 * j + l15) * LC;
          acc3[h][j] = mfma(lds8(wr + kk + 8 * q), av, acc3[h][j]);
          if constexpr (SPL) {
            acc3[h][j] = mfma(lds8(sm + O_W3T + h * F * LC + (16 * j + l15) * LC + kk + 8 * q), av, acc3[h][j]);
            // P2_lo W3_hi^T: the lo fragment of k-step kk / 32 straight from the stage-2 results
            // (tiles 2s, 2s + 1: k = kk + 4 q + r and kk + 16 + 4 q + r), W3_hi read in that order
            const int s2 = kk / 32;
            const bf16x8 pl = {f2bf_lo(acc2[h][2 * s2][0]), f2bf_lo(acc2[h][2 * s2][1]),
                               f2bf_lo(acc2[h][2 * s2][2]), f2bf_lo(acc2[h][2 * s2][3]),
                               f2bf_lo(acc2[h][2 * s2 + 1][0]), f2bf_lo(acc2[h][2 * s2 + 1][1]),
                               f2bf_lo(acc2[h][2 * s2 + 1][2]), f2bf_lo(acc2[h][2 * s2 + 1][3])};
            const bf16x4 w0 = *reinterpret_cast<const bf16x4*>(wr + kk + 4 * q);
            const bf16x4 w1 = *reinterpret_cast<const bf16x4*>(wr + kk + 16 + 4 * q);
            acc3[h][j] = mfma(bf16x8{w0[0], w0[1], w0[2], w0[3], w1[0], w1[1], w1[2], w1[3]}, pl, acc3[h][j]);
          }
        }
      }
#pragma unroll
      for (int j = 0; j < NF; ++j) {
        const int col = 16 * j + 4 * q;
        const f32x4 bb = *reinterpret_cast<const f32x4*>(sbias + 2 * C + h * F + col);
#pragma unroll
        for (int r = 0; r < 4; ++r) acc3[h][j][r] += bb[r];
        if (rv) *reinterpret_cast<f32x4*>(a.OUT[h] + (size_t)grow * F + col) = acc3[h][j];
      }
    }

    // ---- stage 4: reconstruction loss, masked partial sum, gradient wrt (mu, log_var)
    bool m = false;
    if (rv) m = grow % a.T < valid_frames(lenb, a.T);
    const float sc = m ? a.rec_scale * inv_cnt : 0.f;
    float lsum = 0.f;
#pragma unroll
    for (int j = 0; j < NF; ++j) {
      const int col = 16 * j + 4 * q;
      f32x4 gm, gv;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float mu = acc3[0][j][r], d = xv[j][r] - mu;
        float rr, gmu, glv = 0.f;
        if (lik) {
          const float lv = acc3[1][j][r];
          const float elv = expf(lv), ev = elv + 1e-5f;
          rr = 0.5f * (LOG_2PI_H + lv + d * d / ev);
          gmu = -d / ev;
          glv = 0.5f * (1.f - d * d * elv / (ev * ev));
        } else {
          rr = d * d;
          gmu = -2.f * d;
        }
        if (m) lsum += rr;
        gm[r] = sc * gmu;
        gv[r] = sc * glv;
      }
      rows16_to_lds(gm, &bred[wave][16 * j], lane);
      rows16_to_lds(gv, &bred[wave][F + 16 * j], lane);
      st4bf(sm + O_DO + lrow * LF + col, gm);
      st4bf(sm + O_DO + RT * LF + lrow * LF + col, gv);
      if (SAVE && rv) {
        st_saved(a.dOUT[0], (size_t)grow * F + col, gm, 1);
        if (lik) st_saved(a.dOUT[1], (size_t)grow * F + col, gv, 1);
      }
    }
    lsum = wave_sum(lsum);
    if (lane == 0) red[wave] = lsum;
    if constexpr (WG) {
      // dW3_h += dOUT_h^T P2_h over the tile's 64 rows (every wave's rows: a barrier before, and
      // one after -- stage 5 overwrites the P2 images with dP2)
      lds_barrier();
#pragma unroll
      for (int i = 0; i < NT3W; ++i) {
        const int t = wave * NT3W + i, h = t / ((F / 16) * NC), fb = (t / NC) % (F / 16), cb = t % NC;
        if (h < nh) {
#pragma unroll
          for (int kk = 0; kk < RT; kk += 32)
            aw3[i] = mfma(trk(sm + O_DO + h * RT * LF, LF, 16 * fb, kk, lane),
                          trk(sm + O_P2 + h * RT * LC, LC, 16 * cb, kk, lane), aw3[i]);
        }
      }
      lds_barrier();
    }

    // ---- stages 5-6 per head: dP2 = (dOUT W3) * lrelu'(P2), dP1_h = (dP2 W2) * lrelu'(P1_h);
    // every image a wave reads here is its own rows: no workgroup barrier until the sums
    for (int h = 0; h < 2; ++h) {
      f32x4 acc5[NC];
#pragma unroll
      for (int j = 0; j < NC; ++j) acc5[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (h < nh) {
#pragma unroll
        for (int kk = 0; kk < FK; kk += 32) {
          const bf16x8 av = lds8(sm + O_DO + h * RT * LF + lrow * LF + kk + 8 * q);
#pragma unroll
          for (int j = 0; j < NC; ++j)
            acc5[j] = mfma(SPL ? trk(sm + O_W3I + h * W3R * LC, LC, 16 * j, kk, lane)
                               : lds8(sm + O_W3T + h * C * LF + (16 * j + l15) * LF + kk + 8 * q), av, acc5[j]);
        }
      }
#pragma unroll
      for (int j = 0; j < NC; ++j) {
        const int col = 16 * j + 4 * q;
#pragma unroll
        for (int r = 0; r < 4; ++r) acc5[j][r] *= lrelu_d(acc2[h][j][r]);
        rows16_to_lds(acc5[j], &bred[wave][2 * F + h * C + 16 * j], lane);
        st4bf(sm + O_P2 + h * RT * LC + lrow * LC + col, acc5[j]);
        if (SAVE && rv && h < nh) st_saved(a.dP2[h], (size_t)grow * C + col, acc5[j], 1);
      }
      f32x4 acc6[NC];
#pragma unroll
      for (int j = 0; j < NC; ++j) acc6[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (h < nh) {
#pragma unroll
        for (int kk = 0; kk < C; kk += 32) {
          const bf16x8 av = lds8(sm + O_P2 + h * RT * LC + lrow * LC + kk + 8 * q);
#pragma unroll
          for (int j = 0; j < NC; ++j)
            acc6[j] = mfma(SPL ? trk(sm + O_W2I + h * C * LC, LC, 16 * j, kk, lane)
                               : lds8(sm + O_W2T + h * C * LC + (16 * j + l15) * LC + kk + 8 * q), av, acc6[j]);
        }
      }
#pragma unroll
      for (int j = 0; j < NC; ++j) {
        const int col = h * C + 16 * j + 4 * q;
#pragma unroll
        for (int r = 0; r < 4; ++r) acc6[j][r] *= lrelu_d(p1r[h * NC + j][r]);
        rows16_to_lds(acc6[j], &bred[wave][2 * F + 2 * C + h * C + 16 * j], lane);
        if (rv) st_saved(a.dP1, (size_t)grow * C2 + col, acc6[j], 1);
      }
    }
    // (LDS-only barriers: the tile's saved-intermediate stores and the next tile's prefetch stay
    // in flight)
    lds_barrier();  // every wave's sums of this tile are in bred / red
    for (int c = tid; c < NBS; c += 256)
      a.bias_ws[(size_t)tile * NBS + c] = (bred[0][c] + bred[1][c]) + (bred[2][c] + bred[3][c]);
    if (tid == 0) a.partials[tile] = red[0] + red[1] + red[2] + red[3];
    if constexpr (WG) {
      // dW2_h += dP2_h^T P1_h (the dP2 images of every wave are complete at the barrier above;
      // the next tile rewrites them and the P1 image only after the one below)
#pragma unroll
      for (int i = 0; i < NT2W; ++i) {
        const int t = wave * NT2W + i, h = t / (NC * NC), ob = (t / NC) % NC, ib = t % NC;
        if (h < nh) {
#pragma unroll
          for (int kk = 0; kk < RT; kk += 32)
            aw2[i] = mfma(trk(sm + O_P2 + h * RT * LC, LC, 16 * ob, kk, lane),
                          trk(sm + O_P1, L2C, h * C + 16 * ib, kk, lane), aw2[i]);
        }
      }
    }
    lds_barrier();  // bred / red are rewritten by the next tile
  }
  if constexpr (WG) {  // this workgroup's slab, in fragment order (16-byte stores, lane-contiguous)
    float* slab = a.wg_ws + (size_t)blockIdx.x * wg_slab<C, F>();
#pragma unroll
    for (int i = 0; i < NT3W; ++i)
      *reinterpret_cast<f32x4*>(slab + ((size_t)(wave * NT3W + i) * 64 + lane) * 4) = aw3[i];
#pragma unroll
    for (int i = 0; i < NT2W; ++i)
      *reinterpret_cast<f32x4*>(slab + ((size_t)(nt3<C, F>() + wave * NT2W + i) * 64 + lane) * 4) = aw2[i];
  }
}

// bias gradients = the per-workgroup column sums summed over workgroups, in two fixed-order
// stages (deterministic): stage 1 -- block (column block of 32, slice z of RSL) sums its slice's
// workgroups with 8 row groups into slices[z]; stage 2 sums the RSL slices in order.  One block
// per column block walking all 2,000 workgroups took 96 us (latency-bound).
constexpr int RSL = 32;
__global__ __launch_bounds__(256) void heads_bias_reduce1(int nwg, int nbs, const float* __restrict__ ws,
                                                          float* __restrict__ slices) {
  __shared__ float part[8][32];
  const int c = blockIdx.x * 32 + (threadIdx.x & 31), g = threadIdx.x >> 5, z = blockIdx.y;
  const int per = (nwg + RSL - 1) / RSL, w0 = z * per, w1 = min(nwg, w0 + per);
  float v = 0.f;
  if (c < nbs)
#pragma unroll 8
    for (int w = w0 + g; w < w1; w += 8) v += ws[(size_t)w * nbs + c];
  part[g][threadIdx.x & 31] = v;
  __syncthreads();
  if (g != 0 || c >= nbs) return;
  const int e = threadIdx.x & 31;
  slices[(size_t)z * nbs + c] = ((part[0][e] + part[1][e]) + (part[2][e] + part[3][e])) +
                                ((part[4][e] + part[5][e]) + (part[6][e] + part[7][e]));
}
__global__ __launch_bounds__(256) void heads_bias_reduce2(int nbs, int F, int C, int n1,
                                                          const float* __restrict__ slices, float* db3m,
                                                          float* db3v, float* db2m, float* db2v, float* db1) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= nbs) return;
  float t = 0.f;
#pragma unroll 8
  for (int z = 0; z < RSL; ++z) t += slices[(size_t)z * nbs + c];
  if (c < F) db3m[c] = t;
  else if (c < 2 * F) { if (db3v) db3v[c - F] = t; }
  else if (c < 2 * F + C) db2m[c - 2 * F] = t;
  else if (c < 2 * F + 2 * C) { if (db2v) db2v[c - 2 * F - C] = t; }
  else if (c - 2 * F - 2 * C < n1) db1[c - 2 * F - 2 * C] = t;
}

template <int C, int F>
int launch_heads(const HeadArgs& a, hipStream_t st) {
  constexpr int FK = (F + 31) / 32 * 32, LC = C + 8, LF = FK + 8, L2C = 2 * C + 8;
  constexpr size_t lds = (size_t)(2 * C * LC * 2 + 2 * F * LC + 2 * C * LF + RT * L2C + 2 * RT * LC +
                                  2 * RT * LF) * sizeof(short);
  auto k = heads_kernel<C, F>;
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
        hipSuccess) {
      mlvae_set_error("heads: cannot reserve %zu B LDS", lds);
      return 2;
    }
    attr = true;
  }
  k<<<(a.N + RT - 1) / RT, 256, lds, st>>>(a);
  MLVAE_CHECK_LAUNCH();
  return 0;
}

// ---- the split form's two first-layer products on a 128-row kernel (instead of 256² tiles
// with a 128-wide N or K: 500 tiles in two rounds at c3).  C[M x Nn] = A[M x K] . B[Nn x K]^T,
// bf16 operands (both k-contiguous), fp32 accumulation:
//   P1 = lrelu(rnn_out W1^T + b1) -> bf16   (Nn = 2C = 128, K = 2H)
//   dY = dP1 W1                  -> bf16 / fp32 (Nn = 2H, K = 2C = 128; B = W1^T)
// A workgroup (8 waves, one 16-row slice each) walks 128-row blocks; per block the (n-chunk,
// k-chunk) pieces of B [128 x 128] pass through LDS (register double buffer, loaded one piece
// ahead), A fragments come straight from global memory into registers (each used by all 8
// n-tiles) and are kept across the n-chunks when K is one chunk.  Swapped MFMA operands: lane
// (l15, q) holds C[row 16 w + l15][16 nt + 4 q + r] -- 8- / 16-byte row stores.
constexpr int HNT_BN = 128;
// SPB (split-bf16 B, the accurate-ELBO step's P1): B is [Nn][2K'] with each 128-wide k-chunk holding
// [B_hi k 64c .. 64c+63 | B_lo same k] (mlvae_bf16_split_rows), K = 2K'; a piece's A fragments cover
// the 64 k of its chunk and are used twice, so P1 = A (W1_hi + W1_lo)^T at one pass over A.
template <bool LRELU, int HNT_BK, bool SPB = false>
__global__ __launch_bounds__(512) void heads_nt_kernel(int M, int Nn, int K, const unsigned short* __restrict__ A,
                                                       int lda, const unsigned short* __restrict__ B, int ldb,
                                                       void* __restrict__ Cv, int ldc, const float* __restrict__ bias,
                                                       int out_bf16) {
  constexpr int HNT_LB = HNT_BK + 8;  // LDS row stride (bf16)
  constexpr int BPT = HNT_BN * HNT_BK / 8 / 512;  // 16-byte B pieces per thread
  extern __shared__ __attribute__((aligned(16))) short hsm[];  // [2][HNT_BN][HNT_LB]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l15 = lane & 15, q = lane >> 4;
  const int nch = Nn / HNT_BN, kch = K / HNT_BK, npc = nch * kch;  // pieces per block
  const int nblk = (M + 127) / 128;
  // B piece p = (n-chunk p / kch, k-chunk p % kch): 128 x HNT_BK bf16 in 16-byte pieces
  u32x4 bq[BPT];
  auto bload = [&](int p) {
    const int nc = p / kch, kc = p - nc * kch;
#pragma unroll
    for (int i = 0; i < BPT; ++i) {
      const int idx = tid + 512 * i, n = idx / (HNT_BK / 8), k16 = idx % (HNT_BK / 8);
      bq[i] = *reinterpret_cast<const u32x4*>(B + (size_t)(nc * HNT_BN + n) * ldb + kc * HNT_BK + 8 * k16);
    }
  };
  auto bstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < BPT; ++i) {
      const int idx = tid + 512 * i, n = idx / (HNT_BK / 8), k16 = idx % (HNT_BK / 8);
      *reinterpret_cast<u32x4*>(hsm + buf * HNT_BN * HNT_LB + n * HNT_LB + 8 * k16) = bq[i];
    }
  };
  // A fragments of piece p of block b: rows 16 w + l15 of the block, k-chunk p % kch (a new chunk
  // per piece when K has several chunks; once per block when it has one)
  constexpr int AKC = SPB ? HNT_BK / 2 : HNT_BK;  // A's k per piece
  auto aload = [&](bf16x8 (&af)[AKC / 32], int b, int p) {
    const int row = b * 128 + 16 * wave + l15;
    const unsigned short* arow = A + (size_t)(row < M ? row : M - 1) * lda + (p % kch) * AKC;
#pragma unroll
    for (int ks = 0; ks < AKC / 32; ++ks) af[ks] = *reinterpret_cast<const bf16x8*>(arow + 32 * ks + 8 * q);
  };
  int blk = blockIdx.x;
  if (blk >= nblk) return;
  bf16x8 afr[AKC / 32], anx[AKC / 32];
  bload(0);
  aload(afr, blk, 0);
  int buf = 0;
  f32x4 acc[HNT_BN / 16];
  for (; blk < nblk; blk += gridDim.x) {
    const int row = blk * 128 + 16 * wave + l15;
    const bool rv = row < M;
    for (int p = 0; p < npc; ++p) {
      const int nc = p / kch, kc = p - nc * kch;
      // piece p: registers -> LDS buffer (its previous piece, p - 2, was read before every wave
      // passed the barrier of p - 1); the next piece's B and, when it needs new ones, A fragments
      // are loaded behind it and land under this piece's MFMAs
      bstore(buf);
      __syncthreads();
      const int nb = p + 1 < npc ? blk : blk + (int)gridDim.x, np = p + 1 < npc ? p + 1 : 0;
      const bool more = nb < nblk, new_a = more && (kch > 1 || np == 0);
      if (more) bload(np);
      if (new_a) aload(anx, nb, np);
      if (kc == 0) {
#pragma unroll
        for (int nt = 0; nt < HNT_BN / 16; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
      const short* bb = hsm + buf * HNT_BN * HNT_LB;
      // n-tile pair (2 t, 2 t + 1) covers columns 32 t .. 32 t + 31 with MFMA row i of tile 2 t + h
      // on column 32 t + 8 (i >> 2) + 4 h + (i & 3): lane (l15, q) then holds 8 consecutive
      // columns 32 t + 8 q .. + 7 of its row -- one 16-byte bf16 store per pair
#pragma unroll
      for (int ks = 0; ks < HNT_BK / 32; ++ks)
#pragma unroll
        for (int nt = 0; nt < HNT_BN / 16; ++nt) {
          const int brow = 32 * (nt >> 1) + 8 * (l15 >> 2) + 4 * (nt & 1) + (l15 & 3);
          acc[nt] = mfma(*reinterpret_cast<const bf16x8*>(bb + brow * HNT_LB + 32 * ks + 8 * q),
                         afr[ks % (AKC / 32)], acc[nt]);
        }
      buf ^= 1;
      if (kc == kch - 1 && rv) {
#pragma unroll
        for (int t = 0; t < HNT_BN / 32; ++t) {
          const int col = nc * HNT_BN + 32 * t + 8 * q;
          f32x4 v0 = acc[2 * t], v1 = acc[2 * t + 1];
          if (LRELU) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              v0[r] = lrelu(v0[r] + bias[col + r]);
              v1[r] = lrelu(v1[r] + bias[col + 4 + r]);
            }
          }
          if (out_bf16) {
            *reinterpret_cast<bf16x8*>(static_cast<unsigned short*>(Cv) + (size_t)row * ldc + col) =
                bf16x8{f2bf(v0[0]), f2bf(v0[1]), f2bf(v0[2]), f2bf(v0[3]), f2bf(v1[0]), f2bf(v1[1]), f2bf(v1[2]),
                       f2bf(v1[3])};
          } else {
            float* cr = static_cast<float*>(Cv) + (size_t)row * ldc + col;
            *reinterpret_cast<f32x4*>(cr) = v0;
            *reinterpret_cast<f32x4*>(cr + 4) = v1;
          }
        }
      }
      if (new_a) {
#pragma unroll
        for (int ks = 0; ks < AKC / 32; ++ks) afr[ks] = anx[ks];
      }
    }
  }
}

int heads_cus();
// split_b: B is the split-bf16 [Nn][2K] image (SPB above; K is A's depth, the kernel runs 2K)
int heads_nt(bool lrelu_bias, int M, int Nn, int K, const void* A, int lda, const void* B, int ldb, void* C,
             int ldc, const float* bias, bool out_bf16, hipStream_t st, bool split_b = false) {
  if (M <= 0) return 0;
  if (Nn % HNT_BN || K % 128 || lda % 8 || ldb % 8 || ldc % 8 || (lrelu_bias && !bias) ||
      (split_b && (!lrelu_bias || ldb < 2 * K))) {
    mlvae_set_error("heads_nt: Nn %% 128, K %% 128, 16-byte rows and a bias with the LReLU epilogue");
    return 1;
  }
  // k-chunks of 128, two workgroups per CU (k-chunks of 256 at one per CU: c3 heads 0.367 -> 0.375 ms)
  constexpr size_t lds = (size_t)2 * HNT_BN * (128 + 8) * sizeof(short);
  const int nblk = (M + 127) / 128, grid = nblk < 2 * heads_cus() ? nblk : 2 * heads_cus();
  const int ki = split_b ? 2 : lrelu_bias ? 1 : 0;
  auto k = split_b ? heads_nt_kernel<true, 128, true>
                   : lrelu_bias ? heads_nt_kernel<true, 128> : heads_nt_kernel<false, 128>;
  if (split_b) K *= 2;
  static bool attr[3] = {false, false, false};
  if (!attr[ki]) {
    if (hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) {
      mlvae_set_error("heads_nt: cannot reserve %zu B LDS", lds);
      return 2;
    }
    attr[ki] = true;
  }
  k<<<grid, 512, lds, st>>>(M, Nn, K, static_cast<const unsigned short*>(A), lda,
                            static_cast<const unsigned short*>(B), ldb, C, ldc, bias, out_bf16 ? 1 : 0);
  MLVAE_CHECK_LAUNCH();
  return 0;
}
// 0: the 256² GEMM for the two products; 1 (default): the 128-row kernel from 64K frames; 2: the
// 128-row kernel at every size (tests).  MLVAE_HEADS_NT sets the initial mode (A/B timing).
int g_heads_nt = [] {
  const char* e = getenv("MLVAE_HEADS_NT");
  return e ? atoi(e) : 1;
}();

int heads_cus() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}
// persistent heads_mid grid: one workgroup per CU (the LDS holds one), ~8 tiles each at c3
int mid_grid(int N) {
  const int ntiles = (N + RT - 1) / RT, cus = heads_cus();
  return ntiles < cus ? ntiles : cus;
}

template <int C, int F, bool WG, bool SPL>
int launch_mid(const HeadArgs& a, hipStream_t st) {
  constexpr int FK = (F + 31) / 32 * 32, LC = C + 8, LF = FK + 8, L2C = 2 * C + 8;
  constexpr size_t lds = (size_t)(2 * C * LC * 2 + 2 * (SPL ? FK : F) * LC + 2 * C * LF + RT * L2C +
                                  2 * RT * LC + 2 * RT * LF) * sizeof(short);
  auto k = heads_mid_kernel<C, F, WG, SPL>;
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
        hipSuccess) {
      mlvae_set_error("heads_mid: cannot reserve %zu B LDS", lds);
      return 2;
    }
    attr = true;
  }
  k<<<mid_grid(a.N), 256, lds, st>>>(a);
  MLVAE_CHECK_LAUNCH();
  return 0;
}

// the fused weight gradients' slabs: stage 1 sums slice z of the workgroups (fixed order) per
// element, stage 2 the WG_NZ slices in order and scatters fragment order to the four matrices
constexpr int WG_NZ = 16;
__global__ __launch_bounds__(256) void heads_wg_reduce1(const float* __restrict__ slabs, int G, int S,
                                                        float* __restrict__ part) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= S) return;
  const int z = blockIdx.y, g0 = z * G / WG_NZ, g1 = (z + 1) * G / WG_NZ;
  float v = 0.f;
#pragma unroll 8  // loads in flight; the adds keep their order
  for (int g = g0; g < g1; ++g) v += slabs[(size_t)g * S + e];
  part[(size_t)z * S + e] = v;
}
template <int C, int F>
__global__ __launch_bounds__(256) void heads_wg_reduce2(const float* __restrict__ part, float* dw3m,
                                                        float* dw3v, float* dw2m, float* dw2v) {
  constexpr int S = wg_slab<C, F>(), NC = C / 16, NF = F / 16;
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= S) return;
  float v = 0.f;
#pragma unroll
  for (int z = 0; z < WG_NZ; ++z) v += part[(size_t)z * S + e];
  const int r = e & 3, lane = (e >> 2) & 63, tp = e >> 8;
  const int m = 4 * (lane >> 4) + r, n = lane & 15;
  if (tp < nt3<C, F>()) {
    const int h = tp / (NF * NC), fb = (tp / NC) % NF, cb = tp % NC;
    float* d = h ? dw3v : dw3m;
    if (d) d[(16 * fb + m) * C + 16 * cb + n] = v;
  } else {
    const int t = tp - nt3<C, F>(), h = t / (NC * NC), ob = (t / NC) % NC, ib = t % NC;
    float* d = h ? dw2v : dw2m;
    if (d) d[(16 * ob + m) * C + 16 * ib + n] = v;
  }
}
template <int C, int F>
int launch_wg_reduce(const HeadArgs& a, float* dw3m, float* dw3v, float* dw2m, float* dw2v, hipStream_t st) {
  constexpr int S = wg_slab<C, F>();
  const int G = mid_grid(a.N);
  float* part = a.wg_ws + (size_t)G * S;
  heads_wg_reduce1<<<dim3((S + 255) / 256, WG_NZ), 256, 0, st>>>(a.wg_ws, G, S, part);
  MLVAE_CHECK_LAUNCH();
  heads_wg_reduce2<C, F><<<(S + 255) / 256, 256, 0, st>>>(part, dw3m, dw3v, dw2m, dw2v);
  MLVAE_CHECK_LAUNCH();
  return 0;
}

template <int C, int F>
int launch_bias_reduce(const HeadArgs& a, int n1, float* db3m, float* db3v, float* db2m, float* db2v,
                       float* db1, hipStream_t st) {
  constexpr int NBS = nbs<C, F>();
  const int nwg = (a.N + RT - 1) / RT;
  float* slices = a.bias_ws + (size_t)nwg * NBS;
  heads_bias_reduce1<<<dim3((NBS + 31) / 32, RSL), 256, 0, st>>>(nwg, NBS, a.bias_ws, slices);
  MLVAE_CHECK_LAUNCH();
  heads_bias_reduce2<<<(NBS + 255) / 256, 256, 0, st>>>(NBS, F, C, n1, slices, db3m, db3v, db2m, db2v, db1);
  MLVAE_CHECK_LAUNCH();
  return 0;
}

}  // namespace

extern "C" int mlvae_gemm_bf16(int trans_a, int trans_b, int M, int N, int K, int batch,
                               const void* A, int lda, long long a_bstride, const void* B, int ldb,
                               long long b_bstride, float* C, int ldc, long long c_bstride,
                               float beta, const float* bias1, const float* bias2, int epi,
                               const float* aux, int ldaux, int kshift_T, int kshift,
                               int kshift_bstep, unsigned long long drop_seed,
                               unsigned long long drop_offset, float drop_p,
                               float* ws, size_t ws_bytes, void* stream);

extern "C" int mlvae_heads_partials_count(int B, int T) { return (B * T + RT - 1) / RT; }

extern "C" int mlvae_heads_supported(int C, int F, int H2) {
  return C == 64 && (F == 64 || F == 80) && H2 > 0 && H2 % 128 == 0;
}

extern "C" size_t mlvae_heads_bias_workspace_size(int B, int T, int F, int C) {
  return (size_t)((B * T + RT - 1) / RT + RSL) * (2 * F + 4 * C) * sizeof(float);
}

// the fused small weight gradients (mlvae_heads_fused_ex2): per-workgroup slabs + WG_NZ partials
extern "C" int mlvae_heads_set_nt_mode(int mode) {
  if (mode < 0 || mode > 2) {
    mlvae_set_error("heads: nt mode %d (0 off, 1 auto, 2 always)", mode);
    return 1;
  }
  g_heads_nt = mode;
  return 0;
}
extern "C" size_t mlvae_heads_wgrad_workspace_size(int B, int T, int F, int C) {
  if (C != 64 || (F != 64 && F != 80) || B <= 0 || T <= 0) return 0;
  const size_t S = F == 80 ? wg_slab<64, 80>() : wg_slab<64, 64>();
  return ((size_t)mid_grid(B * T) + WG_NZ) * S * sizeof(float);
}

static int heads_impl(int B, int T, int F, int C, int H2, int loss_type, int train,
                      const void* y_bf16, const void* w1_bf16, const void* w1t_bf16,
                      const float* b1, const float* w2m, const float* b2m,
                      const float* w3m, const float* b3m, const float* w2v,
                      const float* b2v, const float* w3v, const float* b3v,
                      const float* x, const float* lens, const int* count,
                      float rec_scale, float* p1, float* p2m, float* p2v, float* mux,
                      float* lvx, float* dmux, float* dlvx, float* dp2m, float* dp2v,
                      float* dp1, float* dy, float* partials, float* bias_ws, size_t bias_ws_bytes,
                      float* db3m, float* db3v, float* db2m, float* db2v, float* db1, int saved_bf16,
                      float* wg_ws, size_t wg_ws_bytes, float* dw3m, float* dw3v, float* dw2m,
                      float* dw2v, const void* w1_split, void* stream);

extern "C" int mlvae_heads_fused(int B, int T, int F, int C, int H2, int loss_type, int train,
                                 const void* y_bf16, const void* w1_bf16, const void* w1t_bf16,
                                 const float* b1, const float* w2m, const float* b2m,
                                 const float* w3m, const float* b3m, const float* w2v,
                                 const float* b2v, const float* w3v, const float* b3v,
                                 const float* x, const float* lens, const int* count,
                                 float rec_scale, float* p1, float* p2m, float* p2v, float* mux,
                                 float* lvx, float* dmux, float* dlvx, float* dp2m, float* dp2v,
                                 float* dp1, float* dy, float* partials, void* stream) {
  return heads_impl(B, T, F, C, H2, loss_type, train, y_bf16, w1_bf16, w1t_bf16, b1, w2m, b2m, w3m,
                    b3m, w2v, b2v, w3v, b3v, x, lens, count, rec_scale, p1, p2m, p2v, mux, lvx, dmux,
                    dlvx, dp2m, dp2v, dp1, dy, partials, nullptr, 0, nullptr, nullptr, nullptr, nullptr,
                    nullptr, 0, nullptr, 0, nullptr, nullptr, nullptr, nullptr, nullptr, stream);
}

extern "C" int mlvae_heads_fused_ex(int B, int T, int F, int C, int H2, int loss_type, int train,
                                    const void* y_bf16, const void* w1_bf16, const void* w1t_bf16,
                                    const float* b1, const float* w2m, const float* b2m,
                                    const float* w3m, const float* b3m, const float* w2v,
                                    const float* b2v, const float* w3v, const float* b3v,
                                    const float* x, const float* lens, const int* count,
                                    float rec_scale, float* p1, float* p2m, float* p2v, float* mux,
                                    float* lvx, float* dmux, float* dlvx, float* dp2m, float* dp2v,
                                    float* dp1, float* dy, float* partials, float* bias_ws,
                                    size_t bias_ws_bytes, float* db3m, float* db3v, float* db2m,
                                    float* db2v, float* db1, int saved_bf16, void* stream) {
  return heads_impl(B, T, F, C, H2, loss_type, train, y_bf16, w1_bf16, w1t_bf16, b1, w2m, b2m, w3m,
                    b3m, w2v, b2v, w3v, b3v, x, lens, count, rec_scale, p1, p2m, p2v, mux, lvx, dmux,
                    dlvx, dp2m, dp2v, dp1, dy, partials, bias_ws, bias_ws_bytes, db3m, db3v, db2m, db2v,
                    db1, saved_bf16, nullptr, 0, nullptr, nullptr, nullptr, nullptr, nullptr, stream);
}

// ... and, with wg_ws, the four small weight gradients dW3 / dW2 of both heads too (written to
// dw3m / dw3v [F, C], dw2m / dw2v [C, C]; the log_var head's pointers may be null under mse):
// split form only (train, bias sums, bf16 saved intermediates).  P2 / dOUT / dP2 are then not
// written (p2m, p2v, dmux, dlvx, dp2m, dp2v may still be passed; nothing reads them)
extern "C" int mlvae_heads_fused_ex2(int B, int T, int F, int C, int H2, int loss_type, int train,
                                     const void* y_bf16, const void* w1_bf16, const void* w1t_bf16,
                                     const float* b1, const float* w2m, const float* b2m,
                                     const float* w3m, const float* b3m, const float* w2v,
                                     const float* b2v, const float* w3v, const float* b3v,
                                     const float* x, const float* lens, const int* count,
                                     float rec_scale, float* p1, float* p2m, float* p2v, float* mux,
                                     float* lvx, float* dmux, float* dlvx, float* dp2m, float* dp2v,
                                     float* dp1, float* dy, float* partials, float* bias_ws,
                                     size_t bias_ws_bytes, float* db3m, float* db3v, float* db2m,
                                     float* db2v, float* db1, int saved_bf16, float* wg_ws,
                                     size_t wg_ws_bytes, float* dw3m, float* dw3v, float* dw2m,
                                     float* dw2v, void* stream) {
  return heads_impl(B, T, F, C, H2, loss_type, train, y_bf16, w1_bf16, w1t_bf16, b1, w2m, b2m, w3m,
                    b3m, w2v, b2v, w3v, b3v, x, lens, count, rec_scale, p1, p2m, p2v, mux, lvx, dmux,
                    dlvx, dp2m, dp2v, dp1, dy, partials, bias_ws, bias_ws_bytes, db3m, db3v, db2m, db2v,
                    db1, saved_bf16, wg_ws, wg_ws_bytes, dw3m, dw3v, dw2m, dw2v, nullptr, stream);
}

// ... and, with w1_split (mlvae_bf16_split_rows of the stacked W1 [2C, 2H], chunk 64), the split-bf16
// forward: P1 = Y (W1_hi + W1_lo)^T and stages 2-3 on split W2 / W3 / P2 (heads_mid_kernel SPL)
extern "C" int mlvae_heads_fused_ex3(int B, int T, int F, int C, int H2, int loss_type, int train,
                                     const void* y_bf16, const void* w1_bf16, const void* w1t_bf16,
                                     const float* b1, const float* w2m, const float* b2m,
                                     const float* w3m, const float* b3m, const float* w2v,
                                     const float* b2v, const float* w3v, const float* b3v,
                                     const float* x, const float* lens, const int* count,
                                     float rec_scale, float* p1, float* p2m, float* p2v, float* mux,
                                     float* lvx, float* dmux, float* dlvx, float* dp2m, float* dp2v,
                                     float* dp1, float* dy, float* partials, float* bias_ws,
                                     size_t bias_ws_bytes, float* db3m, float* db3v, float* db2m,
                                     float* db2v, float* db1, int saved_bf16, float* wg_ws,
                                     size_t wg_ws_bytes, float* dw3m, float* dw3v, float* dw2m,
                                     float* dw2v, const void* w1_split, void* stream) {
  return heads_impl(B, T, F, C, H2, loss_type, train, y_bf16, w1_bf16, w1t_bf16, b1, w2m, b2m, w3m,
                    b3m, w2v, b2v, w3v, b3v, x, lens, count, rec_scale, p1, p2m, p2v, mux, lvx, dmux,
                    dlvx, dp2m, dp2v, dp1, dy, partials, bias_ws, bias_ws_bytes, db3m, db3v, db2m, db2v,
                    db1, saved_bf16, wg_ws, wg_ws_bytes, dw3m, dw3v, dw2m, dw2v, w1_split, stream);
}

// dst [rows][2 cols] bf16: each chunk-wide column block c of src [rows][cols] fp32 becomes
// [hi(src block c) | lo(src block c)] at columns 2 c chunk .. (split-bf16 operand images)
__global__ void bf16_split_rows_kernel(const float* __restrict__ src, int rows, int cols, int chunk,
                                       unsigned short* __restrict__ dst) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long long)rows * cols) return;
  const int r = (int)(i / cols), c = (int)(i % cols), blk = c / chunk, w = c % chunk;
  const float v = src[i];
  unsigned short* d = dst + (size_t)r * 2 * cols + (size_t)blk * 2 * chunk + w;
  d[0] = (unsigned short)f2bf(v);
  d[chunk] = (unsigned short)f2bf_lo(v);
}
extern "C" int mlvae_bf16_split_rows(const float* src, int rows, int cols, int chunk, void* dst, void* stream) {
  if (rows <= 0 || cols <= 0) return 0;
  if (!src || !dst || chunk <= 0 || cols % chunk) {
    mlvae_set_error("mlvae_bf16_split_rows: null pointer or cols %% chunk");
    return 1;
  }
  const long long n = (long long)rows * cols;
  bf16_split_rows_kernel<<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(
      src, rows, cols, chunk, static_cast<unsigned short*>(dst));
  MLVAE_CHECK_LAUNCH();
  return 0;
}

static int heads_impl(int B, int T, int F, int C, int H2, int loss_type, int train,
                                 const void* y_bf16, const void* w1_bf16, const void* w1t_bf16,
                                 const float* b1, const float* w2m, const float* b2m,
                                 const float* w3m, const float* b3m, const float* w2v,
                                 const float* b2v, const float* w3v, const float* b3v,
                                 const float* x, const float* lens, const int* count,
                                 float rec_scale, float* p1, float* p2m, float* p2v, float* mux,
                                 float* lvx, float* dmux, float* dlvx, float* dp2m, float* dp2v,
                                 float* dp1, float* dy, float* partials, float* bias_ws, size_t bias_ws_bytes,
                                 float* db3m, float* db3v, float* db2m, float* db2v, float* db1,
                                 int saved_bf16, float* wg_ws, size_t wg_ws_bytes, float* dw3m, float* dw3v,
                                 float* dw2m, float* dw2v, const void* w1_split, void* stream) {
  if (B <= 0 || T <= 0) return 0;
  if (!mlvae_heads_supported(C, F, H2)) {
    mlvae_set_error("heads: unsupported shape C=%d F=%d 2H=%d (C 64, F 64|80, 2H %% 128)", C, F, H2);
    return 1;
  }
  if (loss_type != 0 && loss_type != 1) { mlvae_set_error("Invalid loss type: %d", loss_type); return 1; }
  if (!y_bf16 || !w1_bf16 || !b1 || !w2m || !w3m || !w2v || !w3v || !b2m || !b3m || !b2v || !b3v ||
      !x || !lens || !mux || !lvx || !partials ||
      (train && (!w1t_bf16 || !p1 || !p2m || !p2v || !dmux || (loss_type == 0 && !dlvx) || !dp2m ||
                 !dp2v || !dp1 || !dy))) {
    mlvae_set_error("heads: null pointer");
    return 1;
  }
  HeadArgs a;
  a.B = B; a.T = T; a.N = B * T; a.H2 = H2; a.loss_type = loss_type; a.train = train;
  a.Y = static_cast<const unsigned short*>(y_bf16);
  a.W1 = static_cast<const unsigned short*>(w1_bf16);
  a.W1t = static_cast<const unsigned short*>(w1t_bf16);
  a.b1 = b1;
  a.W2[0] = w2m; a.b2[0] = b2m; a.W3[0] = w3m; a.b3[0] = b3m;
  a.W2[1] = w2v; a.b2[1] = b2v; a.W3[1] = w3v; a.b3[1] = b3v;
  a.x = x; a.lens = lens; a.count = count; a.rec_scale = rec_scale;
  a.P1 = p1; a.P2[0] = p2m; a.P2[1] = p2v; a.OUT[0] = mux; a.OUT[1] = lvx;
  a.dOUT[0] = dmux; a.dOUT[1] = dlvx; a.dP2[0] = dp2m; a.dP2[1] = dp2v; a.dP1 = dp1; a.dY = dy;
  a.partials = partials;
  a.sbf = (saved_bf16 & 1) ? 1 : 0;
  const bool dy_bf16 = (saved_bf16 & 2) != 0;  // split form: dY written as bf16 [N, H2]
  a.bias_ws = nullptr;
  if (bias_ws) {  // the five bias gradients from in-kernel column sums (train only)
    const bool mse = loss_type == 1;
    if (!train || bias_ws_bytes < mlvae_heads_bias_workspace_size(B, T, F, C) || !db3m || !db2m || !db1 ||
        (!mse && (!db3v || !db2v))) {
      mlvae_set_error("heads: bias sums need train, a workspace of %zu B and the bias gradients",
                      mlvae_heads_bias_workspace_size(B, T, F, C));
      return 1;
    }
    a.bias_ws = bias_ws;
  }
  hipStream_t st = (hipStream_t)stream;
  int rc;
  const bool split = train && bias_ws && (saved_bf16 & 1);
  a.wg_ws = nullptr;
  if (wg_ws) {
    const bool mse = loss_type == 1;
    if (!split || wg_ws_bytes < mlvae_heads_wgrad_workspace_size(B, T, F, C) || !dw3m || !dw2m ||
        (!mse && (!dw3v || !dw2v))) {
      mlvae_set_error("heads: fused weight gradients need the split form, a workspace of %zu B and "
                      "the weight gradients", mlvae_heads_wgrad_workspace_size(B, T, F, C));
      return 1;
    }
    a.wg_ws = wg_ws;
  }
  if (w1_split && !split) {
    mlvae_set_error("heads: the split-bf16 forward (w1_split) needs the split form (train, bias_ws, saved_bf16)");
    return 1;
  }
  if (dy_bf16 && !split) {
    mlvae_set_error("heads: bf16 dY (saved_bf16 bit 1) needs the split form (train, bias_ws, saved_bf16 bit 0)");
    return 1;
  }
  if (split) {
    // split form: P1 GEMM, the persistent middle stages, dY GEMM (heads_mid_kernel comment)
    constexpr int EPI_LRELU_BF16 = 1 | 32;  // gemm_fast.hip: EPI_LRELU | EPI_OUT_BF16
    // (the 256² GEMM below 64K frames: the 128-row kernel's blocks then leave CUs idle, c2 +6 us)
    const bool nt = g_heads_nt != 0 && (2 * C) % HNT_BN == 0 && H2 % 128 == 0 &&
                    (a.N >= 65536 || g_heads_nt == 2);
    // the split-bf16 forward runs P1 on the 128-row kernel at every size (its split-B form)
    rc = w1_split ? heads_nt(true, a.N, 2 * C, H2, y_bf16, H2, w1_split, 2 * H2, p1, 2 * C, b1, true, st, true)
         : nt ? heads_nt(true, a.N, 2 * C, H2, y_bf16, H2, w1_bf16, H2, p1, 2 * C, b1, true, st)
              : mlvae_gemm_bf16(0, 1, a.N, 2 * C, H2, 1, y_bf16, H2, 0, w1_bf16, H2, 0, p1, 2 * C, 0, 0.f, b1,
                                nullptr, EPI_LRELU_BF16, nullptr, 0, 0, 0, 0, 0ull, 0ull, 0.f, nullptr, 0, stream);
    if (rc) return rc;
    const bool spl = w1_split != nullptr;
    if (a.wg_ws) rc = F == 80 ? (spl ? launch_mid<64, 80, true, true>(a, st) : launch_mid<64, 80, true, false>(a, st))
                              : (spl ? launch_mid<64, 64, true, true>(a, st) : launch_mid<64, 64, true, false>(a, st));
    else rc = F == 80 ? (spl ? launch_mid<64, 80, false, true>(a, st) : launch_mid<64, 80, false, false>(a, st))
                      : (spl ? launch_mid<64, 64, false, true>(a, st) : launch_mid<64, 64, false, false>(a, st));
    if (rc) return rc;
    if (a.wg_ws) {
      const bool mse = loss_type == 1;
      rc = F == 80 ? launch_wg_reduce<64, 80>(a, dw3m, mse ? nullptr : dw3v, dw2m, mse ? nullptr : dw2v, st)
                   : launch_wg_reduce<64, 64>(a, dw3m, mse ? nullptr : dw3v, dw2m, mse ? nullptr : dw2v, st);
      if (rc) return rc;
    }
    rc = nt ? heads_nt(false, a.N, H2, 2 * C, dp1, 2 * C, w1t_bf16, 2 * C, dy, H2, nullptr, dy_bf16, st)
            : mlvae_gemm_bf16(0, 1, a.N, H2, 2 * C, 1, dp1, 2 * C, 0, w1t_bf16, 2 * C, 0, dy, H2, 0, 0.f, nullptr,
                              nullptr, dy_bf16 ? 32 : 0 /* EPI_OUT_BF16 */, nullptr, 0, 0, 0, 0, 0ull, 0ull, 0.f,
                              nullptr, 0, stream);
  } else {
    rc = F == 80 ? launch_heads<64, 80>(a, st) : launch_heads<64, 64>(a, st);
  }
  if (rc || !bias_ws) return rc;
  // mse: the log_var head gets no gradient (torch leaves its grads None): its bias gradients and
  // the log_var half of the stacked first-layer bias are not written
  const bool mse = loss_type == 1;
  const int n1 = mse ? C : 2 * C;
  return F == 80 ? launch_bias_reduce<64, 80>(a, n1, db3m, mse ? nullptr : db3v, db2m, mse ? nullptr : db2v, db1, st)
                 : launch_bias_reduce<64, 64>(a, n1, db3m, mse ? nullptr : db3v, db2m, mse ? nullptr : db2v, db1, st);
}
