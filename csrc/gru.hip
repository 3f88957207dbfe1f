// GRU(256) recurrent Q-net on minute-bar sequences (BASELINE config 5), MI355X-native.
//
// Not in the reference (its Q-net is a 203->200->3 MLP over a flattened 201-price
// window, QDecisionPolicyActor.scala:38-50); this is the north-star recurrent variant
// of the same Buy/Sell/Hold agent (action order 0,1,2 as QDecisionPolicyActor.scala:17).
//
// Actor (gru_act_kernel) — the fp8 MFMA path:
//   * one workgroup = 8 waves owns a chunk of 32 envs and runs S env steps on-chip;
//     wave w owns hidden units 32w..32w+31 of all three gates (r, z, n: torch.nn.GRUCell
//     order), so the whole GRU update of a unit happens in the lane that holds it;
//   * W_hh (768x256) lives in VGPRs for the life of the kernel as block-scaled MX-fp8
//     (OCP e4m3 + one E8M0 scale per 32-element block: the gfx950 scaled MFMA
//     v_mfma_scale_f32_16x16x128_f8f6f4, 2x the bf16 MFMA rate); W_ih (x part, K=32)
//     is bf16 in LDS (one 16x16x32 bf16 MFMA per tile);
//   * 16x16x128 operand layout (measured, tools/mx_layout_probe.py): lane l = i + 16g holds
//     row/col i, K = [16g, 16g+16) in bytes 0..15 and [64+16g, 64+16g+16) in bytes 16..31;
//     the E8M0 scale of (row i, K-block s = [32s, 32s+32)) is read from lane i + 16s --
//     so a lane's scale is NOT the scale of its own bytes;
//   * h is fp32 in registers (exact recurrence) and is re-quantized every step into an
//     LDS fp8 tile with per-(env, 32-unit block) E8M0 scales -- each scale block is
//     exactly one wave's unit range, so amax is a 4-lane reduction;
//   * Q = W_q h is reduced across waves through LDS; wave 0 runs epsilon-greedy
//     (Philox), the minute-bar trading env, and writes the replay segment.
// Learner: csrc/gru_learn.hip.
#include "gru_common.h"

namespace st {

// ---------------------------------------------------------------- synthetic minute bars
struct MinuteBars {
  float* close;        // [E][T]
  bf16_t* feat;        // [E][T][RMF]
  int E, T, day;       // bars per session (U-shaped intraday volatility / volume)
  float sigma, phi, alpha, beta, p0;
  uint32_t key0, key1;
};

// one thread per env, sequential over time: AR(1) log returns with GARCH(1,1) variance
// and a U-shaped intraday profile; OHLC + volume -> 8 features per bar.
__global__ void __launch_bounds__(256) minute_bars_kernel(MinuteBars g) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= g.E) return;
  uint32_t c0 = (uint32_t)e, c1 = 0xFFFFFFFFu, c2 = 0u, c3 = 0x4D424152u;
  philox4x32(c0, c1, c2, c3, g.key0, g.key1);
  float c = g.p0 * (0.5f + u24(c0));
  float var = g.sigma * g.sigma, rprev = 0.f;
  const float omega = g.sigma * g.sigma * (1.f - g.alpha - g.beta);
  float r1 = 0.f, r2 = 0.f, r3 = 0.f, r4 = 0.f;   // previous 4 returns (5-bar momentum)
  for (int t = 0; t < g.T; ++t) {
    uint32_t a0 = (uint32_t)e, a1 = (uint32_t)t, a2 = 0u, a3 = 0x4D424152u;
    philox4x32(a0, a1, a2, a3, g.key0, g.key1);
    const float u0 = fmaxf(u24(a0), 1e-7f), u1 = u24(a1), u2 = fmaxf(u24(a2), 1e-7f), u3 = u24(a3);
    const float rad0 = sqrtf(-2.f * logf(u0)), rad1 = sqrtf(-2.f * logf(u2));
    const float n1 = rad0 * cosf(6.2831853f * u1), n2 = rad0 * sinf(6.2831853f * u1);
    const float n3 = rad1 * cosf(6.2831853f * u3), n4 = rad1 * sinf(6.2831853f * u3);
    const int tod = t % g.day;
    const float x = (2.f * (float)tod / (float)g.day) - 1.f;
    const float ush = 1.f + 0.8f * x * x;
    const float sig = sqrtf(var) * ush;
    const float ret = g.phi * rprev + sig * n1;
    const float open = c;
    c = open * expf(ret);
    const float hi = fmaxf(open, c) * expf(0.5f * sig * fabsf(n2));
    const float lo = fminf(open, c) * expf(-0.5f * sig * fabsf(n3));
    const float vol = expf(0.5f * n4) * ush;
    const float dsr = ret / ush;   // de-seasonalised: the U-shape must not feed the GARCH recursion
    var = omega + g.alpha * dsr * dsr + g.beta * var;
    const float mom = ret + r1 + r2 + r3 + r4;
    r4 = r3; r3 = r2; r2 = r1; r1 = ret;
    rprev = ret;
    const float ang = 6.2831853f * (float)tod / (float)g.day;
    const size_t o = (size_t)e * g.T + t;
    g.close[o] = c;
    uint4 w;
    w.x = pack_bf2(ret * 100.f, (hi - lo) / c * 100.f);
    w.y = pack_bf2((c - lo) / fmaxf(hi - lo, 1e-12f) - 0.5f, logf(vol));
    w.z = pack_bf2(sinf(ang), cosf(ang));
    w.w = pack_bf2(mom * 100.f, sig * 100.f);
    *reinterpret_cast<uint4*>(g.feat + o * RMF) = w;
  }
}

// ---------------------------------------------------------------- actor weight packing
struct GruPack {
  const float* w_hh;   // [RG][RH] fp32 master
  const float* w_ih;   // [RG][RFL] fp32 master (the actor uses the first RF columns)
  const float* b_ih;
  const float* b_hh;   // [RG]
  const float* w_q;    // [3][RH]
  const float* b_q;    // [3]
  i8v* whh8;           // [RW][3][2][2][64] fragments
  int* whhs;           // [RW][3][2][2][64] E8M0 scales (byte 0)
  s8v* wih;            // [RW][3][2][64]
  float* bias4;        // [4][RH]: b_ir+b_hr, b_iz+b_hz, b_in, b_hn
  float* wq;           // [4][RH]: W_q rows, row 3 = b_q (first 3 entries)
  // optional: W_hh^T as MX-fp8 A fragments of the learner's backward dh GEMM (rows = units,
  // K = the 768 gate rows): [RW][2 m][6 ks][64] fragments + scales, or null
  i8v* whhT8;
  int* whhTs;
};

// one thread per (wave, gate, m-tile, k-step, lane) fragment
__global__ void __launch_bounds__(256) gru_pack_kernel(GruPack p) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  if (tid < RH) {
    const int u = tid;
    // pre-scaled gate biases (gru_common.h GS_RZ / GS_N)
    p.bias4[u] = (p.b_ih[u] + p.b_hh[u]) * GS_RZ;
    p.bias4[RH + u] = (p.b_ih[RH + u] + p.b_hh[RH + u]) * GS_RZ;
    p.bias4[2 * RH + u] = p.b_ih[2 * RH + u] * GS_N;
    p.bias4[3 * RH + u] = p.b_hh[2 * RH + u] * GS_N;
    for (int a = 0; a < 3; ++a) p.wq[a * RH + u] = p.w_q[a * RH + u];
    p.wq[3 * RH + u] = u < 3 ? p.b_q[u] : 0.f;
  }
  if (tid >= RW * 3 * 2 * 2 * 64) return;
  const int lane = tid & 63, f = tid >> 6;
  const int ks = f & 1, m = (f >> 1) & 1, g = (f >> 2) % 3, w = (f >> 2) / 3;
  const int row = g * RH + 32 * w + 16 * m + (lane & 15);
  const int gl = lane >> 4;
  const float* wr = p.w_hh + (size_t)row * RH + 128 * ks;
  const float gs = g == 2 ? GS_N : GS_RZ;   // the gate's pre-scale, applied before quantization
  // block exponent of K-block b (32 columns) of this row within the K step
  auto blk_e = [&](int b) {
    float amax = 0.f;
    for (int j = 0; j < 32; ++j) amax = fmaxf(amax, fabsf(wr[32 * b + j] * gs));
    return mx_exp(amax);
  };
  const int e_lo = blk_e(gl >> 1), e_hi = blk_e(2 + (gl >> 1));   // blocks of this lane's two 16-byte halves
  const float* lo = wr + 16 * gl;
  const float* hi = wr + 64 + 16 * gl;
  i8v frag;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    frag[j] = (int)fp8x4(ldexpf(lo[4 * j] * gs, -e_lo), ldexpf(lo[4 * j + 1] * gs, -e_lo),
                         ldexpf(lo[4 * j + 2] * gs, -e_lo), ldexpf(lo[4 * j + 3] * gs, -e_lo));
    frag[4 + j] = (int)fp8x4(ldexpf(hi[4 * j] * gs, -e_hi), ldexpf(hi[4 * j + 1] * gs, -e_hi),
                             ldexpf(hi[4 * j + 2] * gs, -e_hi), ldexpf(hi[4 * j + 3] * gs, -e_hi));
  }
  p.whh8[tid] = frag;
  p.whhs[tid] = blk_e(gl) + 127;      // the scale slot of lane i + 16g belongs to K-block g
  if (p.whhT8 != nullptr) {
    // backward fragment: the same thread count covers [RW][2][6][64]
    const int f2 = tid >> 6, ks2 = f2 % 6, m2 = (f2 / 6) & 1, w2 = f2 / 12;
    const int u = 32 * w2 + 16 * m2 + (lane & 15);      // row of W_hh^T = hidden unit
    const float* col = p.w_hh + (size_t)(128 * ks2) * RH + u;   // W_hh[g][u], g = 128 ks2 + ...
    auto blk_t = [&](int b) {
      float amax = 0.f;
      for (int j = 0; j < 32; ++j) amax = fmaxf(amax, fabsf(col[(size_t)(32 * b + j) * RH]));
      return mx_exp(amax);
    };
    const int t_lo = blk_t(gl >> 1), t_hi = blk_t(2 + (gl >> 1));
    i8v fr;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float* lo2 = col + (size_t)(16 * gl + 4 * j) * RH;
      const float* hi2 = col + (size_t)(64 + 16 * gl + 4 * j) * RH;
      fr[j] = (int)fp8x4(ldexpf(lo2[0], -t_lo), ldexpf(lo2[RH], -t_lo), ldexpf(lo2[2 * RH], -t_lo),
                         ldexpf(lo2[3 * RH], -t_lo));
      fr[4 + j] = (int)fp8x4(ldexpf(hi2[0], -t_hi), ldexpf(hi2[RH], -t_hi), ldexpf(hi2[2 * RH], -t_hi),
                             ldexpf(hi2[3 * RH], -t_hi));
    }
    p.whhT8[tid] = fr;
    p.whhTs[tid] = blk_t(gl) + 127;
  }
  if (ks == 0) {
    s8v x;
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = (short)f2bf(p.w_ih[(size_t)row * RFL + 8 * (lane >> 4) + j] * gs);
    p.wih[((w * 3 + g) * 2 + m) * 64 + lane] = x;
  }
}

// ---------------------------------------------------------------- actor
struct GruAct {
  const i8v* whh8;
  const int* whhs;
  const s8v* wih;
  const float* bias4;
  const float* wq;
  const bf16_t* feat;          // [E][T][RMF]
  const float* close;          // [E][T]
  const float* ret;            // [E][T]: (close[t+1] / close[t] - 1) * 100 (last bar 0)
  int E, T, S, ep_len;
  float eps, inv_ramp, cost, inv_ep_len;
  float* h;                    // [E][RH] fp32 recurrent state between launches
  int* pos;                    // [E] bar index
  int* ep_start;
  int* position;               // 0 flat / 1 long
  float* entry;
  float* ep_ret;
  int* episodes;
  float* last_ret;
  // replay: one segment (S steps) per env per launch
  bf16_t* rx;                  // [cap][S+1][RF]
  unsigned char* ra;           // [cap][S]
  float* rr;                   // [cap][S]
  unsigned char* rd;           // [cap][S]
  bf16_t* rh0;                 // [cap][RH]
  unsigned long long* rctrl;   // [0] segments written (monotonic), [1] size
  int cap;
  uint32_t key0, key1;
  unsigned long long* ctrl;    // [0] actor launches so far
  float* stats;                // [4] reward sum, explore count, episodes done, finished-episode return sum
  float* q_out;                // optional [E][4]: Q of the last step (tests)
  unsigned long long* stamps;  // optional debug: s_memtime of workgroup 0, waves 0 and 1: [step][2][8]
  unsigned* done_ctr;          // optional (pair actor): workgroups finished; the last one advances rctrl /
                               // ctrl itself and re-zeroes it (else a separate advance launch follows)
};

struct ActLds {
  static constexpr int WX = 0;                                   // RW*6*64 s8v
  static constexpr int X = WX + RW * 6 * 64 * 16;                // [2][RN*XS] bf16
  static constexpr int H8 = X + 2 * RN * XS * 2;                 // [2][RN*HS] bytes
  static constexpr int SC = H8 + 2 * RN * HS;                    // [2][RN*SCS] int
  static constexpr int B = SC + 2 * RN * SCS * 4;                // [4*RH] float
  static constexpr int WQ = B + 4 * RH * 4;                      // [4*RH] float
  static constexpr int QP = WQ + 4 * RH * 4;                     // [RW][3][RN] float
  static constexpr int DN = QP + RW * 3 * RN * 4;                // [RN] int
  static constexpr int U = DN + RN * 4;                          // [S<=64][RN][4] float: Philox draws
  static constexpr int BYTES = U + 64 * RN * 16;
};
static_assert(ActLds::BYTES <= 160 * 1024, "actor LDS");

// build the x row (bf16 [RF]) from bar features mf / close c into LDS and (if rx_row) the replay segment
ST_DEV void build_x(const GruAct& p, uint4 mf, float c, int t, int es, int pz, float entry, bf16_t* sx_row,
                    bf16_t* rx_row) {
  const float upnl = pz ? (c / entry - 1.f) * 100.f : 0.f;
  uint4 w1;
  w1.x = pack_bf2((float)pz, upnl);
  w1.y = pack_bf2((float)(t - es) * p.inv_ep_len, 1.f);
  w1.z = 0u;
  w1.w = 0u;
  const uint4 z = {0u, 0u, 0u, 0u};
  uint4* d = reinterpret_cast<uint4*>(sx_row);
  d[0] = mf; d[1] = w1; d[2] = z; d[3] = z;
  if (rx_row) {
    uint4* r = reinterpret_cast<uint4*>(rx_row);
    r[0] = mf; r[1] = w1; r[2] = z; r[3] = z;
  }
}
ST_DEV uint4 bar_feat(const GruAct& p, int e, int t) {
  return *reinterpret_cast<const uint4*>(p.feat + ((size_t)e * p.T + t) * RMF);
}

__global__ void __launch_bounds__(RT, 1) gru_act_kernel(GruAct p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const s8v* sWx = reinterpret_cast<const s8v*>(lds + ActLds::WX);
  bf16_t* sX = reinterpret_cast<bf16_t*>(lds + ActLds::X);
  unsigned char* sH8 = lds + ActLds::H8;
  int* sSc = reinterpret_cast<int*>(lds + ActLds::SC);
  float* sB = reinterpret_cast<float*>(lds + ActLds::B);
  float* sWq = reinterpret_cast<float*>(lds + ActLds::WQ);
  float* sQp = reinterpret_cast<float*>(lds + ActLds::QP);
  int* sDone = reinterpret_cast<int*>(lds + ActLds::DN);
  f4v* sU = reinterpret_cast<f4v*>(lds + ActLds::U);

  const int tid = threadIdx.x, lane = tid & 63, l16 = lane & 15, g4 = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  for (int i = tid; i < RW * 6 * 64; i += RT) reinterpret_cast<s8v*>(lds + ActLds::WX)[i] = p.wih[i];
  for (int i = tid; i < 4 * RH; i += RT) {
    sB[i] = p.bias4[i];
    sWq[i] = p.wq[i];
  }
  // resident MX-fp8 W_hh fragments of this wave's 32 units x 3 gates (96 VGPRs + 12 scales)
  i8v Wh[3][2][2];
  int Ws4[3] = {0, 0, 0};   // 12 E8M0 scales packed 4 per VGPR: (g, m, ks) -> reg g, byte 2m + ks
#pragma unroll
  for (int g = 0; g < 3; ++g)
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int idx = (((wave * 3 + g) * 2 + m) * 2 + ks) * 64 + lane;
        Wh[g][m][ks] = p.whh8[idx];
        Ws4[g] |= (p.whhs[idx] & 0xFF) << (8 * (2 * m + ks));
      }
  const s8v* myWx = sWx + wave * 6 * 64 + lane;
  // Q head as one bf16 MFMA per env tile: A = W_q rows (a < 3, zero-padded to 16) over this
  // wave's 32 units, K ordered like the GRU accumulators the B operand is built from:
  // element j of lane group q <-> unit 32w + (j < 4 ? 4q + j : 16 + 4q + j - 4)
  s8v WqA;
  {
    const int a = l16;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int u = 32 * wave + (j < 4 ? 4 * g4 + j : 16 + 4 * g4 + j - 4);
      WqA[j] = (short)f2bf(a < 3 ? p.wq[a * RH + u] : 0.f);
    }
  }
  const unsigned long long launch = p.ctrl[0];
  const unsigned long long seg0 = p.rctrl[0];
  const int nchunks = p.E / RN, S = p.S;
  __syncthreads();

  for (int chunk = blockIdx.x; chunk < nchunks; chunk += gridDim.x) {
    const int e0 = chunk * RN;
    float hr[2][2][4];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        const int e = e0 + 16 * n + l16, u0 = 32 * wave + 16 * m + 4 * g4;
        const float4 v = *reinterpret_cast<const float4*>(p.h + (size_t)e * RH + u0);
        hr[m][n][0] = v.x; hr[m][n][1] = v.y; hr[m][n][2] = v.z; hr[m][n][3] = v.w;
        const size_t slot = (size_t)((seg0 + (unsigned long long)e) % (unsigned long long)p.cap);
        lds_st4(p.rh0 + slot * RH + u0, v.x, v.y, v.z, v.w);   // 8-byte global store of h0 (bf16)
      }
    quant_h(hr, sH8, sSc, wave, l16, g4);
    // env state lives in wave 0: lane l and l + 32 both carry env e0 + (l & 31) (the upper half
    // mirrors the lower one so every load is unconditional; only lanes < RN store)
    int t_ = 0, es_ = 0, pz_ = 0, eps_ = 0;
    float en_ = 0.f, er_ = 0.f, lr_ = 0.f;
    float cA = 0.f, cB = 0.f;      // close[t], close[t+1] (prefetched one env phase ahead)
    float rA = 0.f, rB = 0.f;      // ret[t], ret[t+1]
    uint4 fB = {0u, 0u, 0u, 0u};   // features of bar t+1
    float st_rew = 0.f, st_exp = 0.f, st_fin = 0.f, st_dn = 0.f;
    size_t slot_ = 0;
    const int me = e0 + (lane & (RN - 1));
    const bool writer = lane < RN;
    if (wave == 0) {
      t_ = p.pos[me]; es_ = p.ep_start[me]; pz_ = p.position[me]; en_ = p.entry[me]; er_ = p.ep_ret[me];
      eps_ = p.episodes[me]; lr_ = p.last_ret[me];
      slot_ = (size_t)((seg0 + (unsigned long long)me) % (unsigned long long)p.cap);
      const size_t o = (size_t)me * p.T + t_;
      cA = p.close[o];
      cB = p.close[o + 1];
      rA = p.ret[o];
      rB = p.ret[o + 1];
      fB = bar_feat(p, me, t_ + 1);
      const uint4 f0 = bar_feat(p, me, t_);
      if (writer) build_x(p, f0, cA, t_, es_, pz_, en_, sX + lane * XS, p.rx + slot_ * (size_t)(S + 1) * RF);
    }
    // the chunk's Philox draws for all S steps, by every thread (off the env phase's serial path)
    for (int i = tid; i < S * RN; i += RT) {
      const int ss = i / RN, e = e0 + (i % RN);
      const unsigned long long step = launch * (unsigned long long)S + (unsigned long long)ss;
      uint32_t c0 = (uint32_t)e, c1 = (uint32_t)(step & 0xFFFFFFFFull), c2 = (uint32_t)(step >> 32),
               c3 = 0x47525531u;
      philox4x32(c0, c1, c2, c3, p.key0, p.key1);
      f4v u;
      u[0] = u24(c0); u[1] = u24(c1); u[2] = u24(c2); u[3] = (float)step;
      sU[i] = u;
    }
    __syncthreads();

    for (int s = 0; s < S; ++s) {
      const int cur = s & 1, nxt = cur ^ 1;
      // debug phase stamps (tools/stamp_gru.py): slot 0 step start, 1 after MFMAs of tile 0,
      // 2 after tile 1 + GRU update, 3 after quantization, 4 after barrier 1, 5 after the env
      // phase, 6 after barrier 2
#define GR_STAMP(I)                                                                                       \
  if (p.stamps != nullptr && blockIdx.x == 0 && chunk == 0 && wave < 2 && lane == 0)                      \
    p.stamps[((size_t)s * 2 + wave) * 8 + (I)] = __builtin_amdgcn_s_memtime();
      GR_STAMP(0)
      const bf16_t* cX = sX + cur * RN * XS;
      const unsigned char* cH = sH8 + cur * RN * HS;
      const int* cS = sSc + cur * RN * SCS;
      // one 16-env tile at a time keeps the accumulators at 32 VGPRs (W_hh holds 108)
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        f4v ar[2], az[2], anx[2], anh[2];   // accumulators start at the biases (b_ir+b_hr, b_iz+b_hz, b_in, b_hn)
#pragma unroll
        for (int m = 0; m < 2; ++m) {
          const int u0 = 32 * wave + 16 * m + 4 * g4;
          ar[m] = *reinterpret_cast<const f4v*>(sB + u0);
          az[m] = *reinterpret_cast<const f4v*>(sB + RH + u0);
          anx[m] = *reinterpret_cast<const f4v*>(sB + 2 * RH + u0);
          anh[m] = *reinterpret_cast<const f4v*>(sB + 3 * RH + u0);
        }
        const int row = 16 * n + l16;
        // x part: bf16 16x16x32 (W_ih fragments from LDS)
        {
          const s8v xb = lds_ld8(cX + row * XS + 8 * g4);
#pragma unroll
          for (int m = 0; m < 2; ++m) {
            ar[m] = mfma32(myWx[(0 * 2 + m) * 64], xb, ar[m]);
            az[m] = mfma32(myWx[(1 * 2 + m) * 64], xb, az[m]);
            anx[m] = mfma32(myWx[(2 * 2 + m) * 64], xb, anx[m]);
          }
        }
        // h part: MX-fp8 16x16x128, two K steps over the 256 hidden units
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          // bytes 0..15: units 128ks + 16g4 + [0,16); bytes 16..31: units 128ks + 64 + 16g4 + [0,16)
          const uint4 h0 = *reinterpret_cast<const uint4*>(cH + row * HS + 128 * ks + 16 * g4);
          const uint4 h1 = *reinterpret_cast<const uint4*>(cH + row * HS + 128 * ks + 64 + 16 * g4);
          i8v hb;
          hb[0] = (int)h0.x; hb[1] = (int)h0.y; hb[2] = (int)h0.z; hb[3] = (int)h0.w;
          hb[4] = (int)h1.x; hb[5] = (int)h1.y; hb[6] = (int)h1.z; hb[7] = (int)h1.w;
          const int sc = cS[row * SCS + 4 * ks + g4];   // scale of K-block g4 = units of wave 4ks + g4
#define ST_MX3(M, KS)                                                              \
  ar[M] = mx_mfma_sel<2 * (M) + (KS)>(Wh[0][M][KS], hb, ar[M], Ws4[0], sc);          \
  az[M] = mx_mfma_sel<2 * (M) + (KS)>(Wh[1][M][KS], hb, az[M], Ws4[1], sc);          \
  anh[M] = mx_mfma_sel<2 * (M) + (KS)>(Wh[2][M][KS], hb, anh[M], Ws4[2], sc);
          if (ks == 0) { ST_MX3(0, 0) ST_MX3(1, 0) } else { ST_MX3(0, 1) ST_MX3(1, 1) }
#undef ST_MX3
        }
        if (n == 0) { GR_STAMP(1) }
        // GRU update in registers (lane: units u0..u0+3 of tile m, env 16n + l16)
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float r = sigm_ps(ar[m][i]);
            const float z = sigm_ps(az[m][i]);
            const float nn = tanh_ps(__builtin_fmaf(r, anh[m][i], anx[m][i]));
            hr[m][n][i] = __builtin_fmaf(z, hr[m][n][i] - nn, nn);
          }
        // Q partials of this wave's units: one MFMA, h (bf16) taken straight from the accumulator layout
        {
          s8v hb;
          const uint32_t p0 = pack_bf2(hr[0][n][0], hr[0][n][1]), p1 = pack_bf2(hr[0][n][2], hr[0][n][3]);
          const uint32_t p2 = pack_bf2(hr[1][n][0], hr[1][n][1]), p3 = pack_bf2(hr[1][n][2], hr[1][n][3]);
          hb[0] = (short)(p0 & 0xFFFF); hb[1] = (short)(p0 >> 16); hb[2] = (short)(p1 & 0xFFFF); hb[3] = (short)(p1 >> 16);
          hb[4] = (short)(p2 & 0xFFFF); hb[5] = (short)(p2 >> 16); hb[6] = (short)(p3 & 0xFFFF); hb[7] = (short)(p3 >> 16);
          const f4v qp = mfma32(WqA, hb, zero4());
          if (g4 == 0) {   // rows a = 0..2 of the 16x16 result live in lanes 0..15, registers 0..2
            sQp[(wave * 3 + 0) * RN + row] = qp[0];
            sQp[(wave * 3 + 1) * RN + row] = qp[1];
            sQp[(wave * 3 + 2) * RN + row] = qp[2];
          }
        }
      }
      GR_STAMP(2)
      quant_h(hr, sH8 + nxt * RN * HS, sSc + nxt * RN * SCS, wave, l16, g4);
      GR_STAMP(3)
      if (p.stamps != nullptr && blockIdx.x == 0 && chunk == 0 && lane == 0)   // every wave: arrival at barrier 1
        p.stamps[(size_t)S * 16 + (size_t)s * RW + wave] = __builtin_amdgcn_s_memtime();
      __syncthreads();
      GR_STAMP(4)
      // ---------------------------------------------------------- env step (wave 0)
      if (wave == 0) {
        float q[3];
#pragma unroll
        for (int a = 0; a < 3; ++a) {
          float v = sWq[3 * RH + a];
#pragma unroll
          for (int w = 0; w < RW; ++w) v += sQp[(w * 3 + a) * RN + (lane & (RN - 1))];
          q[a] = v;
        }
        int greedy = 0;
        const float qg = q[1] > q[0] ? q[1] : q[0];   // select chain: no stack-indexed q[greedy]
        if (q[1] > q[0]) greedy = 1;
        if (q[2] > qg) greedy = 2;
        const f4v u = sU[s * RN + (lane & (RN - 1))];   // (explore coin, random action, reset, step)
        const bool exploit = u[0] < fminf(p.eps, u[3] * p.inv_ramp);
        const int rnd = min((int)(u[1] * 3.0f), 2);
        const int a = exploit ? greedy : rnd;
        const int np = a == 0 ? 1 : (a == 1 ? 0 : pz_);
        const bool trade = np != pz_;
        if (trade && np == 1) en_ = cA;
        const float rew = (float)np * rA - (trade ? p.cost : 0.f);
        er_ += rew;
        int t1 = t_ + 1;
        const bool done = (t1 - es_) >= p.ep_len;
        float fin = 0.f;
        if (done) {
          eps_ += 1;
          lr_ = er_;
          fin = er_;
          es_ = min((int)(u[2] * (float)(p.T - p.ep_len - 1)), p.T - p.ep_len - 2);
          t1 = es_;
          pz_ = 0;
          er_ = 0.f;
        } else {
          pz_ = np;
        }
        t_ = t1;
        // bar t1's features: prefetched unless the episode restarted (rare: load now)
        uint4 fx = fB;
        float cx = cB, rx = rB;
        if (__builtin_amdgcn_ballot_w64(done) != 0ull) {
          const size_t o = (size_t)me * p.T + t_;
          const uint4 fr = bar_feat(p, me, t_);
          const float cr = p.close[o], rr = p.ret[o];
          fx.x = done ? fr.x : fx.x;   // per component: a uint4 ternary lowers to a stack select
      fx.y = done ? fr.y : fx.y;
      fx.z = done ? fr.z : fx.z;
      fx.w = done ? fr.w : fx.w;
          cx = done ? cr : cx;
          rx = done ? rr : rx;
        }
        if (writer) {
          p.ra[slot_ * S + s] = (unsigned char)a;
          p.rr[slot_ * S + s] = rew;
          p.rd[slot_ * S + s] = done ? 1 : 0;
          build_x(p, fx, cx, t_, es_, pz_, en_, sX + nxt * RN * XS + lane * XS,
                  p.rx + (slot_ * (size_t)(S + 1) + (size_t)(s + 1)) * RF);
          sDone[lane] = done ? 1 : 0;
          if (done) {   // the next step starts from h = 0
            uint4* hz = reinterpret_cast<uint4*>(sH8 + nxt * RN * HS + lane * HS);
            const uint4 z = {0u, 0u, 0u, 0u};
#pragma unroll
            for (int j = 0; j < RH / 16; ++j) hz[j] = z;
          }
          if (p.q_out && s == S - 1) {
            float* qo = p.q_out + (size_t)me * 4;
            qo[0] = q[0]; qo[1] = q[1]; qo[2] = q[2]; qo[3] = (float)a;
          }
          st_rew += rew;
          st_exp += exploit ? 0.f : 1.f;
          st_fin += fin;
          st_dn += done ? 1.f : 0.f;
        }
        // prefetch bar t1+1 for the next env phase (issued last: a whole MFMA phase to land)
        cA = cx;
        rA = rx;
        const size_t o1 = (size_t)me * p.T + min(t_ + 1, p.T - 1);
        cB = p.close[o1];
        rB = p.ret[o1];
        fB = *reinterpret_cast<const uint4*>(p.feat + o1 * RMF);
      }
      GR_STAMP(5)
      __syncthreads();
      GR_STAMP(6)
#pragma unroll
      for (int n = 0; n < 2; ++n)
        if (sDone[16 * n + l16]) {
#pragma unroll
          for (int m = 0; m < 2; ++m)
#pragma unroll
            for (int i = 0; i < 4; ++i) hr[m][n][i] = 0.f;
        }
    }
    // write back
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        const int e = e0 + 16 * n + l16, u0 = 32 * wave + 16 * m + 4 * g4;
        *reinterpret_cast<float4*>(p.h + (size_t)e * RH + u0) =
            make_float4(hr[m][n][0], hr[m][n][1], hr[m][n][2], hr[m][n][3]);
      }
    if (wave == 0) {
      st_rew = wave_sum(st_rew);
      st_exp = wave_sum(st_exp);
      st_fin = wave_sum(st_fin);
      st_dn = wave_sum(st_dn);
      if (lane == 0) {
        atomicAdd(p.stats + 0, st_rew);
        atomicAdd(p.stats + 1, st_exp);
        atomicAdd(p.stats + 2, st_dn);
        atomicAdd(p.stats + 3, st_fin);
      }
    }
    if (wave == 0 && writer) {
      p.pos[me] = t_; p.ep_start[me] = es_; p.position[me] = pz_; p.entry[me] = en_; p.ep_ret[me] = er_;
      p.episodes[me] = eps_; p.last_ret[me] = lr_;
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------- two-chunk actor
// gru_act_kernel runs each env step as [MFMA phase: every wave] -> barrier -> [env phase: wave 0 alone,
// ~1.45k of the ~8.5k cycles of a step, the other seven waves idle] -> barrier
// (profiles/r1_stamps_gru_actor.md).  Here a workgroup holds TWO 32-env chunks (slots A, B) and
// alternates: wave 0 runs slot A's env phase of step s while every wave runs slot B's MFMA phase of
// step s, then slot B's env phase beside slot A's MFMA phase of step s+1 -- each barrier interval
// pairs one chunk's serial env work with the other chunk's matrix work.  Per chunk the arithmetic
// and its order are those of gru_act_kernel (bit-identical env / replay / h), so the same tests
// hold.  LDS: the shared weights + two slot images (S <= 32 Philox rows each) = 146 KB.
constexpr int PAIR_SMAX = 32;
struct Act2Lds {
  static constexpr int WX = 0;                                   // RW*6*64 s8v
  static constexpr int B = WX + RW * 6 * 64 * 16;                // [4*RH] float
  static constexpr int WQ = B + 4 * RH * 4;                      // [4*RH] float
  static constexpr int SLOT0 = WQ + 4 * RH * 4;
  // one slot (offsets from its base)
  static constexpr int X = 0;                                    // [2][RN*XS] bf16
  static constexpr int H8 = X + 2 * RN * XS * 2;                 // [2][RN*HS] bytes
  static constexpr int SC = H8 + 2 * RN * HS;                    // [2][RN*SCS] int
  static constexpr int QP = SC + 2 * RN * SCS * 4;               // [RW][3][RN] float
  static constexpr int DN = QP + RW * 3 * RN * 4;                // [RN] int
  static constexpr int U = DN + RN * 4;                          // [PAIR_SMAX][RN][4] float: Philox draws
  static constexpr int ENV = U + PAIR_SMAX * RN * 16;            // [16][64] words: wave 0's env state
  static constexpr int SLOT = ENV + 16 * 64 * 4;
  static constexpr int BYTES = SLOT0 + 2 * SLOT;
};
static_assert(Act2Lds::BYTES <= 160 * 1024, "two-chunk actor LDS");
static_assert(Act2Lds::SLOT0 % 16 == 0 && Act2Lds::SLOT % 16 == 0, "16-byte aligned slots");

struct ActEnv {
  int t, es, pz, eps;
  float en, er, lr, cA, cB, rA, rB;
  uint4 fB;
  unsigned slot;
};

template <int V>
struct ActSlot {
  static constexpr int v = V;
};

__global__ void __launch_bounds__(RT, 1) gru_act_pair_kernel(GruAct p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const s8v* sWx = reinterpret_cast<const s8v*>(lds + Act2Lds::WX);
  float* sB = reinterpret_cast<float*>(lds + Act2Lds::B);
  float* sWq = reinterpret_cast<float*>(lds + Act2Lds::WQ);

  const int tid = threadIdx.x, lane = tid & 63, l16 = lane & 15, g4 = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  for (int i = tid; i < RW * 6 * 64; i += RT) reinterpret_cast<s8v*>(lds + Act2Lds::WX)[i] = p.wih[i];
  for (int i = tid; i < 4 * RH; i += RT) {
    sB[i] = p.bias4[i];
    sWq[i] = p.wq[i];
  }
  i8v Wh[3][2][2];
  int Ws4[3] = {0, 0, 0};
#pragma unroll
  for (int g = 0; g < 3; ++g)
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int idx = (((wave * 3 + g) * 2 + m) * 2 + ks) * 64 + lane;
        Wh[g][m][ks] = p.whh8[idx];
        Ws4[g] |= (p.whhs[idx] & 0xFF) << (8 * (2 * m + ks));
      }
  const s8v* myWx = sWx + wave * 6 * 64 + lane;
  s8v WqA;
  {
    const int a = l16;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int u = 32 * wave + (j < 4 ? 4 * g4 + j : 16 + 4 * g4 + j - 4);
      WqA[j] = (short)f2bf(a < 3 ? p.wq[a * RH + u] : 0.f);
    }
  }
  const unsigned long long launch = p.ctrl[0];
  const unsigned long long seg0 = p.rctrl[0];
  const int nchunks = p.E / RN, S = p.S;
  const int npairs = (nchunks + 1) / 2;
  const bool writer = lane < RN;
  __syncthreads();

  // ---------------------------------------------------------------- per-slot state
  // h lives in registers (every wave, both slots); wave 0's env state of the slot that is not in its
  // env phase is parked in LDS (ActEnv) so it does not hold registers through the other slot's MFMAs
  float hr[2][2][2][4];
  int e0_[2] = {0, 0};
  bool valid_[2] = {false, false};
  float st_rew = 0.f, st_exp = 0.f, st_fin = 0.f, st_dn = 0.f;
  auto base = [&](auto sl) { return lds + Act2Lds::SLOT0 + decltype(sl)::v * Act2Lds::SLOT; };
  auto env_ld = [&](auto sl) {
    const unsigned* w = reinterpret_cast<const unsigned*>(base(sl) + Act2Lds::ENV) + lane;
    ActEnv v;
    v.t = (int)w[0 * 64]; v.es = (int)w[1 * 64]; v.pz = (int)w[2 * 64]; v.eps = (int)w[3 * 64];
    v.en = __uint_as_float(w[4 * 64]); v.er = __uint_as_float(w[5 * 64]); v.lr = __uint_as_float(w[6 * 64]);
    v.cA = __uint_as_float(w[7 * 64]); v.cB = __uint_as_float(w[8 * 64]);
    v.rA = __uint_as_float(w[9 * 64]); v.rB = __uint_as_float(w[10 * 64]);
    v.fB = make_uint4(w[11 * 64], w[12 * 64], w[13 * 64], w[14 * 64]);
    v.slot = w[15 * 64];
    return v;
  };
  // (next = false: the next step's cB / rB / fB are not stored -- the env phase DMAs them in)
  auto env_st = [&](auto sl, const ActEnv& v, bool next = true) {
    unsigned* w = reinterpret_cast<unsigned*>(base(sl) + Act2Lds::ENV) + lane;
    w[0 * 64] = (unsigned)v.t; w[1 * 64] = (unsigned)v.es; w[2 * 64] = (unsigned)v.pz; w[3 * 64] = (unsigned)v.eps;
    w[4 * 64] = __float_as_uint(v.en); w[5 * 64] = __float_as_uint(v.er); w[6 * 64] = __float_as_uint(v.lr);
    w[7 * 64] = __float_as_uint(v.cA);
    w[9 * 64] = __float_as_uint(v.rA);
    if (next) {
      w[8 * 64] = __float_as_uint(v.cB);
      w[10 * 64] = __float_as_uint(v.rB);
      w[11 * 64] = v.fB.x; w[12 * 64] = v.fB.y; w[13 * 64] = v.fB.z; w[14 * 64] = v.fB.w;
    }
    w[15 * 64] = v.slot;
  };
  // one dword per lane from global memory into LDS at base + 4 * lane (LDS-DMA; base wave-uniform)
  auto dma4 = [&](const void* src, unsigned* base) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)base, 4, 0, 0);
  };

  // load a chunk into a slot: h (fp32 registers + fp8 LDS tile 0), env state (wave 0), x_0, Philox draws
  auto init = [&](auto sl, int chunk, bool valid) {
    constexpr int K = decltype(sl)::v;
    unsigned char* sb = base(sl);
    bf16_t* sX = reinterpret_cast<bf16_t*>(sb + Act2Lds::X);
    f4v* sU = reinterpret_cast<f4v*>(sb + Act2Lds::U);
    const int cc = valid ? chunk : nchunks - 1;   // an empty slot computes on a clamped chunk, writes nothing
    const int e0 = cc * RN;
    valid_[K] = valid;
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        const int e = e0 + 16 * n + l16, u0 = 32 * wave + 16 * m + 4 * g4;
        const float4 v = *reinterpret_cast<const float4*>(p.h + (size_t)e * RH + u0);
        hr[K][m][n][0] = v.x; hr[K][m][n][1] = v.y; hr[K][m][n][2] = v.z; hr[K][m][n][3] = v.w;
        if (valid) {
          const size_t slot = (size_t)((seg0 + (unsigned long long)e) % (unsigned long long)p.cap);
          lds_st4(p.rh0 + slot * RH + u0, v.x, v.y, v.z, v.w);
        }
      }
    quant_h(hr[K], sb + Act2Lds::H8, reinterpret_cast<int*>(sb + Act2Lds::SC), wave, l16, g4);
    e0_[K] = e0;
    if (wave == 0) {
      const int me = e0 + (lane & (RN - 1));
      ActEnv v;
      v.t = p.pos[me]; v.es = p.ep_start[me]; v.pz = p.position[me]; v.en = p.entry[me];
      v.er = p.ep_ret[me]; v.eps = p.episodes[me]; v.lr = p.last_ret[me];
      v.slot = (unsigned)((seg0 + (unsigned long long)me) % (unsigned long long)p.cap);
      const size_t o = (size_t)me * p.T + v.t;
      v.cA = p.close[o];
      v.cB = p.close[o + 1];
      v.rA = p.ret[o];
      v.rB = p.ret[o + 1];
      v.fB = bar_feat(p, me, v.t + 1);
      const uint4 f0 = bar_feat(p, me, v.t);
      if (writer)
        build_x(p, f0, v.cA, v.t, v.es, v.pz, v.en, sX + lane * XS,
                valid ? p.rx + (size_t)v.slot * (size_t)(S + 1) * RF : nullptr);
      env_st(sl, v);
    }
    for (int i = tid; i < S * RN; i += RT) {
      const int ss = i / RN, e = e0 + (i % RN);
      const unsigned long long step = launch * (unsigned long long)S + (unsigned long long)ss;
      uint32_t c0 = (uint32_t)e, c1 = (uint32_t)(step & 0xFFFFFFFFull), c2 = (uint32_t)(step >> 32),
               c3 = 0x47525531u;
      philox4x32(c0, c1, c2, c3, p.key0, p.key1);
      f4v u;
      u[0] = u24(c0); u[1] = u24(c1); u[2] = u24(c2); u[3] = (float)step;
      sU[i] = u;
    }
  };

  // MFMA phase of one step of a slot: gates from x (bf16) and h (MX-fp8), GRU update in registers,
  // Q partials -> LDS, h re-quantized into the other fp8 tile (reads tile `cur`, writes `cur ^ 1`)
  auto mfma_phase = [&](auto sl, int cur) {
    constexpr int K = decltype(sl)::v;
    unsigned char* sb = base(sl);
    const bf16_t* cX = reinterpret_cast<const bf16_t*>(sb + Act2Lds::X) + cur * RN * XS;
    const unsigned char* cH = sb + Act2Lds::H8 + cur * RN * HS;
    const int* cS = reinterpret_cast<const int*>(sb + Act2Lds::SC) + cur * RN * SCS;
    float* sQp = reinterpret_cast<float*>(sb + Act2Lds::QP);
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      f4v ar[2], az[2], anx[2], anh[2];
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const int u0 = 32 * wave + 16 * m + 4 * g4;
        ar[m] = *reinterpret_cast<const f4v*>(sB + u0);
        az[m] = *reinterpret_cast<const f4v*>(sB + RH + u0);
        anx[m] = *reinterpret_cast<const f4v*>(sB + 2 * RH + u0);
        anh[m] = *reinterpret_cast<const f4v*>(sB + 3 * RH + u0);
      }
      const int row = 16 * n + l16;
      {
        const s8v xb = lds_ld8(cX + row * XS + 8 * g4);
#pragma unroll
        for (int m = 0; m < 2; ++m) {
          ar[m] = mfma32(myWx[(0 * 2 + m) * 64], xb, ar[m]);
          az[m] = mfma32(myWx[(1 * 2 + m) * 64], xb, az[m]);
          anx[m] = mfma32(myWx[(2 * 2 + m) * 64], xb, anx[m]);
        }
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const uint4 h0 = *reinterpret_cast<const uint4*>(cH + row * HS + 128 * ks + 16 * g4);
        const uint4 h1 = *reinterpret_cast<const uint4*>(cH + row * HS + 128 * ks + 64 + 16 * g4);
        i8v hb;
        hb[0] = (int)h0.x; hb[1] = (int)h0.y; hb[2] = (int)h0.z; hb[3] = (int)h0.w;
        hb[4] = (int)h1.x; hb[5] = (int)h1.y; hb[6] = (int)h1.z; hb[7] = (int)h1.w;
        const int sc = cS[row * SCS + 4 * ks + g4];
#define ST_MX3P(M, KS)                                                             \
  ar[M] = mx_mfma_sel<2 * (M) + (KS)>(Wh[0][M][KS], hb, ar[M], Ws4[0], sc);          \
  az[M] = mx_mfma_sel<2 * (M) + (KS)>(Wh[1][M][KS], hb, az[M], Ws4[1], sc);          \
  anh[M] = mx_mfma_sel<2 * (M) + (KS)>(Wh[2][M][KS], hb, anh[M], Ws4[2], sc);
        if (ks == 0) { ST_MX3P(0, 0) ST_MX3P(1, 0) } else { ST_MX3P(0, 1) ST_MX3P(1, 1) }
#undef ST_MX3P
      }
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float r = sigm_ps(ar[m][i]);
          const float z = sigm_ps(az[m][i]);
          const float nn = tanh_ps(__builtin_fmaf(r, anh[m][i], anx[m][i]));
          hr[K][m][n][i] = __builtin_fmaf(z, hr[K][m][n][i] - nn, nn);
        }
      {
        s8v hb;
        const uint32_t p0 = pack_bf2(hr[K][0][n][0], hr[K][0][n][1]), p1 = pack_bf2(hr[K][0][n][2], hr[K][0][n][3]);
        const uint32_t p2 = pack_bf2(hr[K][1][n][0], hr[K][1][n][1]), p3 = pack_bf2(hr[K][1][n][2], hr[K][1][n][3]);
        hb[0] = (short)(p0 & 0xFFFF); hb[1] = (short)(p0 >> 16); hb[2] = (short)(p1 & 0xFFFF); hb[3] = (short)(p1 >> 16);
        hb[4] = (short)(p2 & 0xFFFF); hb[5] = (short)(p2 >> 16); hb[6] = (short)(p3 & 0xFFFF); hb[7] = (short)(p3 >> 16);
        const f4v qp = mfma32(WqA, hb, zero4());
        if (g4 == 0) {
          sQp[(wave * 3 + 0) * RN + row] = qp[0];
          sQp[(wave * 3 + 1) * RN + row] = qp[1];
          sQp[(wave * 3 + 2) * RN + row] = qp[2];
        }
      }
    }
    quant_h(hr[K], sb + Act2Lds::H8 + (cur ^ 1) * RN * HS, reinterpret_cast<int*>(sb + Act2Lds::SC) + (cur ^ 1) * RN * SCS,
            wave, l16, g4);
  };

  // env phase of step s of a slot (wave 0): Q, epsilon-greedy, trading env, replay segment, next x
  // into tile `nxt`, done flags (+ the next tile's h rows zeroed for finished episodes)
  auto env_phase = [&](auto sl, int s, int nxt) {
    constexpr int K = decltype(sl)::v;
    unsigned char* sb = base(sl);
    const float* sQp = reinterpret_cast<const float*>(sb + Act2Lds::QP);
    const f4v* sU = reinterpret_cast<const f4v*>(sb + Act2Lds::U);
    int* sDone = reinterpret_cast<int*>(sb + Act2Lds::DN);
    const int me = e0_[K] + (lane & (RN - 1));
    const bool valid = valid_[K];
    // this slot's LDS-DMA of cB / rB / fB (issued by this wave in its previous env phase, two barrier
    // intervals ago) has landed: vmcnt(0) (a workgroup barrier does not wait for a wave's own loads)
    __builtin_amdgcn_s_waitcnt(0xF70);
    ActEnv v = env_ld(sl);
    float q[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      float v = sWq[3 * RH + a];
#pragma unroll
      for (int w = 0; w < RW; ++w) v += sQp[(w * 3 + a) * RN + (lane & (RN - 1))];
      q[a] = v;
    }
    int greedy = 0;
    const float qg = q[1] > q[0] ? q[1] : q[0];
    if (q[1] > q[0]) greedy = 1;
    if (q[2] > qg) greedy = 2;
    const f4v u = sU[s * RN + (lane & (RN - 1))];
    const bool exploit = u[0] < fminf(p.eps, u[3] * p.inv_ramp);
    const int rnd = min((int)(u[1] * 3.0f), 2);
    const int a = exploit ? greedy : rnd;
    const int np = a == 0 ? 1 : (a == 1 ? 0 : v.pz);
    const bool trade = np != v.pz;
    if (trade && np == 1) v.en = v.cA;
    const float rew = (float)np * v.rA - (trade ? p.cost : 0.f);
    v.er += rew;
    int t1 = v.t + 1;
    const bool done = (t1 - v.es) >= p.ep_len;
    float fin = 0.f;
    if (done) {
      v.eps += 1;
      v.lr = v.er;
      fin = v.er;
      v.es = min((int)(u[2] * (float)(p.T - p.ep_len - 1)), p.T - p.ep_len - 2);
      t1 = v.es;
      v.pz = 0;
      v.er = 0.f;
    } else {
      v.pz = np;
    }
    v.t = t1;
    uint4 fx = v.fB;
    float cx = v.cB, rx = v.rB;
    if (__builtin_amdgcn_ballot_w64(done) != 0ull) {
      const size_t o = (size_t)me * p.T + v.t;
      const uint4 fr = bar_feat(p, me, v.t);
      const float cr = p.close[o], rr = p.ret[o];
      fx.x = done ? fr.x : fx.x;   // per component: a uint4 ternary lowers to a stack select
      fx.y = done ? fr.y : fx.y;
      fx.z = done ? fr.z : fx.z;
      fx.w = done ? fr.w : fx.w;
      cx = done ? cr : cx;
      rx = done ? rr : rx;
    }
    if (writer) {
      const size_t sl_ = v.slot;
      if (valid) {
        p.ra[sl_ * S + s] = (unsigned char)a;
        p.rr[sl_ * S + s] = rew;
        p.rd[sl_ * S + s] = done ? 1 : 0;
      }
      build_x(p, fx, cx, v.t, v.es, v.pz, v.en,
              reinterpret_cast<bf16_t*>(sb + Act2Lds::X) + nxt * RN * XS + lane * XS,
              valid ? p.rx + (sl_ * (size_t)(S + 1) + (size_t)(s + 1)) * RF : nullptr);
      sDone[lane] = done ? 1 : 0;
      if (done) {
        uint4* hz = reinterpret_cast<uint4*>(sb + Act2Lds::H8 + nxt * RN * HS + lane * HS);
        const uint4 z = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int j = 0; j < RH / 16; ++j) hz[j] = z;
      }
      if (valid && p.q_out && s == S - 1) {
        float* qo = p.q_out + (size_t)me * 4;
        qo[0] = q[0]; qo[1] = q[1]; qo[2] = q[2]; qo[3] = (float)a;
      }
      if (valid) {
        st_rew += rew;
        st_exp += exploit ? 0.f : 1.f;
        st_fin += fin;
        st_dn += done ? 1.f : 0.f;
      }
    }
    v.cA = cx;
    v.rA = rx;
    const size_t o1 = (size_t)me * p.T + min(v.t + 1, p.T - 1);
    // the next step's close / return / bar features go straight from HBM into the parked env state by
    // LDS-DMA (one dword per lane and field, the parking layout): nothing in this env phase waits for them
    // -- they land behind the other slot's MFMA phase, and the barrier closing it retires them (a register
    // load stored with the rest of the state held the env phase for a whole HBM round trip)
    env_st(sl, v, false);
    unsigned* w = reinterpret_cast<unsigned*>(base(sl) + Act2Lds::ENV);
    dma4(p.close + o1, w + 8 * 64);             // cB
    dma4(p.ret + o1, w + 10 * 64);             // rB
    const unsigned* f = reinterpret_cast<const unsigned*>(p.feat + o1 * RMF);
#pragma unroll
    for (int j = 0; j < 4; ++j) dma4(f + j, w + (11 + j) * 64);   // fB
  };

  // h of envs whose episode ended restarts from 0 (after the env phase's barrier)
  auto reset = [&](auto sl) {
    constexpr int K = decltype(sl)::v;
    const int* sDone = reinterpret_cast<const int*>(base(sl) + Act2Lds::DN);
#pragma unroll
    for (int n = 0; n < 2; ++n)
      if (sDone[16 * n + l16]) {
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
          for (int i = 0; i < 4; ++i) hr[K][m][n][i] = 0.f;
      }
  };

  auto writeback = [&](auto sl) {
    constexpr int K = decltype(sl)::v;
    if (!valid_[K]) return;
    int e0 = e0_[K];
    asm volatile("" : "+s"(e0));   // (the h row addresses recomputed here, not kept from init() across the step loop)
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        const int e = e0 + 16 * n + l16, u0 = 32 * wave + 16 * m + 4 * g4;
        *reinterpret_cast<float4*>(p.h + (size_t)e * RH + u0) =
            make_float4(hr[K][m][n][0], hr[K][m][n][1], hr[K][m][n][2], hr[K][m][n][3]);
      }
    if (wave == 0 && writer) {
      const int me = e0 + lane;
      const ActEnv v = env_ld(sl);
      p.pos[me] = v.t; p.ep_start[me] = v.es; p.position[me] = v.pz; p.entry[me] = v.en;
      p.ep_ret[me] = v.er; p.episodes[me] = v.eps; p.last_ret[me] = v.lr;
    }
  };

  constexpr ActSlot<0> A{};
  constexpr ActSlot<1> Bs{};
  for (int pr = blockIdx.x; pr < npairs; pr += gridDim.x) {
    init(A, 2 * pr, true);
    init(Bs, 2 * pr + 1, 2 * pr + 1 < nchunks);
    __syncthreads();
    mfma_phase(A, 0);                              // slot A, step 0
    __syncthreads();
    for (int s = 0; s < S; ++s) {
      const int cur = s & 1, nxt = cur ^ 1;
      // debug interval stamps (tools/stamp_gru.py --kernel pair), first pair of workgroup 0, waves 0
      // and 4 (same SIMD): 0 start, 1 after env A, 2 after MFMA B, 3 after barrier + reset A,
      // 4 after env B, 5 after MFMA A, 6 after barrier + reset B
#define GP_STAMP(I)                                                                                        \
  if (p.stamps != nullptr && blockIdx.x == 0 && pr == 0 && (wave & 3) == 0 && lane == 0)                   \
    p.stamps[((size_t)s * 2 + (wave >> 2)) * 8 + (I)] = __builtin_amdgcn_s_memtime();
      GP_STAMP(0)
      if (wave == 0) env_phase(A, s, nxt);         // A: env of step s   | B: MFMA of step s
      GP_STAMP(1)
      mfma_phase(Bs, cur);
      GP_STAMP(2)
      __syncthreads();
      reset(A);
      GP_STAMP(3)
      if (wave == 0) env_phase(Bs, s, nxt);        // B: env of step s   | A: MFMA of step s + 1
      GP_STAMP(4)
      if (s + 1 < S) mfma_phase(A, nxt);
      GP_STAMP(5)
      __syncthreads();
      reset(Bs);
      GP_STAMP(6)
#undef GP_STAMP
    }
    writeback(A);
    writeback(Bs);
    __syncthreads();
  }
  if (wave == 0) {
    st_rew = wave_sum(st_rew);
    st_exp = wave_sum(st_exp);
    st_fin = wave_sum(st_fin);
    st_dn = wave_sum(st_dn);
    if (lane == 0) {
      atomicAdd(p.stats + 0, st_rew);
      atomicAdd(p.stats + 1, st_exp);
      atomicAdd(p.stats + 2, st_dn);
      atomicAdd(p.stats + 3, st_fin);
    }
  }
  // the launch's counters advance in its last workgroup (every workgroup read them at its start, and the
  // last one to finish runs after all of those reads): no separate one-thread launch on the iteration's
  // critical path
  if (p.done_ctr != nullptr && tid == 0) {
    __threadfence();
    if (atomicAdd(p.done_ctr, 1u) == gridDim.x - 1) {
      const unsigned long long w = p.rctrl[0] + (unsigned long long)p.E;
      p.rctrl[0] = w;
      p.rctrl[1] = w < (unsigned long long)p.cap ? w : (unsigned long long)p.cap;
      p.ctrl[0] = p.ctrl[0] + 1;
      *p.done_ctr = 0u;
      __threadfence();
    }
  }
}

__global__ void gru_advance_kernel(unsigned long long* rctrl, unsigned long long* ctrl, int E, int cap) {
  rctrl[0] += (unsigned long long)E;
  rctrl[1] = rctrl[0] < (unsigned long long)cap ? rctrl[0] : (unsigned long long)cap;
  ctrl[0] += 1;
}

// MX-fp8 MFMA probe: D = (A * 2^(sa-127)) . (B * 2^(sb-127))^T for one 16x16x128 tile (layout tests)
__global__ void mx_probe_kernel(const i8v* a, const i8v* b, const int* sa, const int* sb, f4v* d) {
  const int l = threadIdx.x;
  d[l] = mx_mfma(a[l], b[l], zero4(), sa[l], sb[l]);
}

}  // namespace st

// ---------------------------------------------------------------- C ABI
extern "C" hipError_t st_minute_bars(const st::MinuteBars* g, hipStream_t s) {
  if (g->E <= 0 || g->T <= 1 || g->day <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(st::minute_bars_kernel, dim3((g->E + 255) / 256), dim3(256), 0, s, *g);
  return hipGetLastError();
}

extern "C" hipError_t st_gru_pack(const st::GruPack* p, hipStream_t s) {
  const int n = st::RW * 3 * 2 * 2 * 64;
  hipLaunchKernelGGL(st::gru_pack_kernel, dim3((n + 255) / 256), dim3(256), 0, s, *p);
  return hipGetLastError();
}

extern "C" int st_gru_act_lds_bytes() { return st::ActLds::BYTES; }

extern "C" hipError_t st_gru_act(const st::GruAct* p, int grid, hipStream_t s) {
  if (p->E % st::RN || p->S <= 0 || p->S > 64 || p->ep_len <= 0 || p->T < p->ep_len + 3 || p->cap <= 0 || grid <= 0)
    return hipErrorInvalidValue;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)st::gru_act_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       st::ActLds::BYTES);
    if (e != hipSuccess) return e;
    attr = true;
  }
  const int nch = p->E / st::RN;
  hipLaunchKernelGGL(st::gru_act_kernel, dim3(grid < nch ? grid : nch), dim3(st::RT), st::ActLds::BYTES, s, *p);
  hipLaunchKernelGGL(st::gru_advance_kernel, dim3(1), dim3(1), 0, s, p->rctrl, p->ctrl, p->E, p->cap);
  return hipGetLastError();
}






extern "C" int st_gru_act_pair_smax() { return st::PAIR_SMAX; }

extern "C" hipError_t st_gru_act_pair(const st::GruAct* p, int grid, hipStream_t s) {
  if (p->E % st::RN || p->S <= 0 || p->S > st::PAIR_SMAX || p->ep_len <= 0 || p->T < p->ep_len + 3 || p->cap <= 0 ||
      grid <= 0)
    return hipErrorInvalidValue;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)st::gru_act_pair_kernel,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, st::Act2Lds::BYTES);
    if (e != hipSuccess) return e;
    attr = true;
  }
  const int npairs = (p->E / st::RN + 1) / 2;
  hipLaunchKernelGGL(st::gru_act_pair_kernel, dim3(grid < npairs ? grid : npairs), dim3(st::RT), st::Act2Lds::BYTES,
                     s, *p);
  if (p->done_ctr == nullptr)   // (else the kernel's last workgroup advanced the counters)
    hipLaunchKernelGGL(st::gru_advance_kernel, dim3(1), dim3(1), 0, s, p->rctrl, p->ctrl, p->E, p->cap);
  return hipGetLastError();
}

extern "C" hipError_t st_mx_probe(const void* a, const void* b, const int* sa, const int* sb, float* d,
                                  hipStream_t s) {
  hipLaunchKernelGGL(st::mx_probe_kernel, dim3(1), dim3(64), 0, s, (const st::i8v*)a, (const st::i8v*)b, sa, sb,
                     (f4v*)d);
  return hipGetLastError();
}

// struct sizes of this file's launch ABI, for the host mirrors' check (tests/test_abi.py; no HIP call)
extern "C" int st_abi_gru(int* out, int n) {
  const int sz[] = {(int)sizeof(st::MinuteBars), (int)sizeof(st::GruPack), (int)sizeof(st::GruAct)};
  const int m = (int)(sizeof(sz) / sizeof(sz[0]));
  for (int i = 0; i < n && i < m; ++i) out[i] = sz[i];
  return m;
}
