// Paired-slot fused online-DQN engine step on CDNA4 (gfx950): the step of qstep_wide.hip
// (gather -> Q(x) -> epsilon-greedy + env step -> Q(x') -> TD -> backward -> per-workgroup
// weight-gradient slabs; QDecisionPolicyActor.scala:54-77, TrainerChildActor.scala:82-146) with
// the chunk loop software-pipelined over TWO chunk slots.
//
// Why: the 64-env-chunk kernel runs ten barrier-separated phases per chunk with all eight waves in
// the same phase, so each phase's LDS latency, VALU tail and MFMA time add up (~20.4k cycles per
// chunk, MFMA pipes ~25 % busy; profiles/r1_stamps_wide_step_1m_envs.md).  Here every workgroup
// holds two 32-env chunks in flight, in separate LDS slots, five phases apart: each barrier
// interval runs phase k of slot A's chunk and phase k+5 of slot B's chunk, so the latency-bound
// phases (gather P0, env step P3, TD target P6) always share an interval with MFMA phases of the
// other chunk:
//
//     interval   0      1      2      3      4      5      6      7      8      9
//     slot A     P0     P1     P2     P3     P4     P5     P6     P7     P8     P9
//     slot B     P5     P6     P7     P8     P9     P0     P1     P2     P3     P4
//
// Ten barriers per 64 envs as before, but each interval holds two independent dependency chains.
// Weights (W0 fragments in VGPRs, W1 / W2 images in LDS) and the weight-gradient accumulators
// (VGPRs) are shared by both slots: a gradient is a sum over envs, so both chunks accumulate into
// the same registers.  Per-slot LDS: the activation images of one 32-env chunk (~60 KB); two slots
// + weights = 163,168 of the 163,840 bytes a workgroup may declare.
//
// The epsilon-greedy draw (Philox) is computed in P1 by one wave for the whole chunk (it depends only
// on the env id, the step and the env position), taking ~60 dependent VALU ops off the P3 critical
// path; P3 only resolves exploit ? argmax : random action.  Same draws, same actions as the other
// kernels.
//
// Pipeline fill / drain: every interval runs both slots unconditionally (one basic block per
// interval, no uniform branches around the phases); a slot without a chunk computes on a clamped
// chunk index with dQ forced to zero (every gradient contribution exactly 0: the slot buffers are
// zero-filled at launch, so no NaN can enter), no global writes and zero statistics.
#include "qstep.h"

namespace st {
namespace pair {

constexpr int C = 32;            // envs per chunk (per slot)
constexpr int NW = 8;            // waves: two per SIMD
constexpr int NT = 64 * NW;
constexpr int NET = C / 16;      // env tiles per chunk (2)
constexpr int RPW = C / NW;      // gather rows per wave (4)
constexpr int SQ = OUTP + 8;
constexpr int ENVF = 6;          // fp32 words per env in sEnv
#ifndef ST_PAIR_DW0_PIPE
#define ST_PAIR_DW0_PIPE 3
#endif
constexpr int DW0_PIPE = ST_PAIR_DW0_PIPE;
#ifndef ST_PAIR_STAGGER
#define ST_PAIR_STAGGER 0   // 1: duplicated phase code per wave half -- 134 VGPR spills, not usable
#endif
#ifndef ST_PAIR_PRIO
#define ST_PAIR_PRIO 0      // 1: waves 4-7 at s_setprio 1 through the chunk loop -- measured no gain
#endif

// activation images: 16-byte unit of column c of row r stored at c ^ 8 * bit2(r) (see qstep_wide.hip)
ST_DEV int asw(int r, int lo) { return lo ^ ((r & 4) << 1); }
ST_DEV s8v afrag_row(const bf16_t* img, int S, int r0, int k0, int l16, int g4) {
  const int r = r0 + l16;
  return lds_ld8(img + r * S + k0 + asw(r, 8 * g4));
}
ST_DEV s8v afrag_trp(const bf16_t* img, int S, int k0, int c0, int l16, int g4) {
  const int r = k0 + 4 * g4 + (l16 >> 2);
  const bf16_t* q = img + r * S + c0 + asw(r, 4 * (l16 & 3));
  s4v lo = lds_tr4(q);
  s4v hi = lds_tr4(q + 16 * S);
  s8v v;
  v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
  v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
  return v;
}

template <int INP, int H1P, int H2P>
struct Geo {
  static constexpr int SW1 = H1P + 8, SW2 = H2P + 8;
  static constexpr int SX = INP + 16, SH1 = H1P + 16, SH2 = H2P + 16;
  // shared weight images (bf16 element offsets from the LDS base)
  static constexpr int oW1 = 0;
  static constexpr int oW2 = oW1 + H2P * SW1;
  static constexpr int W_END = oW2 + OUTP * SW2;
  // one slot (bf16 element offsets from the slot base)
  static constexpr int oX = 0;
  static constexpr int oH1 = oX + C * SX;
  static constexpr int oH2 = oH1 + C * SH1;
  static constexpr int oR0 = oH2 + C * SH2;          // X' / H2' / dZ2
  static constexpr int R0SZ = (C * SX > C * SH2) ? C * SX : C * SH2;
  static constexpr int oR1 = oR0 + R0SZ;             // H1' / dZ1
  static constexpr int oDQ = oR1 + C * SH1;
  static constexpr int SLOT_BF = oDQ + C * SQ;
  // slot fp32 region (byte offsets from the slot base)
  static constexpr int fQ = SLOT_BF * 2;             // q(x) [C][4]; P6 -> P7: per-env statistics
  static constexpr int fENV = fQ + C * 16;           // [C][ENVF] floats
  static constexpr int fENVI = fENV + C * ENVF * 4;  // [C][4] ints
  static constexpr int SLOT_BYTES = fENVI + C * 16;
  static constexpr int SLOT0 = W_END * 2;            // byte offset of slot 0
  static constexpr int fB1 = SLOT0 + 2 * SLOT_BYTES; // b1 [H2P] fp32
  static constexpr int fB2 = fB1 + H2P * 4;          // b2 [16]
  static constexpr int fST = fB2 + OUTP * 4;         // step statistics [NSTAT] (end of launch)
  static constexpr int BYTES = fST + NSTAT * 4;
  static_assert(BYTES <= 163840, "LDS budget exceeded");
  static_assert(SLOT0 % 16 == 0 && SLOT_BYTES % 16 == 0, "16-byte aligned slots");
  static_assert(H1P == 16 * NW && H2P == 16 * NW, "one 16-unit m-tile per wave in each hidden layer");
  static_assert(INP % 32 == 0, "padding");
  static constexpr int KS0 = INP / 32;               // layer-1 k-steps
  static constexpr int NT0 = INP / 16 - 1;           // in-col tiles of dW0 (last tile is pure padding)
  static constexpr int NT1 = H1P / 16;
};

// out^T[m][env] for this wave's 16 units and the chunk's NET env tiles (B = activation rows); epilogue
// + bias, ReLU, bf16 store into out image [env][m]
template <int K, int SB, int SO, typename AFrag>
ST_DEV void fwd_hidden(AFrag afrag, const bf16_t* sB, bf16_t* sO, const float* bias, int m0, int l16, int g4) {
  float bb[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) bb[j] = bias ? bias[m0 + 4 * g4 + j] : 0.f;
  f4v acc[NET];
#pragma unroll
  for (int n = 0; n < NET; ++n) acc[n] = zero4();
#pragma unroll
  for (int ks = 0; ks < K / 32; ++ks) {
    s8v b[NET];
#pragma unroll
    for (int n = 0; n < NET; ++n) b[n] = afrag_row(sB, SB, 16 * n, ks * 32, l16, g4);
    const s8v a = afrag(ks);
#pragma unroll
    for (int n = 0; n < NET; ++n) acc[n] = mfma32(a, b[n], acc[n]);
  }
#pragma unroll
  for (int n = 0; n < NET; ++n) {
    const f4v v = acc[n];
    lds_st4(sO + (16 * n + l16) * SO + m0 + asw(l16, 4 * g4), fmaxf(v[0] + bb[0], 0.f), fmaxf(v[1] + bb[1], 0.f),
            fmaxf(v[2] + bb[2], 0.f), fmaxf(v[3] + bb[3], 0.f));
  }
}

// q^T[a][env] of env tile nt (lanes g4 == 0 hold q[0..3] of env 16*nt + l16)
template <int K, int SA, int SB>
ST_DEV f4v fwd_out(const bf16_t* sA, const bf16_t* sB, int nt, int l16, int g4) {
  f4v acc = zero4();
#pragma unroll
  for (int ks = 0; ks < K / 32; ++ks) acc = mfma32(frag_row(sA, SA, 0, ks * 32, l16, g4), afrag_row(sB, SB, 16 * nt, ks * 32, l16, g4), acc);
  return acc;
}

// dA^T[m][env] = sum_k W[m][k] dZ[env][k] (W read transposed from the W^T image [k][m]), masked by
// act[env][m] > 0, bf16 store into out image [env][m]
template <int K, int SW, int SD, int SACT, int SO>
ST_DEV void bwd_data(const bf16_t* sWT, const bf16_t* sDZ, const bf16_t* sAct, bf16_t* sO, int m0, int l16, int g4) {
  s4v hm[NET];
#pragma unroll
  for (int n = 0; n < NET; ++n) hm[n] = lds_ld4(sAct + (16 * n + l16) * SACT + m0 + asw(l16, 4 * g4));
  f4v acc[NET];
#pragma unroll
  for (int n = 0; n < NET; ++n) acc[n] = zero4();
  if constexpr (K == 16) {
    const s4v a = lds_tr4(sWT + (4 * g4 + (l16 >> 2)) * SW + m0 + 4 * (l16 & 3));
#pragma unroll
    for (int n = 0; n < NET; ++n) acc[n] = mfma16(a, lds_ld4(sDZ + (16 * n + l16) * SD + 4 * g4), acc[n]);
  } else {
#pragma unroll
    for (int ks = 0; ks < K / 32; ++ks) {
      s8v b[NET];
#pragma unroll
      for (int n = 0; n < NET; ++n) b[n] = afrag_row(sDZ, SD, 16 * n, ks * 32, l16, g4);
      const s8v a = frag_tr(sWT, SW, ks * 32, m0, l16, g4);
#pragma unroll
      for (int n = 0; n < NET; ++n) acc[n] = mfma32(a, b[n], acc[n]);
    }
  }
#pragma unroll
  for (int n = 0; n < NET; ++n) {
    const s4v h = hm[n];
    const f4v v = acc[n];
    lds_st4(sO + (16 * n + l16) * SO + m0 + asw(l16, 4 * g4), h[0] > 0 ? v[0] : 0.f, h[1] > 0 ? v[1] : 0.f,
            h[2] > 0 ? v[2] : 0.f, h[3] > 0 ? v[3] : 0.f);
  }
}

template <int V>
struct SlotT {
  static constexpr int v = V;
};

template <int INP, int H1P, int H2P, int FEAT>
__global__ void __launch_bounds__(NT, 1) qstep_pair_kernel(QStepParams p) {
  using G = Geo<INP, H1P, H2P>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* const sW1 = reinterpret_cast<bf16_t*>(smem) + G::oW1;
  bf16_t* const sW2 = reinterpret_cast<bf16_t*>(smem) + G::oW2;
  float* const sB1 = reinterpret_cast<float*>(smem + G::fB1);
  float* const sB2 = reinterpret_cast<float*>(smem + G::fB2);
  float* const sSt = reinterpret_cast<float*>(smem + G::fST);

  const int tid = threadIdx.x, lane = tid & 63, l16 = lane & 15, g4 = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H = p.H;
  const unsigned long long step = p.ctrl[0];
  const int m0 = 16 * wave;   // this wave's hidden units in both hidden layers
  const int nch = p.E / C;    // 32-env chunks
  const int grid = (int)gridDim.x, bid = (int)blockIdx.x;
  // slot A runs chunks bid + 2k*grid (cycle k), slot B chunks bid + (2k+1)*grid
  const int ncyc = (nch - bid + 2 * grid - 1) / (2 * grid);   // cycles with a slot-A chunk
#define STP_STAMPX(I) \
  if (p.stamps != nullptr && bid == 0 && tid == 0) p.stamps[(ncyc + 1) * 16 + 8 + (I)] = __builtin_amdgcn_s_memtime();
  STP_STAMPX(0);

  // ---------------------------------------------------------------- per-slot register state
  // env scalars of the slot's next chunk (row-owner lanes), price windows of it
  int e_pos[2] = {0, 0}, e_sh[2] = {0, 0}, e_ep[2] = {0, 0};
  float e_b[2] = {0.f, 0.f}, e_val[2] = {0.f, 0.f}, e_rs[2] = {0.f, 0.f};
  float4 w[2][RPW];
  float wl[2] = {0.f, 0.f}, wv[2] = {0.f, 0.f};
#define STP_LOAD_ENV(S, CH)                                                \
  {                                                                        \
    const int e_ = min((CH), nch - 1) * C + wave * RPW + min(lane, RPW - 1); \
    e_pos[S] = ENV_I(ER_POS, e_); e_b[S] = ENV_F(ER_BUDGET, e_); e_sh[S] = ENV_I(ER_SHARES, e_);   \
    e_val[S] = ENV_F(ER_VALUE, e_); e_rs[S] = ENV_F(ER_RET_SUM, e_); e_ep[S] = ENV_I(ER_EPISODES, e_); \
  }
#define STP_LOAD_PRICES(S, CH)                                             \
  {                                                                        \
    const int row_ = min((CH), nch - 1) * C + wave * RPW + min(lane, RPW - 1); \
    const int pos_ = e_pos[S];                                             \
    const int sh_ = pos_ & 3;                                              \
    const size_t off_ = ((size_t)sh_ * p.E + (size_t)row_) * p.T4 + (size_t)(pos_ - sh_); \
    const unsigned long long a_ = (unsigned long long)(p.prices4 + off_);  \
    const unsigned alo_ = (unsigned)a_, ahi_ = (unsigned)(a_ >> 32);       \
    _Pragma("unroll") for (int rr = 0; rr < RPW; ++rr) {                   \
      const unsigned long long b_ =                                        \
          ((unsigned long long)__builtin_amdgcn_readlane(ahi_, rr) << 32) | \
          (unsigned)__builtin_amdgcn_readlane(alo_, rr);                   \
      typedef float f4g_ __attribute__((ext_vector_type(4)));              \
      const f4g_ v_ = reinterpret_cast<const __attribute__((address_space(1))) f4g_*>(b_)[lane]; \
      w[S][rr] = make_float4(v_.x, v_.y, v_.z, v_.w);                      \
    }                                                                      \
    const float* pl_ = p.prices + (size_t)row_ * p.T + pos_ + H;           \
    wl[S] = pl_[-1];                                                       \
    wv[S] = pl_[0];                                                        \
  }
  STP_LOAD_ENV(0, bid)

  // ---------------------------------------------------------------- weights (once per launch)
  s8v aW0[G::KS0];
  {
    const bf16_t* w0 = p.wq + p.off_w0 + (size_t)(m0 + l16) * INP + 8 * g4;
#pragma unroll
    for (int ks = 0; ks < G::KS0; ++ks) aW0[ks] = *reinterpret_cast<const s8v*>(w0 + ks * 32);
  }
  {
    const bf16_t* w1 = p.wq + p.off_w1;
    for (int i = tid; i < H2P * H1P / 8; i += NT) {
      const int r = i / (H1P / 8), c = (i % (H1P / 8)) * 8;
      *reinterpret_cast<uint4*>(sW1 + r * G::SW1 + c) = *reinterpret_cast<const uint4*>(w1 + r * H1P + c);
    }
    const bf16_t* w2 = p.wq + p.off_w2;
    for (int i = tid; i < OUTP * H2P / 8; i += NT) {
      const int r = i / (H2P / 8), c = (i % (H2P / 8)) * 8;
      *reinterpret_cast<uint4*>(sW2 + r * G::SW2 + c) = *reinterpret_cast<const uint4*>(w2 + r * H2P + c);
    }
    for (int i = tid; i < H2P; i += NT) sB1[i] = p.wf[p.off_b1 + i];
    if (tid < OUTP) sB2[tid] = p.wf[p.off_b2 + tid];
    // slot buffers zero-filled: the pipeline-fill phases of slot B read them before any write
    uint4* z = reinterpret_cast<uint4*>(smem + G::SLOT0);
    for (int i = tid; i < 2 * G::SLOT_BYTES / 16; i += NT) z[i] = make_uint4(0u, 0u, 0u, 0u);
  }

  // ---------------------------------------------------------------- gradient accumulators
  // wave w owns h1 rows 16w.. of dW0^T (13 column tiles), h2 rows 16w.. of dW1^T (8 tiles) + db1,
  // dW2^T column tile w, db2 (every wave; wave 0 writes it)
  constexpr int B0 = G::NT0, B1 = G::NT1;
  f4v gW0[B0], gW1[B1], gB1 = zero4(), gW2 = zero4(), gB2 = zero4();
#pragma unroll
  for (int n = 0; n < B0; ++n) gW0[n] = zero4();
#pragma unroll
  for (int n = 0; n < B1; ++n) gW1[n] = zero4();
  s8v ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (l16 == 0) ? (short)0x3F80 : (short)0;
  float sa0 = 0.f, sa1 = 0.f;   // statistics fold (waves NET..NET+3, lane = env row)

  STP_LOAD_PRICES(0, bid)
  __syncthreads();
  STP_STAMPX(1);

  // ================================================================ phases (slot S = compile time)
  // Slot base: an opaque scalar, re-materialised once per phase.  Every lane-dependent LDS address is
  // then (lane part, loop-invariant and shared by both slots) + (slot base, SGPR) + (immediate < 64 KB);
  // with compile-time slot bases hipcc hoisted a separate address register per image, pattern and slot
  // out of the chunk loop (slot 1 lies past the 64 KB ds-offset reach) and spilled them.
  auto slot_base = [&](auto s) {
    int o = G::SLOT0 + decltype(s)::v * G::SLOT_BYTES;
    asm volatile("" : "+s"(o));
    return smem + o;
  };

#define SB_BF(SB, OFF) (reinterpret_cast<bf16_t*>(SB) + (OFF))
#define SB_FL(SB, OFF) (reinterpret_cast<float*>((SB) + (OFF)))
#define SB_IN(SB, OFF) (reinterpret_cast<int*>((SB) + (OFF)))
  // P0: windows -> feature rows x, x'; env scalars -> LDS (row-owner lanes)
  auto P0 = [&](auto s) {
    constexpr int S = decltype(s)::v;
    char* const sb = slot_base(s);
    bf16_t* sX = SB_BF(sb, G::oX);
    bf16_t* sR0 = SB_BF(sb, G::oR0);
    float* sEnv = SB_FL(sb, G::fENV);
    int* sEnvI = SB_IN(sb, G::fENVI);
    float r_inv = 0.f, r_invn = 0.f;
    if (lane < RPW) {
      const int r = wave * RPW + lane;
      sEnv[r * ENVF + 0] = e_b[S];
      sEnv[r * ENVF + 1] = e_val[S];
      sEnv[r * ENVF + 2] = wv[S];
      sEnv[r * ENVF + 5] = e_rs[S];
      sEnvI[r * 4 + 0] = e_pos[S];
      sEnvI[r * 4 + 1] = e_sh[S];
      sEnvI[r * 4 + 3] = e_ep[S];
      r_inv = __fdiv_rn(1.0f, wl[S]);
      r_invn = __fdiv_rn(1.0f, wv[S]);
    }
    if (lane < INP / 4) {
      bf16_t* px = sX + (wave * RPW) * G::SX + 4 * lane;
      bf16_t* pxn = sR0 + (wave * RPW) * G::SX + 4 * lane;
#pragma unroll
      for (int rr = 0; rr < RPW; ++rr) {
        const float inv = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(r_inv), rr));
        const float invn = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(r_invn), rr));
        const float w4 = dpp_next_lane(w[S][rr].x);
        f32x2_t x01 = {w[S][rr].x, w[S][rr].y}, x23 = {w[S][rr].z, w[S][rr].w};
        f32x2_t n01 = {w[S][rr].y, w[S][rr].z}, n23 = {w[S][rr].w, w4};
        if (FEAT) {
          const f32x2_t iv = {inv, inv}, ivn = {invn, invn}, one = {1.0f, 1.0f};
          x01 = x01 * iv - one; x23 = x23 * iv - one;
          n01 = n01 * ivn - one; n23 = n23 * ivn - one;
        }
        const int cw = asw(wave * RPW + rr, (4 * lane) & 15) - ((4 * lane) & 15);
        lds_st4(px + rr * G::SX + cw, x01.x, x01.y, x23.x, x23.y);
        lds_st4(pxn + rr * G::SX + cw, n01.x, n01.y, n23.x, n23.y);
      }
    }
    if (lane < RPW) {   // x tail: (budget, shares, 1)
      const int rw = wave * RPW + lane;
      bf16_t* xt = sX + rw * G::SX;
      xt[(H & ~15) + asw(rw, H & 15)] = f2bf(feat_budget(e_b[S], p.inv_b0, FEAT));
      xt[((H + 1) & ~15) + asw(rw, (H + 1) & 15)] = f2bf(feat_shares(e_sh[S], wl[S], p.inv_b0, FEAT));
      xt[((H + 2) & ~15) + asw(rw, (H + 2) & 15)] = f2bf(1.0f);
    }
  };
  auto a_w0 = [&](int ks) { return aW0[ks]; };
  auto a_w1 = [&](int ks) { return frag_row(sW1, G::SW1, m0, ks * 32, l16, g4); };
  // P1 / P2: hidden layers of Q(x); P4 / P5: of Q(x').  P1 also draws the chunk's epsilon-greedy
  // decisions on ONE wave (DRAW_WAVE, lanes = the 32 envs; its SIMD partner is not a P3 / P6 wave):
  // Philox is ~60 dependent VALU ops with quarter-rate multiplies, paid once per chunk instead of by
  // every wave's row-owner lanes; P3 reads the result two intervals later.
  constexpr int DRAW_WAVE = 2;
  auto P1 = [&](auto s, int ch) {
    char* const sb = slot_base(s);
    if (wave == DRAW_WAVE && lane < C) {
      int* sEnvI = SB_IN(sb, G::fENVI);
      const int pos = sEnvI[lane * 4 + 0];
      uint32_t c0 = (uint32_t)(p.env_offset + ch * C + lane), c1 = (uint32_t)(step & 0xFFFFFFFFull),
               c2 = (uint32_t)(step >> 32), c3 = 0u;
      philox4x32(c0, c1, c2, c3, p.key0, p.key1);
      const float u1 = u24(c0), u2 = u24(c1);
      const bool exploit = u1 < fminf(p.eps, __fmul_rn((float)pos, p.inv_ramp));
      int rnd = (int)(u2 * 3.0f);
      rnd = rnd > 2 ? 2 : rnd;
      sEnvI[lane * 4 + 2] = rnd | (exploit ? 8 : 0);   // exploit flag (bit 3) + random action
    }
    fwd_hidden<INP, G::SX, G::SH1>(a_w0, SB_BF(sb, G::oX), SB_BF(sb, G::oH1), nullptr, m0, l16, g4);
  };
  auto P2 = [&](auto s) {
    char* const sb = slot_base(s);
    fwd_hidden<H1P, G::SH1, G::SH2>(a_w1, SB_BF(sb, G::oH1), SB_BF(sb, G::oH2), sB1, m0, l16, g4);
  };
  auto P4 = [&](auto s) {
    char* const sb = slot_base(s);
    fwd_hidden<INP, G::SX, G::SH1>(a_w0, SB_BF(sb, G::oR0), SB_BF(sb, G::oR1), nullptr, m0, l16, g4);
  };
  auto P5 = [&](auto s) {
    char* const sb = slot_base(s);
    fwd_hidden<H1P, G::SH1, G::SH2>(a_w1, SB_BF(sb, G::oR1), SB_BF(sb, G::oR0), sB1, m0, l16, g4);
  };
  // P3: Q(x), action, Buy/Sell/Hold env step, x' tail (waves < NET; lanes g4 == 0 own env 16w + l16)
  auto P3 = [&](auto s, int ch, bool valid) {
    if (wave >= NET) return;
    char* const sb = slot_base(s);
    float* sQ = SB_FL(sb, G::fQ);
    float* sEnv = SB_FL(sb, G::fENV);
    int* sEnvI = SB_IN(sb, G::fENVI);
    const f4v qa = fwd_out<H2P, G::SW2, G::SH2>(sW2, SB_BF(sb, G::oH2), wave, l16, g4);
    if (g4 == 0) {
      const int r = 16 * wave + l16, e = ch * C + r;
      float q[3];
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        q[j] = qa[j] + sB2[j];
        if (p.output_relu) q[j] = fmaxf(q[j], 0.f);
      }
      sQ[r * 4 + 0] = q[0];
      sQ[r * 4 + 1] = q[1];
      sQ[r * 4 + 2] = q[2];
      int greedy = 0;
      float best = q[0];
      if (q[1] > best) { best = q[1]; greedy = 1; }
      if (q[2] > best) { best = q[2]; greedy = 2; }
      const int draw = sEnvI[r * 4 + 2];
      const bool exploit = (draw & 8) != 0;
      const int a = exploit ? greedy : (draw & 3);
      const float b = sEnv[r * ENVF + 0], vprev = sEnv[r * ENVF + 1], vnew = sEnv[r * ENVF + 2];
      const int sh = sEnvI[r * 4 + 1];
      const float bd = p.compat_env ? p.b0 : b;
      const int sd = p.compat_env ? p.s0 : sh;
      const bool buy = (a == 0) && (bd >= vnew);
      const bool sell = (a == 1) && (sd > 0);
      const float b2 = buy ? __fsub_rn(bd, vnew) : (sell ? __fadd_rn(bd, vnew) : bd);
      const int s2 = buy ? sd + 1 : (sell ? sd - 1 : sd);
      const float cur = __fadd_rn(b, __fmul_rn((float)sh, vprev));
      const float nw = __fadd_rn(b2, __fmul_rn((float)s2, vnew));
      float rew = __fsub_rn(nw, cur);
      if (p.reward_mode) rew = cur > 0.f ? __fdiv_rn(rew, cur) : 0.f;
      sEnv[r * ENVF + 3] = b2;
      sEnv[r * ENVF + 4] = rew;
      sEnvI[r * 4 + 1] = s2;
      sEnvI[r * 4 + 2] = a | (exploit ? 0 : 4);
      bf16_t* xn = SB_BF(sb, G::oR0) + r * G::SX;
      xn[(H & ~15) + asw(r, H & 15)] = f2bf(feat_budget(b2, p.inv_b0, FEAT));
      xn[((H + 1) & ~15) + asw(r, (H + 1) & 15)] = f2bf(feat_shares(s2, vnew, p.inv_b0, FEAT));
      xn[((H + 2) & ~15) + asw(r, (H + 2) & 15)] = f2bf(1.0f);
      if (valid) {
        ENV_I(ER_ACTION, e) = a;
        ENV_F(ER_REWARD, e) = rew;
      }
    }
  };
  // P6: Q(x'), TD target, dQ row, env state write-back, per-env statistics -> LDS
  auto P6 = [&](auto s, int ch, bool valid) {
    if (wave >= NET) return;
    char* const sb = slot_base(s);
    float* sQ = SB_FL(sb, G::fQ);
    float* sEnv = SB_FL(sb, G::fENV);
    int* sEnvI = SB_IN(sb, G::fENVI);
    const f4v qn = fwd_out<H2P, G::SW2, G::SH2>(sW2, SB_BF(sb, G::oR0), wave, l16, g4);
    if (g4 == 0) {
      const int r = 16 * wave + l16, e = ch * C + r;
      float n[3];
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        n[j] = qn[j] + sB2[j];
        if (p.output_relu) n[j] = fmaxf(n[j], 0.f);
      }
      int am = 0;
      float mx = n[0];
      if (n[1] > mx) { mx = n[1]; am = 1; }
      if (n[2] > mx) { mx = n[2]; am = 2; }
      const int araw = sEnvI[r * 4 + 2], a = araw & 3;
      const float rew = sEnv[r * ENVF + 4];
      const int slot = p.target_compat ? am : a;
      const float y = __fadd_rn(rew, __fmul_rn(p.gamma, mx));
      const float qs = sQ[r * 4 + slot];
      const float diff = __fsub_rn(qs, y);
      float dq = p.loss_coef * (p.td_clip > 0.f ? fminf(fmaxf(diff, -p.td_clip), p.td_clip) : diff);
      if ((p.output_relu && !(qs > 0.f)) || !valid) dq = 0.f;
      const uint32_t dqb = (uint32_t)f2bf(dq);
      const uint32_t wd0 = (slot == 0) ? dqb : (slot == 1) ? (dqb << 16) : 0u, wd1 = (slot == 2) ? dqb : 0u;
      uint4* dqr = reinterpret_cast<uint4*>(SB_BF(sb, G::oDQ) + r * SQ);
      dqr[0] = make_uint4(wd0, wd1, 0u, 0u);
      dqr[1] = make_uint4(0u, 0u, 0u, 0u);
      const float b2 = sEnv[r * ENVF + 3], vnew = sEnv[r * ENVF + 2];
      const int s2 = sEnvI[r * 4 + 1];
      const int np = sEnvI[r * 4 + 0] + 1;
      const float rs = sEnv[r * ENVF + 5] + rew;
      float fdone = 0.f, ndone = 0.f;
      const bool done = np >= p.T - H;
      if (done) {
        fdone = __fadd_rn(b2, __fmul_rn((float)s2, vnew));
        ndone = 1.f;
      }
      if (valid) {
        if (done) {
          ENV_F(ER_LAST_FINAL, e) = fdone;
          ENV_I(ER_EPISODES, e) = sEnvI[r * 4 + 3] + 1;
          ENV_F(ER_BUDGET, e) = p.b0;
          ENV_I(ER_SHARES, e) = p.s0;
          ENV_F(ER_VALUE, e) = 0.f;
          ENV_I(ER_POS, e) = 0;
          ENV_F(ER_RET_SUM, e) = 0.f;
        } else {
          ENV_F(ER_BUDGET, e) = b2;
          ENV_I(ER_SHARES, e) = s2;
          ENV_F(ER_VALUE, e) = vnew;
          ENV_I(ER_POS, e) = np;
          ENV_F(ER_RET_SUM, e) = rs;
        }
      }
      // per-env statistics for the folding waves (sQ / sEnv[0..1] are dead until P0 / P3)
      const float vf = valid ? 1.f : 0.f;
      sQ[r * 4 + 0] = vf * rew;
      sQ[r * 4 + 1] = vf * (diff * diff);
      sQ[r * 4 + 2] = vf * qs;
      sQ[r * 4 + 3] = vf * ((araw >> 2) ? 1.f : 0.f);
      sEnv[r * ENVF + 0] = vf * fdone;
      sEnv[r * ENVF + 1] = vf * ndone;
    }
  };
  // P7: statistics fold (waves NET..NET+3), layer-2 data backward + dW2 / db2
  auto P7 = [&](auto s) {
    char* const sb = slot_base(s);
    {
      const int sw = wave - NET;
      // selects, not branches on the accumulators (a branch per accumulator made hipcc address
      // sa0 / sa1 through the stack)
      float x0 = 0.f, x1 = 0.f;
      if (sw >= 0 && sw < 4 && lane < C) {
        const f4v q = *reinterpret_cast<const f4v*>(SB_FL(sb, G::fQ) + lane * 4);
        const float f0 = SB_FL(sb, G::fENV)[lane * ENVF + 0], f1 = SB_FL(sb, G::fENV)[lane * ENVF + 1];
        x0 = sw == 0 ? q[0] : sw == 1 ? q[2] : sw == 2 ? f0 : f1;
        x1 = sw == 0 ? q[1] : sw == 1 ? q[3] : sw == 2 ? f0 * f0 : 0.f;
      }
      sa0 += x0;
      sa1 += x1;
    }
    bwd_data<OUTP, G::SW2, SQ, G::SH2, G::SH2>(sW2, SB_BF(sb, G::oDQ), SB_BF(sb, G::oH2), SB_BF(sb, G::oR0), m0, l16, g4);
    const s8v aq = frag_trp(SB_BF(sb, G::oDQ), SQ, 0, 0, l16, g4);
    gW2 = mfma32(aq, afrag_trp(SB_BF(sb, G::oH2), G::SH2, 0, m0, l16, g4), gW2);
    gB2 = mfma32(aq, ones, gB2);
  };
  // P8: layer-1 data backward + dW1 / db1 (dZ2 = R0, H1)
  auto P8 = [&](auto s) {
    char* const sb = slot_base(s);
    bwd_data<H2P, G::SW1, G::SH2, G::SH1, G::SH1>(sW1, SB_BF(sb, G::oR0), SB_BF(sb, G::oH1), SB_BF(sb, G::oR1), m0, l16, g4);
    const s8v a2 = afrag_trp(SB_BF(sb, G::oR0), G::SH2, 0, m0, l16, g4);
#pragma unroll
    for (int n = 0; n < B1; ++n) gW1[n] = mfma32(a2, afrag_trp(SB_BF(sb, G::oH1), G::SH1, 0, 16 * n, l16, g4), gW1[n]);
    gB1 = mfma32(a2, ones, gB1);
  };
  // P9: dW0^T[h1][in] += dZ1^T . X over the chunk's 32 envs (one k-step), software-pipelined strip
  auto P9 = [&](auto s) {
    char* const sb = slot_base(s);
    const bf16_t* sX = SB_BF(sb, G::oX);
    const s8v a1 = afrag_trp(SB_BF(sb, G::oR1), G::SH1, 0, m0, l16, g4);
    s8v bq[DW0_PIPE];
#pragma unroll
    for (int d = 0; d < DW0_PIPE; ++d) bq[d] = afrag_trp(sX, G::SX, 0, 16 * d, l16, g4);
    __builtin_amdgcn_sched_group_barrier(0x100, 2 * (DW0_PIPE + 1), 0);
#pragma unroll
    for (int n = 0; n < B0; ++n) {
      const s8v bx = bq[n % DW0_PIPE];
      gW0[n] = mfma32(a1, bx, gW0[n]);
      __builtin_amdgcn_sched_group_barrier(0x8, 1, 0);
      if (n + DW0_PIPE < B0) {
        bq[n % DW0_PIPE] = afrag_trp(sX, G::SX, 0, 16 * (n + DW0_PIPE), l16, g4);
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
      }
    }
  };
#undef SB_BF
#undef SB_FL
#undef SB_IN

  // Stagger (ST_PAIR_STAGGER): the two waves sharing a SIMD (w and w + 4) run an interval's two phases
  // in opposite orders, so while one issues one phase's MFMAs the other is in the other phase's
  // LDS / VALU work instead of both contending for the same pipe at the same time.
  auto both = [&](auto&& x, auto&& y) {
    if (ST_PAIR_STAGGER && wave >= 4) {
      y();
      x();
    } else {
      x();
      y();
    }
  };
  constexpr SlotT<0> A{};
  constexpr SlotT<1> B{};
  int iter = 0;
#define STP_STAMP(I) \
  if (p.stamps != nullptr && bid == 0 && tid == 0) p.stamps[iter * 16 + (I)] = __builtin_amdgcn_s_memtime();
  if (ST_PAIR_PRIO && wave >= 4) __builtin_amdgcn_s_setprio(1);
  for (int k = 0;; ++k) {
    const int ca = bid + 2 * k * grid;         // slot A: P0..P9 in intervals 0..9
    const int cbp = ca - grid;                 // slot B, second half (P5..P9 in intervals 0..4)
    const int cb = ca + grid;                  // slot B, first half (P0..P4 in intervals 5..9)
    const bool va = ca < nch, vbp = k > 0 && cbp < nch, vb = cb < nch;
    if (!va && !vbp) break;
    STP_STAMP(0);
    const int cac = min(ca, nch - 1), cbpc = min(max(cbp, 0), nch - 1), cbc = min(cb, nch - 1);
    // I0: A.P0 | B.P5 (+ env state of B's next chunk: three intervals ahead of its window loads' use)
    STP_LOAD_ENV(1, cb)
    both([&] { P0(A); }, [&] { P5(B); });
    __syncthreads();
    STP_STAMP(1);
    // I1: B.P6 (waves < NET, latency chain first) | A.P1
    both([&] { P6(B, cbpc, vbp); }, [&] { P1(A, cac); });
    __syncthreads();
    STP_STAMP(2);
    // I2: A.P2 | B.P7 (+ price windows of B's next chunk, used in I5)
    STP_LOAD_PRICES(1, cb)
    both([&] { P7(B); }, [&] { P2(A); });
    __syncthreads();
    STP_STAMP(3);
    // I3: A.P3 | B.P8
    both([&] { P3(A, cac, va); }, [&] { P8(B); });
    __syncthreads();
    STP_STAMP(4);
    // I4: A.P4 | B.P9
    both([&] { P9(B); }, [&] { P4(A); });
    __syncthreads();
    STP_STAMP(5);
    if (!va) break;   // drain: the rest of this cycle would be slot A's and slot B's empty phases
    // I5: A.P5 | B.P0 (+ env state of A's next chunk)
    STP_LOAD_ENV(0, ca + 2 * grid)
    both([&] { P0(B); }, [&] { P5(A); });
    __syncthreads();
    STP_STAMP(6);
    // I6: A.P6 | B.P1
    both([&] { P6(A, cac, va); }, [&] { P1(B, cbc); });
    __syncthreads();
    STP_STAMP(7);
    // I7: A.P7 | B.P2 (+ price windows of A's next chunk, used in I0)
    STP_LOAD_PRICES(0, ca + 2 * grid)
    both([&] { P7(A); }, [&] { P2(B); });
    __syncthreads();
    STP_STAMP(8);
    // I8: A.P8 | B.P3
    both([&] { P3(B, cbc, vb); }, [&] { P8(A); });
    __syncthreads();
    STP_STAMP(9);
    // I9: A.P9 | B.P4
    both([&] { P9(A); }, [&] { P4(B); });
    __syncthreads();
    STP_STAMP(10);
    ++iter;
  }
#undef STP_LOAD_ENV
#undef STP_LOAD_PRICES
#undef STP_STAMP
  if (ST_PAIR_PRIO) __builtin_amdgcn_s_setprio(0);

  STP_STAMPX(2);
  // ---------------------------------------------------------------- per-workgroup stats (-> LDS -> slab)
  {
    const int sw = wave - NET;
    if (sw >= 0 && sw < 4) {   // the four folding waves write all NSTAT slots (slot 7 is unused: 0)
      const float v0 = wave_sum(sa0), v1 = wave_sum(sa1);
      if (lane == 0) {
        constexpr int k0[4] = {0, 6, 4, 3}, k1[4] = {1, 2, 5, 7};
        sSt[k0[sw]] = v0;
        sSt[k1[sw]] = sw < 3 ? v1 : 0.f;
      }
    }
    __syncthreads();
    if (tid < NSTAT) p.stats[(size_t)bid * NSTAT + tid] = sSt[tid];
  }
  // ---------------------------------------------------------------- gradient slab write-out
  auto write_slab = [&](auto rowp, auto put_w, auto put_b) {
    {
      const int h = m0 + 4 * g4;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const auto rp = rowp(p.off_w0 + (h + j) * INP);
#pragma unroll
        for (int n = 0; n < B0; ++n) put_w(rp, n * 16, gW0[n][j]);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const auto rp = rowp(p.off_w1 + (h + j) * H1P);
#pragma unroll
        for (int n = 0; n < B1; ++n) put_w(rp, n * 16, gW1[n][j]);
      }
      if (l16 == 0)
#pragma unroll
        for (int j = 0; j < 4; ++j) put_b(p.off_b1 + h + j, gB1[j]);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) put_w(rowp(p.off_w2 + (4 * g4 + j) * H2P), m0, gW2[j]);
    if (wave == 0 && l16 == 0)
#pragma unroll
      for (int j = 0; j < 4; ++j) put_b(p.off_b2 + 4 * g4 + j, gB2[j]);
  };
  if (p.slab_bf16) {
    bf16_t* const sb = reinterpret_cast<bf16_t*>(p.slab) + (size_t)bid * 32 + l16;
    const size_t BS = (size_t)p.slab_rows * 32;
    write_slab([&](int row) { return sb + (size_t)(row >> 5) * BS; },
               [&](bf16_t* rp, int cb, float v) { rp[(size_t)(cb >> 5) * BS + (cb & 31)] = f2bf(v); },
               [&](int i, float v) { sb[(size_t)(i >> 5) * BS + (i & 31) - l16] = f2bf(v); });
  } else {
    float* const sf = p.slab + (size_t)bid * p.P + l16;
    write_slab([&](int row) { return sf + row; }, [&](float* rp, int cb, float v) { rp[cb] = v; },
               [&](int i, float v) { sf[i - l16] = v; });
  }
  STP_STAMPX(3);
  if (bid == 0 && tid == 0) p.ctrl[1] = step + 1;  // 1-based update count for the optimizer
  STP_STAMPX(4);
#undef STP_STAMPX
}

template <int INP, int H1P, int H2P, int FEAT>
static hipError_t launch_f(const QStepParams& p, int grid, hipStream_t stream) {
  using G = Geo<INP, H1P, H2P>;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)qstep_pair_kernel<INP, H1P, H2P, FEAT>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, G::BYTES);
    if (e != hipSuccess) return e;
    attr = true;
  }
  hipLaunchKernelGGL((qstep_pair_kernel<INP, H1P, H2P, FEAT>), dim3(grid), dim3(NT), G::BYTES, stream, p);
  return hipGetLastError();
}

}  // namespace pair
}  // namespace st

extern "C" int st_qstep_pair_lds_bytes(int inp, int h1p, int h2p) {
  if (inp == 224 && h1p == 128 && h2p == 128) return st::pair::Geo<224, 128, 128>::BYTES;
  return -1;
}

// Preconditions (checked here and by the host, sharetrade/trainer/engine.py): E % 32 == 0,
// 1 <= grid <= E / 64 (each workgroup holds two 32-env chunk slots), static chunk schedule,
// H + 3 <= inp - 16, 8-element aligned weight offsets.
extern "C" hipError_t st_qstep_pair_launch(const st::QStepParams* p, int inp, int h1p, int h2p, int grid,
                                           hipStream_t stream) {
  if (p->E % st::pair::C != 0 || grid < 1 || 2 * grid > p->E / st::pair::C) return hipErrorInvalidValue;
  if ((p->off_w0 | p->off_w1 | p->off_w2) & 7) return hipErrorInvalidValue;
  if (p->H + 3 > inp - 16) return hipErrorInvalidValue;
  if (p->chunk_heads) return hipErrorInvalidValue;   // static schedule only
  if (p->slab_bf16 && (p->slab_rows != grid || p->P % 32 != 0 || ((p->off_w0 | p->off_w1 | p->off_w2) & 31) ||
                       inp % 32 || h1p % 32 || h2p % 32))
    return hipErrorInvalidValue;
  if (inp == 224 && h1p == 128 && h2p == 128)
    return p->feat_mode ? st::pair::launch_f<224, 128, 128, 1>(*p, grid, stream)
                        : st::pair::launch_f<224, 128, 128, 0>(*p, grid, stream);
  return hipErrorInvalidValue;
}
