// Wide-chunk fused online-DQN engine step on CDNA4 (gfx950): the same step as
// qstep_fused.hip (gather -> Q(x) -> epsilon-greedy + env step -> Q(x') -> TD ->
// backward -> per-workgroup weight-gradient slabs; QDecisionPolicyActor.scala:54-77,
// TrainerChildActor.scala:82-146), re-tiled so that every workgroup barrier covers
// twice the work.
//
// qstep_fused.hip keeps all bf16 weights (~94 KB) resident in LDS, which leaves room
// for 32-env activation chunks only; its chunk loop is latency/barrier bound (in-kernel
// stamps: ~15.7k cycles per 32-env chunk, MFMA pipes ~11 % busy, profiles/).  Here:
//
//  * layer-1 weights (W0^T, the 59 KB image) live in VGPRs: a wave owning 16 hidden units of both
//    hidden layers holds one 16x224 A operand = 7 fragments = 28 VGPRs per lane, loaded once per
//    launch straight from the bf16 parameters;
//  * LDS holds W1^T / W2^T (forward row reads + hardware-transposed backward reads) and 64-env
//    activation chunks: the barriers of a chunk serve 64 envs instead of 32 and every A fragment
//    feeds 4 MFMAs (4 env tiles);
//  * the output layer runs on 4 waves (one 16-env tile each) and the epsilon-greedy + Buy/Sell/Hold
//    env step / TD target run in the lanes that hold the Q values (16 lanes x 4 waves instead of
//    one wave), removing a barrier per forward;
//  * the next chunk's price windows are issued at the start of the weight-gradient phase, so their
//    registers are live only from there to the gather (not across the forward / backward phases);
//  * two builds: 8 waves (two per SIMD, 256 registers per lane, 16 units per wave; this file via
//    qstep_wide8.hip, the engine default: fastest measured, profiles/r1_stamps_wide_step.md) and
//    4 waves (one per SIMD, 512 registers, 32 units per wave; this file).
#include "qstep.h"

#ifndef ST_WIDE_NS
#define ST_WIDE_NS wide
#define ST_WIDE_API(name) name
#endif

namespace st {
namespace ST_WIDE_NS {

constexpr int C = 64;          // envs per chunk
#ifndef ST_WIDE_WAVES
#define ST_WIDE_WAVES 4
#endif
constexpr int NW = ST_WIDE_WAVES;   // waves per workgroup (4: one per SIMD, 8: two per SIMD)
constexpr int NT = 64 * NW;
constexpr int NET = C / 16;    // env tiles per chunk
constexpr int RPW = C / NW;    // gather rows per wave
#ifndef ST_WIDE_PF_LATE
#define ST_WIDE_PF_LATE 1
#endif
constexpr bool PF_LATE = ST_WIDE_PF_LATE;
#ifndef ST_WIDE_PF_AFTER_DW0
#define ST_WIDE_PF_AFTER_DW0 0
#endif
#ifndef ST_WIDE_GTILE
#define ST_WIDE_GTILE 0
#endif
#ifndef ST_WIDE_STATW
#define ST_WIDE_STATW 1
#endif
#ifndef ST_WIDE_GRAD_EARLY
#define ST_WIDE_GRAD_EARLY 1
#endif
constexpr bool GRAD_EARLY = ST_WIDE_GRAD_EARLY;
#ifndef ST_WIDE_DW0_PIPE
#define ST_WIDE_DW0_PIPE 3
#endif
constexpr int DW0_PIPE = ST_WIDE_DW0_PIPE;   // X fragments in flight in the dW0 strip (0 = compiler order)
#ifndef ST_WIDE_KPIPE
#define ST_WIDE_KPIPE 0
#endif
constexpr int KPIPE = ST_WIDE_KPIPE;   // double-buffered k-loops (bits): 1 layer-1 forward, 2 layer-2 forward, 4 data backward
#ifndef ST_WIDE_ASWZ
#define ST_WIDE_ASWZ 1
#endif
// Activation images (rows = envs: X, X', H1, H2, H1', H2', dZ1, dZ2) store the 16-byte unit of
// column c of row r at c ^ 8 * bit2(r).  Fragment reads stay conflict-free (tools/lds_bank_sim.py);
// the epilogue ds_write_b64 of 16 env rows at one column drops from 4-way to 2-way bank conflicts
// (rows r and r + 4 no longer share banks).  Weight images and the dQ rows are not swizzled.
constexpr bool ASWZ = ST_WIDE_ASWZ;
#ifndef ST_WIDE_PRIO
#define ST_WIDE_PRIO 0   // 1: the second-dispatched half of the waves at s_setprio 1 through the chunk loop
#endif
#ifndef ST_WIDE_DRAW_EARLY
#define ST_WIDE_DRAW_EARLY 0
#endif
// DRAW_EARLY (off: A/B in profiles/r2_pair_kernel.md, P3 -330 ticks but P1-2 / P6 +600): the chunk's epsilon-greedy draws (Philox: ~60 dependent VALU ops with quarter-rate
// multiplies) are computed in P1 by the last wave for all 64 envs (lane = env row) and left in
// sEnvI[.][2]; P3 only resolves exploit ? argmax : random action.  Same draws, same actions.
constexpr bool DRAW_EARLY = ST_WIDE_DRAW_EARLY;
#ifndef ST_WIDE_OFOLD
#define ST_WIDE_OFOLD 0
#endif
// OFOLD: the output layer of Q(x) folded into layer 2's epilogue -- each wave multiplies its own 16
// bf16-rounded h2 units (its accumulator tile IS the B operand of a 16x16x16 MFMA) by its W2 slice and
// leaves a partial q in LDS (R1, dead from P1 to P4); P3 sums the eight partials in wave order instead
// of running the 4-deep dependent fwd_out chain (same operands, fp32 summation order differs).
constexpr bool OFOLD = ST_WIDE_OFOLD;
#ifndef ST_WIDE_WSWZ
#define ST_WIDE_WSWZ 0
#endif
// WSWZ: the weight images W1^T / W2^T at an unpadded 128-element row stride with their 16-byte units
// XOR-swizzled by row: unit u of row R sits at u ^ wf(R & 15), wf(r) = 2 (r & 7) ^ 9 bit3(r).  Both read
// forms are then conflict-free (tools/lds_bank_sim.py): the row-fragment reads of the forwards (16 rows
// per ds_read_b128 lane group; stride 136 costs 2x) and the transposed reads of the backward (8 rows x
// 32 bytes per ds_read_b64_tr_b16 group; stride 136 costs 2x), and the images shrink by 2.3 KB.
constexpr bool WSWZ = ST_WIDE_WSWZ;
ST_DEV int wf(int r) { return ((r & 7) << 1) ^ (((r >> 3) & 1) * 9); }
// element offset of (row R, column c) in a weight image of row stride S
ST_DEV int wsw(int R, int c, int S) { return WSWZ ? R * S + ((((c >> 3) ^ wf(R & 15))) << 3) + (c & 7) : R * S + c; }
// frag_row / frag_tr / the K=16 transposed read on a weight image
ST_DEV s8v wfrag_row(const bf16_t* img, int S, int r0, int k0, int l16, int g4) {
  return lds_ld8(img + wsw(r0 + l16, k0 + 8 * g4, S));
}
ST_DEV s8v wfrag_tr(const bf16_t* img, int S, int k0, int c0, int l16, int g4) {
  const int R = k0 + 8 * g4 + (l16 >> 2), c = c0 + 4 * (l16 & 3);
  s4v lo = lds_tr4(img + wsw(R, c, S));
  s4v hi = lds_tr4(img + wsw(R + 4, c, S));
  s8v r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}
// asw(r, lo): the swizzled offset of column base + lo for a base that is a multiple of 16 and lo < 16
// (then (base + lo) ^ 8 bit2(r) = base + (lo ^ 8 bit2(r)): the base stays an immediate offset)
ST_DEV int asw(int r, int lo) { return ASWZ ? (lo ^ ((r & 4) << 1)) : lo; }
// frag_row / frag_trp (csrc/qstep.h) on a swizzled activation image (k0, c0: multiples of 16)
ST_DEV s8v afrag_row(const bf16_t* img, int S, int r0, int k0, int l16, int g4) {
  const int r = r0 + l16;
  return lds_ld8(img + r * S + k0 + asw(r, 8 * g4));
}
ST_DEV s8v afrag_trp(const bf16_t* img, int S, int k0, int c0, int l16, int g4) {
  const int r = k0 + 4 * g4 + (l16 >> 2);   // the second read is row r + 16: same bit 2
  const bf16_t* q = img + r * S + c0 + asw(r, 4 * (l16 & 3));
  s4v lo = lds_tr4(q);
  s4v hi = lds_tr4(q + 16 * S);
  s8v v;
  v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
  v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
  return v;
}
constexpr int SQ = OUTP + 8;
constexpr int ENVF = 6;        // fp32 words per env in sEnv
static_assert(NW >= NET, "the output layer / env step maps env tile w to wave w < NET");

template <int INP, int H1P, int H2P>
struct Geo {
  static constexpr int SW1 = WSWZ ? H1P : H1P + 8, SW2 = WSWZ ? H2P : H2P + 8;
  static constexpr int SX = INP + 16, SH1 = H1P + 16, SH2 = H2P + 16;
  static constexpr int oW1 = 0;
  static constexpr int oW2 = oW1 + H2P * SW1;
  static constexpr int oX = oW2 + OUTP * SW2;
  static constexpr int oH1 = oX + C * SX;
  static constexpr int oH2 = oH1 + C * SH1;
  static constexpr int oR0 = oH2 + C * SH2;          // X' / H2' / dZ2
  static constexpr int R0SZ = (C * SX > C * SH2) ? C * SX : C * SH2;
  static constexpr int oR1 = oR0 + R0SZ;             // H1' / dZ1
  static constexpr int oDQ = oR1 + C * SH1;
  static constexpr int BF16_END = oDQ + C * SQ;
  static constexpr int fQ = BF16_END * 2;            // q(x)   [C][4] fp32 (also the end-of-launch stats scratch)
  static constexpr int fENV = fQ + C * 4 * 4;        // [C][ENVF] floats
  static constexpr int fENVI = fENV + C * ENVF * 4;  // [C][4] ints
  static constexpr int fB1 = fENVI + C * 4 * 4;      // b1 [H2P]
  static constexpr int fB2 = fB1 + H2P * 4;          // b2 [16]
  static constexpr int fST = fB2 + OUTP * 4;          // step statistics [NSTAT] fp32 (end of launch)
  static constexpr int fCL = fST + NSTAT * 4;         // dynamic schedule: claimed chunk (broadcast slot)
  static constexpr int BYTES = fCL + 16;
  static_assert(BYTES <= 163840, "LDS budget exceeded");
  static_assert(H1P % (16 * NW) == 0 && H2P % (16 * NW) == 0 && H1P == H2P, "m-tiles per wave");
  static_assert(INP % 32 == 0 && H1P % 32 == 0, "padding");
  static constexpr int MT = H1P / (16 * NW);   // 16-unit m-tiles per wave in each hidden layer
  static constexpr int KS0 = INP / 32;         // layer-1 k-steps
  static constexpr int NT0 = INP / 16 - 1;     // in-col tiles of dW0 (last tile is pure padding)
  static constexpr int NT1 = H1P / 16;
};

// out^T[m][env] for this wave's MT m-tiles and the chunk's NET env tiles; A fragments given per
// (m-tile, k-step) by the functor, B = activation rows.  Epilogue: + bias, ReLU, bf16 store into
// out image [env][m].
template <int MT, int K, int SB, int SO, bool ALDS, typename AFrag, bool OF = false, int SW2_ = 0>
ST_DEV void fwd_hidden(AFrag afrag, const bf16_t* sB, bf16_t* sO, const float* bias, int m0, int l16, int g4,
                       const bf16_t* sW2 = nullptr, float* sPart = nullptr, int wave = 0) {
  float bb[MT][4];   // bias read up front (its LDS latency under the MFMAs)
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) bb[i][j] = bias ? bias[m0 + 16 * i + 4 * g4 + j] : 0.f;
  f4v acc[MT][NET];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int n = 0; n < NET; ++n) acc[i][n] = zero4();
  if constexpr ((KPIPE & (ALDS ? 2 : 1)) != 0) {
    // double-buffered k-loop: k-step ks+1's fragments are read while ks's MFMAs issue (order pinned;
    // hipcc's own order waits lgkmcnt(0) for each k-step's reads right before its MFMAs)
    constexpr int KS = K / 32, NR = NET + (ALDS ? MT : 0);
    s8v b[2][NET], a[2][MT];
#pragma unroll
    for (int n = 0; n < NET; ++n) b[0][n] = afrag_row(sB, SB, 16 * n, 0, l16, g4);
    if constexpr (ALDS)
#pragma unroll
      for (int i = 0; i < MT; ++i) a[0][i] = afrag(i, 0);
    __builtin_amdgcn_sched_group_barrier(0x100, NR, 0);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int c = ks & 1;
      if (ks + 1 < KS) {
#pragma unroll
        for (int n = 0; n < NET; ++n) b[c ^ 1][n] = afrag_row(sB, SB, 16 * n, (ks + 1) * 32, l16, g4);
        if constexpr (ALDS)
#pragma unroll
          for (int i = 0; i < MT; ++i) a[c ^ 1][i] = afrag(i, ks + 1);
        __builtin_amdgcn_sched_group_barrier(0x100, NR, 0);
      }
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const s8v aa = ALDS ? a[c][i] : afrag(i, ks);
#pragma unroll
        for (int n = 0; n < NET; ++n) acc[i][n] = mfma32(aa, b[c][n], acc[i][n]);
      }
      __builtin_amdgcn_sched_group_barrier(0x8, MT * NET, 0);
    }
  } else
#pragma unroll
  for (int ks = 0; ks < K / 32; ++ks) {
    s8v b[NET];
#pragma unroll
    for (int n = 0; n < NET; ++n) b[n] = afrag_row(sB, SB, 16 * n, ks * 32, l16, g4);
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const s8v a = afrag(i, ks);
#pragma unroll
      for (int n = 0; n < NET; ++n) acc[i][n] = mfma32(a, b[n], acc[i][n]);
    }
  }
  if constexpr (OF) {
    // partial q^T[a][env] = W2[a][this wave's units] . h2[units][env]: lane (env l16, g4) holds units
    // 4 g4 .. 4 g4 + 3 of its accumulator -- the B-operand layout of v_mfma_f32_16x16x16_bf16
    s4v aw[MT];
#pragma unroll
    for (int i = 0; i < MT; ++i) aw[i] = lds_ld4(sW2 + wsw(l16, m0 + 16 * i + 4 * g4, SW2_));
#pragma unroll
    for (int n = 0; n < NET; ++n) {
      f4v pq = zero4();
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const f4v v = acc[i][n];
        uint2 hv;
        hv.x = pack_bf2(fmaxf(v[0] + bb[i][0], 0.f), fmaxf(v[1] + bb[i][1], 0.f));
        hv.y = pack_bf2(fmaxf(v[2] + bb[i][2], 0.f), fmaxf(v[3] + bb[i][3], 0.f));
        *reinterpret_cast<uint2*>(sO + (16 * n + l16) * SO + m0 + 16 * i + asw(l16, 4 * g4)) = hv;
        pq = mfma16(aw[i], __builtin_bit_cast(s4v, hv), pq);
      }
      if (g4 == 0) *reinterpret_cast<f4v*>(sPart + (wave * C + 16 * n + l16) * 4) = pq;   // actions 0..3
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int m = m0 + 16 * i + 4 * g4;
#pragma unroll
    for (int n = 0; n < NET; ++n) {
      const f4v v = acc[i][n];
      lds_st4(sO + (16 * n + l16) * SO + m0 + 16 * i + asw(l16, 4 * g4), fmaxf(v[0] + bb[i][0], 0.f), fmaxf(v[1] + bb[i][1], 0.f),
              fmaxf(v[2] + bb[i][2], 0.f), fmaxf(v[3] + bb[i][3], 0.f));
    }
  }
}

// q^T[a][env] of env tile `nt` (lanes g4 == 0 end up holding q[0..3] of env 16*nt + l16)
template <int K, int SA, int SB>
ST_DEV f4v fwd_out(const bf16_t* sA, const bf16_t* sB, int nt, int l16, int g4) {
  f4v acc = zero4();
#pragma unroll
  for (int ks = 0; ks < K / 32; ++ks) {
    const s8v a = wfrag_row(sA, SA, 0, ks * 32, l16, g4);
    const s8v b = afrag_row(sB, SB, 16 * nt, ks * 32, l16, g4);
    acc = mfma32(a, b, acc);
  }
  return acc;
}

// dA^T[m][env] = sum_k W[m][k] * dZ[env][k] (W read transposed from the W^T image [k][m]),
// masked by (act[env][m] > 0), bf16 store into out image [env][m].
template <int MT, int K, int SW, int SD, int SACT, int SO>
ST_DEV void bwd_data(const bf16_t* sWT, const bf16_t* sDZ, const bf16_t* sAct, bf16_t* sO, int m0, int l16, int g4) {
  // ReLU masks (forward activations) read up front: their LDS latency hides under the MFMAs, and the
  // epilogue has no load between its stores (hipcc kept each mask read right before its store:
  // one LDS round trip per tile)
  s4v hm[MT][NET];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int n = 0; n < NET; ++n) hm[i][n] = lds_ld4(sAct + (16 * n + l16) * SACT + m0 + 16 * i + asw(l16, 4 * g4));
  f4v acc[MT][NET];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int n = 0; n < NET; ++n) acc[i][n] = zero4();
  if constexpr (K == 16) {
    s4v b[NET];
#pragma unroll
    for (int n = 0; n < NET; ++n) b[n] = lds_ld4(sDZ + (16 * n + l16) * SD + 4 * g4);
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const s4v a = lds_tr4(sWT + wsw(4 * g4 + (l16 >> 2), m0 + 16 * i + 4 * (l16 & 3), SW));
#pragma unroll
      for (int n = 0; n < NET; ++n) acc[i][n] = mfma16(a, b[n], acc[i][n]);
    }
  } else if constexpr ((KPIPE & 4) != 0) {
    constexpr int KS = K / 32, NR = NET + 2 * MT;   // frag_tr = 2 reads
    s8v b[2][NET], a[2][MT];
#pragma unroll
    for (int n = 0; n < NET; ++n) b[0][n] = afrag_row(sDZ, SD, 16 * n, 0, l16, g4);
#pragma unroll
    for (int i = 0; i < MT; ++i) a[0][i] = wfrag_tr(sWT, SW, 0, m0 + 16 * i, l16, g4);
    __builtin_amdgcn_sched_group_barrier(0x100, NR, 0);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int c = ks & 1;
      if (ks + 1 < KS) {
#pragma unroll
        for (int n = 0; n < NET; ++n) b[c ^ 1][n] = afrag_row(sDZ, SD, 16 * n, (ks + 1) * 32, l16, g4);
#pragma unroll
        for (int i = 0; i < MT; ++i) a[c ^ 1][i] = wfrag_tr(sWT, SW, (ks + 1) * 32, m0 + 16 * i, l16, g4);
        __builtin_amdgcn_sched_group_barrier(0x100, NR, 0);
      }
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int n = 0; n < NET; ++n) acc[i][n] = mfma32(a[c][i], b[c][n], acc[i][n]);
      __builtin_amdgcn_sched_group_barrier(0x8, MT * NET, 0);
    }
  } else {
#pragma unroll
    for (int ks = 0; ks < K / 32; ++ks) {
      s8v b[NET];
#pragma unroll
      for (int n = 0; n < NET; ++n) b[n] = afrag_row(sDZ, SD, 16 * n, ks * 32, l16, g4);
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const s8v a = wfrag_tr(sWT, SW, ks * 32, m0 + 16 * i, l16, g4);
#pragma unroll
        for (int n = 0; n < NET; ++n) acc[i][n] = mfma32(a, b[n], acc[i][n]);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int m = m0 + 16 * i + 4 * g4;
#pragma unroll
    for (int n = 0; n < NET; ++n) {
      const int env = 16 * n + l16;
      const s4v h = hm[i][n];
      const f4v v = acc[i][n];
      lds_st4(sO + env * SO + m0 + 16 * i + asw(l16, 4 * g4), h[0] > 0 ? v[0] : 0.f, h[1] > 0 ? v[1] : 0.f, h[2] > 0 ? v[2] : 0.f,
              h[3] > 0 ? v[3] : 0.f);
    }
  }
}

template <int INP, int H1P, int H2P, int FEAT, bool DYN>
__global__ void __launch_bounds__(NT, 1) qstep_wide_kernel(QStepParams p) {
  using G = Geo<INP, H1P, H2P>;
  constexpr int MT = G::MT;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* sbf = reinterpret_cast<bf16_t*>(smem);
  bf16_t* sW1 = sbf + G::oW1;
  bf16_t* sW2 = sbf + G::oW2;
  bf16_t* sX = sbf + G::oX;
  bf16_t* sH1 = sbf + G::oH1;
  bf16_t* sH2 = sbf + G::oH2;
  bf16_t* sR0 = sbf + G::oR0;
  bf16_t* sR1 = sbf + G::oR1;
  bf16_t* sDQ = sbf + G::oDQ;
  float* sQ = reinterpret_cast<float*>(smem + G::fQ);
  float* sEnv = reinterpret_cast<float*>(smem + G::fENV);
  int* sEnvI = reinterpret_cast<int*>(smem + G::fENVI);
  float* sB1 = reinterpret_cast<float*>(smem + G::fB1);
  float* sB2 = reinterpret_cast<float*>(smem + G::fB2);
  float* sSt = reinterpret_cast<float*>(smem + G::fST);

  const int tid = threadIdx.x, lane = tid & 63, l16 = lane & 15, g4 = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H = p.H;
  const unsigned long long step = p.ctrl[0];
  const int m0 = 16 * MT * wave;   // this wave's hidden units in both hidden layers
  // debug stamps outside the chunk loop: row (chunks of this workgroup) of the stamp array, slots 8..12
  const int nmy = (p.E / C - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;
#define STW_STAMPX(I) \
  if (p.stamps != nullptr && blockIdx.x == 0 && tid == 0) p.stamps[nmy * 16 + 8 + (I)] = __builtin_amdgcn_s_memtime();
  STW_STAMPX(0);

  // ---------------------------------------------------------------- chunk schedule
  // static: chunk k of this workgroup = blockIdx.x + k * gridDim.x.  dynamic (p.chunk_heads): the
  // chunks of XCD x (chunk % 8 == x; workgroup i runs on XCD i % 8) are handed out by that XCD's
  // claim head -- a workgroup's first chunk is fixed, later ones are claimed (one returning atomic by
  // thread 0, two chunks ahead, broadcast through LDS).  Workgroups that start late (their CU still
  // held by a concurrent RCCL kernel in overlapped DP) then take fewer chunks instead of stretching
  // the launch's tail.  Per-XCD heads: one device-scope word serves ~88 claims/us.
  constexpr bool dyn = DYN;   // (a template flag: the static build keeps its scalar registers)
  int* sCl = reinterpret_cast<int*>(smem + G::fCL);
  const int xcd = blockIdx.x & 7;
  unsigned* const head = dyn ? p.chunk_heads + 32 * xcd : nullptr;
  const int gx = (int)gridDim.x >> 3;   // workgroups per XCD (dynamic mode: grid % 8 == 0)
  unsigned claim_v = 0u;                // thread 0: the claim in flight (consumed at the next publish)
  if (dyn && tid == 0) claim_v = atomicAdd(head, 1u);
  // k-th chunk of a sequence: static = blockIdx.x + k * grid; dynamic = xcd + 8 * j
  auto dyn_chunk = [&](unsigned j) { return (int)min(j * 8u + (unsigned)xcd, 0x7FFFFFF0u); };

  // ---------------------------------------------------------------- gather state + first env loads
  // (issued before the weight loads: the first chunk's price windows depend on its env positions,
  // two dependent HBM round trips that now overlap the weight traffic of the prologue)
  const int nchunks = p.E / C;
  int eA_pos = 0, eA_sh = 0, eA_ep = 0, eB_pos = 0, eB_sh = 0, eB_ep = 0;
  float eA_b = 0.f, eA_val = 0.f, eA_rs = 0.f, eB_b = 0.f, eB_val = 0.f, eB_rs = 0.f;
  float4 w[RPW];
  float wl = 0.f, wv = 0.f;
#define STW_LOAD_ENV(CH, POS, B, SH, VAL, RS, EP)                          \
  {                                                                        \
    const int ch_ = min((CH), nchunks - 1);                                \
    const int e_ = ch_ * C + wave * RPW + min(lane, RPW - 1);              \
    POS = ENV_I(ER_POS, e_); B = ENV_F(ER_BUDGET, e_); SH = ENV_I(ER_SHARES, e_);                  \
    VAL = ENV_F(ER_VALUE, e_); RS = ENV_F(ER_RET_SUM, e_); EP = ENV_I(ER_EPISODES, e_);            \
  }
#define STW_LOAD_PRICES(CH, POS)                                           \
  {                                                                        \
    const int ch_ = min((CH), nchunks - 1);                                \
    const int sh_ = (POS) & 3;                                             \
    const size_t off_ = ((size_t)sh_ * p.E + (size_t)(ch_ * C + wave * RPW + min(lane, RPW - 1))) \
        * p.T4 + (size_t)((POS) - sh_);                                    \
    const unsigned long long a_ = (unsigned long long)(p.prices4 + off_);  \
    const unsigned alo_ = (unsigned)a_, ahi_ = (unsigned)(a_ >> 32);       \
    _Pragma("unroll") for (int rr = 0; rr < RPW; ++rr) {                   \
      const unsigned long long b_ =                                        \
          ((unsigned long long)__builtin_amdgcn_readlane(ahi_, rr) << 32) | \
          (unsigned)__builtin_amdgcn_readlane(alo_, rr);                   \
      typedef float f4g_ __attribute__((ext_vector_type(4)));              \
      const f4g_ v_ = reinterpret_cast<const __attribute__((address_space(1))) f4g_*>(b_)[lane]; \
      w[rr] = make_float4(v_.x, v_.y, v_.z, v_.w);                         \
    }                                                                      \
    const float* pl_ = p.prices +                                          \
        (size_t)(ch_ * C + wave * RPW + min(lane, RPW - 1)) * p.T + (POS) + H; \
    wl = pl_[-1];                                                          \
    wv = pl_[0];                                                           \
  }
  // chunk = the chunk being computed, c1 = the next one (env state loaded), c2 = the one after
  int chunk = blockIdx.x, c1 = blockIdx.x + gridDim.x, c2 = c1;
  STW_LOAD_ENV(chunk, eA_pos, eA_b, eA_sh, eA_val, eA_rs, eA_ep)

  // ---------------------------------------------------------------- weights (once per launch)
  // W0^T rows m0 + 16i + l16 -> MT x KS0 A fragments in VGPRs (global dwordx4; the 57 KB image is
  // L2-resident across the workgroups of an XCD)
  s8v aW0[MT][G::KS0];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const bf16_t* w0 = p.wq + p.off_w0 + (size_t)(m0 + 16 * i + l16) * INP + 8 * g4;
#pragma unroll
    for (int ks = 0; ks < G::KS0; ++ks) aW0[i][ks] = *reinterpret_cast<const s8v*>(w0 + ks * 32);
  }
  {
    const bf16_t* w1 = p.wq + p.off_w1;
    for (int i = tid; i < H2P * H1P / 8; i += NT) {
      const int r = i / (H1P / 8), c = (i % (H1P / 8)) * 8;
      *reinterpret_cast<uint4*>(sW1 + wsw(r, c, G::SW1)) = *reinterpret_cast<const uint4*>(w1 + r * H1P + c);
    }
    const bf16_t* w2 = p.wq + p.off_w2;
    for (int i = tid; i < OUTP * H2P / 8; i += NT) {
      const int r = i / (H2P / 8), c = (i % (H2P / 8)) * 8;
      *reinterpret_cast<uint4*>(sW2 + wsw(r, c, G::SW2)) = *reinterpret_cast<const uint4*>(w2 + r * H2P + c);
    }
    for (int i = tid; i < H2P; i += NT) sB1[i] = p.wf[p.off_b1 + i];
    if (tid < OUTP) sB2[tid] = p.wf[p.off_b2 + tid];
  }

  // ---------------------------------------------------------------- gradient accumulators
  // Weight-gradient tiling (independent of the forward split): wave w owns GA0 row tiles (h1) x B0
  // column tiles of dW0^T and GA1 x B1 of dW1^T.  ST_WIDE_GTILE=1 splits dW0 of the 8-wave build in 2
  // column groups (a 2x7 block: 9 fragment reads per k-step instead of 1+13): P9 drops ~15 %, but the
  // extra live registers slow P3 / P6 and the whole step measured 2-3 % slower
  // (profiles/r1_wide_step_variants.md), so the default is the 1x13 strip.
  constexpr int GA0 = ST_WIDE_GTILE ? 2 : G::MT;       // dW0 row tiles per wave
  constexpr int GC0 = NW / (H1P / 16 / GA0);           // dW0 column groups
  constexpr int GA1 = (NW >= 8) ? 1 : 2;               // dW1 row tiles per wave (registers: 8 waves)
  constexpr int GC1 = NW / (H2P / 16 / GA1);
  static_assert(GC0 >= 1 && (H1P / 16 / GA0) * GC0 == NW && (H2P / 16 / GA1) * GC1 == NW, "gradient tiling");
  static_assert(GC0 == 1 || (INP / 16) % GC0 == 0, "dW0 column groups");
  constexpr int B0 = (GC0 == 1) ? G::NT0 : (INP / 16) / GC0;
  constexpr int B1 = (H1P / 16) / GC1;
  const int ghb0 = GA0 * (wave / GC0), gcg0 = wave % GC0;   // row-tile base, column group
  const int ghb1 = GA1 * (wave / GC1), gcg1 = wave % GC1;
  f4v gW0[GA0][B0];
  f4v gW1[GA1][B1];
  f4v gB1[GA1], gW2[MT];
  f4v gB2 = zero4();
#pragma unroll
  for (int i = 0; i < GA0; ++i)
#pragma unroll
    for (int n = 0; n < B0; ++n) gW0[i][n] = zero4();
#pragma unroll
  for (int i = 0; i < GA1; ++i) {
#pragma unroll
    for (int n = 0; n < B1; ++n) gW1[i][n] = zero4();
    gB1[i] = zero4();
  }
#pragma unroll
  for (int i = 0; i < MT; ++i) gW2[i] = zero4();
  // ones fragment for bias gradients: B[k][n] = (n == 0)
  s8v ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (l16 == 0) ? (short)0x3F80 : (short)0;

  // step statistics.  8-wave build (STATW): the Q-holding lanes (waves < NET) leave their per-env
  // values in LDS at the end of P6 and the waves that idle through P3 / P6 (NET..2*NET-1) fold them
  // into two lane accumulators at the start of P7 -- 2 live registers instead of 7 (those were the
  // spill victims of the 256-register build) and no reduction work on the P6 critical path.
  // 4-wave build: per-lane accumulators in the Q-holding lanes (512 registers).
  constexpr bool STATW = ST_WIDE_STATW && NW >= 2 * NET;
  float sa0 = 0.f, sa1 = 0.f;
  float st_reward = 0.f, st_loss = 0.f, st_explore = 0.f, st_done = 0.f, st_fsum = 0.f, st_fsq = 0.f,
        st_qslot = 0.f;

  int iter = 0;
#define STW_STAMP(I) \
  if (p.stamps != nullptr && blockIdx.x == 0 && tid == 0 && (!dyn || iter < nmy)) p.stamps[iter * 16 + (I)] = __builtin_amdgcn_s_memtime();

  // ---------------------------------------------------------------- software-pipelined gather
  // (same scheme as qstep_fused.hip: env state two chunks ahead, price windows one chunk ahead,
  // every load unconditional with clamped indices; lanes rr < RPW own one row each)
// next chunk's price windows + the env state of the one after (PF_LATE: issued at the start of the
// weight-gradient phase, so the window registers are live only from there to the next gather)
#define STW_PREFETCH_NEXT()                                                \
  {                                                                        \
    const int nxt_ = dyn ? c1 : chunk + (int)gridDim.x;                    \
    STW_LOAD_PRICES(nxt_, eB_pos)                                          \
    eA_pos = eB_pos; eA_b = eB_b; eA_sh = eB_sh; eA_val = eB_val; eA_rs = eB_rs; eA_ep = eB_ep; \
    if constexpr (dyn) c2 = __builtin_amdgcn_readfirstlane(sCl[0]);        \
    STW_LOAD_ENV(dyn ? c2 : nxt_ + (int)gridDim.x, eB_pos, eB_b, eB_sh, eB_val, eB_rs, eB_ep) \
  }
  STW_LOAD_PRICES(chunk, eA_pos)
  if (dyn) {
    if (tid == 0) sCl[0] = dyn_chunk((unsigned)gx + claim_v);
    __syncthreads();
    c1 = __builtin_amdgcn_readfirstlane(sCl[0]);
  }
  STW_LOAD_ENV(dyn ? c1 : chunk + (int)gridDim.x, eB_pos, eB_b, eB_sh, eB_val, eB_rs, eB_ep)
  __syncthreads();
  STW_STAMPX(1);

  if (ST_WIDE_PRIO && wave >= NW / 2) __builtin_amdgcn_s_setprio(1);
  while (chunk < nchunks) {
    STW_STAMP(0);
    if (dyn && tid == 0) claim_v = atomicAdd(head, 1u);   // the chunk after c1 (published after P1)
    const int ebase = chunk * C;
    // ------------------------------------------------------------ P0: windows -> feature rows
    // row-owner lanes (lane rr < RPW owns row wave*RPW + rr): env scalars -> LDS, 1/last, 1/new
    float r_inv = 0.f, r_invn = 0.f;
    if (lane < RPW) {
      const int r = wave * RPW + lane;
      sEnv[r * ENVF + 0] = eA_b;
      sEnv[r * ENVF + 1] = eA_val;
      sEnv[r * ENVF + 2] = wv;
      sEnv[r * ENVF + 5] = eA_rs;
      sEnvI[r * 4 + 0] = eA_pos;
      sEnvI[r * 4 + 1] = eA_sh;
      sEnvI[r * 4 + 3] = eA_ep;
      r_inv = __fdiv_rn(1.0f, wl);
      r_invn = __fdiv_rn(1.0f, wv);
    }
    // lane L < INP/4 owns window columns k = 4L..4L+3 of every row: price features; one 8-byte LDS
    // store per row for x and one for x'.  Columns H..H+2 are overwritten with the (budget, shares, 1)
    // tail (x: below, by the row owners of this wave; x': by the env step in P3).  Columns >= H+3 keep
    // the (finite) features of the prices past the window: the layer-1 weights of those padding
    // columns are zero (engine invariant, re-applied on load; the optimizer masks them), so they add
    // exactly 0 to Q -- no per-element select (64 VALU per wave and chunk).  Their weight gradient is
    // masked in the slab pass.
    if (lane < INP / 4) {
      bf16_t* px = sX + (wave * RPW) * G::SX + 4 * lane;
      bf16_t* pxn = sR0 + (wave * RPW) * G::SX + 4 * lane;
#pragma unroll
      for (int rr = 0; rr < RPW; ++rr) {
        const float inv = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(r_inv), rr));
        const float invn = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(r_invn), rr));
        const float w4 = dpp_next_lane(w[rr].x);
        // packed fp32 (v_pk_mul_f32 / v_pk_add_f32): same IEEE rounding as feat_price, half the VALU ops
        f32x2_t x01 = {w[rr].x, w[rr].y}, x23 = {w[rr].z, w[rr].w};
        f32x2_t n01 = {w[rr].y, w[rr].z}, n23 = {w[rr].w, w4};
        if (FEAT) {
          const f32x2_t iv = {inv, inv}, ivn = {invn, invn}, one = {1.0f, 1.0f};
          x01 = x01 * iv - one; x23 = x23 * iv - one;
          n01 = n01 * ivn - one; n23 = n23 * ivn - one;
        }
        const int cw = asw(wave * RPW + rr, (4 * lane) & 15) - ((4 * lane) & 15);   // swizzle shift of this row
        lds_st4(px + rr * G::SX + cw, x01.x, x01.y, x23.x, x23.y);
        lds_st4(pxn + rr * G::SX + cw, n01.x, n01.y, n23.x, n23.y);
      }
    }
    if (lane < RPW) {   // x tail: (budget, shares, 1) features (same wave, after its row stores)
      const int rw = wave * RPW + lane;
      bf16_t* xt = sX + rw * G::SX;
      xt[(H & ~15) + asw(rw, H & 15)] = f2bf(feat_budget(eA_b, p.inv_b0, FEAT));
      xt[((H + 1) & ~15) + asw(rw, (H + 1) & 15)] = f2bf(feat_shares(eA_sh, wl, p.inv_b0, FEAT));
      xt[((H + 2) & ~15) + asw(rw, (H + 2) & 15)] = f2bf(1.0f);
    }
    if constexpr (!PF_LATE) STW_PREFETCH_NEXT();
    __syncthreads();
    STW_STAMP(1);
    // ------------------------------------------------------------ P1-P2: hidden layers of Q(x)
    auto a_w0 = [&](int i, int ks) { return aW0[i][ks]; };
    auto a_w1 = [&](int i, int ks) { return wfrag_row(sW1, G::SW1, m0 + 16 * i, ks * 32, l16, g4); };
    if (DRAW_EARLY && wave == NW - 1) {
      const int pos = sEnvI[lane * 4 + 0];
      uint32_t c0 = (uint32_t)(p.env_offset + ebase + lane), c1 = (uint32_t)(step & 0xFFFFFFFFull),
               c2 = (uint32_t)(step >> 32), c3 = 0u;
      philox4x32(c0, c1, c2, c3, p.key0, p.key1);
      const float u1 = u24(c0), u2 = u24(c1);
      const bool exploit = u1 < fminf(p.eps, __fmul_rn((float)pos, p.inv_ramp));
      int rnd = (int)(u2 * 3.0f);
      rnd = rnd > 2 ? 2 : rnd;
      sEnvI[lane * 4 + 2] = rnd | (exploit ? 8 : 0);   // exploit flag (bit 3) + random action
    }
    fwd_hidden<MT, INP, G::SX, G::SH1, false>(a_w0, sX, sH1, nullptr, m0, l16, g4);
    if (dyn && tid == 0) sCl[0] = dyn_chunk((unsigned)gx + claim_v);   // read in P9
    __syncthreads();
    float* sPart = reinterpret_cast<float*>(sR1);   // OFOLD: [NW][C][4] partial q (R1 is dead until P4)
    if constexpr (OFOLD)
      fwd_hidden<MT, H1P, G::SH1, G::SH2, true, decltype(a_w1), true, G::SW2>(a_w1, sH1, sH2, sB1, m0, l16, g4, sW2,
                                                                            sPart, wave);
    else
      fwd_hidden<MT, H1P, G::SH1, G::SH2, true>(a_w1, sH1, sH2, sB1, m0, l16, g4);
    __syncthreads();
    STW_STAMP(2);
    // ------------------------------------------------------------ P3: Q(x), epsilon-greedy, env step
    // wave w < NET: output tile of env tile w; lanes g4 == 0 own env 16*w + l16
    if (wave < NET) {
      f4v qa;
      if constexpr (OFOLD) {
        qa = zero4();
        if (g4 == 0) {
#pragma unroll
          for (int w = 0; w < NW; ++w) qa += *reinterpret_cast<const f4v*>(sPart + (w * C + 16 * wave + l16) * 4);
        }
      } else {
        qa = fwd_out<H2P, G::SW2, G::SH2>(sW2, sH2, wave, l16, g4);
      }
      if (g4 == 0) {
        const int r = 16 * wave + l16, e = ebase + r;
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
        bool exploit;
        int rnd;
        if constexpr (DRAW_EARLY) {
          const int draw = sEnvI[r * 4 + 2];
          exploit = (draw & 8) != 0;
          rnd = draw & 3;
        } else {
          const int ps = sEnvI[r * 4 + 0];
          uint32_t c0 = (uint32_t)(p.env_offset + e), c1 = (uint32_t)(step & 0xFFFFFFFFull),
                   c2 = (uint32_t)(step >> 32), c3 = 0u;
          philox4x32(c0, c1, c2, c3, p.key0, p.key1);
          const float u1 = u24(c0), u2 = u24(c1);
          exploit = u1 < fminf(p.eps, __fmul_rn((float)ps, p.inv_ramp));
          rnd = (int)(u2 * 3.0f);
          rnd = rnd > 2 ? 2 : rnd;
        }
        const int a = exploit ? greedy : rnd;
        const float b = sEnv[r * ENVF + 0], vprev = sEnv[r * ENVF + 1], vnew = sEnv[r * ENVF + 2];
        const int s = sEnvI[r * 4 + 1];
        const float bd = p.compat_env ? p.b0 : b;
        const int sd = p.compat_env ? p.s0 : s;
        const bool buy = (a == 0) && (bd >= vnew);
        const bool sell = (a == 1) && (sd > 0);
        const float b2 = buy ? __fsub_rn(bd, vnew) : (sell ? __fadd_rn(bd, vnew) : bd);
        const int s2 = buy ? sd + 1 : (sell ? sd - 1 : sd);
        const float cur = __fadd_rn(b, __fmul_rn((float)s, vprev));
        const float nw = __fadd_rn(b2, __fmul_rn((float)s2, vnew));
        float rew = __fsub_rn(nw, cur);
        if (p.reward_mode) rew = cur > 0.f ? __fdiv_rn(rew, cur) : 0.f;
        if (p.reward_mode == 2) rew = __fsub_rn(rew, __fmul_rn(__fmul_rn(rew, 0.5f), rew));   // growth: log1p to 2nd order
        sEnv[r * ENVF + 3] = b2;
        sEnv[r * ENVF + 4] = rew;
        sEnvI[r * 4 + 1] = s2;
        sEnvI[r * 4 + 2] = STATW ? (a | (exploit ? 0 : 4)) : a;   // (8-wave: explore flag in bit 2)
        bf16_t* xn = sR0 + r * G::SX;
        xn[(H & ~15) + asw(r, H & 15)] = f2bf(feat_budget(b2, p.inv_b0, FEAT));
        xn[((H + 1) & ~15) + asw(r, (H + 1) & 15)] = f2bf(feat_shares(s2, vnew, p.inv_b0, FEAT));
        xn[((H + 2) & ~15) + asw(r, (H + 2) & 15)] = f2bf(1.0f);
        if constexpr (!STATW) st_explore += exploit ? 0.f : 1.f;
        ENV_I(ER_ACTION, e) = a;
        ENV_F(ER_REWARD, e) = rew;
      }
    }
    __syncthreads();
    STW_STAMP(3);
    // ------------------------------------------------------------ P4-P5: hidden layers of Q(x')
    fwd_hidden<MT, INP, G::SX, G::SH1, false>(a_w0, sR0, sR1, nullptr, m0, l16, g4);
    __syncthreads();
    fwd_hidden<MT, H1P, G::SH1, G::SH2, true>(a_w1, sR1, sR0, sB1, m0, l16, g4);
    __syncthreads();
    STW_STAMP(4);
    // ------------------------------------------------------------ P6: Q(x'), TD target, dQ, state write-back
    if (wave < NET) {
      const f4v qn = fwd_out<H2P, G::SW2, G::SH2>(sW2, sR0, wave, l16, g4);
      if (g4 == 0) {
        const int r = 16 * wave + l16, e = ebase + r;
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
        if (p.output_relu && !(qs > 0.f)) dq = 0.f;
        // dQ row: one nonzero at `slot`, written as two 16-byte stores
        // (slot < 3: only the first two words can be nonzero)
        const uint32_t dqb = (uint32_t)f2bf(dq);
        const uint32_t wd0 = (slot == 0) ? dqb : (slot == 1) ? (dqb << 16) : 0u, wd1 = (slot == 2) ? dqb : 0u;
        uint4* dqr = reinterpret_cast<uint4*>(sDQ + r * SQ);
        dqr[0] = make_uint4(wd0, wd1, 0u, 0u);
        dqr[1] = make_uint4(0u, 0u, 0u, 0u);
        const float b2 = sEnv[r * ENVF + 3], vnew = sEnv[r * ENVF + 2];
        const int s2 = sEnvI[r * 4 + 1];
        const int np = sEnvI[r * 4 + 0] + 1;
        const float rs = sEnv[r * ENVF + 5] + rew;
        float fdone = 0.f, ndone = 0.f;
        if (np >= p.T - H) {
          const float fin = __fadd_rn(b2, __fmul_rn((float)s2, vnew));
          ENV_F(ER_LAST_FINAL, e) = fin;
          ENV_I(ER_EPISODES, e) = sEnvI[r * 4 + 3] + 1;
          ENV_F(ER_BUDGET, e) = p.b0;
          ENV_I(ER_SHARES, e) = p.s0;
          ENV_F(ER_VALUE, e) = 0.f;
          ENV_I(ER_POS, e) = 0;
          ENV_F(ER_RET_SUM, e) = 0.f;
          fdone = fin;
          ndone = 1.f;
        } else {
          ENV_F(ER_BUDGET, e) = b2;
          ENV_I(ER_SHARES, e) = s2;
          ENV_F(ER_VALUE, e) = vnew;
          ENV_I(ER_POS, e) = np;
          ENV_F(ER_RET_SUM, e) = rs;
        }
        if constexpr (STATW) {
          // per-env stats for the idle waves (sQ / sEnv[0..1] are dead until the next chunk's P0 / P3)
          sQ[r * 4 + 0] = rew;
          sQ[r * 4 + 1] = diff * diff;
          sQ[r * 4 + 2] = qs;
          sQ[r * 4 + 3] = (araw >> 2) ? 1.f : 0.f;
          sEnv[r * ENVF + 0] = fdone;
          sEnv[r * ENVF + 1] = ndone;
        } else {
          st_reward += rew;
          st_loss += diff * diff;
          st_qslot += qs;
          st_done += ndone;
          st_fsum += fdone;
          st_fsq += fdone * fdone;
        }
      }
    }
    __syncthreads();
    STW_STAMP(5);
    // ------------------------------------------------------------ P7-P8: backward (data)
    if constexpr (STATW) {
      // stats fold (lane = env row of the chunk): wave NET: reward, loss; +1: qslot, explore;
      // +2: final portfolio sum, sum of squares; +3: episodes done
      // (row index re-derived from tid behind an opaque move: a loop-invariant address kept live
      // across the chunk would cost a register of the 256-register build)
      const int sw = wave - NET;
      int ln = tid;
      asm volatile("" : "+v"(ln));
      ln &= 63;
      if (sw == 0) { sa0 += sQ[ln * 4 + 0]; sa1 += sQ[ln * 4 + 1]; }
      else if (sw == 1) { sa0 += sQ[ln * 4 + 2]; sa1 += sQ[ln * 4 + 3]; }
      else if (sw == 2) { const float f = sEnv[ln * ENVF + 0]; sa0 += f; sa1 += f * f; }
      else if (sw == 3) { sa0 += sEnv[ln * ENVF + 1]; }
    }
    // dW2^T[out][h2] += dQ^T . H2, db2 += dQ^T . 1  (reads dQ, H2)
    auto grad_w2 = [&]() {
#pragma unroll
      for (int ks = 0; ks < C / 32; ++ks) {
        const int k0 = 32 * ks;
        const s8v aq = frag_trp(sDQ, SQ, k0, 0, l16, g4);
#pragma unroll
        for (int i = 0; i < MT; ++i) gW2[i] = mfma32(aq, afrag_trp(sH2, G::SH2, k0, m0 + 16 * i, l16, g4), gW2[i]);
        gB2 = mfma32(aq, ones, gB2);   // every wave (branch-free accumulators); wave 0 writes it
      }
    };
    // dW1^T[h2][h1] += dZ2^T . H1, db1 += dZ2^T . 1  (reads dZ2 = R0, H1)
    auto grad_w1 = [&]() {
#pragma unroll
      for (int ks = 0; ks < C / 32; ++ks) {
        const int k0 = 32 * ks;
        s8v a2[GA1];
#pragma unroll
        for (int i = 0; i < GA1; ++i) a2[i] = afrag_trp(sR0, G::SH2, k0, (ghb1 + i) * 16, l16, g4);
#pragma unroll
        for (int n = 0; n < B1; ++n) {
          const s8v bh = afrag_trp(sH1, G::SH1, k0, (gcg1 * B1 + n) * 16, l16, g4);
#pragma unroll
          for (int i = 0; i < GA1; ++i) gW1[i][n] = mfma32(a2[i], bh, gW1[i][n]);
        }
#pragma unroll
        for (int i = 0; i < GA1; ++i) gB1[i] = mfma32(a2[i], ones, gB1[i]);
      }
    };
    // dW0^T[h1][in] += dZ1^T . X  (reads dZ1 = R1, X)
    auto grad_w0 = [&]() {
      if constexpr (DW0_PIPE > 0 && GA0 == 1) {
        // software-pipelined strip: DW0_PIPE X fragments in flight ahead of the MFMA that consumes
        // them, order pinned with sched_group_barrier (hipcc otherwise reuses ONE fragment buffer:
        // read, wait, MFMA, read, ... -- the LDS latency of all 2 x 13 reads in series)
#pragma unroll
        for (int ks = 0; ks < C / 32; ++ks) {
          const int k0 = 32 * ks;
          const s8v a1 = afrag_trp(sR1, G::SH1, k0, ghb0 * 16, l16, g4);
          s8v bq[DW0_PIPE > 0 ? DW0_PIPE : 1];
#pragma unroll
          for (int d = 0; d < DW0_PIPE; ++d) bq[d] = afrag_trp(sX, G::SX, k0, (gcg0 * B0 + d) * 16, l16, g4);
          __builtin_amdgcn_sched_group_barrier(0x100, 2 * (DW0_PIPE + 1), 0);
#pragma unroll
          for (int n = 0; n < B0; ++n) {
            const s8v bx = bq[n % DW0_PIPE];
            gW0[0][n] = mfma32(a1, bx, gW0[0][n]);
            __builtin_amdgcn_sched_group_barrier(0x8, 1, 0);
            if (n + DW0_PIPE < B0) {
              bq[n % DW0_PIPE] = afrag_trp(sX, G::SX, k0, (gcg0 * B0 + n + DW0_PIPE) * 16, l16, g4);
              __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
            }
          }
        }
        return;
      }
#pragma unroll
      for (int ks = 0; ks < C / 32; ++ks) {
        const int k0 = 32 * ks;
        s8v a1[GA0];
#pragma unroll
        for (int i = 0; i < GA0; ++i) a1[i] = afrag_trp(sR1, G::SH1, k0, (ghb0 + i) * 16, l16, g4);
#pragma unroll
        for (int n = 0; n < B0; ++n) {
          const s8v bx = afrag_trp(sX, G::SX, k0, (gcg0 * B0 + n) * 16, l16, g4);
#pragma unroll
          for (int i = 0; i < GA0; ++i) gW0[i][n] = mfma32(a1[i], bx, gW0[i][n]);
        }
      }
    };
    // GRAD_EARLY: each weight gradient runs in the first phase where its operands are final -- dW2 beside
    // the layer-2 data backward (P7), dW1 beside the layer-1 data backward (P8) -- filling those
    // latency-bound phases; P9 keeps dW0 only.  (P7 writes only R0, P8 only R1: no read hazards.)
    bwd_data<MT, OUTP, G::SW2, SQ, G::SH2, G::SH2>(sW2, sDQ, sH2, sR0, m0, l16, g4);
    if constexpr (GRAD_EARLY) grad_w2();
    __syncthreads();
    bwd_data<MT, H2P, G::SW1, G::SH2, G::SH1, G::SH1>(sW1, sR0, sH1, sR1, m0, l16, g4);
    if constexpr (GRAD_EARLY) grad_w1();
    __syncthreads();
    STW_STAMP(6);
    // ------------------------------------------------------------ P9: weight gradients (sum over the chunk's envs)
    if constexpr (PF_LATE && !ST_WIDE_PF_AFTER_DW0) STW_PREFETCH_NEXT();
    grad_w0();
    // the next chunk's windows land during the rest of the phase, the barrier and the next gather's
    // row-owner work; their registers are not live across the forward / backward / dW0 phases
    if constexpr (PF_LATE && ST_WIDE_PF_AFTER_DW0) STW_PREFETCH_NEXT();
    if constexpr (!GRAD_EARLY) {
      grad_w1();
      grad_w2();
    }
    __syncthreads();
    STW_STAMP(7);
    ++iter;
    if constexpr (dyn) {
      chunk = c1;
      c1 = c2;
    } else {
      chunk += gridDim.x;
    }
  }
#undef STW_LOAD_ENV
#undef STW_LOAD_PRICES
#undef STW_PREFETCH_NEXT
#undef STW_STAMP

  if (ST_WIDE_PRIO) __builtin_amdgcn_s_setprio(0);
  STW_STAMPX(2);
  // ---------------------------------------------------------------- per-workgroup stats (-> LDS -> slab)
  // (before the slab write-out, so its barrier does not wait for the slab stores; the chunk loop
  // ends on a barrier; sSt is outside every chunk buffer)
  if constexpr (STATW) {
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
    if (tid < NSTAT) p.stats[(size_t)blockIdx.x * NSTAT + tid] = sSt[tid];
  } else {
    const float v[NSTAT - 1] = {st_reward, st_loss, st_explore, st_done, st_fsum, st_fsq, st_qslot};
    float* so = sQ + wave * NSTAT;   // waves -> LDS, then a fixed-order fold (deterministic)
#pragma unroll
    for (int k = 0; k < NSTAT - 1; ++k) {
      const float t = wave_sum(v[k]);
      if (lane == 0) so[k] = t;
    }
    if (lane == 0) so[NSTAT - 1] = 0.f;
    __syncthreads();
    if (tid < NSTAT) {
      float t = 0.f;
#pragma unroll
      for (int k = 0; k < NW; ++k) t += sQ[k * NSTAT + tid];
      p.stats[(size_t)blockIdx.x * NSTAT + tid] = t;
    }
  }
  // ---------------------------------------------------------------- gradient slab write-out
  // (bf16 slabs: each workgroup's fp32 partial is rounded once; csrc/optim.hip sums them in fp32)
  // rowp(row): this lane's pointer for the weight row whose first parameter index is `row`;
  // put_w(rp, cb, v): weight (row, cb + l16) with a wave-uniform column tile base cb (multiple of 16);
  // put_b(i, v): bias parameter i
  auto write_slab = [&](auto rowp, auto put_w, auto put_b) {
#pragma unroll
    for (int i = 0; i < GA0; ++i) {
      const int h = (ghb0 + i) * 16 + 4 * g4;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const auto rp = rowp(p.off_w0 + (h + j) * INP);
#pragma unroll
        for (int n = 0; n < B0; ++n) put_w(rp, (gcg0 * B0 + n) * 16, gW0[i][n][j]);
      }
    }
#pragma unroll
    for (int i = 0; i < GA1; ++i) {
      const int h = (ghb1 + i) * 16 + 4 * g4;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const auto rp = rowp(p.off_w1 + (h + j) * H1P);
#pragma unroll
        for (int n = 0; n < B1; ++n) put_w(rp, (gcg1 * B1 + n) * 16, gW1[i][n][j]);
      }
      if (gcg1 == 0 && l16 == 0)
#pragma unroll
        for (int j = 0; j < 4; ++j) put_b(p.off_b1 + h + j, gB1[i][j]);
    }
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) put_w(rowp(p.off_w2 + (4 * g4 + j) * H2P), m0 + 16 * i, gW2[i][j]);
    if (wave == 0 && l16 == 0)
#pragma unroll
      for (int j = 0; j < 4; ++j) put_b(p.off_b2 + 4 * g4 + j, gB2[j]);
  };
  if (p.slab_bf16) {
    // column-blocked [P/32][G][32] (csrc/optim.hip): parameter i of this workgroup at
    // ((i >> 5) * G + blockIdx.x) * 32 + (i & 31).  Weight rows start on 32-parameter boundaries
    // (segment offsets and padded row lengths are multiples of 32; checked by the launcher), so a
    // lane's row costs one multiply and each column tile is a scalar offset from it (the 128-wide
    // blocks this replaced took a shift / mask / multiply per element: ~1,170 VALU per wave)
    bf16_t* const sb = reinterpret_cast<bf16_t*>(p.slab) + (size_t)blockIdx.x * 32 + l16;
    const size_t BS = (size_t)p.slab_rows * 32;
    write_slab([&](int row) { return sb + (size_t)(row >> 5) * BS; },
               [&](bf16_t* rp, int cb, float v) { rp[(size_t)(cb >> 5) * BS + (cb & 31)] = f2bf(v); },
               [&](int i, float v) { sb[(size_t)(i >> 5) * BS + (i & 31) - l16] = f2bf(v); });
  } else {
    float* const sf = p.slab + (size_t)blockIdx.x * p.P + l16;
    write_slab([&](int row) { return sf + row; }, [&](float* rp, int cb, float v) { rp[cb] = v; },
               [&](int i, float v) { sf[i - l16] = v; });
  }

  STW_STAMPX(3);
  if (blockIdx.x == 0 && tid == 0) p.ctrl[1] = step + 1;  // 1-based update count for the optimizer
  STW_STAMPX(4);
#undef STW_STAMPX
}

template <int INP, int H1P, int H2P, int FEAT, bool DYN>
static hipError_t launch_fd(const QStepParams& p, int grid, hipStream_t stream) {
  using G = Geo<INP, H1P, H2P>;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)qstep_wide_kernel<INP, H1P, H2P, FEAT, DYN>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, G::BYTES);
    if (e != hipSuccess) return e;
    attr = true;
  }
  hipLaunchKernelGGL((qstep_wide_kernel<INP, H1P, H2P, FEAT, DYN>), dim3(grid), dim3(NT), G::BYTES, stream, p);
  return hipGetLastError();
}

template <int INP, int H1P, int H2P, int FEAT>
static hipError_t launch_f(const QStepParams& p, int grid, hipStream_t stream) {
  return p.chunk_heads ? launch_fd<INP, H1P, H2P, FEAT, true>(p, grid, stream)
                       : launch_fd<INP, H1P, H2P, FEAT, false>(p, grid, stream);
}

}  // namespace ST_WIDE_NS
}  // namespace st

extern "C" int ST_WIDE_API(st_qstep_wide_lds_bytes)(int inp, int h1p, int h2p) {
  if (inp == 224 && h1p == 128 && h2p == 128) return st::ST_WIDE_NS::Geo<224, 128, 128>::BYTES;
  return -1;
}

// Preconditions (checked here and by the host, sharetrade/trainer/engine.py): E % 64 == 0,
// 1 <= grid <= E / 64, H + 3 <= inp - 16, 8-element aligned weight offsets (16-byte fragment loads).
extern "C" hipError_t ST_WIDE_API(st_qstep_wide_launch)(const st::QStepParams* p, int inp, int h1p, int h2p, int grid,
                                           hipStream_t stream) {
  if (p->E % st::ST_WIDE_NS::C != 0 || grid < 1 || grid > p->E / st::ST_WIDE_NS::C) return hipErrorInvalidValue;
  if ((p->off_w0 | p->off_w1 | p->off_w2) & 7) return hipErrorInvalidValue;
  if (p->H + 3 > inp - 16) return hipErrorInvalidValue;
  if (p->slab_bf16 && (p->slab_rows != grid || p->P % 32 != 0 || ((p->off_w0 | p->off_w1 | p->off_w2) & 31) ||
                       inp % 32 || h1p % 32 || h2p % 32))
    return hipErrorInvalidValue;   // 32-parameter column blocks, weight rows block-aligned
  if (p->chunk_heads && (!st::ST_WIDE_NS::PF_LATE || grid % 8 != 0 || (p->E / st::ST_WIDE_NS::C) % 8 != 0)) return hipErrorInvalidValue;
  if (inp == 224 && h1p == 128 && h2p == 128)
    return p->feat_mode ? st::ST_WIDE_NS::launch_f<224, 128, 128, 1>(*p, grid, stream)
                        : st::ST_WIDE_NS::launch_f<224, 128, 128, 0>(*p, grid, stream);
  return hipErrorInvalidValue;
}
