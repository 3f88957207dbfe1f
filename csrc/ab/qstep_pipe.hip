// Unit-sliced, weight-stationary, software-pipelined fused online-DQN engine step on CDNA4 (gfx950):
// the step of csrc/qstep_ws.hip (gather -> Q(x) -> epsilon-greedy + Buy/Sell/Hold env step -> Q(x') -> TD
// target -> backward -> per-workgroup weight-gradient slabs; QDecisionPolicyActor.scala:54-77,
// TrainerChildActor.scala:82-146) reorganised so that each SIMD always has several tiles' independent work
// instead of one tile's dependent chain.
//
// Why a new kernel (docs/PERFORMANCE.md, "where this design's ceiling is"): qstep_ws.hip runs each 16-env
// tile as ONE dependent chain in one data wave (features -> layer 1 -> layer 2 -> output -> env step ->
// Q(x') -> TD -> dZ2: ~12.8k cycles per tile for ~3k cycles of its own MFMA work), with the weights in LDS
// and one tile in flight per SIMD; its registers (246 of 256) and LDS (all 160 KiB) leave no room for a
// second chain.  Here:
//
//  * every wave owns 16 hidden units of each layer (wave w: units 16 w .. 16 w + 15) and keeps its slices of
//    W0 (26 VGPRs) and of W1's rows (16) in registers for the whole launch, and its slices of the weight
//    gradients (dW0 52, dW1 32, dW2 4); W1's columns (the dZ1 product) are a transposed LDS image;
//  * the activations of a tile go through LDS (X, X', H1, H1', dZ2 images, partial output sums), and
//  * the step of a tile is cut into stages that are a barrier apart.  Iteration `it` has two phases, each
//    ended by one s_barrier, and runs one stage of each of five tiles:
//        P0(it):  features of tile it (window -> X, X', env record)          [all waves]
//                 layer 2 of Q(x) of tile it-1 + this wave's output share    [all]   -> Q partials
//                 layer 2 of Q(x') of tile it-2 + output share               [all]   -> Q' partials
//                 dZ1 of tile it-3 (this wave's units)                        [all]
//        P1(it):  epsilon-greedy + env step of tile it-1, TD target of it-2  [waves 0-3, handed to 4-7]
//                 layer 1 of Q(x) and of Q(x')'s window of tile it          [all]   -> H1
//                 weight gradients of a PAIR of tiles (K = 32 envs per MFMA) [all]
//                 Q(x')'s layer-1 tail of tile it-1, dZ2 and dW2 of it-2     [all]   -> H1', dZ2
//    so a wave issues five tiles' independent MFMA / VALU / LDS work between two barriers, and the two waves of
//    a SIMD run them in complementary orders (waves 0-3 start P1 with the VALU-heavy env step and TD, waves
//    4-7 with the MFMAs).
//
// The env step and the TD target need the whole output layer (the sum of the 8 waves' partial Q) and every
// wave needs their results (the x' tail features for its Z1' rows, dQ for its dZ2 rows): waves 0-3 compute
// both redundantly (one per SIMD) and hand them to their SIMD partner (waves 4-7) through an LDS flag word per
// producer inside the phase; the partners use them at the end of it.  The next tile's price windows and env rows
// are brought into LDS by LDS-DMA (global_load_lds) during P1, so no VGPR holds a load in flight across the
// MFMA stages.  Per-env uniforms (the Philox draw of qstep_ws.hip) are computed once per launch in the
// prologue into the env's action row, which the env step overwrites with the action.
//
// Numerics: the rounding points of qstep_ws.hip (bf16 operands, fp32 accumulation, dZ2 / dQ products exact);
// fp32 summation orders differ (per-wave unit slices, pairs of tiles per weight-gradient MFMA).  A workgroup
// accumulates its tiles in a fixed order: bit-exact replays.
//
// Specialised to the flagship geometry: window H = 201, padded dims 224-128-128-16 (input slots 208),
// 64-env chunks (4 tiles of 16 envs), static chunk schedule.
#include "../qstep.h"

#ifndef PIPE_STAMPS
#define PIPE_STAMPS 0   // debug builds (csrc/ab/qstep_pipe_stamps.hip): s_memtime at 8 points per iteration of
#endif                  // workgroup 0, waves 0 and 4 (tools/stamp_pipe.py)
#ifndef PIPE_NS
#define PIPE_NS pipe
#define PIPE_API(name) name
#endif

// scheduling fence between stages: keeps a stage's loads from being hoisted into the previous one
#define PIPE_SB() __builtin_amdgcn_sched_barrier(0)
#define PIPE_SGB(MASK, N) __builtin_amdgcn_sched_group_barrier(MASK, N, 0)

namespace st {
namespace PIPE_NS {

// instruction-group pattern inside a stage: PF groups of NLD LDS reads ahead, then (NMF MFMAs, NLD reads)
template <int N, int PF, int NLD, int NMF>
ST_DEV void pattern() {
#pragma unroll
  for (int i = 0; i < PF && i < N; ++i) PIPE_SGB(0x100, NLD);
#pragma unroll
  for (int i = 0; i < N; ++i) {
    PIPE_SGB(0x008, NMF);
    if (i + PF < N) PIPE_SGB(0x100, NLD);
  }
}

constexpr int NW = 8, NT = 64 * NW;
constexpr int NP = 4;            // producer waves (env step, TD); wave w + 4 is wave w's SIMD partner
constexpr int TE = 16;           // envs per tile
constexpr int C = 64;            // envs per chunk
constexpr int INP = 224, HP = 128, KX = 208, HWIN = 201;
constexpr int XS = 216;          // row stride (bf16) of the X / X' images
constexpr int HS = 136;          // row stride (bf16) of the 128-wide images (H1, H1', dZ2, W1^T)
constexpr int NXB = 6, NH1 = 5, NDZ = 3;
constexpr int NJOB = TE * 26;    // feature jobs per tile: (env, group of 8 input slots)
constexpr int DRAIN = 4;         // iterations past the last tile (the second half of its pair)

// ---------------------------------------------------------------------------------- LDS layout (bytes)
constexpr int X_BYTES = TE * XS * 2, H_BYTES = TE * HS * 2;
constexpr int oXB = 0;                              // X   [NXB][16][XS] bf16 (input slot order)
constexpr int oXP = oXB + NXB * X_BYTES;            // X'  [16][XS] bf16 (slots 192..195 zero: the env step's)
constexpr int oH1 = oXP + X_BYTES;                  // H1  [NH1][16][HS] bf16
constexpr int oH1P = oH1 + NH1 * H_BYTES;           // H1' [16][HS]
constexpr int oDZ = oH1P + H_BYTES;                 // dZ2 [NDZ][16][HS]
constexpr int oW1T = oDZ + NDZ * H_BYTES;           // W1^T [128][128] bf16 (u1 rows, u2 columns; 16-B units
constexpr int oQP = oW1T + HP * HP * 2;             //   XOR-swizzled by the row)  Q partials [NW][16] f32x4
constexpr int oQPP = oQP + NW * TE * 16;            // Q' partials [NW][16] f32x4
constexpr int oENVR = oQPP + NW * TE * 16;          // TD record [2][16][8] words (wave 0: env step -> TD)
constexpr int oEREC = oENVR + 2 * TE * 32;          // env record [2][16][8] words (features -> env step)
constexpr int oTAIL = oEREC + 2 * TE * 32;          // x' tail features [NP][16] 4 bf16 (producer -> partner)
constexpr int oDQ = oTAIL + NP * TE * 8;            // dQ [NP][16] 4 bf16 (producer -> partner)
constexpr int oSCR = oDQ + NP * TE * 8;             // per wave: H2^T [16][16] bf16; then one shared dQ^T [16][16]
constexpr int NJW = (NJOB + 63) / 64;               // waves with feature jobs (7)
constexpr int STG_BYTES = NJW * 2048;               // LDS-DMA staging of one tile: per job wave 2 x 1 KiB (window
constexpr int oSTG = oSCR + NW * 512 + 512;         //   dwords 0-3 | 4-7), two tiles in flight
// job wave 6 fills only lanes 0..31 of its two KiB: the env rows of the tile (wave 7's DMA, [8][16] words) go to
// its upper half of the first KiB, and lane groups with no result store to the second (a write-only sink)
constexpr int ESTG_OFF = 6 * 2048 + 512, SINK_OFF = 6 * 2048 + 1024 + 512;
constexpr int oW2 = oSTG + 2 * STG_BYTES;           // W2  [4][128] bf16 (row 3 zero)
constexpr int oW2T = oW2 + 4 * HP * 2;              // W2^T [128][4] bf16 (column 3 zero)
constexpr int oB1 = oW2T + HP * 4 * 2;              // b1 [128] f32
constexpr int oZERO = oB1 + HP * 4;                 // 64 zero bytes
constexpr int oCTL = oZERO + 64;                    // ints: [0..3] tail flags, [4..7] dQ flags, [12] abort
constexpr int oST = oCTL + 64;                      // [NW][NSTAT] f32
constexpr int LDS_BYTES = oST + NW * NSTAT * 4;
static_assert(LDS_BYTES <= 163840, "LDS budget");
static_assert((X_BYTES % 16) == 0 && (H_BYTES % 16) == 0 && (oW1T % 16) == 0 && (oSTG % 16) == 0, "alignment");
static_assert(NJW == 7 && NJOB <= 6 * 64 + 32, "wave 7 stages the env rows into wave 6's free half");
constexpr int CTL_TAIL = 0, CTL_DQ = 4, CTL_ABORT = 12;
constexpr int SPIN_LIMIT = 1 << 22;

// input slot -> flat-layout column of W0^T (the permutation of qstep_ws.hip: the last 16-wide k-step puts
// budget, shares, the constant 1 and the window's last price in lane group 0)
ST_DEV int slot_col(int s) {
  if (s < 192) return s;
  const int t = s - 192, g = t >> 2, j = t & 3;
  if (g == 0) return j < 3 ? 201 + j : 200;
  if (g == 1) return 192 + j;
  if (g == 2) return 196 + j;
  return 204 + j;
}

// W1^T image: 16-byte unit c / 8 of row r at (c / 8) ^ (r & 15): the dZ1 B-fragment reads (16 rows, one unit
// each) hit 16 different bank groups
ST_DEV int w1t_off(int r, int c) { return r * HP + ((((c >> 3) ^ (r & 15))) << 3) + (c & 7); }

ST_DEV s4v zero_s4() { s4v z = {0, 0, 0, 0}; return z; }
ST_DEV s8v cat8(s4v a, s4v b) {
  s8v r;
  r[0] = a[0]; r[1] = a[1]; r[2] = a[2]; r[3] = a[3];
  r[4] = b[0]; r[5] = b[1]; r[6] = b[2]; r[7] = b[3];
  return r;
}
ST_DEV s4v pk4(float a, float b, float c, float d) {
  uint2 v;
  v.x = pack_bf2(a, b);
  v.y = pack_bf2(c, d);
  return __builtin_bit_cast(s4v, v);
}
ST_DEV s8v pk8(const float* v) {
  uint4 r;
  r.x = pack_bf2(v[0], v[1]);
  r.y = pack_bf2(v[2], v[3]);
  r.z = pack_bf2(v[4], v[5]);
  r.w = pack_bf2(v[6], v[7]);
  return __builtin_bit_cast(s8v, r);
}
typedef short s2v __attribute__((ext_vector_type(2)));
// relu then bf16 == bf16 then relu on the bits (a negative bf16 is a negative int16)
ST_DEV s4v relu_bf(f4v v) {
  const s2v z = {0, 0};
  const s2v a = __builtin_elementwise_max(__builtin_bit_cast(s2v, pack_bf2(v[0], v[1])), z);
  const s2v b = __builtin_elementwise_max(__builtin_bit_cast(s2v, pack_bf2(v[2], v[3])), z);
  s4v r = {a[0], a[1], b[0], b[1]};
  return r;
}
// bf16(v) * [act > 0] on packed integers (act: relu'd bf16 bits, >= 0): bits * min(act, 1)
ST_DEV unsigned mask2(unsigned x, unsigned act) {
  unsigned m, r;
  asm("v_pk_min_u16 %0, %1, %2" : "=v"(m) : "v"(act), "v"(0x00010001u));
  asm("v_pk_mul_lo_u16 %0, %1, %2" : "=v"(r) : "v"(x), "v"(m));
  return r;
}
ST_DEV s4v mask_pk(f4v v, s4v act) {
  const uint2 a = __builtin_bit_cast(uint2, act);
  uint2 r;
  r.x = mask2(pack_bf2(v[0], v[1]), a.x);
  r.y = mask2(pack_bf2(v[2], v[3]), a.y);
  return __builtin_bit_cast(s4v, r);
}
ST_DEV f4v ld_f4(const void* p) { return *reinterpret_cast<const f4v*>(p); }
ST_DEV int lds_acq(const int* w) {
  return __builtin_amdgcn_readfirstlane(__hip_atomic_load(w, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
}
// LDS-DMA from inline asm (csrc/qserve.hip): the builtin makes hipcc order every later LDS store behind the
// DMA; the kernel retires it itself (s_waitcnt vmcnt(0) before the phase's barrier).  lds_off: wave-uniform
// byte offset of the wave-instruction's destination (lane i lands at lds_off + 16 i / 4 i).
ST_DEV void glds16(const void* gsrc, unsigned lds_off) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(lds_off) : "memory");
}
// env rows: sc1 (L2; the draw words were stored by this launch's prologue)
ST_DEV void glds4_sc1(const void* gsrc, unsigned lds_off) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off sc1\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(lds_off) : "memory");
}
ST_DEV void wait_vm0() { __builtin_amdgcn_s_waitcnt((0x7 << 4) | (0xF << 8)); }
#define wait_vm(N) __builtin_amdgcn_s_waitcnt((N) | (0x7 << 4) | (0xF << 8))   // vmcnt(N), N < 16
ST_DEV unsigned lds_base(char* p) {   // a generic pointer into LDS -> its LDS byte address
  return (unsigned)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) char*)p);
}

template <int FEAT>
__global__ void __launch_bounds__(NT, 1) qstep_pipe_kernel(QStepParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, l16 = lane & 15, g4 = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool producer = w < NP;
  const unsigned long long step = p.ctrl[0];
  const int nchunks = p.E / C;
  const int nmy = (nchunks - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;
  const int ntile = 4 * nmy;
  int* ctl = reinterpret_cast<int*>(smem + oCTL);
  auto tile_env0 = [&](int t) { return ((int)blockIdx.x + (t >> 2) * (int)gridDim.x) * C + TE * (t & 3); };
  auto bf = [&](int off) { return reinterpret_cast<bf16_t*>(smem + off); };
  const unsigned smem_base = lds_base(smem);

  // ------------------------------------------------------------------ prologue
  // every ring starts zeroed: stages that run before the first tile (pipeline fill) compute on finite data
  for (int i = tid; i < LDS_BYTES / 16; i += NT) reinterpret_cast<int4*>(smem)[i] = make_int4(0, 0, 0, 0);
  __syncthreads();
  {
    const bf16_t* w2 = p.wq + p.off_w2;
    for (int i = tid; i < 4 * HP; i += NT) {
      const int a = i / HP, u = i % HP;
      const bf16_t v = a < 3 ? w2[a * HP + u] : (bf16_t)0;
      bf(oW2)[a * HP + u] = v;
      bf(oW2T)[u * 4 + a] = v;
    }
    const bf16_t* w1 = p.wq + p.off_w1;
    for (int i = tid; i < HP * HP; i += NT) {          // W1^T[u1][u2] = W1[u2][u1]  (W1 stored [u2][u1])
      const int u2 = i / HP, u1 = i % HP;
      bf(oW1T)[w1t_off(u1, u2)] = w1[i];
    }
    for (int i = tid; i < HP; i += NT) reinterpret_cast<float*>(smem + oB1)[i] = p.wf[p.off_b1 + i];
    // per-env uniforms of this step (Philox4x32-10 keyed by (global env, step), the draw of qstep_ws.hip):
    // packed u1 (24 bits) | random action << 30, into the env's action row until the env step replaces it
    for (int i = tid; i < nmy * C; i += NT) {
      const int e = ((int)blockIdx.x + (i / C) * (int)gridDim.x) * C + (i % C);
      uint32_t c0 = (uint32_t)(p.env_offset + e), c1 = (uint32_t)(step & 0xFFFFFFFFull),
               c2 = (uint32_t)(step >> 32), c3 = 0u;
      philox4x32(c0, c1, c2, c3, p.key0, p.key1);
      int rnd = (int)(u24(c1) * 3.0f);
      rnd = rnd > 2 ? 2 : rnd;
      p.env[(size_t)ER_ACTION * p.E + e] = (int)((c0 >> 8) | ((uint32_t)rnd << 30));
    }
    wait_vm0();          // the draws are read back (by LDS-DMA) by other waves of this workgroup
  }
  __syncthreads();
  // this wave's weight slices (bf16 images of the live weights), in MFMA operand layouts
  s8v W0s[6];     // A of layer 1: lane (unit l16, g4): W0[16 w + l16][32 ks + 8 g4 + j]
  s4v W0t;        //   the 16-wide tail k-step (input slots 192 + 4 g4 + j)
  s8v W1r[4];     // A of layer 2: W1[16 w + l16][32 ks + 8 g4 + j]  (W1 stored [u2][u1])
  {
    const bf16_t* w0 = p.wq + p.off_w0 + (size_t)(16 * w + l16) * INP;
#pragma unroll
    for (int ks = 0; ks < 6; ++ks) W0s[ks] = *reinterpret_cast<const s8v*>(w0 + 32 * ks + 8 * g4);
#pragma unroll
    for (int j = 0; j < 4; ++j) W0t[j] = (short)w0[slot_col(192 + 4 * g4 + j)];
    const bf16_t* w1 = p.wq + p.off_w1;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
      W1r[ks] = *reinterpret_cast<const s8v*>(w1 + (size_t)(16 * w + l16) * HP + 32 * ks + 8 * g4);
  }
  const float b2v0 = p.wf[p.off_b2], b2v1 = p.wf[p.off_b2 + 1], b2v2 = p.wf[p.off_b2 + 2];
  // weight-gradient slices: dW0 rows / dW1 rows of this wave's units, dW2 columns
  f4v gW0[13], gW1[8], gW2 = zero4();
  float gB1[4] = {0.f, 0.f, 0.f, 0.f};   // per-lane partial sums of dZ2 (units 16 w + 4 g4 + j)
#pragma unroll
  for (int n = 0; n < 13; ++n) gW0[n] = zero4();
#pragma unroll
  for (int n = 0; n < 8; ++n) gW1[n] = zero4();
  // statistics, per wave: 0 (reward, explore), 4 (loss, qslot, done), 5 (fsum, fsq), 6 db2[0..2]
  float sA = 0.f, sB = 0.f, sC = 0.f;
  // cross-phase carries: Z1' partial of tile it (P1 -> P1 of it + 1), H2 (P0 -> P1 of it + 1), dZ1 of a pair
  f4v zpOld = zero4();
  s4v h2A = zero_s4();   // H2 of tile it - 2 during P1 (made by P0 of it - 1)
  s4v dza = zero_s4(), dzb = zero_s4();

  // feature job of this lane: (env jenv of the tile, 8-slot group jkq); the window positions of the job's env
  // in tiles it .. it + 2 (the DMA of tile t is issued in P1 of t - 2 and needs its position)
  const bool jvalid = tid < NJOB;
  const int jenv = tid / 26, jkq = tid % 26;
  const int jbase = jkq < 24 ? 8 * jkq : (jkq == 24 ? 192 : 196);
  int jcur = 0, jn1 = 0, jn2 = 0;
  auto load_pos = [&](int t) { return p.env[(size_t)ER_POS * p.E + tile_env0(t) + jenv]; };
  // stage tile t into LDS buffer t & 1: each job lane's 8 window floats (two 16-B DMAs); wave 7: the env rows
  auto stage = [&](int t, int pos) {
    const unsigned sb = smem_base + oSTG + (t & 1) * STG_BYTES;
    if (w < NJW) {
      if (jvalid) {
        const int pc = min(max(pos, 0), p.T - HWIN - 1);
        const float* b = p.prices4 + (size_t)(tile_env0(t) + jenv) * p.T4 + (size_t)pc + jbase;
        glds16(b, __builtin_amdgcn_readfirstlane(sb + w * 2048));
        glds16(b + 4, __builtin_amdgcn_readfirstlane(sb + w * 2048 + 1024));
      }
    } else {
      // lane (row r = lane / 16, env l16): rows budget, shares, value, ret_sum (first DMA); episodes and the
      // draw (second DMA; lanes 32..63 duplicate the draw)
      const int rr = lane >> 4;
      const int e = tile_env0(t) + l16;
      glds4_sc1(p.env + (size_t)(ER_BUDGET + rr) * p.E + e, __builtin_amdgcn_readfirstlane(sb + ESTG_OFF));
      const int row1 = rr == 0 ? ER_EPISODES : ER_ACTION;
      glds4_sc1(p.env + (size_t)row1 * p.E + e, __builtin_amdgcn_readfirstlane(sb + ESTG_OFF + 256));
    }
  };
  if (ntile > 0) {
    if (jvalid) {
      jcur = load_pos(0);
      if (ntile > 1) jn1 = load_pos(1);
      if (ntile > 2) jn2 = load_pos(2);
    }
    stage(0, jcur);
    if (ntile > 1) stage(1, jn1);
    wait_vm0();
  }
  __syncthreads();

  // ------------------------------------------------------------------ per-stage helpers
  const int a_row = min(l16, 3);                     // W2 image row of this lane (row 3 zero)
  auto wait_flag = [&](int idx, int want) {
    for (int spin = 0; lds_acq(ctl + idx) < want; ++spin) {
      if (lds_acq(ctl + CTL_ABORT)) break;
      __builtin_amdgcn_s_sleep(1);
      if (spin > SPIN_LIMIT) {
        if (lane == 0) {
          __hip_atomic_store(ctl + CTL_ABORT, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          if (p.err != nullptr) atomicOr(p.err, 2u);
        }
        break;
      }
    }
  };
  auto sum_partials = [&](int off, float& a0, float& a1, float& a2) {   // fixed order over the 8 waves
    a0 = b2v0; a1 = b2v1; a2 = b2v2;
#pragma unroll
    for (int v = 0; v < NW; ++v) {
      const f4v q = ld_f4(smem + off + (v * TE + l16) * 16);
      a0 += q[0]; a1 += q[1]; a2 += q[2];
    }
  };
  // layer 2 (Q(x) or Q(x')) of this wave's units for one tile: H2 slice + its share of the output layer
  auto layer2 = [&](int hoff, s4v& h2, f4v& qp) {
    f4v z = ld_f4(smem + oB1 + (16 * w + 4 * g4) * 4);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
      z = mfma32(W1r[ks], lds_ld8(bf(hoff) + l16 * HS + 32 * ks + 8 * g4), z);
    h2 = relu_bf(z);
    const s4v w2a = lds_ld4(bf(oW2) + a_row * HP + 16 * w + 4 * g4);
    qp = mfma16(w2a, h2, zero4());
  };
  // two tiles' transposed fragments side by side: K = 32 envs (index 8 g4 + j = env 4 g4 + (j & 3) of a / b)
  auto trp = [&](int offa, int offb, int S, int c0) {
    const int o = (4 * g4 + (l16 >> 2)) * S + c0 + 4 * (l16 & 3);
    return cat8(lds_tr4(bf(offa) + o), lds_tr4(bf(offb) + o));
  };

  // ------------------------------------------------------------------ the pipeline
  // Stages run for every iteration index, valid tile or not (pipeline fill / drain): the rings are indexed by
  // the iteration, sized so that no write lands on data still in use, and zero-initialised, so an idle stage
  // computes on finite data; only what leaves the pipeline is gated (dQ = 0 outside the tiles, env write-back
  // and statistics of real tiles, weight gradients of real pairs).  Stores of lane groups that hold no result
  // go to a sink instead of being predicated: no divergent branch splits a phase's scheduling region.
  unsigned long long* const stamps =
      (PIPE_STAMPS && p.stamps != nullptr && blockIdx.x == 0 && (w == 0 || w == 4)) ? p.stamps + (w == 4 ? 8 : 0) : nullptr;
#define PIPE_STAMP(I) \
  if (PIPE_STAMPS && stamps != nullptr && lane == 0) stamps[(size_t)it * 16 + (I)] = __builtin_amdgcn_s_memtime();
  const float relu_floor = p.output_relu ? 0.f : -INFINITY;   // the output ReLU as a max
  const float clip = p.td_clip > 0.f ? p.td_clip : INFINITY;
  char* const sink = smem + oSTG + SINK_OFF;                  // write-only (16 B per lane l16)
  for (int it = 0; it < ntile + DRAIN; ++it) {
    const bool v1 = it >= 1 && it - 1 < ntile, v2 = it >= 2 && it - 2 < ntile;
    // ================================================================ P0
    PIPE_STAMP(0);
    s4v h2N, dzN;
    {
      // ------------------------------------------------ features of tile it (staged by P1 of it - 1)
      const float* stg = reinterpret_cast<const float*>(smem + oSTG + (it & 1) * STG_BYTES);
      auto stA = [&](int j) { return stg + (j >> 6) * 512 + (j & 63) * 4; };   // job j's dwords 0-3
      const float4 A = *reinterpret_cast<const float4*>(stA(tid));
      const float4 B = *reinterpret_cast<const float4*>(stA(tid) + 256);
      const float* s25 = stA(26 * jenv + 25) + 256;   // job 25 of the env: window 200..203
      const float last = s25[0], vnew = s25[1];
      const float cnext = jkq == 24 ? last : stA(tid + 1)[0];   // window 8 kq + 8 (job kq + 1's first)
      const float inv = FEAT ? __fdiv_rn(1.0f, last) : 0.f, invn = FEAT ? __fdiv_rn(1.0f, vnew) : 0.f;
      auto fx = [&](float v) { return FEAT ? __fmaf_rn(v, inv, -1.0f) : v; };
      auto fxn = [&](float v) { return FEAT ? __fmaf_rn(v, invn, -1.0f) : v; };
      const int* es = reinterpret_cast<const int*>(smem + oSTG + (it & 1) * STG_BYTES + ESTG_OFF);  // [row][env]
      const int eb = es[0 * TE + (jenv & 15)], esh = es[1 * TE + (jenv & 15)];
      // slot groups: kq < 24 window 8 kq .. 8 kq + 7; kq 24: budget, shares, 1, last | window 192..195;
      // kq 25: window 196..199 | pads.  X' (x'): the window shifted by one, lane group 0 of kq 24 zero.
      const float g[8] = {fx(A.x), fx(A.y), fx(A.z), fx(A.w), fx(B.x), fx(B.y), fx(B.z), fx(B.w)};
      const float gp[8] = {fxn(A.y), fxn(A.z), fxn(A.w), fxn(B.x), fxn(B.y), fxn(B.z), fxn(B.w), fxn(cnext)};
      const bool k24 = jkq == 24, kt = jkq >= 24;
      const float tl[4] = {feat_budget(__int_as_float(eb), p.inv_b0, FEAT), feat_shares(esh, last, p.inv_b0, FEAT),
                           1.0f, fx(last)};
      float x[8], xp[8];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        x[i] = k24 ? tl[i] : g[i];
        x[4 + i] = kt ? (k24 ? g[i] : 0.f) : g[4 + i];
        xp[i] = k24 ? 0.f : gp[i];
        xp[4 + i] = kt ? (k24 ? gp[i] : 0.f) : gp[4 + i];
      }
      *reinterpret_cast<s8v*>(jvalid ? reinterpret_cast<char*>(bf(oXB + (it % NXB) * X_BYTES) + jenv * XS + 8 * jkq)
                                     : sink + l16 * 16) = pk8(x);
      *reinterpret_cast<s8v*>(jvalid ? reinterpret_cast<char*>(bf(oXP) + jenv * XS + 8 * jkq) : sink + l16 * 16) =
          pk8(xp);
      {
        char* er = (jvalid && k24) ? smem + oEREC + (((it & 1) * TE) + jenv) * 32 : sink + l16 * 16;
        *reinterpret_cast<int4*>(er) = make_int4(jcur, eb, esh, es[2 * TE + (jenv & 15)]);
        *reinterpret_cast<int4*>(er + 16) = make_int4(es[3 * TE + (jenv & 15)], es[4 * TE + (jenv & 15)],
                                                      es[5 * TE + (jenv & 15)], __float_as_int(vnew));
      }
      // ------------------------------------------------ layer 2 + output share of Q(x), tile it - 1
      f4v qp, qpp;
      layer2(oH1 + ((it + NH1 - 1) % NH1) * H_BYTES, h2N, qp);
      // ------------------------------------------------ layer 2 + output share of Q(x'), tile it - 2
      s4v h2n;
      layer2(oH1P, h2n, qpp);
      // ------------------------------------------------ dZ1 = (dZ2 W1) * [H1 > 0] of this wave's units, tile it - 3
      {
        const bf16_t* dr = bf(oDZ + ((it + NDZ - 3) % NDZ) * H_BYTES) + l16 * HS + 8 * g4;
        const int wrow = 16 * w + l16;
        f4v c = zero4();
#pragma unroll
        for (int ks = 0; ks < 4; ++ks)
          c = mfma32(lds_ld8(dr + 32 * ks), lds_ld8(bf(oW1T) + w1t_off(wrow, 32 * ks + 8 * g4)), c);
        // c: lane (unit l16, g4)[j] = dZ1[16 w + l16][env 4 g4 + j]; the mask: H1 of the same (env, unit)
        const s4v hm = lds_tr4(bf(oH1 + ((it + 2 * NH1 - 3) % NH1) * H_BYTES) + (4 * g4 + (l16 >> 2)) * HS +
                               16 * w + 4 * (l16 & 3));
        dzN = mask_pk(c, hm);
      }
      // stores: lane group 0 holds the partial output sums; feature lanes their slot groups
      *reinterpret_cast<f4v*>(g4 == 0 ? smem + oQP + (w * TE + l16) * 16 : sink + l16 * 16) = qp;
      *reinterpret_cast<f4v*>(g4 == 0 ? smem + oQPP + (w * TE + l16) * 16 : sink + l16 * 16) = qpp;
    }
    PIPE_STAMP(2);
    __syncthreads();
    PIPE_STAMP(3);

    // ================================================================ P1
    // the role's VALU chain (env step or TD target) beside layer 1 of tile it: one scheduling region
    f4v zpN;
    s4v tail, dqf;
    float rew = 0.f, b2 = 0.f, q0 = 0.f, q1 = 0.f, q2 = 0.f, vnew_e = 0.f, rs_new = 0.f, fin = 0.f;
    int s2 = 0, act = 0, pos_new = 0, ep_new = 0;
    bool done = false, exploit = false;
    float diff = 0.f, qs = 0.f, fdone = 0.f;
    int dslot = 0;
    s4v dv = zero_s4();
    {
      if (producer) {
        // ------------------------------------------------ epsilon-greedy + env step, tile it - 1
        const int* er = reinterpret_cast<const int*>(smem + oEREC + ((((it + 1) & 1) * TE) + l16) * 32);
        const int4 r0 = *reinterpret_cast<const int4*>(er);
        const int4 r1 = *reinterpret_cast<const int4*>(er + 4);
        const int pos = r0.x, sh0 = r0.z, ep0 = r1.y, rw = r1.z;
        const float bud0 = __int_as_float(r0.y), vprev = __int_as_float(r0.w), rs0 = __int_as_float(r1.x);
        vnew_e = __int_as_float(r1.w);
        sum_partials(oQP, q0, q1, q2);
        q0 = fmaxf(q0, relu_floor); q1 = fmaxf(q1, relu_floor); q2 = fmaxf(q2, relu_floor);
        int greedy = 0;
        float best = q0;
        greedy = q1 > best ? 1 : greedy; best = fmaxf(best, q1);
        greedy = q2 > best ? 2 : greedy;
        const float u1 = (float)(rw & 0xFFFFFF) * (1.0f / 16777216.0f);
        const int rnd = (int)((unsigned)rw >> 30);
        exploit = u1 < fminf(p.eps, __fmul_rn((float)pos, p.inv_ramp));
        act = exploit ? greedy : rnd;
        const float bd = p.compat_env ? p.b0 : bud0;
        const int sd = p.compat_env ? p.s0 : sh0;
        const bool buy = (act == 0) && (bd >= vnew_e);
        const bool sell = (act == 1) && (sd > 0);
        b2 = buy ? __fsub_rn(bd, vnew_e) : (sell ? __fadd_rn(bd, vnew_e) : bd);
        s2 = buy ? sd + 1 : (sell ? sd - 1 : sd);
        const float cur = __fadd_rn(bud0, __fmul_rn((float)sh0, vprev));
        const float nw = __fadd_rn(b2, __fmul_rn((float)s2, vnew_e));
        rew = __fsub_rn(nw, cur);
        const float rrel = cur > 0.f ? __fdiv_rn(rew, cur) : 0.f;
        rew = p.reward_mode ? rrel : rew;
        if (p.reward_mode == 2) rew = __fsub_rn(rew, __fmul_rn(__fmul_rn(rew, 0.5f), rew));   // growth
        const float invn = FEAT ? __fdiv_rn(1.0f, vnew_e) : 0.f;
        const float fvn = FEAT ? __fmaf_rn(vnew_e, invn, -1.0f) : vnew_e;
        const s4v tl = pk4(feat_budget(b2, p.inv_b0, FEAT), feat_shares(s2, vnew_e, p.inv_b0, FEAT), 1.0f, fvn);
        tail = g4 == 0 ? tl : zero_s4();
        pos_new = pos + 1;
        done = pos_new >= p.T - HWIN;
        ep_new = done ? ep0 + 1 : ep0;
        fin = __fadd_rn(b2, __fmul_rn((float)s2, vnew_e));
        rs_new = rs0 + rew;
        dqf = zero_s4();
      } else {
        // ------------------------------------------------ TD target, tile it - 2
        float n0, n1, n2;
        sum_partials(oQPP, n0, n1, n2);
        n0 = fmaxf(n0, relu_floor); n1 = fmaxf(n1, relu_floor); n2 = fmaxf(n2, relu_floor);
        int am = 0;
        float mx = n0;
        am = n1 > mx ? 1 : am; mx = fmaxf(mx, n1);
        am = n2 > mx ? 2 : am; mx = fmaxf(mx, n2);
        const int* tr = reinterpret_cast<const int*>(smem + oENVR + ((((it + 2) & 1) * TE) + l16) * 32);
        const int4 r0 = *reinterpret_cast<const int4*>(tr);
        const int4 r1 = *reinterpret_cast<const int4*>(tr + 4);
        const float tq0 = __int_as_float(r0.x), tq1 = __int_as_float(r0.y), tq2 = __int_as_float(r0.z),
                    trew = __int_as_float(r0.w), tb2 = __int_as_float(r1.x), tvnew = __int_as_float(r1.y);
        const int ts2 = r1.z, tact = r1.w & 255;
        const bool tdone = (r1.w >> 8) != 0;
        dslot = p.target_compat ? am : tact;
        const float y = __fadd_rn(trew, __fmul_rn(p.gamma, mx));
        qs = dslot == 0 ? tq0 : (dslot == 1 ? tq1 : tq2);
        diff = __fsub_rn(qs, y);
        float dq = p.loss_coef * fminf(fmaxf(diff, -clip), clip);
        dq = (p.output_relu && !(qs > 0.f)) || !v2 ? 0.f : dq;
        dv = pk4(dslot == 0 ? dq : 0.f, dslot == 1 ? dq : 0.f, dslot == 2 ? dq : 0.f, 0.f);
        dqf = g4 == 0 ? dv : zero_s4();
        fdone = tdone ? __fadd_rn(tb2, __fmul_rn((float)ts2, tvnew)) : 0.f;
        done = tdone;
        tail = zero_s4();
      }
      // ------------------------------------------------ layer 1 of Q(x) and of Q(x')'s window, tile it
      const bf16_t* xr = bf(oXB + (it % NXB) * X_BYTES) + l16 * XS + 8 * g4;
      const bf16_t* xpr = bf(oXP) + l16 * XS + 8 * g4;
      f4v z = zero4(), zp = zero4();
#pragma unroll
      for (int ks = 0; ks < 6; ++ks) {
        z = mfma32(W0s[ks], lds_ld8(xr + 32 * ks), z);
        zp = mfma32(W0s[ks], lds_ld8(xpr + 32 * ks), zp);
      }
      z = mfma16(W0t, lds_ld4(xr + 192 - 4 * g4), z);     // (slot 192 + 4 g4: the row base already has 8 g4)
      zp = mfma16(W0t, lds_ld4(xpr + 192 - 4 * g4), zp);
      zpN = zp;
      *reinterpret_cast<s4v*>(bf(oH1 + (it % NH1) * H_BYTES) + l16 * HS + 16 * w + 4 * g4) = relu_bf(z);
      // hand the role's result to the SIMD partner (lane group 0; the others write the sink)
      if (producer) {
        *reinterpret_cast<s4v*>(g4 == 0 ? smem + oTAIL + (w * TE + l16) * 8 : sink + l16 * 16) = tail;
      } else {
        *reinterpret_cast<s4v*>(g4 == 0 ? smem + oDQ + ((w - NP) * TE + l16) * 8 : sink + l16 * 16) = dqf;
      }
    }
    if (lane == 0)
      __hip_atomic_store(ctl + (producer ? CTL_TAIL + w : CTL_DQ + w - NP), it + 1, __ATOMIC_RELEASE,
                         __HIP_MEMORY_SCOPE_WORKGROUP);
    PIPE_STAMP(4);
    // ------------------------------------------------ env record, write-back, statistics (lane group 0)
    if (producer) {
      if (w == 0) {   // TD record (read by the TD of P1 of it + 1)
        int* tr = reinterpret_cast<int*>(g4 == 0 ? smem + oENVR + ((((it + 1) & 1) * TE) + l16) * 32 : sink);
        *reinterpret_cast<int4*>(tr) = make_int4(__float_as_int(q0), __float_as_int(q1), __float_as_int(q2),
                                                 __float_as_int(rew));
        *reinterpret_cast<int4*>(tr + 4) = make_int4(__float_as_int(b2), __float_as_int(vnew_e), s2,
                                                     act | (done ? 256 : 0));
      }
      if (w == 0 && v1 && g4 == 0) {   // env-state write-back (TrainerChildActor.scala:136-146)
        const int e = tile_env0(it - 1) + l16;
        float* envf = reinterpret_cast<float*>(p.env);
        const size_t E = (size_t)p.E;
        envf[ER_BUDGET * E + e] = done ? p.b0 : b2;
        p.env[ER_SHARES * E + e] = done ? p.s0 : s2;
        envf[ER_VALUE * E + e] = done ? 0.f : vnew_e;
        p.env[ER_POS * E + e] = done ? 0 : pos_new;
        envf[ER_RET_SUM * E + e] = done ? 0.f : rs_new;
        p.env[ER_ACTION * E + e] = act;
        envf[ER_REWARD * E + e] = rew;
        if (done) {
          envf[ER_LAST_FINAL * E + e] = fin;
          p.env[ER_EPISODES * E + e] = ep_new;
        }
      }
      if (w == 0 && v1) {
        sA += g4 == 0 ? rew : 0.f;
        sB += (g4 == 0 && !exploit) ? 1.f : 0.f;
      }
    } else if (v2) {
      const bool lg = g4 == 0;
      if (w == 4) {
        sA += lg ? diff * diff : 0.f;
        sB += lg ? qs : 0.f;
        sC += (lg && done) ? 1.f : 0.f;
      } else if (w == 5) {
        sA += lg ? fdone : 0.f;
        sB += lg ? fdone * fdone : 0.f;
      } else if (w == 6) {   // db2: the bf16-rounded dQ, as the weight-gradient MFMAs see it
        sA += lg ? bf2f((bf16_t)dv[0]) : 0.f;
        sB += lg ? bf2f((bf16_t)dv[1]) : 0.f;
        sC += lg ? bf2f((bf16_t)dv[2]) : 0.f;
      }
    }
    // ------------------------------------------------ stage tile it + 2 into LDS (LDS-DMA; after this phase's global
    // stores, so that the counted wait at the end of the phase covers the DMA of the previous phase only)
    if (it + 2 < ntile) stage(it + 2, jn2);
    jcur = jn1;
    jn1 = jn2;
    if (jvalid && it + 3 < ntile) jn2 = load_pos(it + 3);
    // ------------------------------------------------ weight gradients of the pair (tb - 1, tb)
    {
      const int tb1 = it - 3, tb2 = it - 4;
      if ((tb1 & 1) && tb1 >= 1 && tb1 < ntile) {
        // first half (dZ1 of tb is this iteration's): dW1 = dZ2^T H1 of this wave's u2 rows, dW0 slot groups 0..2
        const int ta = tb1 - 1, tb = tb1;
        const s8v a0 = cat8(dza, dzN);
        const s8v a1 = trp(oDZ + (ta % NDZ) * H_BYTES, oDZ + (tb % NDZ) * H_BYTES, HS, 16 * w);
        const int ha = oH1 + (ta % NH1) * H_BYTES, hb = oH1 + (tb % NH1) * H_BYTES;
#pragma unroll
        for (int n = 0; n < 8; ++n) gW1[n] = mfma32(a1, trp(ha, hb, HS, 16 * n), gW1[n]);
        const int xa = oXB + (ta % NXB) * X_BYTES, xb = oXB + (tb % NXB) * X_BYTES;
#pragma unroll
        for (int n = 0; n < 3; ++n) gW0[n] = mfma32(a0, trp(xa, xb, XS, 16 * n), gW0[n]);
        dzb = dzN;
      } else if ((tb2 & 1) && tb2 >= 1 && tb2 < ntile) {
        // second half: dW0 slot groups 3..12
        const int ta = tb2 - 1, tb = tb2;
        const s8v a0 = cat8(dza, dzb);
        const int xa = oXB + (ta % NXB) * X_BYTES, xb = oXB + (tb % NXB) * X_BYTES;
#pragma unroll
        for (int n = 3; n < 13; ++n) gW0[n] = mfma32(a0, trp(xa, xb, XS, 16 * n), gW0[n]);
        dza = dzN;   // (this iteration's dZ1 is tile tb2 + 1: the next pair's first)
      } else {
        dza = dzN;   // pipeline edges: the first tile's dZ1
      }
    }
    PIPE_STAMP(5);
    // ------------------------------------------------ the partner's result; Q(x') layer-1 tail of it - 1; dZ2 of it - 2
    if (producer) {
      wait_flag(CTL_DQ + w, it + 1);
      dqf = g4 == 0 ? *reinterpret_cast<const s4v*>(smem + oDQ + (w * TE + l16) * 8) : zero_s4();
    } else {
      wait_flag(CTL_TAIL + w - NP, it + 1);
      tail = g4 == 0 ? *reinterpret_cast<const s4v*>(smem + oTAIL + ((w - NP) * TE + l16) * 8) : zero_s4();
    }
    {
      const f4v z = mfma16(W0t, tail, zpOld);
      *reinterpret_cast<s4v*>(bf(oH1P) + l16 * HS + 16 * w + 4 * g4) = relu_bf(z);
      const s4v w2t = lds_ld4(g4 == 0 ? bf(oW2T) + (16 * w + l16) * 4 : bf(oZERO));
      const f4v zt = mfma16(w2t, dqf, zero4());   // lane (env l16, g4)[j]: unit 16 w + 4 g4 + j (exact products)
      const s4v dz = mask_pk(zt, h2A);
      *reinterpret_cast<s4v*>(bf(oDZ + ((it + NDZ - 2) % NDZ) * H_BYTES) + l16 * HS + 16 * w + 4 * g4) = dz;
#pragma unroll
      for (int j = 0; j < 4; ++j) gB1[j] += bf2f((bf16_t)dz[j]);
      // dW2[a][u2] += dQ[a][env] H2[u2][env]: both operands transposed through this wave's scratch
      bf16_t* h2t = bf(oSCR + w * 512);
      bf16_t* dqt = bf(oSCR + NW * 512);   // shared: every wave holds the same dQ (columns 4..15 stay zero)
      *reinterpret_cast<s4v*>(h2t + l16 * 16 + 4 * g4) = h2A;
      *reinterpret_cast<s4v*>(g4 == 0 ? dqt + l16 * 16 : reinterpret_cast<bf16_t*>(sink + l16 * 16)) = dqf;
      const int o = (4 * g4 + (l16 >> 2)) * 16 + 4 * (l16 & 3);
      gW2 = mfma16(lds_tr4(dqt + o), lds_tr4(h2t + o), gW2);
    }
    // ------------------------------------------------ carries; the DMA of P1 of it - 1 landed; barrier
    zpOld = zpN;
    h2A = h2N;
    PIPE_STAMP(6);
    // every global access but this phase's DMA and position load done (counted: 2 DMAs, 1 load on job waves):
    // the DMA of P1 of it - 1, i.e. tile it + 1, is in LDS for P0 of it + 1
    if (it + 3 < ntile) {
      if (w < NJW) wait_vm(3); else wait_vm(2);
    } else if (it + 2 < ntile) {
      wait_vm(2);
    } else {
      wait_vm0();
    }
    PIPE_STAMP(7);
    __syncthreads();
  }

  // ------------------------------------------------------------------ gradient slab write-out
  auto put = [&](int idx, float v) {
    if (p.slab_bf16) {
      bf16_t* sbf = reinterpret_cast<bf16_t*>(p.slab);
      sbf[((size_t)(idx >> 5) * p.slab_rows + blockIdx.x) * 32 + (idx & 31)] = f2bf(v);
    } else {
      p.slab[(size_t)blockIdx.x * p.P + idx] = v;
    }
  };
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int u = 16 * w + 4 * g4 + j;
#pragma unroll
    for (int n = 0; n < 13; ++n) put(p.off_w0 + u * INP + slot_col(16 * n + l16), gW0[n][j]);
#pragma unroll
    for (int n = 0; n < 8; ++n) put(p.off_w1 + u * HP + 16 * n + l16, gW1[n][j]);
  }
  if (g4 == 0) {
#pragma unroll
    for (int j = 0; j < 3; ++j) put(p.off_w2 + j * HP + 16 * w + l16, gW2[j]);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float v = row16_sum(gB1[j]);   // over the 16 envs of a lane group
    if (l16 == 15) put(p.off_b1 + 16 * w + 4 * g4 + j, v);
  }
  // statistics: per-lane sums (lane group 0 only) -> one row per workgroup
  float* sSt = reinterpret_cast<float*>(smem + oST);
  {
    const float a = wave_sum(g4 == 0 ? sA : 0.f), b = wave_sum(g4 == 0 ? sB : 0.f), c = wave_sum(g4 == 0 ? sC : 0.f);
    if (lane == 0) {
      float* r = sSt + w * NSTAT;
#pragma unroll
      for (int s = 0; s < NSTAT; ++s) r[s] = 0.f;
      // NSTAT rows: reward, loss, explore, done, fsum, fsq, qslot
      if (w == 0) { r[0] = a; r[2] = b; }
      if (w == 4) { r[1] = a; r[6] = b; r[3] = c; }
      if (w == 5) { r[4] = a; r[5] = b; }
      if (w == 6) {   // db2
        put(p.off_b2 + 0, a);
        put(p.off_b2 + 1, b);
        put(p.off_b2 + 2, c);
      }
    }
  }
  __syncthreads();
  if (tid < NSTAT) {
    float t = 0.f;
#pragma unroll
    for (int v = 0; v < NW; ++v) t += sSt[v * NSTAT + tid];
    p.stats[(size_t)blockIdx.x * NSTAT + tid] = t;
  }
  if (blockIdx.x == 0 && tid == 0) p.ctrl[1] = step + 1;   // 1-based update count for the optimizer
}

template <int FEAT>
static hipError_t launch_f(const QStepParams& p, int grid, hipStream_t stream) {
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)qstep_pipe_kernel<FEAT>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    if (e != hipSuccess) return e;
    attr = true;
  }
  hipLaunchKernelGGL((qstep_pipe_kernel<FEAT>), dim3(grid), dim3(NT), LDS_BYTES, stream, p);
  return hipGetLastError();
}

}  // namespace PIPE_NS
}  // namespace st

extern "C" int PIPE_API(st_qstep_pipe_lds_bytes)(int inp, int h1p, int h2p) {
  if (inp == st::PIPE_NS::INP && h1p == st::PIPE_NS::HP && h2p == st::PIPE_NS::HP) return st::PIPE_NS::LDS_BYTES;
  return -1;
}

// Preconditions (checked here and by sharetrade/trainer/engine.py): E % 64 == 0, 1 <= grid <= E / 64,
// H == 201, padded dims (224, 128, 128), static schedule (chunk_heads null), bf16 slabs column-blocked by 32.
extern "C" hipError_t PIPE_API(st_qstep_pipe_launch)(const st::QStepParams* p, int inp, int h1p, int h2p, int grid,
                                                     hipStream_t stream) {
  using namespace st::PIPE_NS;
  if (inp != INP || h1p != HP || h2p != HP || p->H != HWIN) return hipErrorInvalidValue;
  if (p->E % C != 0 || grid < 1 || grid > p->E / C) return hipErrorInvalidValue;
  if (p->chunk_heads != nullptr) return hipErrorInvalidValue;
  if (p->T < HWIN + 2 || p->T4 < p->T + 4) return hipErrorInvalidValue;
  if ((p->off_w0 | p->off_w1 | p->off_w2) & 7) return hipErrorInvalidValue;
  if (p->slab_bf16 && (p->slab_rows != grid || p->P % 32 != 0)) return hipErrorInvalidValue;
  return p->feat_mode ? launch_f<1>(*p, grid, stream) : launch_f<0>(*p, grid, stream);
}
