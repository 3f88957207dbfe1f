// Wave-specialised fused online-DQN engine step on CDNA4 (gfx950): the step of qstep_wide.hip
// (gather -> Q(x) -> epsilon-greedy + Buy/Sell/Hold env step -> Q(x') -> TD target -> backward ->
// per-workgroup weight-gradient slabs; QDecisionPolicyActor.scala:54-77, TrainerChildActor.scala:82-146)
// re-organised so that no phase of the chain waits on a workgroup barrier.
//
// Why: qstep_wide.hip splits every layer over the hidden units of all 8 waves, so each of its ten
// phases per 64-env chunk ends in an s_barrier and MFMA, VALU and LDS time add up instead of
// overlapping (profiles/r2_pmc_flagship_set*.md: 24 % MFMA-busy, waves waiting 62 % of their cycles).
//
// Here a 512-thread workgroup has two kinds of waves, one of each on every SIMD:
//
//  * 4 DATA waves (waves 0-3) each run the forward / TD chain for their own 16-env tile with no other
//    wave involved: the tile's price windows go from HBM straight into MFMA B-operand registers, every
//    layer's accumulator tiles become the next layer's B operands in registers (a fixed permutation pi
//    of the hidden units inside each 32-wide k-step, absorbed by the column order of the weight images
//    in LDS: no activation round trip through LDS), the epsilon-greedy draw / env step / TD target run
//    in the 16 lanes that hold an env's Q values (the tail features of the state live in the same lanes),
//    and layer 1 of Q(x') (its price-window part) is issued together with layer 1 of Q(x) -- one read of
//    every W0 fragment feeds both.  A data wave fills a slot of an LDS ring as it goes: X and H1 after
//    layer 1, H2 after layer 2, dZ2 = (W2^T dQ) * [H2 > 0] and dQ at the end of its tile.
//  * 4 GRADIENT waves (waves 4-7) hold the per-workgroup weight-gradient accumulators (188 VGPRs each,
//    split by hidden unit) and consume ring slots in sequence order: the layer-1 data backward for their
//    own 32 hidden units (dZ1^T computed directly in the A-operand layout of the next MFMA: env = k),
//    then transposed fragment reads of the slot images and 16x16x16 MFMAs into dW0 / dW1 / dW2 / db.
//
// The ring (4 slots of 18.5 KB beside the 85.6 KB of bf16 weight images) is the only coupling: an LDS
// sequence counter, a "full" word per slot (release / acquire at workgroup scope) and a "freed" count
// per slot.  Data waves never wait for each other; a gradient wave waits only for the next slot.  The
// co-resident data and gradient waves of a SIMD overlap MFMA, VALU and LDS time.
//
// Specialised to the flagship geometry: window H = 201, padded dims 224-128-128-16 (input slots used:
// 208 = 6 k-steps of 32 + one of 16), 64-env chunks (one 16-env tile per data wave), static chunk
// schedule.  Numerics: bf16 operands, fp32 accumulation, the rounding points of qstep_wide.hip; fp32
// summation order differs (bias added first, k order pi inside MFMAs, per-16-env gradient sums).
#include "qstep.h"

#ifndef WS_STAMPS
#define WS_STAMPS 0     // s_memtime stamps per phase, bit 0 data wave 0, bit 1 gradient wave 0 (debug builds
#endif                  // csrc/ab/qstep_ws_*stamps*.hip only: the stamp code costs registers)
#ifndef WS_GSKIP
#define WS_GSKIP 0      // 1: timing build (csrc/ab/qstep_ws_gskip.hip), gradient waves skip their work
#endif
#if WS_MARKS   // tools/isa.py: assembly comments at the stamp points, to count instructions per phase
#define WS_MARK(W, I) asm volatile(";@" #W " " #I);
#else
#define WS_MARK(W, I)
#endif
#ifndef WS_PD1
#define WS_PD1 8        // data waves: layer-1 W0 fragment pairs read ahead of their MFMAs (10: 0.5 % slower, 12: 1 %)
#endif
#ifndef WS_NOPHIL
#define WS_NOPHIL 0     // timing build csrc/ab/qstep_ws_nophil.hip: no Philox draw (constant u1, u2; wrong results)
#endif
// Production schedule choices, each A/B'd in round 3 (profiles/r3_ws_ab.md; the losing builds were retired):
//  - the next tile's price windows are issued at Q(x')'s layer 2 (earlier issue loses 1.3-2 %, a whole tile
//    ahead spills);
//  - the env-state write-back is issued right after the env step (at TD: 0.5 % slower; deferred: 2.6 %);
//  - the env-state prefetch of the tile after next is issued at layer 1's start;
//  - the output layers' W2 fragments are read in layer 2's last read slots, dZ2's fragments before TD;
//  - window features are w / last - 1 as one fma per value (multiply + subtract: 1.2 % slower);
//  - Q(x)'s first WS_L2PRE layer-2 W1 fragments are read before the slot claim;
//  - gradient waves take ring slots in pairs (K = 32 weight-gradient MFMAs; single slots: 3.4 % slower), the
//    data waves form dZ2 (gradient waves forming it: 13 % slower), no issue priorities (gradient priority: +25 %).
constexpr int WS_GXP = 2;       // paired slots: X fragment pairs read this many dW0 steps ahead
#ifndef WS_L2PRE
#define WS_L2PRE 4
#endif
#ifndef WS_WAIT_UNROLL
#define WS_WAIT_UNROLL -1 // ring-wait poll loops: 0 not unrolled, > 0 unrolled by this count, -1 the compiler's
                          // choice (production: 6x, the round-3 form; not unrolled is 0.8-0.9 % slower,
                          // profiles/r4_ws_ab.md; csrc/ab/qstep_ws_wunroll0.hip)
#endif
#ifndef WS_SLEEP
#define WS_SLEEP 1        // s_sleep argument between ring-wait polls (0 / 2 / 4 A/B'd: profiles/r4_ws_ab.md)
#endif
#ifndef WS_ABORT_WORD
#define WS_ABORT_WORD 1   // ring waits check the workgroup's sticky abort word (0: csrc/ab/qstep_ws_noabort.hip)
#endif
#ifndef WS_NOWB
#define WS_NOWB 0       // timing build csrc/ab/qstep_ws_nowb.hip: no env-state write-back (wrong results)
#endif
#ifndef WS_NOPF
#define WS_NOPF 0       // timing build csrc/ab/qstep_ws_nopf.hip: no price prefetch in the loop (stale windows)
#endif
#ifndef WS_L1REP
#define WS_L1REP 1      // timing builds only (csrc/ab/qstep_ws_l1x2.hip / _l2x2.hip): a phase run twice, to price it in
#endif                  // context (wrong results)
#ifndef WS_L2REP
#define WS_L2REP 1
#endif
#ifndef WS_GST_MASK
#define WS_GST_MASK 0x7F   // which gradient-wave stamps a stamps build takes
#endif
#ifndef WS_NS
#define WS_NS ws
#define WS_API(name) name
#endif

namespace st {
namespace WS_NS {

constexpr int NW = 8, NT = 64 * NW;
constexpr int ND = 4, NG = 4;    // data waves (0..3), gradient waves (4..7)
constexpr int C = 64;            // envs per chunk (one 16-env tile per data wave)
constexpr int INP = 224, HP = 128;
constexpr int KX = 208;          // input slots used by layer 1
constexpr int HWIN = 201;        // window length this kernel is built for
constexpr int NSLOT = 4;
static_assert(NSLOT % ND == 0, "a data wave reuses its own slots (sequence q = ND k + d)");

// ---------------------------------------------------------------------------------- LDS layout (bytes)
constexpr int oW0 = 0;                          // W0p [128][208] bf16: columns in slot order
constexpr int oW1 = oW0 + HP * KX * 2;          // W1p [128][128] bf16: columns in pi order, 16-B units swizzled
constexpr int oW2 = oW1 + HP * HP * 2;          // W2p [5][128] bf16 (rows = actions, rows 3, 4 zero; pi order)
constexpr int oB1 = oW2 + 5 * HP * 2;           // b1 [128] f32
constexpr int oB2 = oB1 + HP * 4;               // b2 [16] f32
constexpr int oSLOT = oB2 + 64;
// one ring slot: X [16][208] (slots 204..207 of each row carry dQ[env][0..3]), H1 / H2 [16][128]
// (8-byte chunks swizzled), DZ2 [16][128] (pi order, 16-byte units swizzled like W1p)
constexpr int sX = 0, sH1 = sX + 16 * KX * 2, sH2 = sH1 + 16 * HP * 2, sDZ2 = sH2 + 16 * HP * 2,
              SLOT_BYTES = sDZ2 + 16 * HP * 2;
constexpr int oCTL = oSLOT + NSLOT * SLOT_BYTES;   // ints: [0] claim, [1..4] full, [5..8] freed, [10..11] zero,
                                                   // [12] abort (sticky)
constexpr int oST = oCTL + 64;                     // [ND][NSTAT] f32
constexpr int LDS_BYTES = oST + ND * NSTAT * 4;
static_assert(LDS_BYTES <= 163840, "LDS budget");
static_assert(SLOT_BYTES % 16 == 0 && oSLOT % 16 == 0, "alignment");

// ---------------------------------------------------------------------------------- index maps
// input slot -> flat-layout column of W0^T.  Slots 0..191 are window columns; the last 16-wide k-step
// is permuted so that the lanes holding an env's Q values (g4 == 0) also hold its tail features:
//   g4 = 0: 201 budget, 202 shares, 203 constant 1 (layer-0 bias column), 200 (the window's last price)
//   g4 = 1: 192..195;  g4 = 2: 196..199;  g4 = 3: pads 204..207
ST_DEV int slot_col(int s) {
  if (s < 192) return s;
  const int t = s - 192, g = t >> 2, j = t & 3;
  if (g == 0) return j < 3 ? 201 + j : 200;
  if (g == 1) return 192 + j;
  if (g == 2) return 196 + j;
  return 204 + j;
}
// pi: position s (0..127, k-step s/32, lane group (s/8)%4, element s%8) of a B operand built in
// registers from accumulator tiles 2*ks and 2*ks+1 -> hidden unit index
ST_DEV int pi_unit(int s) {
  const int ks = s >> 5, g = (s >> 3) & 3, j = s & 7;
  return 32 * ks + 16 * (j >> 2) + 4 * g + (j & 3);
}
// pi position of natural units 16 i + 4 q + (0..3) (4 consecutive positions)
ST_DEV int pi_pos4(int i, int q) { return 32 * (i >> 1) + 8 * q + 4 * (i & 1); }
// pi-ordered images (W1p, DZ2): 16-byte units of row R XOR-swizzled by 2 (R & 7) -- conflict-free 16-byte
// row reads, 2-way transposed reads (the minimum for one half-unit per lane; tools/lds_bank_sim.py)
ST_DEV int w1_off(int R, int s) { return R * HP + ((((s >> 3) ^ (2 * (R & 7)))) << 3) + (s & 7); }
// natural-order 128-wide slot images (H1, H2): 8-byte chunk c8 of row r at c8 ^ (4 (r & 7) | ((r >> 2) & 3)) --
// conflict-free for the data waves' 8-byte row writes / reads (16 rows of one chunk) and the gradient waves'
// transposed reads (8 rows x 4 chunks per 32 lanes) alike (tools/lds_bank_sim.py --ws)
ST_DEV int a_off(int r, int c) {
  return r * HP + ((((c >> 2) ^ ((4 * (r & 7)) | ((r >> 2) & 3)))) << 2) + (c & 3);
}

ST_DEV s4v zero_s4() { s4v z = {0, 0, 0, 0}; return z; }
ST_DEV s8v zero_s8() { s8v z = {0, 0, 0, 0, 0, 0, 0, 0}; return z; }
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
// relu then bf16 == bf16 then relu on the bits: a bf16 with the sign bit set is a negative int16, and
// rounding never changes a sign (-0 -> +0 is fine); one v_pk_max_i16 per two values instead of a
// NaN-canonicalising v_max_f32 pair per value
typedef short s2v __attribute__((ext_vector_type(2)));
ST_DEV s4v relu_bf(f4v v) {
  const s2v z = {0, 0};
  const s2v a = __builtin_elementwise_max(__builtin_bit_cast(s2v, pack_bf2(v[0], v[1])), z);
  const s2v b = __builtin_elementwise_max(__builtin_bit_cast(s2v, pack_bf2(v[2], v[3])), z);
  s4v r = {a[0], a[1], b[0], b[1]};
  return r;
}
// accumulator tile -> bf16 masked by (act > 0) (act: bf16 bits, a positive value has a positive short)
ST_DEV s4v mask_bf(f4v v, s4v act) {
  return pk4(act[0] > 0 ? v[0] : 0.f, act[1] > 0 ? v[1] : 0.f, act[2] > 0 ? v[2] : 0.f, act[3] > 0 ? v[3] : 0.f);
}
// same, on packed integer ops: bf16(v) bits * min(act, 1) (act >= 0 as a short: relu'd bf16 bits)
// (inline asm: written in C, the compiler turns min(act, 1) * x back into a compare + select per value)
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
ST_DEV s4v lo4(s8v v) { s4v r = {v[0], v[1], v[2], v[3]}; return r; }
ST_DEV s4v hi4(s8v v) { s4v r = {v[4], v[5], v[6], v[7]}; return r; }

// acc[i] += W1 (rows 16 i .. 16 i + 15, pi-ordered columns) . H (B operands of 4 k-steps), 32 MFMAs with
// the W1 fragment of pair j + PD2 read while pair j issues (j = 8 ks + i)
// (pre: the first PD2 fragments were read by layer2_pre, earlier in the chain -- their LDS latency off it)
#ifndef WS_PD2
#define WS_PD2 8        // data waves: layer-2 W1 fragments read ahead of their MFMAs (6 and 10: 0.6-0.8 % slower)
#endif
constexpr int PD2 = WS_PD2, NB2 = PD2 + 1;
template <int NPRE>
ST_DEV void layer2_pre(const bf16_t* W1p, int l16, int g4, s8v* A) {
#pragma unroll
  for (int j = 0; j < NPRE; ++j) A[j] = lds_ld8(W1p + w1_off(16 * (j & 7) + l16, 32 * (j >> 3) + 8 * g4));
}
template <int NPRE = 0>
ST_DEV void layer2(const bf16_t* W1p, int l16, int g4, const s8v* H, f4v* acc, const bf16_t* w2row, s8v* w2f,
                   const s8v* Apre = nullptr) {
  s8v A[NB2];
#pragma unroll
  for (int j = 0; j < NPRE; ++j) A[j] = Apre[j];
#pragma unroll
  for (int j = NPRE; j < PD2; ++j) A[j] = lds_ld8(W1p + w1_off(16 * (j & 7) + l16, 32 * (j >> 3) + 8 * g4));
  if (NPRE < PD2) __builtin_amdgcn_sched_group_barrier(0x100, PD2 - NPRE, 0);
#pragma unroll
  for (int j = 0; j < 32; ++j) {
    acc[j & 7] = mfma32(A[j % NB2], H[j >> 3], acc[j & 7]);
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    if (j + PD2 < 32) {
      const int jn = j + PD2;
      A[jn % NB2] = lds_ld8(W1p + w1_off(16 * (jn & 7) + l16, 32 * (jn >> 3) + 8 * g4));
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    } else if (j >= 32 - 4) {   // the output layer's W2 fragments, in the last read slots
      w2f[j - 28] = lds_ld8(w2row + 32 * (j - 28));
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
  }
  __builtin_amdgcn_sched_barrier(0);
}

// every ring wait is bounded (~1 s at s_sleep 1): a protocol bug ends the launch with an error bit in
// p.err instead of leaving waves spinning on the GPU.  The first wait that gives up also sets a sticky
// abort word in the workgroup's control block (ctl[12]); every wait checks it before sleeping, so the
// rest of the launch falls through its waits at once (results are garbage, p.err says so) instead of
// spinning a full SPIN_LIMIT per wait.  The host checks p.err at its synchronisation points
// (VectorEngine.check_kernel_err).
constexpr int SPIN_LIMIT = 1 << 24;
constexpr int CTL_ABORT = 12;
// dynamic chunk schedule (p.chunk_heads, overlapped DP): chunk ids of rounds k + 3 claimed by data wave 0
// and handed to the other waves through a 4-entry ring of tagged words (round tag << 21 | chunk + 1;
// chunk + 1 == 0: no more chunks), and the workgroup's round count + 1 once known (0 = not yet)
constexpr int CTL_NROUNDS = 13;
ST_DEV int cid_word(int r) { const int s = r & 3; return s == 0 ? 0 : (s == 1 ? 9 : (s == 2 ? 14 : 15)); }
constexpr int CID_SHIFT = 21, CID_MASK = (1 << CID_SHIFT) - 1;
ST_DEV int lds_acq(const int* w) {
  return __builtin_amdgcn_readfirstlane(__hip_atomic_load(w, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
}
ST_DEV void ws_fail(const QStepParams& p, int* ctl) {
  if ((threadIdx.x & 63) == 0) {
    __hip_atomic_store(ctl + CTL_ABORT, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (p.err != nullptr) atomicOr(p.err, 1u);
  }
}
// wait until pred(*w) holds: bounded, and abandoned at once once the workgroup has aborted
template <typename Pred>
ST_DEV void ring_wait(const QStepParams& p, int* ctl, const int* w, Pred pred) {
#if WS_WAIT_UNROLL > 0
#pragma clang loop unroll_count(WS_WAIT_UNROLL)
#elif WS_WAIT_UNROLL == 0
#pragma clang loop unroll(disable)
#endif
  for (int spin = 0; !pred(lds_acq(w)); ++spin) {
    if (WS_ABORT_WORD && lds_acq(ctl + CTL_ABORT)) break;
    if (WS_SLEEP > 0) __builtin_amdgcn_s_sleep(WS_SLEEP);
    if (spin > SPIN_LIMIT) { ws_fail(p, ctl); break; }   // never expected: report, do not hang the GPU
  }
}

// 16-byte loads from 4-byte-aligned addresses (the one padded bank copy is read at every shift): a memcpy
// from a float pointer promises the compiler only 4-byte alignment; it is still one dwordx4 load
ST_DEV float4 ldu4(const float* a) {
  float4 v;
  __builtin_memcpy(&v, a, sizeof(v));
  return v;
}

// env-state rows addressed as a uniform row base + a 32-bit byte offset, so the loads / stores use the
// SGPR-base form (no 64-bit VALU address add per access)
ST_DEV int* env_ptr(const QStepParams& p, int R, int e) {
  return reinterpret_cast<int*>(reinterpret_cast<char*>(p.env + (size_t)R * p.E) + (unsigned)e * 4u);
}
#undef ENV_I
#undef ENV_F
#define ENV_I(R, e) (*env_ptr(p, (R), (e)))
#define ENV_F(R, e) (*reinterpret_cast<float*>(env_ptr(p, (R), (e))))

// dynamic schedule, gradient waves: wait for slot sa to hold sequence q, or for the round count to say that
// round q / ND does not exist; true = the run has ended
ST_DEV bool wait_full_or_end(const QStepParams& p, int* ctl, int sa, int q) {
#pragma clang loop unroll(disable)
  for (int spin = 0;; ++spin) {
    if (lds_acq(ctl + 1 + sa) == q + 1) return false;
    const int n = lds_acq(ctl + CTL_NROUNDS);
    if (n != 0 && q / ND >= n - 1) return true;
    if (WS_ABORT_WORD && lds_acq(ctl + CTL_ABORT)) return true;
    __builtin_amdgcn_s_sleep(1);
    if (spin > SPIN_LIMIT) { ws_fail(p, ctl); return true; }
  }
}

// ---------------------------------------------------------------------------------- the kernel
// KN: the learning-quality knobs (target net, double DQN, reward scale, global exploit ramp) -- a separate
// instance, so the production build carries none of their code
// U16: the windows come from the 16-bit tick bank (p.ticks, csrc/series.hip tick16; FEAT only): half the bytes,
// 15 instead of 21 loads per lane and tile, 35 instead of 63 prefetch VGPRs, the same features bit for bit
template <int FEAT, bool DYN, bool KN, bool U16 = false>
__global__ void __launch_bounds__(NT, 1) qstep_ws_kernel(QStepParams p) {
  static_assert(!U16 || FEAT, "the tick bank serves the relative features (w / last - 1) only");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* W0p = reinterpret_cast<bf16_t*>(smem + oW0);
  bf16_t* W1p = reinterpret_cast<bf16_t*>(smem + oW1);
  bf16_t* W2p = reinterpret_cast<bf16_t*>(smem + oW2);
  float* sB1 = reinterpret_cast<float*>(smem + oB1);
  float* sB2 = reinterpret_cast<float*>(smem + oB2);
  int* ctl = reinterpret_cast<int*>(smem + oCTL);
  float* sSt = reinterpret_cast<float*>(smem + oST);

  const int tid = threadIdx.x, lane = tid & 63, l16 = lane & 15, g4 = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const unsigned long long step = p.ctrl[0];
  const int nchunks = p.E / C;
  const int nmy = (nchunks - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;   // chunks of this WG
  // ---------------------------------------------------------------- chunk schedule
  // static: round k of this workgroup is chunk blockIdx.x + k * grid (nmy rounds).  Dynamic (DYN,
  // p.chunk_heads; grid % 8 == 0): rounds 0..2 are those same chunks, later rounds are claimed from
  // per-XCD-group heads -- the chunks x + 8 j (x = blockIdx.x % 8) with j >= 3 grid / 8 are handed out by
  // head x in claim order -- so workgroups that start late (their CU held by a concurrent RCCL kernel in
  // overlapped DP) take fewer chunks instead of stretching the launch's tail.  Every chunk is handed
  // out exactly once whatever the physical XCD placement; the heads are re-zeroed by the slab pass.
  const int xg = (int)blockIdx.x & 7, gx = (int)gridDim.x >> 3;
  auto static_chunk = [&](int k) {
    const int c = (int)blockIdx.x + k * (int)gridDim.x;
    return c < nchunks ? c : -1;
  };

  // ------------------------------------------------------------------ prologue: weight images, ring state
#if defined(WS_PROLOGUE_REPS) && WS_PROLOGUE_REPS > 1   // timing build csrc/ab/qstep_ws_pro2.hip: images built twice
  for (int rep_ = 0; rep_ < WS_PROLOGUE_REPS; ++rep_) {
    __syncthreads();
#else
  {
#endif
   if (p.wimg != nullptr) {
    // the images as one 87,872-byte run (oW0 .. oSLOT, built by the optimizer pass): 16 bytes per lane and
    // LDS-DMA instruction, 11 per wave, all in flight at once (the gather below takes ~10 us per launch:
    // profiles/r5_ws_prologue.md)
    constexpr int NCH = (oSLOT - oW0) / 16;
    for (int j = wave; j * 64 < NCH; j += NT / 64) {
      const int c = j * 64 + lane;
      if (c < NCH)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(p.wimg + 16 * c),
                                         (__attribute__((address_space(3))) void*)(smem + oW0 + 1024 * j), 16, 0, 0);
    }
    __builtin_amdgcn_s_waitcnt(0xF70);   // vmcnt(0): this wave's copies landed (the barrier below joins the waves)
   } else {
    const bf16_t* w0 = p.wq + p.off_w0;
    for (int i = tid; i < HP * KX; i += NT) {          // W0p[r][s] = W0^T[r][slot_col(s)]
      const int r = i / KX, s = i % KX;
      W0p[i] = w0[r * INP + slot_col(s)];
    }
    const bf16_t* w1 = p.wq + p.off_w1;
    for (int i = tid; i < HP * HP; i += NT) {          // W1p[R][s] = W1^T[R][pi(s)] (swizzled)
      const int R = i >> 7, s = i & 127;
      W1p[w1_off(R, s)] = w1[R * HP + pi_unit(s)];
    }
    const bf16_t* w2 = p.wq + p.off_w2;
    for (int i = tid; i < 5 * HP; i += NT) {           // W2p[a][s] = W2^T[a][pi(s)] (rows 3, 4: padding rows)
      const int a = i >> 7, s = i & 127;
      W2p[i] = w2[a * HP + pi_unit(s)];
    }
    for (int i = tid; i < HP; i += NT) sB1[i] = p.wf[p.off_b1 + i];
    if (tid < 16) sB2[tid] = tid < 4 ? p.wf[p.off_b2 + tid] : 0.f;
   }
    if (tid < 16) ctl[tid] = 0;
    if (DYN && tid == 0) {
      int r = 0;
      while (r < 3 && static_chunk(r) >= 0) ++r;
      if (r < 3) ctl[CTL_NROUNDS] = r + 1;   // the static rounds already end the run
    }
  }
  __syncthreads();

  if (wave < ND) {
    // ================================================================ DATA WAVE
    const int d = wave;
    float st_reward = 0.f, st_loss = 0.f, st_explore = 0.f, st_done = 0.f, st_fsum = 0.f, st_fsq = 0.f,
          st_qslot = 0.f;
    const float b2v[3] = {sB2[0], sB2[1], sB2[2]};

    // chunk ids of rounds k, k + 1, k + 2 (uniform); dynamic: -1 = no such round
    int ck0 = DYN ? static_chunk(0) : (int)blockIdx.x, ck1 = DYN ? static_chunk(1) : 0, ck2 = DYN ? static_chunk(2) : 0;
    // dynamic: the chunk id of round r >= 3 from the ring (data wave 0 writes it one tile ahead of use)
    auto ring_chunk = [&](int r) {
      int v = 0;
      ring_wait(p, ctl, ctl + cid_word(r), [&](int w) { v = w; return (w >> CID_SHIFT) == (r & 0x3FF); });
      return (v & CID_MASK) - 1;
    };
    // data wave 0: the claim for round k + 3 in flight (returned value consumed at the end of tile k)
    unsigned claim_v = 0u;
    bool claim_out = false, ended = DYN && ck2 < 0;   // (static rounds already short: no claims at all)
    unsigned* const head = DYN ? p.chunk_heads + 32 * xg : nullptr;
    // env state of the tile of round k (all lanes load their env l16's words); dynamic: the chunk id of that
    // round, a missing round clamped to a real chunk (its loads are never used)
    auto env_of = [&](int k, int rel) {
      if (DYN) {
        const int c = rel == 0 ? ck0 : (rel == 1 ? ck1 : ck2);
        return max(c, 0) * C + 16 * d + l16;
      }
      return (min((int)blockIdx.x + k * (int)gridDim.x, nchunks - 1)) * C + 16 * d + l16;
    };
    int e_pos, e_sh, e_ep, n_pos, n_sh, n_ep;
    float e_b, e_val, e_rs, n_b, n_val, n_rs;
    float e_sc = 1.f, n_sc = 1.f;   // U16: the env's tick size (price = tick * sc)
#define WS_LOAD_ENV(K, REL, POS, B, SH, VAL, RS, EP, SC)                                          \
  {                                                                                              \
    const int e_ = env_of(K, REL);                                                               \
    POS = ENV_I(ER_POS, e_); B = ENV_F(ER_BUDGET, e_); SH = ENV_I(ER_SHARES, e_);                \
    VAL = ENV_F(ER_VALUE, e_); RS = ENV_F(ER_RET_SUM, e_); EP = ENV_I(ER_EPISODES, e_);          \
    if (U16) SC = p.tscale[e_];                                                                  \
  }
    // raw prices of a tile: per 32-wide k-step 9 floats (x uses 8, x' the 8 shifted by one); for the last
    // 16-wide k-step 5 (lanes g4 = 1, 2); the window's last and next price p[pos + 200], p[pos + 201]
    float4 pa[6], pb[6];
    float pc[6];
    float4 pd = make_float4(0.f, 0.f, 0.f, 0.f);
    float pe = 0.f;
    float4 pl;
    // U16 (ticks as u16 pairs): per 32-wide k-step a dwordx4 + a dword from the 4-byte boundary at or below the
    // lane's first tick (10 ticks cover its 9); the last k-step's window columns (lanes g4 = 1, 2) 3 dwords; the
    // window's last and next tick 2 dwords.  An odd position is undone at the features (v_alignbyte).
    uint4 ta[6];
    unsigned tb[6];
    uint2 td = make_uint2(0u, 0u);
    unsigned te = 0u;
    uint2 tl;
#define WS_LOAD_PRICES(K, REL, POS)                                                               \
  if (U16) {                                                                                     \
    const int e_ = env_of(K, REL);                                                               \
    const int pc_ = min(max((POS), 0), p.T - HWIN - 1);                                          \
    const unsigned* b_ = reinterpret_cast<const unsigned*>(p.ticks + (size_t)e_ * p.T16) + (pc_ >> 1); \
    __builtin_memcpy(&tl, b_ + 100, sizeof(tl));                                                 \
    _Pragma("unroll") for (int ks = 0; ks < 6; ++ks) {                                           \
      __builtin_memcpy(&ta[ks], b_ + 16 * ks + 4 * g4, sizeof(uint4));                           \
      tb[ks] = b_[16 * ks + 4 * g4 + 4];                                                         \
    }                                                                                            \
    if (g4 == 1 || g4 == 2) {                                                                    \
      __builtin_memcpy(&td, b_ + 94 + 2 * g4, sizeof(td));                                       \
      te = b_[96 + 2 * g4];                                                                      \
    }                                                                                            \
  } else {                                                                                       \
    const int e_ = env_of(K, REL);                                                               \
    const int pc_ = min(max((POS), 0), p.T - HWIN - 1);   /* address clamp: never read past the bank */ \
    const float* b_ = p.prices4 + (size_t)e_ * p.T4 + (size_t)pc_;  /* 4-B aligned dwordx4 reads */   \
    pl = ldu4(b_ + 200);  /* first: the back edge copies it (see below) */                         \
    _Pragma("unroll") for (int ks = 0; ks < 6; ++ks) {                                           \
      const float* q_ = b_ + 32 * ks + 8 * g4;                                                   \
      pa[ks] = ldu4(q_);                                                                         \
      pb[ks] = ldu4(q_ + 4);                                                                     \
      pc[ks] = q_[8];                                                                            \
    }                                                                                            \
    if (g4 == 1 || g4 == 2) {                                                                    \
      const float* r_ = b_ + 188 + 4 * g4;                                                       \
      pd = ldu4(r_);                                                                             \
      pe = r_[4];                                                                                \
    }                                                                                            \
  }
    WS_LOAD_ENV(0, 0, e_pos, e_b, e_sh, e_val, e_rs, e_ep, e_sc)
    WS_LOAD_PRICES(0, 0, e_pos)
    WS_LOAD_ENV(1, 1, n_pos, n_b, n_sh, n_val, n_rs, n_ep, n_sc)

    unsigned long long* stamps = ((WS_STAMPS & 1) && p.stamps != nullptr && blockIdx.x == 0 && d == 0 && lane == 0)
                                     ? p.stamps : nullptr;
#define WS_STAMP(I) if ((WS_STAMPS & 1) && stamps) stamps[k * 16 + (I)] = __builtin_amdgcn_s_memtime(); WS_MARK(D, I)
#define WS_PIN(V) asm volatile("" ::"v"(V))
#define WS_SB() __builtin_amdgcn_sched_barrier(0)

    // the env-state write-back of tile k is issued in tile k + 1, after its features have waited for their
    // price windows: a store issued after the windows' loads would make that wait (in-order vmcnt) last
    // until the store is acknowledged
    int w_e = -1, w_s = 0, w_pos = 0, w_ep = 0, w_act = 0;
    float w_b = 0.f, w_v = 0.f, w_rs = 0.f, w_fin = 0.f, w_rew = 0.f;
    bool w_done = false;
#define WS_WRITE_BACK()                                                                           \
  if (!WS_NOWB && g4 == 0 && w_e >= 0) {                                                         \
    ENV_F(ER_BUDGET, w_e) = w_b; ENV_I(ER_SHARES, w_e) = w_s; ENV_F(ER_VALUE, w_e) = w_v;        \
    ENV_I(ER_POS, w_e) = w_pos; ENV_F(ER_RET_SUM, w_e) = w_rs;                                   \
    ENV_I(ER_ACTION, w_e) = w_act; ENV_F(ER_REWARD, w_e) = w_rew;                                \
    if (w_done) { ENV_F(ER_LAST_FINAL, w_e) = w_fin; ENV_I(ER_EPISODES, w_e) = w_ep; }           \
  }
    // the env's next state from this tile's env step (pos, bud0 ... of the tile; act, rew, b2, s2 of its step),
    // then the write-back unless it is deferred to the next tile
#define WS_WB_SET()                                                                               \
  {                                                                                              \
    const int np_ = pos + 1;                                                                     \
    w_e = e; w_act = act; w_rew = rew;                                                           \
    w_done = np_ >= p.T - HWIN;                                                                  \
    w_ep = w_done ? ep0 + 1 : ep0;                                                               \
    if (w_done) {                                                                                \
      w_fin = __fadd_rn(b2, __fmul_rn((float)s2, vnew));                                         \
      w_b = p.b0; w_s = p.s0; w_v = 0.f; w_pos = 0; w_rs = 0.f;                                  \
    } else {                                                                                     \
      w_b = b2; w_s = s2; w_v = vnew; w_pos = np_; w_rs = rs0 + rew;                             \
    }                                                                                            \
    WS_WRITE_BACK() w_e = -1;                                                                    \
  }

    for (int k = 0; DYN ? ck0 >= 0 : k < nmy; ++k) {
      WS_STAMP(0);
      const int chunk = DYN ? ck0 : (int)blockIdx.x + k * (int)gridDim.x;
      if (DYN && k >= 1) ck2 = __builtin_amdgcn_readfirstlane(ring_chunk(k + 2));   // for the env prefetch below
      const int e = chunk * C + 16 * d + l16;
      // ---------------------------------------------------------------- features -> X / X' B operands
      // lastw / vnew_w: the window's last and next value in the window's own units (fp32 prices, or U16 ticks:
      // w / last - 1 is the same number either way); last / vnew: prices (U16: tick * the env's tick size, exact)
      float lastw, vnew_w, last, vnew;
      unsigned shb = 0u;   // U16: 2 when the tile's window starts at an odd tick (bytes to drop)
      if (U16) {
        shb = (unsigned)(min(max(e_pos, 0), p.T - HWIN - 1) & 1) * 2u;
        const unsigned t01 = __builtin_amdgcn_alignbyte(tl.y, tl.x, shb);
        lastw = (float)(t01 & 0xFFFFu);
        vnew_w = (float)(t01 >> 16);
        last = __fmul_rn(lastw, e_sc);
        vnew = __fmul_rn(vnew_w, e_sc);
      } else {
        lastw = last = pl.x;
        vnew_w = vnew = pl.y;
      }
      float inv = 0.f, invn = 0.f;
      if (FEAT) {
        inv = __fdiv_rn(1.0f, lastw);
        invn = __fdiv_rn(1.0f, vnew_w);
      }
      auto fx = [&](float w) {
        return FEAT ? __fmaf_rn(w, inv, -1.0f) : w;
      };
      auto fxn = [&](float w) {
        return FEAT ? __fmaf_rn(w, invn, -1.0f) : w;
      };
      auto lo16f = [](unsigned v) { return (float)(v & 0xFFFFu); };
      auto hi16f = [](unsigned v) { return (float)(v >> 16); };
      s8v X[6], Xn[6];
#pragma unroll
      for (int ks = 0; ks < 6; ++ks) {
        if (U16) {
          const unsigned w0 = __builtin_amdgcn_alignbyte(ta[ks].y, ta[ks].x, shb),
                         w1 = __builtin_amdgcn_alignbyte(ta[ks].z, ta[ks].y, shb),
                         w2 = __builtin_amdgcn_alignbyte(ta[ks].w, ta[ks].z, shb),
                         w3 = __builtin_amdgcn_alignbyte(tb[ks], ta[ks].w, shb),
                         w4 = __builtin_amdgcn_alignbyte(0u, tb[ks], shb);
          const float f0 = lo16f(w0), f1 = hi16f(w0), f2 = lo16f(w1), f3 = hi16f(w1), f4 = lo16f(w2),
                      f5 = hi16f(w2), f6 = lo16f(w3), f7 = hi16f(w3), f8 = lo16f(w4);
          X[ks] = cat8(pk4(fx(f0), fx(f1), fx(f2), fx(f3)), pk4(fx(f4), fx(f5), fx(f6), fx(f7)));
          Xn[ks] = cat8(pk4(fxn(f1), fxn(f2), fxn(f3), fxn(f4)), pk4(fxn(f5), fxn(f6), fxn(f7), fxn(f8)));
        } else {
          X[ks] = cat8(pk4(fx(pa[ks].x), fx(pa[ks].y), fx(pa[ks].z), fx(pa[ks].w)),
                       pk4(fx(pb[ks].x), fx(pb[ks].y), fx(pb[ks].z), fx(pb[ks].w)));
          Xn[ks] = cat8(pk4(fxn(pa[ks].y), fxn(pa[ks].z), fxn(pa[ks].w), fxn(pb[ks].x)),
                        pk4(fxn(pb[ks].y), fxn(pb[ks].z), fxn(pb[ks].w), fxn(pc[ks])));
        }
      }
      // last k-step (16 wide, slot order): g4 = 0 (budget, shares, 1, col 200); 1, 2 window columns; 3 pads
      s4v X6, Xn6;
      if (g4 == 0) {
        X6 = pk4(feat_budget(e_b, p.inv_b0, FEAT), feat_shares(e_sh, last, p.inv_b0, FEAT), 1.0f, fx(lastw));
        Xn6 = zero_s4();   // completed after the env step
      } else if (g4 < 3) {
        if (U16) {
          const unsigned v0 = __builtin_amdgcn_alignbyte(td.y, td.x, shb), v1 = __builtin_amdgcn_alignbyte(te, td.y, shb),
                         v2 = __builtin_amdgcn_alignbyte(0u, te, shb);
          const float f0 = lo16f(v0), f1 = hi16f(v0), f2 = lo16f(v1), f3 = hi16f(v1), f4 = lo16f(v2);
          X6 = pk4(fx(f0), fx(f1), fx(f2), fx(f3));
          Xn6 = pk4(fxn(f1), fxn(f2), fxn(f3), fxn(f4));
        } else {
          X6 = pk4(fx(pd.x), fx(pd.y), fx(pd.z), fx(pd.w));
          Xn6 = pk4(fxn(pd.y), fxn(pd.z), fxn(pd.w), fxn(pe));
        }
      } else {
        X6 = zero_s4();
        Xn6 = zero_s4();
      }
      const int pos = e_pos, sh0 = e_sh, ep0 = e_ep;
      const float bud0 = e_b, vprev = e_val, rs0 = e_rs;
      // rotate the prefetched env state; load the one after next
      e_pos = n_pos; e_b = n_b; e_sh = n_sh; e_val = n_val; e_rs = n_rs; e_ep = n_ep; e_sc = n_sc;
      WS_PIN(X[5]); WS_PIN(Xn[5]); WS_PIN(X6);
      WS_SB();
      WS_STAMP(1);
      // (after the features: a store or load issued before them would hold their window wait)
      WS_WRITE_BACK()
      WS_LOAD_ENV(k + 2, 2, n_pos, n_b, n_sh, n_val, n_rs, n_ep, n_sc)
      if (DYN && d == 0 && !ended) {   // the chunk of round k + 3 (used from tile k + 1 on); flags wave-uniform
        if (lane == 0) claim_v = atomicAdd(head, 1u);
        claim_out = true;
      }
      // the epsilon-greedy draw (Philox, ~70 VALU with quarter-rate multiplies) depends only on (env, step):
      // issued here, the scheduler interleaves it with layer 1's MFMAs (VALU slots in the group pattern)
      float u1, u2;
      {
        uint32_t c0 = (uint32_t)(p.env_offset + e), c1 = (uint32_t)(step & 0xFFFFFFFFull),
                 c2 = (uint32_t)(step >> 32), c3 = 0u;
        if (!WS_NOPHIL) philox4x32(c0, c1, c2, c3, p.key0, p.key1);
        u1 = u24(c0);
        u2 = u24(c1);
      }
      // ---------------------------------------------------------------- layer 1 of Q(x) and of Q(x')'s window
      f4v a1[8], a1n[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) { a1[i] = zero4(); a1n[i] = zero4(); }
      {
        // software pipeline: the W0 fragment of pair j + PD1 is read while pair j's two MFMAs issue
        // (j = 8 ks + i; one fragment feeds Q(x) and Q(x')'s window)
        constexpr int PD1 = WS_PD1, NB1 = PD1 + 1;
        const bf16_t* w0b = W0p + l16 * KX + 8 * g4;
        for (int rep = 0; rep < WS_L1REP; ++rep) {
        s8v A[NB1];
#pragma unroll
        for (int j = 0; j < PD1; ++j) A[j] = lds_ld8(w0b + (j & 7) * 16 * KX + 32 * (j >> 3));
        __builtin_amdgcn_sched_group_barrier(0x100, PD1, 0);
#pragma unroll
        for (int j = 0; j < 48; ++j) {
          const int ks = j >> 3, i = j & 7;
          a1[i] = mfma32(A[j % NB1], X[ks], a1[i]);
          a1n[i] = mfma32(A[j % NB1], Xn[ks], a1n[i]);
          __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
          if (j + PD1 < 48) {
            const int jn = j + PD1;
            A[jn % NB1] = lds_ld8(w0b + (jn & 7) * 16 * KX + 32 * (jn >> 3));
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          }
          __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);   // VALU (the Philox draw) between MFMAs
        }
        }
        WS_PIN(u1); WS_PIN(u2);   // (else the draw sinks into the env-step branch)
        WS_SB();
      }
      WS_STAMP(12);   // (sub-phase: layer 1's k-steps 0..5 done)
      s4v w06[8];   // the last k-step's A fragments: used again after the env step (x')
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        w06[i] = lds_ld4(W0p + (16 * i + l16) * KX + 192 + 4 * g4);
        a1[i] = mfma16(w06[i], X6, a1[i]);
      }
      s8v H1[4];
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) H1[ks] = cat8(relu_bf(a1[2 * ks]), relu_bf(a1[2 * ks + 1]));
      f4v a2[8];   // layer 2's accumulators start at the bias (read early: its latency is off the MFMA chain)
#pragma unroll
      for (int i = 0; i < 8; ++i) a2[i] = *reinterpret_cast<const f4v*>(sB1 + 16 * i + 4 * g4);
      WS_PIN(H1[3]); WS_PIN(a1n[7]);
      WS_SB();
      WS_STAMP(2);
      // ---------------------------------------------------------------- claim a ring slot; X and H1 go in now
      // sequence number fixed by (tile, wave): the gradient waves consume the tiles of a workgroup in one
      // order on every run, so the fp32 gradient sums (and every replay of a captured step) are bit-exact
      s8v A2pre[WS_L2PRE];
      layer2_pre<WS_L2PRE>(W1p, l16, g4, A2pre);
      const int q = ND * k + d;
      const int sl = q % NSLOT, round = q / NSLOT;
      ring_wait(p, ctl, ctl + 5 + sl, [&](int v) { return v >= NG * round; });
      WS_STAMP(3);
      char* sb = smem + oSLOT + sl * SLOT_BYTES;
      bf16_t* sx = reinterpret_cast<bf16_t*>(sb + sX);
      bf16_t* sh1 = reinterpret_cast<bf16_t*>(sb + sH1);
      bf16_t* sh2 = reinterpret_cast<bf16_t*>(sb + sH2);
      bf16_t* sz2 = reinterpret_cast<bf16_t*>(sb + sDZ2);
#pragma unroll
      for (int ks = 0; ks < 6; ++ks) *reinterpret_cast<s8v*>(sx + l16 * KX + 32 * ks + 8 * g4) = X[ks];
      if (g4 < 3) *reinterpret_cast<s4v*>(sx + l16 * KX + 192 + 4 * g4) = X6;   // (g4 = 3: dQ, at the end)
#pragma unroll
      for (int i = 0; i < 8; ++i)
        *reinterpret_cast<s4v*>(sh1 + a_off(l16, 16 * i + 4 * g4)) = (i & 1) ? hi4(H1[i >> 1]) : lo4(H1[i >> 1]);
      WS_SB();
      WS_STAMP(4);
      // ---------------------------------------------------------------- layer 2 + output of Q(x)
      const bf16_t* w2row = W2p + min(l16, 4) * HP + 8 * g4;   // rows >= 3 zero: no masked load
      s8v w2f[4];
      layer2<WS_L2PRE>(W1p, l16, g4, H1, a2, w2row, w2f, A2pre);
      s8v H2[4];
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) H2[ks] = cat8(relu_bf(a2[2 * ks]), relu_bf(a2[2 * ks + 1]));
#pragma unroll
      for (int i = 0; i < 8; ++i)
        *reinterpret_cast<s4v*>(sh2 + a_off(l16, 16 * i + 4 * g4)) = (i & 1) ? hi4(H2[i >> 1]) : lo4(H2[i >> 1]);
      WS_PIN(H2[3]);
      WS_SB();
      WS_STAMP(5);
      f4v qa = zero4();
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const s8v a = w2f[ks];
        qa = mfma32(a, H2[ks], qa);
      }
      WS_PIN(qa);
      WS_SB();
      WS_STAMP(6);
      // ---------------------------------------------------------------- epsilon-greedy + env step (lanes g4 == 0)
      float b2 = 0.f, rew = 0.f, q0 = 0.f, q1 = 0.f, q2 = 0.f;
      int s2 = 0, act = 0;
      if (g4 == 0) {
        q0 = qa[0] + b2v[0];
        q1 = qa[1] + b2v[1];
        q2 = qa[2] + b2v[2];
        if (p.output_relu) { q0 = fmaxf(q0, 0.f); q1 = fmaxf(q1, 0.f); q2 = fmaxf(q2, 0.f); }
        int greedy = 0;
        float best = q0;
        if (q1 > best) { best = q1; greedy = 1; }
        if (q2 > best) { best = q2; greedy = 2; }
        const bool exploit = u1 < fminf(p.eps, __fmul_rn((KN && p.ramp_global) ? (float)step : (float)pos, p.inv_ramp));
        int rnd = (int)(u2 * 3.0f);
        rnd = rnd > 2 ? 2 : rnd;
        act = exploit ? greedy : rnd;
        const float bd = p.compat_env ? p.b0 : bud0;
        const int sd = p.compat_env ? p.s0 : sh0;
        const bool buy = (act == 0) && (bd >= vnew);
        const bool sell = (act == 1) && (sd > 0);
        b2 = buy ? __fsub_rn(bd, vnew) : (sell ? __fadd_rn(bd, vnew) : bd);
        s2 = buy ? sd + 1 : (sell ? sd - 1 : sd);
        const float cur = __fadd_rn(bud0, __fmul_rn((float)sh0, vprev));
        const float nw = __fadd_rn(b2, __fmul_rn((float)s2, vnew));
        rew = __fsub_rn(nw, cur);
        if (p.reward_mode) rew = cur > 0.f ? __fdiv_rn(rew, cur) : 0.f;
        if (p.reward_mode == 2) rew = __fsub_rn(rew, __fmul_rn(__fmul_rn(rew, 0.5f), rew));   // growth: log1p to 2nd order
        Xn6 = pk4(feat_budget(b2, p.inv_b0, FEAT), feat_shares(s2, vnew, p.inv_b0, FEAT), 1.0f, fxn(vnew_w));
        st_explore += exploit ? 0.f : 1.f;
      }
      WS_WB_SET()
      WS_PIN(Xn6);
      WS_SB();
      WS_STAMP(7);
      // ---------------------------------------------------------------- Q(x'): finish layer 1, layer 2, output
#pragma unroll
      for (int i = 0; i < 8; ++i) a1n[i] = mfma16(w06[i], Xn6, a1n[i]);
      s8v H1n[4];
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) H1n[ks] = cat8(relu_bf(a1n[2 * ks]), relu_bf(a1n[2 * ks + 1]));
      // the next tile's price windows issued here
      // (issued earlier -- right after the features or after layer 1 -- the u16 windows (35 VGPRs) still spill
      // the data wave: 76-192 B of scratch, round 6)
      WS_LOAD_PRICES(k + 1, 1, e_pos)
#pragma unroll
      for (int i = 0; i < 8; ++i) a2[i] = *reinterpret_cast<const f4v*>(sB1 + 16 * i + 4 * g4);
      WS_SB();
      for (int rep = 0; rep < WS_L2REP; ++rep) layer2(W1p, l16, g4, H1n, a2, w2row, w2f);
      s8v H2n[4];
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) H2n[ks] = cat8(relu_bf(a2[2 * ks]), relu_bf(a2[2 * ks + 1]));
      f4v qn = zero4();
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const s8v a = w2f[ks];
        qn = mfma32(a, H2n[ks], qn);
      }
      WS_PIN(qn);
      WS_SB();
      WS_STAMP(8);
      // ---------------------------------------------------------------- TD target, dQ, state write-back
      // (dZ2's fragments -- W2^T tiles and the H2 mask -- are read first: their latency runs under TD)
      const bf16_t* zchunk = reinterpret_cast<const bf16_t*>(ctl + 10);   // 8 zero bytes
      s4v aw[8], h2m[8];
      auto dz_reads = [&]() {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          aw[i] = lds_tr4(g4 == 0 ? W2p + (l16 >> 2) * HP + pi_pos4(i, l16 & 3) : zchunk);
          h2m[i] = *reinterpret_cast<const s4v*>(sh2 + a_off(l16, 16 * i + 4 * g4));
        }
      };
      dz_reads();
      float dq = 0.f;
      int slot = 0;
      if (g4 == 0) {
        // target net (csrc/qtarget.hip: Q_target of the next state after each action, this step's weights)
        float4 tq = make_float4(0.f, 0.f, 0.f, 0.f);
        if (KN && p.qt != nullptr) tq = *reinterpret_cast<const float4*>(p.qt + ((size_t)e * 3 + act) * 4);
        float n0 = qn[0] + b2v[0], n1 = qn[1] + b2v[1], n2 = qn[2] + b2v[2];
        if (p.output_relu) { n0 = fmaxf(n0, 0.f); n1 = fmaxf(n1, 0.f); n2 = fmaxf(n2, 0.f); }
        int am = 0;
        float mx = n0;
        if (n1 > mx) { mx = n1; am = 1; }
        if (n2 > mx) { mx = n2; am = 2; }
        slot = p.target_compat ? am : act;
        float vnext = mx;   // the online net's max (QDecisionPolicyActor.scala:67-71)
        if (KN && p.qt != nullptr)   // target value: of the online argmax (compat slot, double DQN) or its max
          vnext = (p.target_compat || p.double_dqn) ? (am == 0 ? tq.x : (am == 1 ? tq.y : tq.z))
                                                    : fmaxf(fmaxf(tq.x, tq.y), tq.z);
        const float rsc = (KN && p.reward_scale != 1.0f) ? __fmul_rn(rew, p.reward_scale) : rew;
        const float y = __fadd_rn(rsc, __fmul_rn(p.gamma, vnext));
        const float qs = slot == 0 ? q0 : (slot == 1 ? q1 : q2);
        const float diff = __fsub_rn(qs, y);
        dq = p.loss_coef * (p.td_clip > 0.f ? fminf(fmaxf(diff, -p.td_clip), p.td_clip) : diff);
        if (p.output_relu && !(qs > 0.f)) dq = 0.f;
        float fdone = 0.f, ndone = 0.f;
        if (pos + 1 >= p.T - HWIN) {
          fdone = __fadd_rn(b2, __fmul_rn((float)s2, vnew));
          ndone = 1.f;
        }
        st_reward += rew;
        st_loss += diff * diff;
        st_qslot += qs;
        st_done += ndone;
        st_fsum += fdone;
        st_fsq += fdone * fdone;
      }
      WS_SB();
      WS_STAMP(9);
      // ---------------------------------------------------------------- dZ2 = (W2^T dQ) * [H2 > 0]
      // on the matrix cores: A = W2^T tiles (lanes g4 == 0 hold W2[0..3][u2], a transposed read of W2p's 4
      // rows), B = dQ^T (lanes g4 == 0 hold dQ[env][0..3], where TD left them); the result has the layout of
      // layer 2's accumulators.  dQ has one nonzero entry per env, so every output is one exact fp32 product.
      const s4v bq = g4 == 0 ? pk4(slot == 0 ? dq : 0.f, slot == 1 ? dq : 0.f, slot == 2 ? dq : 0.f, 0.f)
                             : zero_s4();
      s4v dz[8];
      f4v zt[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) zt[i] = mfma16(aw[i], bq, zero4());
#pragma unroll
      for (int i = 0; i < 8; ++i) dz[i] = mask_pk(zt[i], h2m[i]);
      WS_PIN(dz[7]);
      WS_SB();
      WS_STAMP(10);
      // publish: (dZ2, pi order: tiles 2 ks, 2 ks + 1 form k-step ks) dQ in the X row's pad slots
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
        *reinterpret_cast<s8v*>(sz2 + w1_off(l16, 32 * ks + 8 * g4)) = cat8(dz[2 * ks], dz[2 * ks + 1]);
      if (g4 == 0) *reinterpret_cast<s4v*>(sx + l16 * KX + 204) = bq;
      if (lane == 0) __hip_atomic_store(ctl + 1 + sl, q + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (DYN) {
        if (d == 0) {
          // round k + 3's chunk into the ring; the first missing round also fixes the round count
          int c = -1;
          if (claim_out) {
            const unsigned cv = (unsigned)__builtin_amdgcn_readfirstlane((int)claim_v);
            const long long cc = 8ll * (3ll * gx + (long long)cv) + xg;
            c = cc < nchunks ? (int)cc : -1;
            claim_out = false;
          }
          const bool first_end = c < 0 && !ended;
          if (c < 0) ended = true;
          if (lane == 0) {
            if (first_end && ck2 >= 0)
              __hip_atomic_store(ctl + CTL_NROUNDS, k + 3 + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            __hip_atomic_store(ctl + cid_word(k + 3), (((k + 3) & 0x3FF) << CID_SHIFT) | (c + 1), __ATOMIC_RELEASE,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
          }
        }
        ck0 = ck1;
        ck1 = ck2;
      }
      WS_SB();
      WS_STAMP(11);
    }
    WS_WRITE_BACK()   // the last tile's
#undef WS_WRITE_BACK
#undef WS_WB_SET
#undef WS_LOAD_ENV
#undef WS_LOAD_PRICES
#undef WS_STAMP
    // per-wave statistics -> LDS (folded after the final barrier)
    const float v[NSTAT - 1] = {st_reward, st_loss, st_explore, st_done, st_fsum, st_fsq, st_qslot};
#pragma unroll
    for (int s = 0; s < NSTAT - 1; ++s) {
      const float t = wave_sum(v[s]);
      if (lane == 0) sSt[d * NSTAT + s] = t;
    }
    if (lane == 0) sSt[d * NSTAT + NSTAT - 1] = 0.f;
    __syncthreads();
  } else {
    // ================================================================ GRADIENT WAVE
    const int gw = wave - ND;
    // owns hidden units 32 gw .. 32 gw + 31 of both layers, dW2 columns likewise
    f4v gW0[2][13], gW1[2][8], gW2[2];
    // bias gradients as per-lane fp32 sums of the dZ2^T / dQ^T fragments (each lane's 8 envs per slot
    // pair), folded over the 4 lane groups at the write-out: 3 VGPRs instead of 12 + a ones operand
    float gB1s[2] = {0.f, 0.f}, gB2s = 0.f;
    auto sum8 = [](const s8v& v) {
      float acc = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) acc += bf2f((bf16_t)v[j]);
      return acc;
    };
#pragma unroll
    for (int m = 0; m < 2; ++m) {
#pragma unroll
      for (int n = 0; n < 13; ++n) gW0[m][n] = zero4();
#pragma unroll
      for (int n = 0; n < 8; ++n) gW1[m][n] = zero4();
      gW2[m] = zero4();
    }
    s4v ones;
#pragma unroll
    for (int j = 0; j < 4; ++j) ones[j] = (l16 == 0) ? (short)0x3F80 : (short)0;
    const int r4 = 4 * g4 + (l16 >> 2), qq = l16 & 3;   // transposed-read row / chunk of this lane
    const bf16_t* zchunk = reinterpret_cast<const bf16_t*>(ctl + 10);   // 8 zero bytes
    const int nseq = ND * nmy;
    // debug stamps of gradient wave 0 of workgroup 0: per slot (wait begins, slot full, slot done) after the
    // data-wave rows ((nmy + 1) * 16 words in)
    unsigned long long* gst = ((WS_STAMPS & 2) && p.stamps != nullptr && blockIdx.x == 0 && gw == 0 && lane == 0)
                                  ? p.stamps + (size_t)(nmy + 1) * 16 : nullptr;
    // (held in SGPRs and stored once per slot: the gradient wave has no VGPR to spare mid-slot)
    unsigned long long gts[7] = {0, 0, 0, 0, 0, 0, 0};
#define WS_GST(I) if ((WS_STAMPS & 2) && ((WS_GST_MASK >> (I)) & 1)) gts[I] = __builtin_amdgcn_s_memtime(); WS_MARK(G, I)
    // slots in pairs (q, q + 1): the weight-gradient MFMAs run with K = 32 envs -- v_mfma_f32_16x16x32_bf16
    // at the cost of the K = 16 form for twice the work.  K index 8 g4 + j of lane group g4 is env
    // 4 g4 + (j & 3) of slot q (j < 4) or of slot q + 1 (j >= 4): the A and B fragments are the two slots'
    // 4-element fragments side by side (cat8), no data moves between lanes.  dZ1 stays per slot (K = u2);
    // its W1^T fragments are read once for both.
    int nseqv = DYN ? 0x7FFFFFF0 : nseq;   // dynamic: found when the data waves report the round count
    for (int q = 0; q < nseqv; q += 2) {
      const int sa = q % NSLOT, sb = (q + 1) % NSLOT;
      WS_GST(0);
      if (DYN) {
        // the slot pair of round q / ND -- or the end of the run (the round count is known by then)
        if (wait_full_or_end(p, ctl, sa, q)) {
          nseqv = q;
          continue;
        }
      } else {
        ring_wait(p, ctl, ctl + 1 + sa, [&](int v) { return v == q + 1; });
      }
      ring_wait(p, ctl, ctl + 1 + sb, [&](int v) { return v == q + 2; });
      WS_GST(1);
#if WS_GSKIP
      if (lane == 0) {
        __hip_atomic_fetch_add(ctl + 5 + sa, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_fetch_add(ctl + 5 + sb, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      continue;
#endif
      const char* pa_ = smem + oSLOT + sa * SLOT_BYTES;
      const char* pb_ = smem + oSLOT + sb * SLOT_BYTES;
      const bf16_t *xa = reinterpret_cast<const bf16_t*>(pa_ + sX), *xb = reinterpret_cast<const bf16_t*>(pb_ + sX);
      const bf16_t *h1a = reinterpret_cast<const bf16_t*>(pa_ + sH1), *h1b = reinterpret_cast<const bf16_t*>(pb_ + sH1);
      const bf16_t *h2a = reinterpret_cast<const bf16_t*>(pa_ + sH2), *h2b = reinterpret_cast<const bf16_t*>(pb_ + sH2);
      const bf16_t *z2a = reinterpret_cast<const bf16_t*>(pa_ + sDZ2), *z2b = reinterpret_cast<const bf16_t*>(pb_ + sDZ2);
      // both slots' tr4 fragments at one offset, side by side: K = 32 envs
      auto tr8 = [&](const bf16_t* a, const bf16_t* b, int off) { return cat8(lds_tr4(a + off), lds_tr4(b + off)); };
      // ---- dZ1 of both slots for this wave's u1 tiles (result lane (u1, g4): envs 4 g4 .. 4 g4 + 3)
      f4v c1a[2] = {zero4(), zero4()}, c1b[2] = {zero4(), zero4()};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const s8v aza = lds_ld8(z2a + w1_off(l16, 32 * ks + 8 * g4));
        const s8v azb = lds_ld8(z2b + w1_off(l16, 32 * ks + 8 * g4));
        const int R = 32 * ks + 4 * g4 + (l16 >> 2);
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int col = pi_pos4(2 * gw + t, qq);
          const s8v wt = cat8(lds_tr4(W1p + w1_off(R, col)), lds_tr4(W1p + w1_off(R + 16, col)));
          c1a[t] = mfma32(aza, wt, c1a[t]);
          c1b[t] = mfma32(azb, wt, c1b[t]);
        }
      }
      s4v bowna[2], bownb[2];   // own H1 tiles of both slots (the dZ1 mask)
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        bowna[t] = lds_tr4(h1a + a_off(r4, 16 * (2 * gw + t) + 4 * qq));
        bownb[t] = lds_tr4(h1b + a_off(r4, 16 * (2 * gw + t) + 4 * qq));
      }
      constexpr int XD = WS_GXP;   // X fragment pairs read ahead of the dW0 MFMAs
      s8v bx[13];
#pragma unroll
      for (int n = 0; n < XD; ++n) bx[n] = tr8(xa, xb, r4 * KX + 16 * n + 4 * qq);
      WS_PIN(c1a[1]); WS_PIN(c1b[1]);
      WS_SB();
      WS_GST(2);
      s8v a0[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) a0[t] = cat8(mask_pk(c1a[t], bowna[t]), mask_pk(c1b[t], bownb[t]));
      WS_PIN(a0[1]);
      WS_SB();
      WS_GST(3);
      // ---- dW0^T[u1][slot col] += dZ1^T . X (K = 32 envs)
#pragma unroll
      for (int n = 0; n < 13; ++n) {
#pragma unroll
        for (int m = 0; m < 2; ++m) gW0[m][n] = mfma32(a0[m], bx[n], gW0[m][n]);
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
        if (n + XD < 13) {
          bx[n + XD] = tr8(xa, xb, r4 * KX + 16 * (n + XD) + 4 * qq);
          __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
        }
      }
      WS_PIN(gW0[1][12]);
      WS_SB();
      WS_GST(4);
      // ---- dW1^T[u2][u1] += dZ2^T . H1, db1 += dZ2^T . 1 ; dW2^T[a][u2] += dQ^T . H2, db2 += dQ^T . 1
      //      (H1 fragments in two halves; both slots go back once the last fragment has landed)
      s8v a1[2];
#pragma unroll
      for (int m = 0; m < 2; ++m) a1[m] = tr8(z2a, z2b, w1_off(r4, pi_pos4(2 * gw + m, qq)));
#pragma unroll
      for (int m = 0; m < 2; ++m) gB1s[m] += sum8(a1[m]);
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        s8v bh[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) bh[k] = tr8(h1a, h1b, a_off(r4, 16 * (4 * half + k) + 4 * qq));
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
          for (int k = 0; k < 4; ++k) gW1[m][4 * half + k] = mfma32(a1[m], bh[k], gW1[m][4 * half + k]);
      }
      {
        const s8v aq = qq == 0 ? tr8(xa, xb, r4 * KX + 204) : cat8(lds_tr4(zchunk), lds_tr4(zchunk));   // a = l16 < 4
        s8v bh2[2];
#pragma unroll
        for (int k = 0; k < 2; ++k) bh2[k] = tr8(h2a, h2b, a_off(r4, 16 * (2 * gw + k) + 4 * qq));
        if (lane == 0) {
          __hip_atomic_fetch_add(ctl + 5 + sa, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
          __hip_atomic_fetch_add(ctl + 5 + sb, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        WS_GST(5);
#pragma unroll
        for (int n = 0; n < 2; ++n) gW2[n] = mfma32(aq, bh2[n], gW2[n]);
        gB2s += sum8(aq);
      }
      WS_PIN(gW1[1][7]); WS_PIN(gB2s);
      WS_SB();
      WS_GST(6);
      if ((WS_STAMPS & 2) && gst) {
#pragma unroll
        for (int i = 0; i < 7; ++i) gst[8 * q + i] = gts[i];
      }
    }
    __syncthreads();
    // ------------------------------------------------------------------ gradient slab write-out
    // this wave's rows: dW0^T / dW1^T rows 32 gw + 16 m + 4 g4 + j; dW2^T u2 columns 16 (2 gw + n) + l16
    auto put = [&](int idx, float v) {
      if (p.slab_bf16) {
        bf16_t* sbf = reinterpret_cast<bf16_t*>(p.slab);
        sbf[((size_t)(idx >> 5) * p.slab_rows + blockIdx.x) * 32 + (idx & 31)] = f2bf(v);
      } else {
        p.slab[(size_t)blockIdx.x * p.P + idx] = v;
      }
    };
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int u = 32 * gw + 16 * m + 4 * g4 + j;
#pragma unroll
        for (int n = 0; n < 13; ++n) put(p.off_w0 + u * INP + slot_col(16 * n + l16), gW0[m][n][j]);
#pragma unroll
        for (int n = 0; n < 8; ++n) put(p.off_w1 + u * HP + 16 * n + l16, gW1[m][n][j]);
      }
    // bias gradients: fold the 4 lane groups' partial sums (lane (l16, g4): 8 envs of each slot pair)
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      float v = gB1s[m];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      if (g4 == 0) put(p.off_b1 + 32 * gw + 16 * m + l16, v);
    }
    {
      float v = gB2s;
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      if (gw == 0 && g4 == 0 && l16 < 4) put(p.off_b2 + l16, v);
    }
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int j = 0; j < 4; ++j) put(p.off_w2 + (4 * g4 + j) * HP + 16 * (2 * gw + n) + l16, gW2[n][j]);
  }
#undef WS_SB
#undef WS_PIN
#undef WS_GST
  // ------------------------------------------------------------------ workgroup statistics (data waves' sums)
  if (tid < NSTAT) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < ND; ++w) t += sSt[w * NSTAT + tid];
    p.stats[(size_t)blockIdx.x * NSTAT + tid] = t;
  }
  if (blockIdx.x == 0 && tid == 0) p.ctrl[1] = step + 1;   // 1-based update count for the optimizer
}

template <int FEAT, bool DYN, bool KN, bool U16 = false>
static hipError_t launch_f(const QStepParams& p, int grid, hipStream_t stream) {
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)qstep_ws_kernel<FEAT, DYN, KN, U16>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    if (e != hipSuccess) return e;
    attr = true;
  }
  hipLaunchKernelGGL((qstep_ws_kernel<FEAT, DYN, KN, U16>), dim3(grid), dim3(NT), LDS_BYTES, stream, p);
  return hipGetLastError();
}

// the prologue's image entries, inverted: map[parameter] = bf16 element of the image (>= 0), -(fp32 word) - 2
// (biases), or -1 (not in the image; the host fills -1 first).  Same index math as the prologue's gather, so
// the optimizer pass's scatter (csrc/optim.hip) rebuilds exactly the bytes the gather would.
__global__ void __launch_bounds__(256) ws_img_map_kernel(int* map, int off_w0, int off_w1, int off_w2, int off_b1,
                                                         int off_b2) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < HP * KX) map[off_w0 + (i / KX) * INP + slot_col(i % KX)] = oW0 / 2 + i;
  if (i < HP * HP) map[off_w1 + (i >> 7) * HP + pi_unit(i & 127)] = oW1 / 2 + w1_off(i >> 7, i & 127);
  if (i < 5 * HP) map[off_w2 + (i >> 7) * HP + pi_unit(i & 127)] = oW2 / 2 + i;
  if (i < HP) map[off_b1 + i] = -(oB1 / 4 + i) - 2;
  if (i < 4) map[off_b2 + i] = -(oB2 / 4 + i) - 2;
}

}  // namespace WS_NS
}  // namespace st

extern "C" int WS_API(st_qstep_ws_img_bytes)() { return st::WS_NS::oSLOT - st::WS_NS::oW0; }

extern "C" hipError_t WS_API(st_qstep_ws_img_map)(int* map, int off_w0, int off_w1, int off_w2, int off_b1, int off_b2,
                                                  hipStream_t stream) {
  using namespace st::WS_NS;
  static_assert(oW0 == 0 && (oSLOT - oW0) % 16 == 0, "image run");
  hipLaunchKernelGGL(ws_img_map_kernel, dim3((HP * KX + 255) / 256), dim3(256), 0, stream, map, off_w0, off_w1, off_w2,
                     off_b1, off_b2);
  return hipGetLastError();
}

extern "C" int WS_API(st_qstep_ws_lds_bytes)(int inp, int h1p, int h2p) {
  if (inp == st::WS_NS::INP && h1p == st::WS_NS::HP && h2p == st::WS_NS::HP) return st::WS_NS::LDS_BYTES;
  return -1;
}

// Preconditions (checked here and by sharetrade/trainer/engine.py): E % 64 == 0, 1 <= grid <= E / 64,
// H == 201, padded dims (224, 128, 128), 32-aligned weight offsets for bf16 slabs; the dynamic chunk
// schedule (p->chunk_heads, zero at launch) needs grid % 8 == 0 and E / 64 < 2^21.
extern "C" hipError_t WS_API(st_qstep_ws_launch)(const st::QStepParams* p, int inp, int h1p, int h2p, int grid,
                                                 hipStream_t stream) {
  using namespace st::WS_NS;
  if (inp != INP || h1p != HP || h2p != HP || p->H != HWIN) return hipErrorInvalidValue;
  if (p->E % C != 0 || grid < 1 || grid > p->E / C) return hipErrorInvalidValue;
  if (p->chunk_heads != nullptr && (grid % 8 != 0 || p->E / C >= (1 << CID_SHIFT) - 1)) return hipErrorInvalidValue;
  if (p->T < HWIN + 2 || p->T4 < p->T + 4) return hipErrorInvalidValue;
  if ((p->off_w0 | p->off_w1 | p->off_w2) & 7) return hipErrorInvalidValue;
  if (p->slab_bf16 && (p->slab_rows != grid || p->P % 32 != 0)) return hipErrorInvalidValue;
  const bool kn = p->qt != nullptr || p->reward_scale != 1.0f || p->ramp_global || p->double_dqn;
  if (p->ticks != nullptr) {   // the 16-bit tick bank (relative features only)
    if (!p->feat_mode || p->tscale == nullptr || p->T16 < p->T + 8 || p->T16 % 8) return hipErrorInvalidValue;
    if (kn) {
      if (p->chunk_heads != nullptr || (p->double_dqn && p->qt == nullptr)) return hipErrorInvalidValue;
      return launch_f<1, false, true, true>(*p, grid, stream);
    }
    if (p->chunk_heads != nullptr) return launch_f<1, true, false, true>(*p, grid, stream);
    return launch_f<1, false, false, true>(*p, grid, stream);
  }
  if (kn) {   // learning-quality knobs: static schedule only
    if (p->chunk_heads != nullptr || (p->double_dqn && p->qt == nullptr)) return hipErrorInvalidValue;
    return p->feat_mode ? launch_f<1, false, true>(*p, grid, stream) : launch_f<0, false, true>(*p, grid, stream);
  }
  if (p->chunk_heads != nullptr)
    return p->feat_mode ? launch_f<1, true, false>(*p, grid, stream) : launch_f<0, true, false>(*p, grid, stream);
  return p->feat_mode ? launch_f<1, false, false>(*p, grid, stream) : launch_f<0, false, false>(*p, grid, stream);
}
