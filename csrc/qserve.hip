// Batched policy serving on CDNA4 (gfx950): SelectionAction for many requests in one launch.
//
// The reference answers every SelectionAction(state[1,203], step) with its own TF session run
// (QDecisionPolicyActor.scala:56-62: two dense layers, argmax on the host, scala.util.Random
// epsilon-greedy).  Here a batch of raw request rows -- 201 prices + budget + shares, the reference's
// state layout (TrainerChildActor.scala:90-91) -- goes through the flagship 2x128 bf16 Q-net in one
// persistent launch:
//
//   features (raw, or relative to the window's last price: sharetrade/env/trading.py::features)
//   -> layer 1 (224 -> 128, the bias is the constant-1 input column) -> ReLU
//   -> layer 2 (128 -> 128) + b1 -> ReLU -> output (128 -> 3) + b2 [-> ReLU under reference_compat]
//   -> argmax (first max, like TF ArgMax) -> epsilon-greedy (Philox; exploit iff u < min(eps, step/ramp))
//
// Design (MI355X-first, not the engine's step kernel minus the learner):
//  * every weight lives in VGPRs for the whole launch: a wave owns 32 hidden units of both hidden
//    layers (A operands: 2 m-tiles x (7 + 4) k-steps of v_mfma_f32_16x16x32_bf16 fragments) and the
//    output-layer fragments (4 k-steps), 104 registers per lane, loaded once per workgroup;
//  * persistent grid walking 64-row tiles, so the per-workgroup weight load (~106 KB of L2 reads) is
//    paid once per launch, not once per tile;
//  * STREAM (rows at a 16-byte-aligned stride <= 208 floats): the next tile's raw rows stream into a
//    second LDS buffer by LDS-DMA (global_load_lds_dwordx4, one contiguous 64 x ld block) for the
//    whole of the current tile; the phases are separated by raw s_barriers that wait for LDS traffic
//    only, so the DMA stays in flight across them.  One workgroup per CU (156 KB of LDS);
//  * otherwise (any stride): register gather with every load unconditional (clamped indices) and 7
//    quads x 5 loads in flight per thread; activation tiles only in LDS (49 KB), two workgroups per CU.
#include "common.h"

namespace st {
namespace serve {

constexpr int INP = 224, HP = 128, OUTP = 16;   // padded dims of the flagship layout (models/qnet.py)
constexpr int C = 64;                           // request rows per tile
constexpr int NW = 4, NT = 64 * NW;             // register-gather build (STREAM: 8 waves, see the kernel)
constexpr int NET = C / 16;                     // 16-row tiles per tile
constexpr int MT = HP / (16 * NW);              // 16-unit m-tiles per wave (2; STREAM: 1)
constexpr int KS0 = INP / 32, KS1 = HP / 32;
constexpr int SX = INP + 16, SH = HP + 16;      // activation row strides (bf16)
constexpr int MAXLD = 208;                      // STREAM: widest row stride staged (floats)
constexpr int ACT_BYTES = (C * SX + C * SH) * 2;
constexpr int RAW_BYTES = 2 * C * MAXLD * 4;    // two row buffers: tile t+1 lands while tile t runs
constexpr int LDS_BYTES = ACT_BYTES;                                   // register-gather build
constexpr int LDS_BYTES_STREAM = RAW_BYTES + ACT_BYTES + 2 * C * 4;    // + staged rows, steps, 1/last

// s_waitcnt immediates (gfx9 split vmcnt field): lgkmcnt(0) only / vmcnt(0) only
ST_DEV void wait_lgkm0() { __builtin_amdgcn_s_waitcnt(0xF | (0x3 << 14) | (0x7 << 4)); }
ST_DEV void wait_vm0() { __builtin_amdgcn_s_waitcnt((0x7 << 4) | (0xF << 8)); }
// global_load_lds_dwordx4 issued from inline asm: with the builtin, hipcc orders every later LDS store
// behind the DMA (s_waitcnt vmcnt(0) at the first ds_write after it: the MFMA phases' epilogues), which
// drains it one phase after the issue.  The kernel retires it itself (wait_vm0 before reading the rows).
// lds_off: wave-uniform LDS byte offset of this wave-instruction's 1 KiB destination.
ST_DEV void glds16(const float* gsrc, unsigned lds_off) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(lds_off) : "memory");
}

struct ServeParams {
  const float* states;   // [B][ld] fp32 request rows: H prices, budget, shares
  const float* steps;    // [B] the SelectionAction step (exploit ramp), or null = greedy
  const bf16_t* wq;      // bf16 flat params (engine layout)
  const float* wf;       // fp32 flat params (biases)
  float* q_out;          // [B][3] or null
  int* actions;          // [B]
  int B, ld, H;
  int off_w0, off_w1, off_b1, off_w2, off_b2;
  int feat_mode, output_relu;
  float inv_b0, eps, inv_ramp;
  uint32_t key0, key1;
  unsigned long long seq;   // draw counter: (row, seq_lo, seq_hi, stream 2)
};

template <bool STREAM>
__global__ void __launch_bounds__(STREAM ? 512 : 256, STREAM ? 1 : 2) qserve_kernel(ServeParams p) {
  // STREAM: one workgroup per CU (156 KB of LDS) of 8 waves -- two per SIMD, each owning 16 hidden
  // units -- so one wave's MFMAs overlap the other's VALU / LDS work; register gather: 4 waves x 32 units,
  // two workgroups per CU
  constexpr int NWk = STREAM ? 8 : 4, NTk = 64 * NWk, MTk = HP / (16 * NWk), TPR = NTk / C;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* sRaw = reinterpret_cast<float*>(smem);   // STREAM: the tile's raw rows [C][ld]
  bf16_t* sX = reinterpret_cast<bf16_t*>(smem + (STREAM ? RAW_BYTES : 0));   // [C][SX]; H2 [C][SH] later
  bf16_t* sH1 = sX + C * SX;                        // [C][SH]
  float* sSteps = reinterpret_cast<float*>(reinterpret_cast<char*>(sX) + ACT_BYTES);   // STREAM: [C]
  float* sInv = sSteps + C;                                                            // STREAM: [C]
  const int tid = threadIdx.x, lane = tid & 63, l16 = lane & 15, g4 = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int m0 = 16 * MTk * wave;
  const int H = p.H;

  // ---------------------------------------------------------------- weights -> VGPRs (once)
  s8v aW0[MTk][KS0], aW1[MTk][KS1], aW2[KS1];
#pragma unroll
  for (int i = 0; i < MTk; ++i) {
    const bf16_t* w0 = p.wq + p.off_w0 + (size_t)(m0 + 16 * i + l16) * INP + 8 * g4;
#pragma unroll
    for (int ks = 0; ks < KS0; ++ks) aW0[i][ks] = *reinterpret_cast<const s8v*>(w0 + ks * 32);
    const bf16_t* w1 = p.wq + p.off_w1 + (size_t)(m0 + 16 * i + l16) * HP + 8 * g4;
#pragma unroll
    for (int ks = 0; ks < KS1; ++ks) aW1[i][ks] = *reinterpret_cast<const s8v*>(w1 + ks * 32);
  }
  {
    const bf16_t* w2 = p.wq + p.off_w2 + (size_t)l16 * HP + 8 * g4;
#pragma unroll
    for (int ks = 0; ks < KS1; ++ks) aW2[ks] = *reinterpret_cast<const s8v*>(w2 + ks * 32);
  }
  float bb[MTk][4];
#pragma unroll
  for (int i = 0; i < MTk; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) bb[i][j] = p.wf[p.off_b1 + m0 + 16 * i + 4 * g4 + j];
  float b2[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) b2[j] = p.wf[p.off_b2 + j];

  // barrier between phases: STREAM waits for LDS traffic only (a __syncthreads() would also drain the
  // row DMA in flight: vmcnt(0))
  auto bar = [&]() {
    if constexpr (STREAM) {
      wait_lgkm0();
      asm volatile("s_barrier" ::: "memory");
    } else {
      __syncthreads();
    }
  };
  // STREAM: tile t's rows = one contiguous block of C * ld floats = ld / 4 wave-instructions of 64 x 16 B
  // (pieces past the end of the array re-read its last 16 B: those rows are not live)
  const unsigned npieces = (unsigned)p.B * (unsigned)p.ld / 4u;
  auto stage = [&](int t, int buf) {
    const unsigned base = (unsigned)t * (unsigned)C * (unsigned)p.ld / 4u;
    const unsigned raw0 = (unsigned)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) float*)sRaw) +
                          (unsigned)buf * (unsigned)(C * MAXLD * 4);
    for (int j = wave; j < p.ld / 4; j += NWk) {
      const unsigned pc = min(base + (unsigned)(j * 64 + lane), npieces - 1u);
      glds16(p.states + 4u * pc, __builtin_amdgcn_readfirstlane(raw0 + (unsigned)j * 1024u));
    }
  };

  const int ntiles = (p.B + C - 1) / C;
  if constexpr (STREAM) {
    if ((int)blockIdx.x < ntiles) stage(blockIdx.x, 0);
  }
  int it_ = 0;
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x, ++it_) {
    const int r0 = tile * C;
    const float* rows = sRaw + (it_ & 1) * (C * MAXLD);   // STREAM: this tile's staged rows
    if constexpr (STREAM) {
      wait_vm0();   // this wave's row DMA (and the previous tile's output stores) landed
      if (tid < C) sSteps[tid] = p.steps != nullptr ? p.steps[min(r0 + tid, p.B - 1)] : 0.f;
      bar();        // every wave's DMA landed; every wave is done with the other buffer
      // the next tile's rows stream into the other buffer through this whole tile
      if (tile + (int)gridDim.x < ntiles) stage(tile + gridDim.x, (it_ + 1) & 1);
      // one correctly rounded 1 / last price per row (torch: 1.0 / last), not one per column quad
      if (tid < C) sInv[tid] = p.feat_mode ? __fdiv_rn(1.0f, rows[tid * p.ld + H - 1]) : 1.0f;
      bar();
    }
    // -------------------------------------------------------------- P0: request rows -> features
    // Thread = (row tid / TPR, column quads tid % TPR + TPR m): TPR = 4 (register gather, 14 quad slots)
    // or 8 (STREAM, 7 slots).  The row offset, the row's 1 / last price and its liveness are per thread,
    // and quad slot m is a price quad on every lane while 4 (TPR - 1 + TPR m) + 3 < H (a scalar branch:
    // packed fp32 mul / sub, then bf16); only the slots reaching columns H .. H+2 (budget, shares, the
    // constant-1 bias input) take the select chain.  Batches of 7 quads, all loads of a batch in flight
    // before its first use (register gather: unconditional, clamped loads -- loads under per-element
    // branches were issued one wait at a time).
    {
      constexpr int QB = 7, NQ = INP / 4 / TPR;   // quad slots per thread
      static_assert(NQ % QB == 0, "quad batches");
      const int r = tid / TPR, t4 = tid % TPR;
      const bool live = r0 + r < p.B;
      const unsigned ro = (unsigned)min(r0 + r, p.B - 1) * (unsigned)p.ld;   // host: B * ld < 2^30
      const float* rowp = STREAM ? rows + r * p.ld : nullptr;
      const float last = STREAM ? rowp[H - 1] : p.states[ro + (unsigned)(H - 1)];
      const float inv = !p.feat_mode ? 1.0f : STREAM ? sInv[r] : __fdiv_rn(1.0f, last);
      const int cmax = (H + 1) & ~3;   // the last quad holding row data (column H + 1)
      // price quads: x * iv - off with (iv, off) = (1 / last, 1) relative, (1, 0) raw (exact), (0, 0) for a
      // row past B (its clamped, finite values give 0): no per-quad selects
      const float ivq = live ? inv : 0.f, offq = (live && p.feat_mode) ? 1.0f : 0.f;
#pragma unroll 1
      for (int mb = 0; mb < NQ; mb += QB) {
        float v[QB][4];
#pragma unroll
        for (int m = 0; m < QB; ++m) {
          const int c = min(4 * (t4 + TPR * (mb + m)), cmax);
          if constexpr (STREAM) {
            const float4 t = *reinterpret_cast<const float4*>(rowp + c);
            v[m][0] = t.x; v[m][1] = t.y; v[m][2] = t.z; v[m][3] = t.w;
          } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) v[m][q] = p.states[ro + (unsigned)min(c + q, H + 1)];
          }
        }
#pragma unroll
        for (int m = 0; m < QB; ++m) {
          const int c = 4 * (t4 + TPR * (mb + m));
          float x[4];
          if (4 * (TPR - 1 + TPR * (mb + m)) + 3 < H) {   // prices only, on every lane (a scalar branch)
            // packed fp32 mul then sub: the same IEEE roundings as feat_price
            const f32x2_t iv = {ivq, ivq}, off = {offq, offq};
            const f32x2_t x01 = f32x2_t{v[m][0], v[m][1]} * iv - off, x23 = f32x2_t{v[m][2], v[m][3]} * iv - off;
            lds_st4(sX + r * SX + c, x01.x, x01.y, x23.x, x23.y);
          } else {   // quads at / past column H: budget, shares, the constant 1, padding
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const int k = c + q;
              const float w = v[m][q];
              const float fp = p.feat_mode ? __fsub_rn(__fmul_rn(w, inv), 1.0f) : w;
              const float fb = p.feat_mode ? __fmul_rn(w, p.inv_b0) : w;
              const float fs = p.feat_mode ? __fmul_rn(__fmul_rn(w, last), p.inv_b0) : w;
              x[q] = live ? (k < H ? fp : k == H ? fb : k == H + 1 ? fs : k == H + 2 ? 1.0f : 0.0f) : 0.0f;
            }
            lds_st4(sX + r * SX + c, x[0], x[1], x[2], x[3]);
          }
        }
      }
    }
    bar();
    // -------------------------------------------------------------- P1: layer 1
    {
      f4v acc[MTk][NET];
#pragma unroll
      for (int i = 0; i < MTk; ++i)
#pragma unroll
        for (int n = 0; n < NET; ++n) acc[i][n] = zero4();
#pragma unroll
      for (int ks = 0; ks < KS0; ++ks) {
        s8v b[NET];
#pragma unroll
        for (int n = 0; n < NET; ++n) b[n] = lds_ld8(sX + (16 * n + l16) * SX + ks * 32 + 8 * g4);
#pragma unroll
        for (int i = 0; i < MTk; ++i)
#pragma unroll
          for (int n = 0; n < NET; ++n) acc[i][n] = mfma32(aW0[i][ks], b[n], acc[i][n]);
      }
#pragma unroll
      for (int i = 0; i < MTk; ++i)
#pragma unroll
        for (int n = 0; n < NET; ++n) {
          const f4v v = acc[i][n];
          lds_st4(sH1 + (16 * n + l16) * SH + m0 + 16 * i + 4 * g4, fmaxf(v[0], 0.f), fmaxf(v[1], 0.f),
                  fmaxf(v[2], 0.f), fmaxf(v[3], 0.f));
        }
    }
    bar();
    // -------------------------------------------------------------- P2: layer 2 (+ b1) -> H2 (over X)
    bf16_t* sH2 = sX;
    {
      f4v acc[MTk][NET];
#pragma unroll
      for (int i = 0; i < MTk; ++i)
#pragma unroll
        for (int n = 0; n < NET; ++n) acc[i][n] = zero4();
#pragma unroll
      for (int ks = 0; ks < KS1; ++ks) {
        s8v b[NET];
#pragma unroll
        for (int n = 0; n < NET; ++n) b[n] = lds_ld8(sH1 + (16 * n + l16) * SH + ks * 32 + 8 * g4);
#pragma unroll
        for (int i = 0; i < MTk; ++i)
#pragma unroll
          for (int n = 0; n < NET; ++n) acc[i][n] = mfma32(aW1[i][ks], b[n], acc[i][n]);
      }
#pragma unroll
      for (int i = 0; i < MTk; ++i)
#pragma unroll
        for (int n = 0; n < NET; ++n) {
          const f4v v = acc[i][n];
          lds_st4(sH2 + (16 * n + l16) * SH + m0 + 16 * i + 4 * g4, fmaxf(v[0] + bb[i][0], 0.f),
                  fmaxf(v[1] + bb[i][1], 0.f), fmaxf(v[2] + bb[i][2], 0.f), fmaxf(v[3] + bb[i][3], 0.f));
        }
    }
    bar();
    // -------------------------------------------------------------- P3: output, argmax, epsilon-greedy
    if (wave < NET) {
      f4v acc = zero4();   // wave w: 16-row tile w; lanes g4 == 0 end up with q[0..3] of row 16w + l16
#pragma unroll
      for (int ks = 0; ks < KS1; ++ks)
        acc = mfma32(aW2[ks], lds_ld8(sH2 + (16 * wave + l16) * SH + ks * 32 + 8 * g4), acc);
      const int row = r0 + 16 * wave + l16;
      if (g4 == 0 && row < p.B) {
        float q[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          q[j] = acc[j] + b2[j];
          if (p.output_relu) q[j] = fmaxf(q[j], 0.f);
        }
        int a = 0;
        float best = q[0];
        if (q[1] > best) { best = q[1]; a = 1; }
        if (q[2] > best) { best = q[2]; a = 2; }
        if (p.steps != nullptr) {
          uint32_t c0 = (uint32_t)row, c1 = (uint32_t)(p.seq & 0xFFFFFFFFull), c2 = (uint32_t)(p.seq >> 32),
                   c3 = 2u;
          philox4x32(c0, c1, c2, c3, p.key0, p.key1);
          const float u1 = u24(c0), u2 = u24(c1);
          const float st = STREAM ? sSteps[16 * wave + l16] : p.steps[row];
          const bool exploit = u1 < fminf(p.eps, __fmul_rn(st, p.inv_ramp));
          int rnd = (int)(u2 * 3.0f);
          rnd = rnd > 2 ? 2 : rnd;
          a = exploit ? a : rnd;
        }
        p.actions[row] = a;
        if (p.q_out != nullptr) {
          p.q_out[(size_t)row * 3 + 0] = q[0];
          p.q_out[(size_t)row * 3 + 1] = q[1];
          p.q_out[(size_t)row * 3 + 2] = q[2];
        }
      }
    }
    bar();   // the next tile's features overwrite X / H2 (and its steps sSteps)
  }
  if constexpr (STREAM) wait_vm0();
}

}  // namespace serve
}  // namespace st

extern "C" int st_qserve_lds_bytes(int stream) { return stream ? st::serve::LDS_BYTES_STREAM : st::serve::LDS_BYTES; }

// grid <= 0: min(tiles, CUs) (STREAM) or min(tiles, 2 x CUs).  Pre-launch checks: the padded dims are fixed (224 / 128 / 16) and the
// request rows must hold H + 2 values with H + 3 <= 224 (prices, budget, shares, constant 1).
extern "C" hipError_t st_qserve_launch(const st::serve::ServeParams* p, int grid, hipStream_t stream) {
  using namespace st::serve;
  if (p->B <= 0) return hipSuccess;
  if (p->H < 2 || p->H + 3 > INP || p->ld < p->H + 2 || p->states == nullptr || p->actions == nullptr ||
      p->wq == nullptr || p->wf == nullptr || (long long)p->B * p->ld >= (1LL << 30))
    return hipErrorInvalidValue;
  const bool strm = (p->ld % 4 == 0) && p->ld <= MAXLD && ((reinterpret_cast<uintptr_t>(p->states) & 15) == 0);
  if (strm) {
    static bool attr = false;
    if (!attr) {
      hipError_t e = hipFuncSetAttribute((const void*)qserve_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                         LDS_BYTES_STREAM);
      if (e != hipSuccess) return e;
      attr = true;
    }
  }
  const int ntiles = (p->B + C - 1) / C;
  if (grid <= 0) {
    int dev = 0, cus = 256;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    grid = (strm ? 1 : 2) * cus;
  }
  if (grid > ntiles) grid = ntiles;
  if (strm)
    hipLaunchKernelGGL(qserve_kernel<true>, dim3(grid), dim3(512), LDS_BYTES_STREAM, stream, *p);
  else
    hipLaunchKernelGGL(qserve_kernel<false>, dim3(grid), dim3(NT), LDS_BYTES, stream, *p);
  return hipGetLastError();
}

// struct sizes of this file's launch ABI, for the host mirrors' check (tests/test_abi.py; no HIP call)
extern "C" int st_abi_qserve(int* out, int n) {
  const int sz[] = {(int)sizeof(st::serve::ServeParams)};
  const int m = (int)(sizeof(sz) / sizeof(sz[0]));
  for (int i = 0; i < n && i < m; ++i) out[i] = sz[i];
  return m;
}
