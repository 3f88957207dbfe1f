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
//  * LDS holds only the 64-row activation tiles (X, H1; H2 reuses X): 49 KB, so two workgroups share
//    a CU and one's feature gather overlaps the other's MFMA phases;
//  * persistent grid (<= 2 workgroups per CU) walking 64-row tiles, so the per-workgroup weight load
//    (~90 KB of L2 reads) is paid once per launch, not once per tile.
#include "common.h"

namespace st {
namespace serve {

constexpr int INP = 224, HP = 128, OUTP = 16;   // padded dims of the flagship layout (models/qnet.py)
constexpr int C = 64;                           // request rows per tile
constexpr int NW = 4, NT = 64 * NW;
constexpr int NET = C / 16;                     // 16-row tiles per tile
constexpr int MT = HP / (16 * NW);              // 16-unit m-tiles per wave (2)
constexpr int KS0 = INP / 32, KS1 = HP / 32;
constexpr int SX = INP + 16, SH = HP + 16;      // activation row strides (bf16)
constexpr int LDS_BYTES = (C * SX + C * SH) * 2;

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

// VEC: rows 16-byte aligned (ld % 4 == 0, aligned base): one dwordx4 load per column quad
template <bool VEC>
__global__ void __launch_bounds__(NT, 2) qserve_kernel(ServeParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* sX = reinterpret_cast<bf16_t*>(smem);   // [C][SX]; also H2 [C][SH] after layer 1
  bf16_t* sH1 = sX + C * SX;                        // [C][SH]
  const int tid = threadIdx.x, lane = tid & 63, l16 = lane & 15, g4 = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int m0 = 16 * MT * wave;
  const int H = p.H;

  // ---------------------------------------------------------------- weights -> VGPRs (once)
  s8v aW0[MT][KS0], aW1[MT][KS1], aW2[KS1];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
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
  float bb[MT][4];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) bb[i][j] = p.wf[p.off_b1 + m0 + 16 * i + 4 * g4 + j];
  float b2[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) b2[j] = p.wf[p.off_b2 + j];

  const int ntiles = (p.B + C - 1) / C;
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int r0 = tile * C;
    // -------------------------------------------------------------- P0: request rows -> features
    // 64 rows x 56 column quads, 14 quads per thread in two batches of 7: every load unconditional
    // (row and column indices clamped), all of a batch in flight before the first use -- loads under
    // per-element branches were issued one wait at a time (~8 us per tile).  The row's last price
    // (the relative-feature normaliser) is one more load per quad; budget / shares are columns H,
    // H+1 of the quad that covers them.
    constexpr int QPR = INP / 4, QPT = C * QPR / NT, QB = 7;
    static_assert(QPT % QB == 0, "quad batches");
#pragma unroll 1
    for (int qb = 0; qb < QPT; qb += QB) {
      float v[QB][4], lastv[QB];
#pragma unroll
      for (int j = 0; j < QB; ++j) {
        const int it = tid + NT * (qb + j), r = it / QPR, c = 4 * (it - r * QPR);
        // 32-bit element offsets off one uniform base (the host checks B * ld < 2^30)
        const unsigned ro = (unsigned)min(r0 + r, p.B - 1) * (unsigned)p.ld;
        if constexpr (VEC) {
          // quads past the one holding column H+1 re-read it: their columns take no row value
          const float4 t = *reinterpret_cast<const float4*>(p.states + ro + (unsigned)min(c, (H + 1) & ~3));
          v[j][0] = t.x; v[j][1] = t.y; v[j][2] = t.z; v[j][3] = t.w;
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q) v[j][q] = p.states[ro + (unsigned)min(c + q, H + 1)];
        }
        lastv[j] = p.states[ro + (unsigned)(H - 1)];
      }
#pragma unroll
      for (int j = 0; j < QB; ++j) {
        const int it = tid + NT * (qb + j), r = it / QPR, c = 4 * (it - r * QPR);
        const bool live = r0 + r < p.B;
        const float last = lastv[j];
        const float inv = p.feat_mode ? __fdiv_rn(1.0f, last) : 1.0f;
        float x[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int k = c + q;
          const float w = v[j][q];
          float f = 0.f;
          if (k < H) f = p.feat_mode ? __fsub_rn(__fmul_rn(w, inv), 1.0f) : w;
          else if (k == H) f = p.feat_mode ? __fmul_rn(w, p.inv_b0) : w;
          else if (k == H + 1) f = p.feat_mode ? __fmul_rn(__fmul_rn(w, last), p.inv_b0) : w;
          else if (k == H + 2) f = 1.0f;   // constant-1 column: layer 1's bias
          x[q] = live ? f : 0.f;
        }
        lds_st4(sX + r * SX + c, x[0], x[1], x[2], x[3]);
      }
    }
    __syncthreads();
    // -------------------------------------------------------------- P1: layer 1
    {
      f4v acc[MT][NET];
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int n = 0; n < NET; ++n) acc[i][n] = zero4();
#pragma unroll
      for (int ks = 0; ks < KS0; ++ks) {
        s8v b[NET];
#pragma unroll
        for (int n = 0; n < NET; ++n) b[n] = lds_ld8(sX + (16 * n + l16) * SX + ks * 32 + 8 * g4);
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
          for (int n = 0; n < NET; ++n) acc[i][n] = mfma32(aW0[i][ks], b[n], acc[i][n]);
      }
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int n = 0; n < NET; ++n) {
          const f4v v = acc[i][n];
          lds_st4(sH1 + (16 * n + l16) * SH + m0 + 16 * i + 4 * g4, fmaxf(v[0], 0.f), fmaxf(v[1], 0.f),
                  fmaxf(v[2], 0.f), fmaxf(v[3], 0.f));
        }
    }
    __syncthreads();
    // -------------------------------------------------------------- P2: layer 2 (+ b1) -> H2 (over X)
    bf16_t* sH2 = sX;
    {
      f4v acc[MT][NET];
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int n = 0; n < NET; ++n) acc[i][n] = zero4();
#pragma unroll
      for (int ks = 0; ks < KS1; ++ks) {
        s8v b[NET];
#pragma unroll
        for (int n = 0; n < NET; ++n) b[n] = lds_ld8(sH1 + (16 * n + l16) * SH + ks * 32 + 8 * g4);
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
          for (int n = 0; n < NET; ++n) acc[i][n] = mfma32(aW1[i][ks], b[n], acc[i][n]);
      }
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int n = 0; n < NET; ++n) {
          const f4v v = acc[i][n];
          lds_st4(sH2 + (16 * n + l16) * SH + m0 + 16 * i + 4 * g4, fmaxf(v[0] + bb[i][0], 0.f),
                  fmaxf(v[1] + bb[i][1], 0.f), fmaxf(v[2] + bb[i][2], 0.f), fmaxf(v[3] + bb[i][3], 0.f));
        }
    }
    __syncthreads();
    // -------------------------------------------------------------- P3: output, argmax, epsilon-greedy
    {
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
          const bool exploit = u1 < fminf(p.eps, __fmul_rn(p.steps[row], p.inv_ramp));
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
    __syncthreads();   // the next tile's features overwrite X / H2
  }
}

}  // namespace serve
}  // namespace st

extern "C" int st_qserve_lds_bytes() { return st::serve::LDS_BYTES; }

// grid <= 0: min(tiles, 2 x CUs).  Pre-launch checks: the padded dims are fixed (224 / 128 / 16) and the
// request rows must hold H + 2 values with H + 3 <= 224 (prices, budget, shares, constant 1).
extern "C" hipError_t st_qserve_launch(const st::serve::ServeParams* p, int grid, hipStream_t stream) {
  using namespace st::serve;
  if (p->B <= 0) return hipSuccess;
  if (p->H < 2 || p->H + 3 > INP || p->ld < p->H + 2 || p->states == nullptr || p->actions == nullptr ||
      p->wq == nullptr || p->wf == nullptr || (long long)p->B * p->ld >= (1LL << 30))
    return hipErrorInvalidValue;
  const bool vec = (p->ld % 4 == 0) && ((reinterpret_cast<uintptr_t>(p->states) & 15) == 0);
  const int ntiles = (p->B + C - 1) / C;
  if (grid <= 0) {
    int dev = 0, cus = 256;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    grid = 2 * cus;
  }
  if (grid > ntiles) grid = ntiles;
  if (vec)
    hipLaunchKernelGGL(qserve_kernel<true>, dim3(grid), dim3(NT), LDS_BYTES, stream, *p);
  else
    hipLaunchKernelGGL(qserve_kernel<false>, dim3(grid), dim3(NT), LDS_BYTES, stream, *p);
  return hipGetLastError();
}
