// Fused online-DQN engine step for E vectorised trading envs on CDNA4 (gfx950).
//
// One launch = one environment step of every env on this GPU plus the local
// part of the learner update:
//
//   gather state windows (Hankel addressing into the HBM-resident price bank)
//   -> Q(x_t) forward (MFMA)  -> epsilon-greedy action (Philox, in-kernel)
//   -> Buy/Sell/Hold env step + reward        (TrainerChildActor.scala:118-146)
//   -> Q(x_{t+1}) forward     -> TD target    (QDecisionPolicyActor.scala:67-71)
//   -> (y - q)^2 backward     -> per-workgroup weight-gradient accumulation
//
// The reference performs the same sequence as ~6 JNI TF session calls per
// step per worker, serialized through one actor mailbox.
//
// Design (MI355X-first):
//  * one 256-thread workgroup (4 waves, one per SIMD) per CU, persistent over
//    chunks of C=32 envs; the bf16 weights (~94 KB) stay resident in LDS for
//    the whole launch, activations of a chunk never leave LDS;
//  * "transposed orientation": every product is out^T = W^T . act^T so that
//    forward and backward-data products read both operands as 16-byte row
//    fragments (ds_read_b128) of row-major images, and accumulator tiles store
//    back as one 8-byte ds_write per lane; weight-gradient products (sum over
//    envs) read both operands with the gfx950 hardware transpose read
//    ds_read_b64_tr_b16 from the same images — no second copy of anything;
//  * v_mfma_f32_16x16x32_bf16 for all K>=32 products, 16x16x16 for K=16;
//  * weight gradients stay in accumulator registers across all chunks of the
//    workgroup (~190 VGPR/lane) and are written once per launch into a
//    per-workgroup fp32 slab that optim.hip reduces (and RCCL all-reduces).
#include "common.h"

namespace st {

constexpr int C = 32;       // envs per chunk
constexpr int NT = 512;     // threads per workgroup: 8 waves = 2 per SIMD (latency hiding for the
                            // instruction-bound gather / env phases; see profiles/)
constexpr int NW = NT / 64;
constexpr int OUTP = 16;    // padded action dimension
constexpr int SQ = OUTP + 8;
constexpr int NSTAT = 8;

// The launch parameters of this kernel: the leading fields of st::QStepParams (csrc/qstep.h) up to td_clip, in the
// same order -- the host passes its one QStepParams mirror (sharetrade/ops/native.py) to st_qstep_launch, and this
// kernel reads the prefix (pinned by tests/test_abi.py).  Its own name: one definition per struct in the library.
struct FusedStepParams {
  const float* prices;      // [E, T] env-major
  const float* prices4;     // [4][E][T4] shifted replicas (series.hip: replicate4)
  // env state + per-step outputs as ONE struct-of-arrays buffer [ENV_ROWS][E] of 4-byte
  // words (rows below): one base pointer instead of nine keeps the kernel's scalar
  // registers from spilling across the chunk loop
  int* env;
  const bf16_t* wq;         // bf16 flat params (kernel layout)
  const float* wf;          // fp32 flat params (biases read from here)
  float* slab;              // [G][P] per-workgroup partial gradients
  float* stats;             // [G][NSTAT]
  unsigned long long* ctrl;   // ctrl[0] = step index (read), ctrl[1] = step+1 (written by block 0)
  int T, E, H, P, T4;
  int off_w0, off_w1, off_b1, off_w2, off_b2;
  float eps, inv_ramp, gamma, loss_coef, b0, inv_b0;
  int s0, compat_env, target_compat, output_relu, feat_mode;
  uint32_t key0, key1;
  int env_offset;
  unsigned long long* stamps;  // debug: s_memtime per phase of workgroup 0 ([iter][16]) or null
  int slab_bf16, slab_rows;    // (64-env-chunk kernel fields, csrc/qstep.h: same layout)
  unsigned* chunk_heads;
  int reward_mode;             // 0: reward = change of portfolio value; 1: its one-step return
  float td_clip;               // > 0: TD error clamped to [-td_clip, td_clip] (Huber loss)
};

// rows of FusedStepParams::env
enum EnvRow : int { ER_POS = 0, ER_BUDGET, ER_SHARES, ER_VALUE, ER_RET_SUM, ER_EPISODES, ER_LAST_FINAL,
                    ER_ACTION, ER_REWARD, ENV_ROWS };
#define ENV_I(R, e) (p.env[(size_t)(R) * p.E + (e)])
#define ENV_F(R, e) (reinterpret_cast<float*>(p.env)[(size_t)(R) * p.E + (e)])

template <int INP, int H1P, int H2P>
struct Geo {
  // weight images: +8 bf16 row padding; activation images (the hot MFMA B-operand row
  // reads): +16, which makes the 16x16x32 fragment reads bank-conflict-free (stride search
  // in tools/, transposed reads stay 2-way either way)
  static constexpr int SW0 = INP + 8, SW1 = H1P + 8, SW2 = H2P + 8;
  static constexpr int SX = INP + 16, SH1 = H1P + 16, SH2 = H2P + 16;
  static constexpr int oW0 = 0;
  static constexpr int oW1 = oW0 + H1P * SW0;
  static constexpr int oW2 = oW1 + H2P * SW1;
  static constexpr int oX = oW2 + OUTP * SW2;
  static constexpr int oH1 = oX + C * SX;
  static constexpr int oH2 = oH1 + C * SH1;
  static constexpr int oR0 = oH2 + C * SH2;          // X' / H2' / dZ2
  static constexpr int R0SZ = (C * SX > C * SH2) ? C * SX : C * SH2;
  static constexpr int oR1 = oR0 + R0SZ;             // H1' / dZ1
  static constexpr int oDQ = oR1 + C * SH1;
  static constexpr int BF16_END = oDQ + C * SQ;
  // fp32 region (byte offsets)
  static constexpr int fQ = BF16_END * 2;            // q(x)   [C][4]
  static constexpr int fQN = fQ + C * 4 * 4;         // q(x')  [C][4]
  static constexpr int fENV = fQN + C * 4 * 4;       // [C][8] floats
  static constexpr int fENVI = fENV + C * 8 * 4;     // [C][4] ints
  static constexpr int fB1 = fENVI + C * 4 * 4;      // b1 [H2P]
  static constexpr int fB2 = fB1 + H2P * 4;          // b2 [16]
  static constexpr int BYTES = fB2 + OUTP * 4;
  static_assert(BYTES <= 163840, "LDS budget exceeded");
  static_assert(INP % 32 == 0 && H1P % (16 * NW) == 0 && H2P % (16 * NW) == 0, "padding");
  static constexpr int MT1 = H1P / (16 * NW);   // h1 m-tiles per wave
  static constexpr int MT2 = H2P / (16 * NW);   // h2 m-tiles per wave
  static constexpr int NT0 = INP / 16 - 1;  // in-col tiles of dW0 (last tile is pure padding)
  static constexpr int NT1 = H1P / 16;
};

// A/B fragment from a row-major image: rows r0 + l16, k = k0 + 8*g4 .. +7
ST_DEV s8v frag_row(const bf16_t* img, int S, int r0, int k0, int l16, int g4) {
  return lds_ld8(img + (r0 + l16) * S + k0 + 8 * g4);
}
// Fragment with k running down the image rows (hardware transpose read):
// element j of lane (g4, l16) = img[k0 + 8*g4 + j][c0 + l16]
ST_DEV s8v frag_tr(const bf16_t* img, int S, int k0, int c0, int l16, int g4) {
  const bf16_t* p = img + (k0 + 8 * g4 + (l16 >> 2)) * S + c0 + 4 * (l16 & 3);
  s4v lo = lds_tr4(p);
  s4v hi = lds_tr4(p + 4 * S);
  s8v r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}

// value of lane+1 (lane 63 gets 0): DPP wave_shl:1 — one VALU op instead of a ds_bpermute
ST_DEV float dpp_next_lane(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x130, 0xF, 0xF, true));
}

ST_DEV float feat_price(float w, float inv, int mode) {
  return mode ? __fsub_rn(__fmul_rn(w, inv), 1.0f) : w;
}
ST_DEV float feat_budget(float b, float inv_b0, int mode) { return mode ? __fmul_rn(b, inv_b0) : b; }
ST_DEV float feat_shares(int s, float last, float inv_b0, int mode) {
  return mode ? __fmul_rn(__fmul_rn((float)s, last), inv_b0) : (float)s;
}

// out^T[m][env] = sum_k A[m][k] * act[env][k]   (A = W^T image), MT m-tiles per wave x 2 env tiles.
// Epilogue: + bias (fp32 LDS or none), ReLU, bf16 store into out image [env][m].
template <int K, int SA, int SB, int SO, int MT>
ST_DEV void fwd_hidden(const bf16_t* sA, const bf16_t* sB, bf16_t* sO, const float* bias, int mbase,
                       int l16, int g4) {
  f4v acc[MT][2];
#pragma unroll
  for (int i = 0; i < MT; ++i) { acc[i][0] = zero4(); acc[i][1] = zero4(); }
#pragma unroll
  for (int ks = 0; ks < K / 32; ++ks) {
    s8v b0 = frag_row(sB, SB, 0, ks * 32, l16, g4);
    s8v b1 = frag_row(sB, SB, 16, ks * 32, l16, g4);
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      s8v a = frag_row(sA, SA, mbase + 16 * i, ks * 32, l16, g4);
      acc[i][0] = mfma32(a, b0, acc[i][0]);
      acc[i][1] = mfma32(a, b1, acc[i][1]);
    }
  }
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int m = mbase + 16 * i + 4 * g4;
    float bb[4] = {0.f, 0.f, 0.f, 0.f};
    if (bias) { bb[0] = bias[m]; bb[1] = bias[m + 1]; bb[2] = bias[m + 2]; bb[3] = bias[m + 3]; }
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      f4v v = acc[i][n];
      lds_st4(sO + (16 * n + l16) * SO + m, fmaxf(v[0] + bb[0], 0.f), fmaxf(v[1] + bb[1], 0.f),
              fmaxf(v[2] + bb[2], 0.f), fmaxf(v[3] + bb[3], 0.f));
    }
  }
}

// Output layer: q^T[a][env] for the wave's env tile (waves 0,1). q -> fp32 LDS [env][4].
template <int K, int SA, int SB>
ST_DEV void fwd_out(const bf16_t* sA, const bf16_t* sB, float* sQout, const float* b2, int relu, int ntile,
                    int l16, int g4) {
  f4v acc = zero4();
#pragma unroll
  for (int ks = 0; ks < K / 32; ++ks) {
    s8v a = frag_row(sA, SA, 0, ks * 32, l16, g4);
    s8v b = frag_row(sB, SB, 16 * ntile, ks * 32, l16, g4);
    acc = mfma32(a, b, acc);
  }
  if (g4 == 0) {
    const int env = 16 * ntile + l16;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      float q = acc[j] + b2[j];
      if (relu) q = fmaxf(q, 0.f);
      sQout[env * 4 + j] = q;
    }
  }
}

// dA^T[m][env] = sum_k W[m][k] * dZ[env][k], W read transposed from the W^T image [k][m];
// masked by (act[env][m] > 0); bf16 store into out image [env][m].
template <int K, int SW, int SD, int SACT, int SO, int MT>
ST_DEV void bwd_data(const bf16_t* sWT, const bf16_t* sDZ, const bf16_t* sAct, bf16_t* sO, int mbase, int l16,
                     int g4) {
  f4v acc[MT][2];
#pragma unroll
  for (int i = 0; i < MT; ++i) { acc[i][0] = zero4(); acc[i][1] = zero4(); }
  if constexpr (K == 16) {
    s4v b0 = lds_ld4(sDZ + (0 + l16) * SD + 4 * g4);
    s4v b1 = lds_ld4(sDZ + (16 + l16) * SD + 4 * g4);
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      s4v a = lds_tr4(sWT + (4 * g4 + (l16 >> 2)) * SW + mbase + 16 * i + 4 * (l16 & 3));
      acc[i][0] = mfma16(a, b0, acc[i][0]);
      acc[i][1] = mfma16(a, b1, acc[i][1]);
    }
  } else {
#pragma unroll
    for (int ks = 0; ks < K / 32; ++ks) {
      s8v b0 = frag_row(sDZ, SD, 0, ks * 32, l16, g4);
      s8v b1 = frag_row(sDZ, SD, 16, ks * 32, l16, g4);
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        s8v a = frag_tr(sWT, SW, ks * 32, mbase + 16 * i, l16, g4);
        acc[i][0] = mfma32(a, b0, acc[i][0]);
        acc[i][1] = mfma32(a, b1, acc[i][1]);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int m = mbase + 16 * i + 4 * g4;
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      const int env = 16 * n + l16;
      const s4v h = lds_ld4(sAct + env * SACT + m);
      f4v v = acc[i][n];
      lds_st4(sO + env * SO + m, h[0] > 0 ? v[0] : 0.f, h[1] > 0 ? v[1] : 0.f, h[2] > 0 ? v[2] : 0.f,
              h[3] > 0 ? v[3] : 0.f);
    }
  }
}

template <int INP, int H1P, int H2P, int FEAT>
__global__ void __launch_bounds__(NT, 2) qstep_fused_kernel(FusedStepParams p) {
  using G = Geo<INP, H1P, H2P>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* sbf = reinterpret_cast<bf16_t*>(smem);
  bf16_t* sW0 = sbf + G::oW0;
  bf16_t* sW1 = sbf + G::oW1;
  bf16_t* sW2 = sbf + G::oW2;
  bf16_t* sX = sbf + G::oX;
  bf16_t* sH1 = sbf + G::oH1;
  bf16_t* sH2 = sbf + G::oH2;
  bf16_t* sR0 = sbf + G::oR0;
  bf16_t* sR1 = sbf + G::oR1;
  bf16_t* sDQ = sbf + G::oDQ;
  float* sQ = reinterpret_cast<float*>(smem + G::fQ);
  float* sQN = reinterpret_cast<float*>(smem + G::fQN);
  float* sEnv = reinterpret_cast<float*>(smem + G::fENV);
  int* sEnvI = reinterpret_cast<int*>(smem + G::fENVI);
  float* sB1 = reinterpret_cast<float*>(smem + G::fB1);
  float* sB2 = reinterpret_cast<float*>(smem + G::fB2);

  const int tid = threadIdx.x, lane = tid & 63, l16 = lane & 15, g4 = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // scalar: wave-specialised phases branch, not mask
  const int H = p.H;
  const unsigned long long step = p.ctrl[0];

  // ---------------------------------------------------------------- weights -> LDS (once)
  {
    const bf16_t* w0 = p.wq + p.off_w0;
    for (int i = tid; i < H1P * INP / 8; i += NT) {
      const int r = i / (INP / 8), c = (i % (INP / 8)) * 8;
      *reinterpret_cast<uint4*>(sW0 + r * G::SW0 + c) = *reinterpret_cast<const uint4*>(w0 + r * INP + c);
    }
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
  }

  // ---------------------------------------------------------------- gradient accumulators
  constexpr int MT1 = G::MT1, MT2 = G::MT2, NT0 = G::NT0, NT1 = G::NT1;
  f4v gW0[MT1][NT0];
  f4v gW1[MT2][NT1];
  f4v gB1[MT2];
  f4v gW2[MT2];
  f4v gB2;
#pragma unroll
  for (int i = 0; i < MT1; ++i)
#pragma unroll
    for (int n = 0; n < NT0; ++n) gW0[i][n] = zero4();
#pragma unroll
  for (int i = 0; i < MT2; ++i) {
#pragma unroll
    for (int n = 0; n < NT1; ++n) gW1[i][n] = zero4();
    gB1[i] = zero4();
    gW2[i] = zero4();
  }
  gB2 = zero4();
  // ones fragment for bias gradients: B[k][n] = (n == 0)
  s8v ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (l16 == 0) ? (short)0x3F80 : (short)0;

  float st_reward = 0.f, st_loss = 0.f, st_explore = 0.f, st_done = 0.f, st_fsum = 0.f, st_fsq = 0.f,
        st_qslot = 0.f;

  const int nchunks = p.E / C;
  constexpr int RPW = C / NW;
  int iter = 0;
#define ST_STAMP(I) \
  if (p.stamps != nullptr && blockIdx.x == 0 && tid == 0) p.stamps[iter * 16 + (I)] = __builtin_amdgcn_s_memtime();  // rows (envs) per wave in the gather

  // ---------------------------------------------------------------- software-pipelined gather
  // Global traffic of a chunk is a dependent chain (pos -> price window), so it is
  // issued ahead: the env state of chunk i+1 is loaded while chunk i is processed
  // (lanes 0..RPW-1 of each wave own one row each), and chunk i+1's price windows
  // are issued right after chunk i's gather, landing during chunk i's MFMA phases.
  int eA_pos = 0, eA_sh = 0, eA_ep = 0, eB_pos = 0, eB_sh = 0, eB_ep = 0;
  float eA_b = 0.f, eA_val = 0.f, eA_rs = 0.f, eB_b = 0.f, eB_val = 0.f, eB_rs = 0.f;
  float4 w[RPW];              // lane L: prices[ps + 4L .. ps + 4L + 3] of each of the wave's rows
  float wl = 0.f, wv = 0.f;   // lane rr < RPW: prices[pos + H - 1] and prices[pos + H] of row rr
// All gather loads are unconditional (chunk and lane indices clamped instead of branched on):
// exec-masked loads merge with the destination's old value, and the compiler then has to
// drain vmcnt before reusing the register - which serialised the whole prefetch.
#define ST_LOAD_ENV(CH, POS, B, SH, VAL, RS, EP)                           \
  {                                                                        \
    const int ch_ = min((CH), nchunks - 1);                                \
    const int e_ = ch_ * C + wave * RPW + min(lane, RPW - 1);              \
    POS = ENV_I(ER_POS, e_); B = ENV_F(ER_BUDGET, e_); SH = ENV_I(ER_SHARES, e_);                  \
    VAL = ENV_F(ER_VALUE, e_); RS = ENV_F(ER_RET_SUM, e_); EP = ENV_I(ER_EPISODES, e_);            \
  }
// One dwordx4 per lane per row: the window [ps, ps+H] is a run of aligned float4s in the
// shifted replica ps & 3 of the bank (1 KiB contiguous per wave-instruction, no realignment).
#define ST_LOAD_PRICES(CH, POS)                                            \
  {                                                                        \
    const int ch_ = min((CH), nchunks - 1);                                \
    /* each lane forms its own row's 64-bit replica pointer in VALU; the   \
       per-row loads then only readlane the two halves (no SALU chains) */ \
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
      w[rr] = make_float4(v_.x, v_.y, v_.z, v_.w);   /* replicas are tail-padded */ \
    }                                                                      \
    const float* pl_ = p.prices +                                          \
        (size_t)(ch_ * C + wave * RPW + min(lane, RPW - 1)) * p.T + (POS) + H; \
    wl = pl_[-1];                                                          \
    wv = pl_[0];                                                           \
  }
  ST_LOAD_ENV(blockIdx.x, eA_pos, eA_b, eA_sh, eA_val, eA_rs, eA_ep)
  ST_LOAD_PRICES(blockIdx.x, eA_pos)
  ST_LOAD_ENV(blockIdx.x + gridDim.x, eB_pos, eB_b, eB_sh, eB_val, eB_rs, eB_ep)
  __syncthreads();

  for (int chunk = blockIdx.x; chunk < nchunks; chunk += gridDim.x) {
    ST_STAMP(0);
    if (p.stamps != nullptr) {  // debug only: split P0 into (wait for prefetched data) + (work)
      __builtin_amdgcn_s_waitcnt(0);
      ST_STAMP(8);
    }
    const int ebase = chunk * C;
    // ------------------------------------------------------------ P0: gather windows (from registers)
    if (lane < RPW) {
      const int r = wave * RPW + lane;
      sEnv[r * 8 + 0] = eA_b;
      sEnv[r * 8 + 1] = eA_val;
      sEnv[r * 8 + 5] = eA_rs;
      sEnvI[r * 4 + 0] = eA_pos;
      sEnvI[r * 4 + 1] = eA_sh;
      sEnvI[r * 4 + 3] = eA_ep;
    }
    // per-row scalars: lane rr < RPW computes row rr's (1/last, 1/vnew, budget & shares features)
    float r_inv = 0.f, r_invn = 0.f, r_fb = 0.f, r_fs = 0.f;
    if (lane < RPW) {
      r_inv = __fdiv_rn(1.0f, wl);
      r_invn = __fdiv_rn(1.0f, wv);
      r_fb = feat_budget(eA_b, p.inv_b0, FEAT);
      r_fs = feat_shares(eA_sh, wl, p.inv_b0, FEAT);
    }
    // lane L owns window columns k = 4L..4L+3: branch-free features, one 8-byte LDS store per row
    // for x and one for x' (x'[k] = f(prices[k+1]) takes its 4th value from lane L+1)
#pragma unroll
    for (int rr = 0; rr < RPW; ++rr) {
      const int r = wave * RPW + rr;
      const float inv = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(r_inv), rr));
      const float invn = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(r_invn), rr));
      const float fb = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(r_fb), rr));
      const float fs = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(r_fs), rr));
      const float vnew = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(wv), rr));
      // prices[ps + 4L + t], t = 0..4 (t = 4 from lane L+1 via DPP)
      const float win[5] = {w[rr].x, w[rr].y, w[rr].z, w[rr].w, dpp_next_lane(w[rr].x)};
      float xv[4], xnv[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int k = 4 * lane + j;
        // every candidate is materialised first (empty asm pins it) so that the
        // per-lane choice is a v_cndmask, not a divergent branch around 2 VALU ops
        float fp = feat_price(win[j], inv, FEAT);
        float fpn = feat_price(win[j + 1], invn, FEAT);
        float sp = (k == H) ? fb : (k == H + 1) ? fs : (k == H + 2) ? 1.0f : 0.f;
        asm volatile("" : "+v"(fp), "+v"(fpn), "+v"(sp));
        xv[j] = (k < H) ? fp : sp;
        xnv[j] = (k < H) ? fpn : 0.f;
      }
      if (lane < INP / 4) {
        lds_st4(sX + r * G::SX + 4 * lane, xv[0], xv[1], xv[2], xv[3]);
        lds_st4(sR0 + r * G::SX + 4 * lane, xnv[0], xnv[1], xnv[2], xnv[3]);
      }
      if (lane == 0) sEnv[r * 8 + 2] = vnew;
    }
    ST_STAMP(9);
    // next chunk's price windows (its env state arrived during this chunk's predecessor)
    {
      const int nxt = chunk + gridDim.x;
      ST_LOAD_PRICES(nxt, eB_pos)
      eA_pos = eB_pos; eA_b = eB_b; eA_sh = eB_sh; eA_val = eB_val; eA_rs = eB_rs; eA_ep = eB_ep;
      ST_LOAD_ENV(nxt + gridDim.x, eB_pos, eB_b, eB_sh, eB_val, eB_rs, eB_ep)
    }
    ST_STAMP(10);
    __syncthreads();
    ST_STAMP(1);
    // ------------------------------------------------------------ P1-P3: forward Q(x)
    fwd_hidden<INP, G::SW0, G::SX, G::SH1, MT1>(sW0, sX, sH1, nullptr, wave * 16 * MT1, l16, g4);
    __syncthreads();
    fwd_hidden<H1P, G::SW1, G::SH1, G::SH2, MT2>(sW1, sH1, sH2, sB1, wave * 16 * MT2, l16, g4);
    __syncthreads();
    if (wave < 2) fwd_out<H2P, G::SW2, G::SH2>(sW2, sH2, sQ, sB2, p.output_relu, wave, l16, g4);
    __syncthreads();
    ST_STAMP(2);
    // ------------------------------------------------------------ P4: epsilon-greedy + env step
    if (wave == 0 && lane < C) {
      const int r = lane, e = ebase + r;
      const float q0 = sQ[r * 4 + 0], q1 = sQ[r * 4 + 1], q2 = sQ[r * 4 + 2];
      int greedy = 0;
      float best = q0;
      if (q1 > best) { best = q1; greedy = 1; }
      if (q2 > best) { best = q2; greedy = 2; }
      const int ps = sEnvI[r * 4 + 0];
      uint32_t c0 = (uint32_t)(p.env_offset + e), c1 = (uint32_t)(step & 0xFFFFFFFFull),
               c2 = (uint32_t)(step >> 32), c3 = 0u;
      philox4x32(c0, c1, c2, c3, p.key0, p.key1);
      const float u1 = u24(c0), u2 = u24(c1);
      const bool exploit = u1 < fminf(p.eps, __fmul_rn((float)ps, p.inv_ramp));
      int rnd = (int)(u2 * 3.0f);
      rnd = rnd > 2 ? 2 : rnd;
      const int a = exploit ? greedy : rnd;
      const float b = sEnv[r * 8 + 0], vprev = sEnv[r * 8 + 1], vnew = sEnv[r * 8 + 2];
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
      sEnv[r * 8 + 3] = b2;
      sEnv[r * 8 + 4] = rew;
      sEnvI[r * 4 + 1] = s2;
      sEnvI[r * 4 + 2] = a;
      bf16_t* xn = sR0 + r * G::SX;
      xn[H] = f2bf(feat_budget(b2, p.inv_b0, FEAT));
      xn[H + 1] = f2bf(feat_shares(s2, vnew, p.inv_b0, FEAT));
      xn[H + 2] = f2bf(1.0f);
      st_explore += exploit ? 0.f : 1.f;
      ENV_I(ER_ACTION, e) = a;
      ENV_F(ER_REWARD, e) = rew;
    }
    __syncthreads();
    ST_STAMP(3);
    // ------------------------------------------------------------ P5-P7: forward Q(x')
    fwd_hidden<INP, G::SW0, G::SX, G::SH1, MT1>(sW0, sR0, sR1, nullptr, wave * 16 * MT1, l16, g4);
    __syncthreads();
    fwd_hidden<H1P, G::SW1, G::SH1, G::SH2, MT2>(sW1, sR1, sR0, sB1, wave * 16 * MT2, l16, g4);
    __syncthreads();
    if (wave < 2) fwd_out<H2P, G::SW2, G::SH2>(sW2, sR0, sQN, sB2, p.output_relu, wave, l16, g4);
    __syncthreads();
    ST_STAMP(4);
    // ------------------------------------------------------------ P8: TD target, dQ, state write-back
    if (wave == 0 && lane < C) {
      const int r = lane, e = ebase + r;
      const float n0 = sQN[r * 4 + 0], n1 = sQN[r * 4 + 1], n2 = sQN[r * 4 + 2];
      int am = 0;
      float mx = n0;
      if (n1 > mx) { mx = n1; am = 1; }
      if (n2 > mx) { mx = n2; am = 2; }
      const int a = sEnvI[r * 4 + 2];
      const float rew = sEnv[r * 8 + 4];
      const int slot = p.target_compat ? am : a;
      const float y = __fadd_rn(rew, __fmul_rn(p.gamma, mx));
      const float qs = sQ[r * 4 + slot];
      const float diff = __fsub_rn(qs, y);
      float dq = p.loss_coef * (p.td_clip > 0.f ? fminf(fmaxf(diff, -p.td_clip), p.td_clip) : diff);
      if (p.output_relu && !(qs > 0.f)) dq = 0.f;
      bf16_t* dqr = sDQ + r * SQ;
#pragma unroll
      for (int j = 0; j < OUTP; ++j) dqr[j] = (j == slot) ? f2bf(dq) : (bf16_t)0;
      st_loss += diff * diff;
      st_reward += rew;
      st_qslot += qs;
      // env state write-back
      const float b2 = sEnv[r * 8 + 3], vnew = sEnv[r * 8 + 2];
      const int s2 = sEnvI[r * 4 + 1];
      const int np = sEnvI[r * 4 + 0] + 1;
      const float rs = sEnv[r * 8 + 5] + rew;
      if (np >= p.T - H) {
        const float fin = __fadd_rn(b2, __fmul_rn((float)s2, vnew));
        ENV_F(ER_LAST_FINAL, e) = fin;
        ENV_I(ER_EPISODES, e) = sEnvI[r * 4 + 3] + 1;
        ENV_F(ER_BUDGET, e) = p.b0;
        ENV_I(ER_SHARES, e) = p.s0;
        ENV_F(ER_VALUE, e) = 0.f;
        ENV_I(ER_POS, e) = 0;
        ENV_F(ER_RET_SUM, e) = 0.f;
        st_done += 1.f;
        st_fsum += fin;
        st_fsq += fin * fin;
      } else {
        ENV_F(ER_BUDGET, e) = b2;
        ENV_I(ER_SHARES, e) = s2;
        ENV_F(ER_VALUE, e) = vnew;
        ENV_I(ER_POS, e) = np;
        ENV_F(ER_RET_SUM, e) = rs;
      }
    }
    __syncthreads();
    ST_STAMP(5);
    // ------------------------------------------------------------ P9-P10: backward (data)
    bwd_data<OUTP, G::SW2, SQ, G::SH2, G::SH2, MT2>(sW2, sDQ, sH2, sR0, wave * 16 * MT2, l16, g4);
    __syncthreads();
    bwd_data<H2P, G::SW1, G::SH2, G::SH1, G::SH1, MT1>(sW1, sR0, sH1, sR1, wave * 16 * MT1, l16, g4);
    __syncthreads();
    ST_STAMP(6);
    // ------------------------------------------------------------ P11: weight gradients (sum over envs)
    {
      // dW0^T[h1][in] += dZ1^T . X
#pragma unroll
      for (int i = 0; i < MT1; ++i) {
        const s8v a = frag_tr(sR1, G::SH1, 0, (wave * MT1 + i) * 16, l16, g4);
#pragma unroll
        for (int n = 0; n < NT0; ++n) {
          const s8v bx = frag_tr(sX, G::SX, 0, n * 16, l16, g4);
          gW0[i][n] = mfma32(a, bx, gW0[i][n]);
        }
      }
      // dW1^T[h2][h1] += dZ2^T . H1 ; db1 += dZ2^T . 1
#pragma unroll
      for (int i = 0; i < MT2; ++i) {
        const s8v a = frag_tr(sR0, G::SH2, 0, (wave * MT2 + i) * 16, l16, g4);
#pragma unroll
        for (int n = 0; n < NT1; ++n) {
          const s8v bh = frag_tr(sH1, G::SH1, 0, n * 16, l16, g4);
          gW1[i][n] = mfma32(a, bh, gW1[i][n]);
        }
        gB1[i] = mfma32(a, ones, gB1[i]);
      }
      // dW2^T[out][h2] += dQ^T . H2 ; db2 += dQ^T . 1
      const s8v aq = frag_tr(sDQ, SQ, 0, 0, l16, g4);
#pragma unroll
      for (int i = 0; i < MT2; ++i) {
        const s8v bh = frag_tr(sH2, G::SH2, 0, (wave * MT2 + i) * 16, l16, g4);
        gW2[i] = mfma32(aq, bh, gW2[i]);
      }
      if (wave == 0) gB2 = mfma32(aq, ones, gB2);
    }
    __syncthreads();
    ST_STAMP(7);
    ++iter;
  }

  // ---------------------------------------------------------------- gradient slab write-out
  float* sl = p.slab + (size_t)blockIdx.x * p.P;
#pragma unroll
  for (int i = 0; i < MT1; ++i) {
    const int h = (wave * MT1 + i) * 16 + 4 * g4;
#pragma unroll
    for (int n = 0; n < NT0; ++n)
#pragma unroll
      for (int j = 0; j < 4; ++j) sl[p.off_w0 + (h + j) * INP + n * 16 + l16] = gW0[i][n][j];
  }
#pragma unroll
  for (int i = 0; i < MT2; ++i) {
    const int h = (wave * MT2 + i) * 16 + 4 * g4;
#pragma unroll
    for (int n = 0; n < NT1; ++n)
#pragma unroll
      for (int j = 0; j < 4; ++j) sl[p.off_w1 + (h + j) * H1P + n * 16 + l16] = gW1[i][n][j];
    if (l16 == 0)
#pragma unroll
      for (int j = 0; j < 4; ++j) sl[p.off_b1 + h + j] = gB1[i][j];
#pragma unroll
    for (int j = 0; j < 4; ++j) sl[p.off_w2 + (4 * g4 + j) * H2P + (wave * MT2 + i) * 16 + l16] = gW2[i][j];
  }
  if (wave == 0 && l16 == 0)
#pragma unroll
    for (int j = 0; j < 4; ++j) sl[p.off_b2 + 4 * g4 + j] = gB2[j];

  if (blockIdx.x == 0 && tid == 0) p.ctrl[1] = step + 1;  // 1-based update count for the optimizer
  // ---------------------------------------------------------------- per-workgroup stats
  if (wave == 0) {
    const float v0 = wave_sum(st_reward), v1 = wave_sum(st_loss), v2 = wave_sum(st_explore),
                v3 = wave_sum(st_done), v4 = wave_sum(st_fsum), v5 = wave_sum(st_fsq), v6 = wave_sum(st_qslot);
    if (lane == 0) {
      float* so = p.stats + (size_t)blockIdx.x * NSTAT;
      so[0] = v0; so[1] = v1; so[2] = v2; so[3] = v3; so[4] = v4; so[5] = v5; so[6] = v6; so[7] = 0.f;
    }
  }
}

template <int INP, int H1P, int H2P, int FEAT>
static hipError_t launch_f(const FusedStepParams& p, int grid, hipStream_t stream) {
  using G = Geo<INP, H1P, H2P>;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)qstep_fused_kernel<INP, H1P, H2P, FEAT>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, G::BYTES);
    if (e != hipSuccess) return e;
    attr = true;
  }
  hipLaunchKernelGGL((qstep_fused_kernel<INP, H1P, H2P, FEAT>), dim3(grid), dim3(NT), G::BYTES, stream, p);
  return hipGetLastError();
}

template <int INP, int H1P, int H2P>
static hipError_t launch_t(const FusedStepParams& p, int grid, hipStream_t stream) {
  return p.feat_mode ? launch_f<INP, H1P, H2P, 1>(p, grid, stream) : launch_f<INP, H1P, H2P, 0>(p, grid, stream);
}

}  // namespace st

extern "C" int st_qstep_lds_bytes(int inp, int h1p, int h2p) {
  if (inp == 224 && h1p == 128 && h2p == 128) return st::Geo<224, 128, 128>::BYTES;
  return -1;
}

extern "C" hipError_t st_qstep_launch(const st::FusedStepParams* p, int inp, int h1p, int h2p, int grid,
                                      hipStream_t stream) {
  if (inp == 224 && h1p == 128 && h2p == 128) return st::launch_t<224, 128, 128>(*p, grid, stream);
  return hipErrorInvalidValue;
}

// struct sizes of this file's launch ABI, for the host mirrors' check (tests/test_abi.py; no HIP call)
extern "C" int st_abi_qstep_fused(int* out, int n) {
  const int sz[] = {(int)sizeof(st::FusedStepParams)};
  const int m = (int)(sizeof(sz) / sizeof(sz[0]));
  for (int i = 0; i < n && i < m; ++i) out[i] = sz[i];
  return m;
}
