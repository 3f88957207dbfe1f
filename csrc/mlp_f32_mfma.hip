// Batched exact-fp32 engine step on the matrix cores: the reference network's geometry (203 -> 200 -> 3,
// QDecisionPolicyActor.scala:18-22,41-50) -- and any fp32 MLP of the flat layout up to 6 layers -- for
// a LARGE number of vectorised envs (VectorEngine, engine.dtype = "fp32").
//
// csrc/mlp_f32.hip steps every env in its own workgroup with GEMVs on the VALU (right at batch 1..a few
// hundred: an MFMA tile would be >93 % padding).  With thousands of envs that re-reads every weight
// matrix once per env and sums the weight gradient with one thread per parameter over all envs.  Here
// the step is a short chain of launches over all envs at once (graph-captured by the engine):
//
//   f32b_gather   X, X' [E][in_p] from the HBM price bank + env state (features, layer-0 bias column)
//   GEMM          A_{l+1} = relu(A_l . W_l^T + b_l)   for x; last layer -> Q [E][16]
//                 (two-layer nets from 8,192 envs: f32b_fwd2, both layers in one launch)
//   f32b_env      epsilon-greedy (Philox) + Buy/Sell/Hold step: budget / shares columns of X'
//   GEMM          the same forward for x' -> Q' (and, with a target network, for x' on the target copy)
//   f32b_td       TD target (online / target / Double-DQN bootstrap), dQ (one-hot at the target slot),
//                 loss, env write-back, step statistics
//   GEMM          dZ_{l-1} = (dZ_l . W_l) * [A_l > 0]                       (backward, data)
//   GEMM          dW_l^T += dZ_l^T . A_l  (split-K over envs: fp32 atomics, or partial tiles +
//                 f32b_splitsum)                                             (weight gradient)
//   f32b_colsum   db_l += sum_e dZ_l
//   f32_grad_optim (mode 2, csrc/mlp_f32.hip)  AdaGrad (TF ApplyAdagrad) / Adam / SGD
//   f32b_target_sync  the target copy refreshed every target_every steps (device-side condition)
//
// Every product is v_mfma_f32_16x16x4_f32: fp32 operands and accumulation, each product exact in fp32
// (gfx950's f32-input MFMA runs at the fp32 vector rate, so this is about data reuse, not precision);
// only the summation order differs from the row kernels and the PyTorch oracle.  The env arithmetic is
// the row kernel's, operation for operation (TrainerChildActor.scala:118-146; quirks behind the same
// flags).
#include "common.h"

namespace st {

// ------------------------------------------------------------------------------------------- GEMM
// C(m, n) = sum_k A(m, k) B(k, n), operands addressed by strides (either may be transposed in memory):
// A(m, k) = A[m * am + k * ak], B(k, n) = B[k * bk + n * bn], C(m, n) = C[m * ldc + n].
// Epilogues: EPI_STORE (+ bias[n], optional relu), EPI_MASK (C = acc * [aux(m, n) > 0], aux row stride
// ldaux), EPI_ATOMIC (C += acc: split-K over gridDim.z, C zeroed beforehand), EPI_PARTIAL (split z stores its
// partial at C + z * zstride; st_f32b_splitsum adds the partials in split order: deterministic, no atomics).
enum { F32B_STORE = 0, F32B_MASK = 1, F32B_ATOMIC = 2, F32B_PARTIAL = 3 };

struct GemmF32 {
  const float* A;
  const float* B;
  float* C;
  const float* bias;   // [N] or null (EPI_STORE)
  const float* aux;    // EPI_MASK: [M][ldaux]
  int M, N, K;
  long long am, ak, bk, bn, ldc, ldaux;
  int epi, relu, kchunk;   // kchunk: K per split (gridDim.z splits)
  long long zstride;       // EPI_PARTIAL: elements between split z's partial tiles
};

constexpr int GB_M = 64, GB_N = 64, GB_K = 32, GB_T = 256;
// operand tile loaders (a 64 x 32 tile of X(r, k) = P[r * sr + k * sk], r < R, k < kend; zero outside):
//  LD_KF: unit stride along k, 16-byte aligned runs -> 2 float4 per thread;
//  LD_RF: unit stride along r -> 2 float4 per thread;  LD_SC: 8 scalar loads per thread.
// The next k-tile is loaded into registers while the MFMAs run on the current one (one LDS buffer, two
// barriers per k-tile).  The first form (16-wide k-tiles, scalar loads, no prefetch) reached ~46 TF/s on
// the 65,536 x 208 x 208 forward product.
enum { LD_KF = 0, LD_RF = 1, LD_SC = 2 };

template <int MODE>
ST_DEV void tile_ld(const float* P, long long sr, long long sk, int r0, int R, int k0, int kend, float (&v)[8]) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int i = tid + GB_T * j;
    if (MODE == LD_KF) {
      const int r = i >> 3, k = k0 + 4 * (i & 7);
      const float* a = P + (long long)(r0 + r) * sr + k;
      if (r0 + r < R && k + 3 < kend) {
        const float4 x = *reinterpret_cast<const float4*>(a);
        v[4 * j] = x.x; v[4 * j + 1] = x.y; v[4 * j + 2] = x.z; v[4 * j + 3] = x.w;
      } else {
#pragma unroll
        for (int t = 0; t < 4; ++t) v[4 * j + t] = (r0 + r < R && k + t < kend) ? a[t] : 0.f;
      }
    } else if (MODE == LD_RF) {
      const int kk = i >> 4, r = 4 * (i & 15), k = k0 + kk;
      const float* a = P + (long long)(r0 + r) + (long long)k * sk;
      if (r0 + r + 3 < R && k < kend) {
        const float4 x = *reinterpret_cast<const float4*>(a);
        v[4 * j] = x.x; v[4 * j + 1] = x.y; v[4 * j + 2] = x.z; v[4 * j + 3] = x.w;
      } else {
#pragma unroll
        for (int t = 0; t < 4; ++t) v[4 * j + t] = (r0 + r + t < R && k < kend) ? a[t] : 0.f;
      }
    } else {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int q = i * 4 + t, r = q & 63, k = k0 + (q >> 6);
        v[4 * j + t] = (r0 + r < R && k < kend) ? P[(long long)(r0 + r) * sr + (long long)k * sk] : 0.f;
      }
    }
  }
}

// stores a loaded tile k-major into LDS: S[k * ld + r] (S may point at a column offset of a wider tile)
template <int MODE, int ld>
ST_DEV void tile_st(float* S, const float (&v)[8]) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int i = tid + GB_T * j;
    if (MODE == LD_KF) {
      const int r = i >> 3, k = 4 * (i & 7);
#pragma unroll
      for (int t = 0; t < 4; ++t) S[(k + t) * ld + r] = v[4 * j + t];
    } else if (MODE == LD_RF) {
      const int kk = i >> 4, r = 4 * (i & 15);
      *reinterpret_cast<float4*>(&S[kk * ld + r]) = make_float4(v[4 * j], v[4 * j + 1], v[4 * j + 2], v[4 * j + 3]);
    } else {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int q = i * 4 + t;
        S[(q >> 6) * ld + (q & 63)] = v[4 * j + t];
      }
    }
  }
}

template <int AM, int BM>
__global__ void __launch_bounds__(GB_T) f32b_gemm_kernel(GemmF32 g) {
  __shared__ __attribute__((aligned(16))) float As[GB_K][GB_M + 4];
  __shared__ __attribute__((aligned(16))) float Bs[GB_K][GB_N + 4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l16 = lane & 15, g4 = lane >> 4;
  const int m0 = blockIdx.y * GB_M, n0 = blockIdx.x * GB_N;
  const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;
  const int k_begin = blockIdx.z * g.kchunk, k_end = min(g.K, k_begin + g.kchunk);
  f4v acc[2][2];
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int c = 0; c < 2; ++c) acc[r][c] = f4v{0.f, 0.f, 0.f, 0.f};
  float va[8], vb[8];
  tile_ld<AM>(g.A, g.am, g.ak, m0, g.M, k_begin, k_end, va);
  tile_ld<BM>(g.B, g.bn, g.bk, n0, g.N, k_begin, k_end, vb);
  for (int k0 = k_begin; k0 < k_end; k0 += GB_K) {
    tile_st<AM, GB_M + 4>(&As[0][0], va);
    tile_st<BM, GB_N + 4>(&Bs[0][0], vb);
    __syncthreads();
    if (k0 + GB_K < k_end) {   // the next k-tile in flight under this one's MFMAs
      tile_ld<AM>(g.A, g.am, g.ak, m0, g.M, k0 + GB_K, k_end, va);
      tile_ld<BM>(g.B, g.bn, g.bk, n0, g.N, k0 + GB_K, k_end, vb);
    }
#pragma unroll
    for (int ks = 0; ks < GB_K / 4; ++ks) {
      const int kk = 4 * ks + g4;
      float a[2], b[2];
#pragma unroll
      for (int r = 0; r < 2; ++r) a[r] = As[kk][wm + 16 * r + l16];
#pragma unroll
      for (int c = 0; c < 2; ++c) b[c] = Bs[kk][wn + 16 * c + l16];
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int c = 0; c < 2; ++c) acc[r][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[r], b[c], acc[r][c], 0, 0, 0);
    }
    __syncthreads();
  }
  // accumulator tile (r, c): lane (l16, g4) holds C rows 4 g4 + i, column l16
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int n = n0 + wn + 16 * c + l16;
      if (n >= g.N) continue;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = m0 + wm + 16 * r + 4 * g4 + i;
        if (m >= g.M) continue;
        float v = acc[r][c][i];
        float* dst = g.C + (long long)m * g.ldc + n;
        if (g.epi == F32B_PARTIAL) {
          dst[(long long)blockIdx.z * g.zstride] = v;
        } else if (g.epi == F32B_ATOMIC) {
          atomicAdd(dst, v);
        } else if (g.epi == F32B_MASK) {
          *dst = g.aux[(long long)m * g.ldaux + n] > 0.f ? v : 0.f;
        } else {
          if (g.bias) v = v + g.bias[n];
          *dst = g.relu ? fmaxf(v, 0.f) : v;
        }
      }
    }
}

// ------------------------------------------------------------------------------- fused 2-layer forward
// Q = [relu](relu(A W1^T + b1) W2^T + b2) for a two-layer net with N1 <= 256 hidden units and <= 16 outputs,
// 64 rows per workgroup: the first product on 64 x 256 tiles (the A tile is read once, not once per 64
// hidden units), H written for the backward, and the second product from H in registers (per-lane
// partials over the lane's 4 hidden units, 16-lane shuffles, 4-wave LDS fold) -- one launch and no
// re-read of H instead of two GEMM launches.  A: [M][K] (row stride lda), W1: [N1][K], W2: [16][N1] (rows >=
// nout zero), H: [M][N1], Q: [M][16].
struct Fwd2F32 {
  const float* A; const float* W1; const float* b1; const float* W2; const float* b2;
  float* H; float* Q;
  int M, K, N1, nout, relu_out;
  long long lda;
};
constexpr int F2_N = 256;
__global__ void __launch_bounds__(GB_T) f32b_fwd2_kernel(Fwd2F32 p) {
  __shared__ __attribute__((aligned(16))) float As[GB_K][GB_M + 4];
  __shared__ __attribute__((aligned(16))) float Bs[GB_K][F2_N + 4];
  __shared__ float red[4][GB_M][3];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l16 = lane & 15, g4 = lane >> 4;
  const int m0 = blockIdx.x * GB_M, wn = 64 * wave;
  f4v acc[4][4];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[r][c] = f4v{0.f, 0.f, 0.f, 0.f};
  float va[8], vb[4][8];
  auto load = [&](int k0) {
    tile_ld<LD_KF>(p.A, p.lda, 1, m0, p.M, k0, p.K, va);
#pragma unroll
    for (int q = 0; q < 4; ++q) tile_ld<LD_KF>(p.W1, p.K, 1, 64 * q, p.N1, k0, p.K, vb[q]);
  };
  load(0);
  for (int k0 = 0; k0 < p.K; k0 += GB_K) {
    tile_st<LD_KF, GB_M + 4>(&As[0][0], va);
#pragma unroll
    for (int q = 0; q < 4; ++q) tile_st<LD_KF, F2_N + 4>(&Bs[0][64 * q], vb[q]);   // hidden units 64 q ..
    __syncthreads();
    if (k0 + GB_K < p.K) load(k0 + GB_K);
#pragma unroll
    for (int ks = 0; ks < GB_K / 4; ++ks) {
      const int kk = 4 * ks + g4;
      float a[4], b[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) a[r] = As[kk][16 * r + l16];
#pragma unroll
      for (int c = 0; c < 4; ++c) b[c] = Bs[kk][wn + 16 * c + l16];
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[r][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[r], b[c], acc[r][c], 0, 0, 0);
    }
    __syncthreads();
  }
  // epilogue: H = relu(acc + b1) -> global; per-lane layer-2 partials over this lane's 4 hidden units
  float w2[4][3], bb[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int n = wn + 16 * c + l16;
    const bool ok = n < p.N1;
    bb[c] = ok && p.b1 ? p.b1[n] : 0.f;
#pragma unroll
    for (int a = 0; a < 3; ++a) w2[c][a] = (ok && a < p.nout) ? p.W2[a * p.N1 + n] : 0.f;
  }
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int mr = 16 * r + 4 * g4 + i, m = m0 + mr;
      float part[3] = {0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int n = wn + 16 * c + l16;
        const float h = fmaxf(acc[r][c][i] + bb[c], 0.f);
        if (m < p.M && n < p.N1) p.H[(long long)m * p.N1 + n] = h;
#pragma unroll
        for (int a = 0; a < 3; ++a) part[a] = __builtin_fmaf(h, w2[c][a], part[a]);
      }
#pragma unroll
      for (int a = 0; a < 3; ++a) {
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) part[a] += __shfl_xor(part[a], o);
      }
      if (l16 == 0) {
#pragma unroll
        for (int a = 0; a < 3; ++a) red[wave][mr][a] = part[a];
      }
    }
  __syncthreads();
  {
    const int mr = tid >> 2, a0 = 4 * (tid & 3), m = m0 + mr;   // 64 rows x 16 outputs, 4 per thread
    if (m < p.M) {
      float4 o;
      float* ov = reinterpret_cast<float*>(&o);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int a = a0 + t;
        float v = 0.f;
        if (a < p.nout && a < 3) {
          v = (red[0][mr][a] + red[1][mr][a]) + (red[2][mr][a] + red[3][mr][a]);
          if (p.b2) v = v + p.b2[a];
          if (p.relu_out) v = fmaxf(v, 0.f);
        }
        ov[t] = v;
      }
      *reinterpret_cast<float4*>(p.Q + (long long)m * 16 + a0) = o;
    }
  }
}

// loader mode of an operand with row stride sr / k stride sk
inline int ld_mode(const float* P, long long sr, long long sk) {
  const bool al = (reinterpret_cast<uintptr_t>(P) & 15) == 0;
  if (al && sk == 1 && sr % 4 == 0) return LD_KF;
  if (al && sr == 1 && sk % 4 == 0) return LD_RF;
  return LD_SC;
}

// ------------------------------------------------------------------------------------------- env side
struct F32Batch {
  // layout of the padded input row (sharetrade/models/qnet.py): window features [0, H), budget H,
  // shares H + 1, constant 1 at bias_col, zero elsewhere up to in_p
  int E, in_p, H, T, bias_col, feat_mode;
  float* X;            // [E][in_p]
  float* XN;           // [E][in_p]
  const float* Q;      // [E][16]  Q(x)
  const float* QN;     // [E][16]  Q(x')
  float* DQ;           // [E][16]  dL/dz of the output layer
  float* loss;         // [E]
  // per-env scratch between the env and TD launches
  float* s_b2; int* s_s2; float* s_rew; int* s_act;
  // env state (VectorEngine EnvState) + outputs
  const float* prices;
  float* budget; int* shares; float* value; int* pos; int* episodes; float* last_final; float* ret_sum;
  int* actions_out; float* rewards_out;
  const unsigned long long* ctrl;
  int compat_env, target_compat, output_relu, s0, env_offset, reward_mode;
  float eps, inv_ramp, b0, inv_b0, gamma, coef, td_clip;
  uint32_t key0, key1;
  double* stat;        // optional [2]: += sum of rewards, += sum of squared TD errors (VectorEngine.stat_acc)
  // learning experiments (sharetrade/env/trading.py engine_step_ref: target_params / double_dqn /
  // reward_scale / ramp_pos): QT = Q(x') of a target copy of the parameters (null: none)
  const float* QT;
  float reward_scale;
  int double_dqn, ramp_global;
};

ST_DEV float f32b_feat(float w, float inv, int mode) { return mode ? __fsub_rn(__fmul_rn(w, inv), 1.0f) : w; }

// one thread per element of X / X' (the divisions are per env but cheap beside the traffic)
// one thread per (env, 4 consecutive columns) of X / X': the window's reciprocals once per thread and
// float4 stores (one thread per element with 64-bit index math and two IEEE divisions each ran at
// ~1.5 TB/s: 73 us at 65,536 envs)
__global__ void __launch_bounds__(256) f32b_gather_kernel(F32Batch r) {
  const int q4 = r.in_p >> 2;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= r.E * q4) return;
  const int e = i / q4, k0 = 4 * (i - e * q4);
  const int ps = r.pos[e];
  const float* pr = r.prices + (size_t)e * r.T + ps;
  const float last = pr[r.H - 1], vnew = pr[r.H];
  const float inv = __fdiv_rn(1.0f, last), invn = __fdiv_rn(1.0f, vnew);
  float v[4], vn[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int k = k0 + t;
    v[t] = 0.f;
    vn[t] = 0.f;
    if (k < r.H) {
      v[t] = f32b_feat(pr[k], inv, r.feat_mode);
      vn[t] = f32b_feat(pr[k + 1], invn, r.feat_mode);
    } else if (k == r.H) {
      const float b = r.budget[e];
      v[t] = r.feat_mode ? __fmul_rn(b, r.inv_b0) : b;
    } else if (k == r.H + 1) {
      const int s = r.shares[e];
      v[t] = r.feat_mode ? __fmul_rn(__fmul_rn((float)s, last), r.inv_b0) : (float)s;
    } else if (k == r.bias_col) {
      v[t] = 1.f;
      vn[t] = 1.f;
    }
  }
  const size_t o = (size_t)e * r.in_p + k0;
  *reinterpret_cast<float4*>(r.X + o) = make_float4(v[0], v[1], v[2], v[3]);
  *reinterpret_cast<float4*>(r.XN + o) = make_float4(vn[0], vn[1], vn[2], vn[3]);   // budget / shares of x': env step
}

// epsilon-greedy + the trading env, one thread per env (the row kernel's arithmetic, mlp_f32.hip)
__global__ void __launch_bounds__(256) f32b_env_kernel(F32Batch r) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= r.E) return;
  const unsigned long long step = r.ctrl[0];
  const float* q = r.Q + (size_t)e * 16;
  const float q0 = q[0], q1 = q[1], q2 = q[2];
  int greedy = 0;
  float best = q0;
  if (q1 > best) { best = q1; greedy = 1; }
  if (q2 > best) { best = q2; greedy = 2; }
  const int ps = r.pos[e];
  uint32_t c0 = (uint32_t)(r.env_offset + e), c1 = (uint32_t)(step & 0xFFFFFFFFull), c2 = (uint32_t)(step >> 32),
           c3 = 0u;
  philox4x32(c0, c1, c2, c3, r.key0, r.key1);
  const float u1 = u24(c0), u2 = u24(c1);
  const float rpos = r.ramp_global ? (float)step : (float)ps;   // exploit ramp over the step count (global)
  const bool exploit = u1 < fminf(r.eps, __fmul_rn(rpos, r.inv_ramp));
  int rnd = (int)(u2 * 3.0f);
  rnd = rnd > 2 ? 2 : rnd;
  const int a = exploit ? greedy : rnd;
  const float* pr = r.prices + (size_t)e * r.T + ps;
  const float vnew = pr[r.H];
  const float b = r.budget[e], vprev = r.value[e];
  const int s = r.shares[e];
  const float bd = r.compat_env ? r.b0 : b;
  const int sd = r.compat_env ? r.s0 : s;
  const bool buy = (a == 0) && (bd >= vnew);
  const bool sell = (a == 1) && (sd > 0);
  const float b2 = buy ? __fsub_rn(bd, vnew) : (sell ? __fadd_rn(bd, vnew) : bd);
  const int s2 = buy ? sd + 1 : (sell ? sd - 1 : sd);
  const float cur = __fadd_rn(b, __fmul_rn((float)s, vprev));
  const float nw = __fadd_rn(b2, __fmul_rn((float)s2, vnew));
  float rew = __fsub_rn(nw, cur);
  if (r.reward_mode) rew = cur > 0.f ? __fdiv_rn(rew, cur) : 0.f;
        if (r.reward_mode == 2) rew = __fsub_rn(rew, __fmul_rn(__fmul_rn(rew, 0.5f), rew));   // growth: log1p to 2nd order
  r.s_b2[e] = b2;
  r.s_s2[e] = s2;
  r.s_rew[e] = rew;
  r.s_act[e] = a;
  float* xn = r.XN + (size_t)e * r.in_p;
  xn[r.H] = r.feat_mode ? __fmul_rn(b2, r.inv_b0) : b2;
  xn[r.H + 1] = r.feat_mode ? __fmul_rn(__fmul_rn((float)s2, vnew), r.inv_b0) : (float)s2;
  if (r.actions_out) r.actions_out[e] = a;
  if (r.rewards_out) r.rewards_out[e] = rew;
}

// TD target, one-hot dQ, loss, env write-back, one thread per env
__global__ void __launch_bounds__(1024) f32b_td_kernel(F32Batch r) {
  __shared__ double red[2][16];
  const int e = blockIdx.x * 1024 + threadIdx.x;
  double st_r = 0.0, st_l = 0.0;
  if (e < r.E) {
  const float* qn = r.QN + (size_t)e * 16;
  const float n0 = qn[0], n1 = qn[1], n2 = qn[2];
  int am = 0;
  float mx = n0;
  if (n1 > mx) { mx = n1; am = 1; }
  if (n2 > mx) { mx = n2; am = 2; }
  const int slot = r.target_compat ? am : r.s_act[e];
  const float rew = r.s_rew[e];
  // bootstrap value: max of Q(x') (online or target net); compat and Double DQN: the online argmax's value
  float boot = mx;
  if (r.QT != nullptr) {
    const float* qt = r.QT + (size_t)e * 16;
    if (r.target_compat || r.double_dqn) {
      boot = qt[am];
    } else {
      boot = fmaxf(fmaxf(qt[0], qt[1]), qt[2]);
    }
  }
  const float rs = r.reward_scale != 1.f ? __fmul_rn(rew, r.reward_scale) : rew;
  const float y = __fadd_rn(rs, __fmul_rn(r.gamma, boot));
  const float qs = r.Q[(size_t)e * 16 + slot];
  const float diff = __fsub_rn(qs, y);
  float dq = r.coef * (r.td_clip > 0.f ? fminf(fmaxf(diff, -r.td_clip), r.td_clip) : diff);
  if (r.output_relu && !(qs > 0.f)) dq = 0.f;
  float* d = r.DQ + (size_t)e * 16;
#pragma unroll
  for (int j = 0; j < 16; ++j) d[j] = j == slot ? dq : 0.f;
  r.loss[e] = diff * diff;
  st_r = (double)rew;
  st_l = (double)(diff * diff);
  const float b2 = r.s_b2[e];
  const int s2 = r.s_s2[e];
  const int ps = r.pos[e];
  const float vnew = r.prices[(size_t)e * r.T + ps + r.H];
  const int np = ps + 1;
  if (np >= r.T - r.H) {
    r.last_final[e] = __fadd_rn(b2, __fmul_rn((float)s2, vnew));
    r.episodes[e] = r.episodes[e] + 1;
    r.budget[e] = r.b0;
    r.shares[e] = r.s0;
    r.value[e] = 0.f;
    r.pos[e] = 0;
    r.ret_sum[e] = 0.f;
  } else {
    r.budget[e] = b2;
    r.shares[e] = s2;
    r.value[e] = vnew;
    r.pos[e] = np;
    r.ret_sum[e] = r.ret_sum[e] + rew;
  }
  }
  if (r.stat != nullptr) {   // block sums, one double atomic per block and statistic (per-wave atomics on
                             // two addresses serialised: 30 us at 65,536 envs)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      st_r += __shfl_xor(st_r, o);
      st_l += __shfl_xor(st_l, o);
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
      red[0][w] = st_r;
      red[1][w] = st_l;
    }
    __syncthreads();
    if (threadIdx.x < 2) {
      double t = 0.0;
      for (int j = 0; j < (int)(blockDim.x >> 6); ++j) t += red[threadIdx.x][j];
      atomicAdd(r.stat + threadIdx.x, t);
    }
  }
}

// out[n] += sum over rows e of D[e][n] (n < N): a bias gradient; 256 columns x 256 rows per block
// column sums of D[E][N] (bias gradients), N % 4 == 0 and N <= 256: a block reads 256 / (N / 4) rows per
// pass as float4 runs (N / 4 threads per row), sums `rows` rows (~E / 32), folds its row groups in LDS and
// adds one atomic per column.  Other shapes: one thread per column and row group of 256.
__global__ void __launch_bounds__(256) f32b_colsum4_kernel(const float* D, long long ld, int E, int N, int rows,
                                                           float* out, float* partials) {
  __shared__ float4 part[256];
  const int tr = N >> 2, rpi = 256 / tr;
  const int t = threadIdx.x, c4 = t % tr, rg = t / tr;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (rg < rpi) {
    const int e0 = blockIdx.x * rows, e1 = min(E, e0 + rows);
    for (int e = e0 + rg; e < e1; e += rpi) {
      const float4 v = *reinterpret_cast<const float4*>(D + (long long)e * ld + 4 * c4);
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
  }
  part[t] = s;
  __syncthreads();
  if (t < tr) {
    float4 a = part[t];
    for (int g = 1; g < rpi; ++g) {
      const float4 b = part[g * tr + t];
      a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    }
    if (partials) {   // deterministic mode: the block's column sums to its own row (st_f32b_splitsum adds them)
      reinterpret_cast<float4*>(partials + (long long)blockIdx.x * N)[t] = a;
    } else {
      atomicAdd(out + 4 * t, a.x);
      atomicAdd(out + 4 * t + 1, a.y);
      atomicAdd(out + 4 * t + 2, a.z);
      atomicAdd(out + 4 * t + 3, a.w);
    }
  }
}
__global__ void __launch_bounds__(256) f32b_colsum_kernel(const float* D, long long ld, int E, int N, float* out,
                                                          float* partials) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  const int e0 = blockIdx.y * 256, e1 = min(E, e0 + 256);
  float s = 0.f;
  for (int e = e0; e < e1; ++e) s += D[(long long)e * ld + n];
  if (partials)   // deterministic mode: row group y's column sums to its own row (added in order below)
    partials[(long long)blockIdx.y * N + n] = s;
  else
    atomicAdd(out + n, s);
}

// out[i] = sum over z of part[z * zstride + i] in split order, one thread per element: the deterministic sum
// for shapes the float4 form (f32b_splitsum_kernel) does not take -- widths not a multiple of 4, offsets not
// 16-byte aligned (any fp32 MLP of the flat layout, engine.f32_deterministic)
__global__ void __launch_bounds__(256) f32b_splitsum1_kernel(const float* part, int splits, long long zstride,
                                                             float* out, long long n) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  float a = 0.f;
  for (int z = 0; z < splits; ++z) a += part[z * zstride + i];
  out[i] = a;
}

// out[i] = sum over z of part[z * zstride + i] (split-K partials of EPI_PARTIAL, bias column-sum partials):
// a fixed summation order, so bit-reproducible.  A block covers 16 float4 columns x 16 split groups: thread
// (c, g) adds splits g, g + 16, ... (4 loads in flight), then the 16 group sums fold in LDS in group order.
// (The first form -- one thread per float4 walking all splits -- put 49 blocks and a 64-deep dependent load
// chain on the 224 x 224 product: most of the 0.412 -> 0.493 ms of the deterministic mode at 65,536 envs.)
__global__ void __launch_bounds__(256) f32b_splitsum_kernel(const float* part, int splits, long long zstride,
                                                            float* out, long long n4) {
  __shared__ float4 red[16][17];
  const int c = threadIdx.x & 15, g = threadIdx.x >> 4;
  const long long i = (long long)blockIdx.x * 16 + c;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i < n4) {
    const float4* p4 = reinterpret_cast<const float4*>(part) + i;
    const long long zs4 = zstride >> 2;
    int z = g;
    for (; z + 48 < splits; z += 64) {
      const float4 b0 = p4[z * zs4], b1 = p4[(z + 16) * zs4], b2 = p4[(z + 32) * zs4], b3 = p4[(z + 48) * zs4];
      a.x += b0.x; a.y += b0.y; a.z += b0.z; a.w += b0.w;
      a.x += b1.x; a.y += b1.y; a.z += b1.z; a.w += b1.w;
      a.x += b2.x; a.y += b2.y; a.z += b2.z; a.w += b2.w;
      a.x += b3.x; a.y += b3.y; a.z += b3.z; a.w += b3.w;
    }
    for (; z < splits; z += 16) {
      const float4 b = p4[z * zs4];
      a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    }
  }
  red[g][c] = a;
  __syncthreads();
  if (g == 0 && i < n4) {
    float4 s = red[0][c];
    for (int k = 1; k < 16; ++k) {
      const float4 b = red[k][c];
      s.x += b.x; s.y += b.y; s.z += b.z; s.w += b.w;
    }
    reinterpret_cast<float4*>(out)[i] = s;
  }
}

// target network refresh inside the captured step: copy the parameters when the (already advanced) step
// counter is a multiple of `every` (engine_step_ref: after the optimizer step of step s, if (s + 1) % every == 0)
__global__ void __launch_bounds__(256) f32b_target_sync_kernel(const float* params, float* target, long long n,
                                                               const unsigned long long* ctrl, long long every) {
  if (ctrl[0] % (unsigned long long)every != 0ull) return;
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i < n) target[i] = params[i];
}

}  // namespace st

extern "C" hipError_t st_f32b_gemm(const st::GemmF32* g, int splits, hipStream_t stream) {
  using namespace st;
  if (g->M <= 0 || g->N <= 0 || g->K <= 0 || splits < 1) return hipErrorInvalidValue;
  if (splits > 1 && g->epi != F32B_ATOMIC && g->epi != F32B_PARTIAL) return hipErrorInvalidValue;
  if (g->epi == F32B_PARTIAL && g->zstride < (long long)g->M * g->ldc) return hipErrorInvalidValue;
  GemmF32 a = *g;
  a.kchunk = ((g->K + splits - 1) / splits + GB_K - 1) / GB_K * GB_K;
  const int z = (g->K + a.kchunk - 1) / a.kchunk;
  dim3 grid((g->N + GB_N - 1) / GB_N, (g->M + GB_M - 1) / GB_M, z);
  if (grid.y > 65535) return hipErrorInvalidValue;
  const int am = ld_mode(g->A, g->am, g->ak), bm = ld_mode(g->B, g->bn, g->bk);
  using KFn = void (*)(GemmF32);
  static const KFn tab[3][3] = {
      {f32b_gemm_kernel<LD_KF, LD_KF>, f32b_gemm_kernel<LD_KF, LD_RF>, f32b_gemm_kernel<LD_KF, LD_SC>},
      {f32b_gemm_kernel<LD_RF, LD_KF>, f32b_gemm_kernel<LD_RF, LD_RF>, f32b_gemm_kernel<LD_RF, LD_SC>},
      {f32b_gemm_kernel<LD_SC, LD_KF>, f32b_gemm_kernel<LD_SC, LD_RF>, f32b_gemm_kernel<LD_SC, LD_SC>}};
  hipLaunchKernelGGL(tab[am][bm], grid, dim3(GB_T), 0, stream, a);
  return hipGetLastError();
}

extern "C" hipError_t st_f32b_fwd2(const st::Fwd2F32* p, hipStream_t stream) {
  using namespace st;
  if (p->M <= 0 || p->K <= 0 || p->N1 <= 0 || p->N1 > F2_N || p->nout < 1 || p->nout > 3 || p->K % 4 || p->lda % 4 ||
      ((reinterpret_cast<uintptr_t>(p->A) | reinterpret_cast<uintptr_t>(p->W1) | reinterpret_cast<uintptr_t>(p->Q)) & 15))
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(f32b_fwd2_kernel, dim3((p->M + GB_M - 1) / GB_M), dim3(GB_T), 0, stream, *p);
  return hipGetLastError();
}

extern "C" hipError_t st_f32b_splitsum(const float* part, int splits, long long zstride, float* out, long long n,
                                       hipStream_t stream) {
  if (splits < 1 || n <= 0 || zstride < n) return hipErrorInvalidValue;
  if (n % 4 || zstride % 4 || ((reinterpret_cast<uintptr_t>(part) | reinterpret_cast<uintptr_t>(out)) & 15)) {
    // unaligned shapes: the same fixed order, one element per thread
    hipLaunchKernelGGL(st::f32b_splitsum1_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, part,
                       splits, zstride, out, n);
    return hipGetLastError();
  }
  const long long n4 = n / 4;
  hipLaunchKernelGGL(st::f32b_splitsum_kernel, dim3((unsigned)((n4 + 15) / 16)), dim3(256), 0, stream, part, splits,
                     zstride, out, n4);
  return hipGetLastError();
}

extern "C" hipError_t st_f32b_target_sync(const float* params, float* target, long long n,
                                           const unsigned long long* ctrl, long long every, hipStream_t stream) {
  if (n <= 0 || every <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(st::f32b_target_sync_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, params,
                     target, n, ctrl, every);
  return hipGetLastError();
}

extern "C" hipError_t st_f32b_gather(const st::F32Batch* r, hipStream_t stream) {
  if (r->in_p % 4 || (reinterpret_cast<uintptr_t>(r->X) & 15) || (reinterpret_cast<uintptr_t>(r->XN) & 15) ||
      (long long)r->E * (r->in_p / 4) >= (1ll << 31))
    return hipErrorInvalidValue;
  const long long n = (long long)r->E * (r->in_p / 4);
  hipLaunchKernelGGL(st::f32b_gather_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, *r);
  return hipGetLastError();
}

extern "C" hipError_t st_f32b_env(const st::F32Batch* r, hipStream_t stream) {
  hipLaunchKernelGGL(st::f32b_env_kernel, dim3((r->E + 255) / 256), dim3(256), 0, stream, *r);
  return hipGetLastError();
}

extern "C" hipError_t st_f32b_td(const st::F32Batch* r, hipStream_t stream) {
  hipLaunchKernelGGL(st::f32b_td_kernel, dim3((r->E + 1023) / 1024), dim3(1024), 0, stream, *r);
  return hipGetLastError();
}

// part != nullptr (deterministic mode): the column sums of the blocks land in part[block][N] and one
// st_f32b_splitsum adds them into out in block order (returns the block count through *nparts).  N % 4 == 0,
// N <= 256 and 16-byte alignment: <= 32 blocks of the float4 form, part needs 32 * N floats; other shapes:
// one block row per 256 envs, part needs ceil(E / 256) * N floats (st_f32b_colsum_part_floats)
extern "C" hipError_t st_f32b_colsum_det(const float* D, long long ld, int E, int N, float* out, float* part,
                                         int* nparts, hipStream_t stream);
extern "C" hipError_t st_f32b_colsum(const float* D, long long ld, int E, int N, float* out, hipStream_t stream) {
  return st_f32b_colsum_det(D, ld, E, N, out, nullptr, nullptr, stream);
}
extern "C" hipError_t st_f32b_colsum_det(const float* D, long long ld, int E, int N, float* out, float* part,
                                         int* nparts, hipStream_t stream) {
  if (E <= 0 || N <= 0) return hipErrorInvalidValue;
  const bool vec = N % 4 == 0 && N <= 256 && ld % 4 == 0 && (reinterpret_cast<uintptr_t>(D) & 15) == 0 &&
                   (!part || ((reinterpret_cast<uintptr_t>(part) | reinterpret_cast<uintptr_t>(out)) & 15) == 0);
  if (vec) {
    // at most 32 blocks: every block adds one atomic per column, and same-address fp32 atomics serialise
    // (256 blocks on a 16-column output: 16 us at 65,536 rows, mostly the 256-deep atomic queue per column)
    const int rpi = 256 / (N / 4);
    int rows = (E + 31) / 32;
    rows = (rows + rpi - 1) / rpi * rpi;
    if (rows < 4 * rpi) rows = 4 * rpi;
    const int nb = (E + rows - 1) / rows;
    hipLaunchKernelGGL(st::f32b_colsum4_kernel, dim3(nb), dim3(256), 0, stream, D, ld, E, N, rows, out, part);
    if (part) {
      hipError_t e = hipGetLastError();
      if (e != hipSuccess) return e;
      if (nparts) *nparts = nb;
      return st_f32b_splitsum(part, nb, N, out, N, stream);
    }
    return hipGetLastError();
  }
  dim3 grid((N + 255) / 256, (E + 255) / 256);
  if (grid.y > 65535) return hipErrorInvalidValue;
  hipLaunchKernelGGL(st::f32b_colsum_kernel, grid, dim3(256), 0, stream, D, ld, E, N, out, part);
  if (part) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (nparts) *nparts = (int)grid.y;
    return st_f32b_splitsum(part, (int)grid.y, N, out, N, stream);
  }
  return hipGetLastError();
}

// scratch (floats) st_f32b_colsum_det needs for an [E][N] column sum in deterministic mode
extern "C" long long st_f32b_colsum_part_floats(int E, int N) {
  const bool vec = N % 4 == 0 && N <= 256;
  return vec ? 32ll * 256 : (long long)((E + 255) / 256) * N;
}

// struct sizes of this file's launch ABI, for the host mirrors' check (tests/test_abi.py; no HIP call)
extern "C" int st_abi_mlp_f32_mfma(int* out, int n) {
  const int sz[] = {(int)sizeof(st::GemmF32), (int)sizeof(st::Fwd2F32), (int)sizeof(st::F32Batch)};
  const int m = (int)(sizeof(sz) / sizeof(sz[0]));
  for (int i = 0; i < n && i < m; ++i) out[i] = sz[i];
  return m;
}
