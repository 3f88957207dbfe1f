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
//   f32b_env      epsilon-greedy (Philox) + Buy/Sell/Hold step: budget / shares columns of X'
//   GEMM          the same forward for x' -> Q'
//   f32b_td       TD target, dQ (one-hot at the target slot), loss, env write-back
//   GEMM          dZ_{l-1} = (dZ_l . W_l) * [A_l > 0]                       (backward, data)
//   GEMM          dW_l^T += dZ_l^T . A_l  (split-K over envs, fp32 atomics)  (weight gradient)
//   f32b_colsum   db_l += sum_e dZ_l
//   f32_grad_optim (mode 2, csrc/mlp_f32.hip)  AdaGrad (TF ApplyAdagrad) / Adam / SGD
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
// ldaux), EPI_ATOMIC (C += acc: split-K over gridDim.z, C zeroed beforehand).
enum { F32B_STORE = 0, F32B_MASK = 1, F32B_ATOMIC = 2 };

struct GemmF32 {
  const float* A;
  const float* B;
  float* C;
  const float* bias;   // [N] or null (EPI_STORE)
  const float* aux;    // EPI_MASK: [M][ldaux]
  int M, N, K;
  long long am, ak, bk, bn, ldc, ldaux;
  int epi, relu, kchunk;   // kchunk: K per split (gridDim.z splits)
};

constexpr int GB_M = 64, GB_N = 64, GB_K = 16, GB_T = 256;

__global__ void __launch_bounds__(GB_T) f32b_gemm_kernel(GemmF32 g) {
  __shared__ float As[GB_K][GB_M + 4];
  __shared__ float Bs[GB_K][GB_N + 4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l16 = lane & 15, g4 = lane >> 4;
  const int m0 = blockIdx.y * GB_M, n0 = blockIdx.x * GB_N;
  const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;
  const int k_begin = blockIdx.z * g.kchunk, k_end = min(g.K, k_begin + g.kchunk);
  f4v acc[2][2];
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int c = 0; c < 2; ++c) acc[r][c] = f4v{0.f, 0.f, 0.f, 0.f};
  // global -> LDS mapping: the unit-stride dimension runs along consecutive threads
  const bool a_kfast = g.ak == 1, b_nfast = g.bn == 1;
  for (int k0 = k_begin; k0 < k_end; k0 += GB_K) {
#pragma unroll
    for (int j = 0; j < GB_M * GB_K / GB_T; ++j) {
      const int i = tid + GB_T * j;
      const int mm = a_kfast ? i / GB_K : i % GB_M, kk = a_kfast ? i % GB_K : i / GB_M;
      const int m = m0 + mm, k = k0 + kk;
      As[kk][mm] = (m < g.M && k < k_end) ? g.A[(long long)m * g.am + (long long)k * g.ak] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < GB_N * GB_K / GB_T; ++j) {
      const int i = tid + GB_T * j;
      const int nn = b_nfast ? i % GB_N : i / GB_K, kk = b_nfast ? i / GB_N : i % GB_K;
      const int n = n0 + nn, k = k0 + kk;
      Bs[kk][nn] = (n < g.N && k < k_end) ? g.B[(long long)k * g.bk + (long long)n * g.bn] : 0.f;
    }
    __syncthreads();
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
        if (g.epi == F32B_ATOMIC) {
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
};

ST_DEV float f32b_feat(float w, float inv, int mode) { return mode ? __fsub_rn(__fmul_rn(w, inv), 1.0f) : w; }

// one thread per element of X / X' (the divisions are per env but cheap beside the traffic)
__global__ void __launch_bounds__(256) f32b_gather_kernel(F32Batch r) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long long)r.E * r.in_p) return;
  const int e = (int)(i / r.in_p), k = (int)(i % r.in_p);
  const int ps = r.pos[e];
  const float* pr = r.prices + (size_t)e * r.T + ps;
  const float last = pr[r.H - 1], vnew = pr[r.H];
  float v = 0.f, vn = 0.f;
  if (k < r.H) {
    v = f32b_feat(pr[k], __fdiv_rn(1.0f, last), r.feat_mode);
    vn = f32b_feat(pr[k + 1], __fdiv_rn(1.0f, vnew), r.feat_mode);
  } else if (k == r.H) {
    const float b = r.budget[e];
    v = r.feat_mode ? __fmul_rn(b, r.inv_b0) : b;
  } else if (k == r.H + 1) {
    const int s = r.shares[e];
    v = r.feat_mode ? __fmul_rn(__fmul_rn((float)s, last), r.inv_b0) : (float)s;
  } else if (k == r.bias_col) {
    v = 1.f;
    vn = 1.f;
  }
  r.X[i] = v;
  r.XN[i] = vn;   // budget / shares columns of x' come from the env step
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
  const bool exploit = u1 < fminf(r.eps, __fmul_rn((float)ps, r.inv_ramp));
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
__global__ void __launch_bounds__(256) f32b_td_kernel(F32Batch r) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= r.E) return;
  const float* qn = r.QN + (size_t)e * 16;
  const float n0 = qn[0], n1 = qn[1], n2 = qn[2];
  int am = 0;
  float mx = n0;
  if (n1 > mx) { mx = n1; am = 1; }
  if (n2 > mx) { mx = n2; am = 2; }
  const int slot = r.target_compat ? am : r.s_act[e];
  const float rew = r.s_rew[e];
  const float y = __fadd_rn(rew, __fmul_rn(r.gamma, mx));
  const float qs = r.Q[(size_t)e * 16 + slot];
  const float diff = __fsub_rn(qs, y);
  float dq = r.coef * (r.td_clip > 0.f ? fminf(fmaxf(diff, -r.td_clip), r.td_clip) : diff);
  if (r.output_relu && !(qs > 0.f)) dq = 0.f;
  float* d = r.DQ + (size_t)e * 16;
#pragma unroll
  for (int j = 0; j < 16; ++j) d[j] = j == slot ? dq : 0.f;
  r.loss[e] = diff * diff;
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

// out[n] += sum over rows e of D[e][n] (n < N): a bias gradient; 256 columns x 256 rows per block
__global__ void __launch_bounds__(256) f32b_colsum_kernel(const float* D, long long ld, int E, int N, float* out) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  const int e0 = blockIdx.y * 256, e1 = min(E, e0 + 256);
  float s = 0.f;
  for (int e = e0; e < e1; ++e) s += D[(long long)e * ld + n];
  atomicAdd(out + n, s);
}

}  // namespace st

extern "C" hipError_t st_f32b_gemm(const st::GemmF32* g, int splits, hipStream_t stream) {
  using namespace st;
  if (g->M <= 0 || g->N <= 0 || g->K <= 0 || splits < 1) return hipErrorInvalidValue;
  if (splits > 1 && g->epi != F32B_ATOMIC) return hipErrorInvalidValue;
  GemmF32 a = *g;
  a.kchunk = ((g->K + splits - 1) / splits + GB_K - 1) / GB_K * GB_K;
  const int z = (g->K + a.kchunk - 1) / a.kchunk;
  dim3 grid((g->N + GB_N - 1) / GB_N, (g->M + GB_M - 1) / GB_M, z);
  if (grid.y > 65535) return hipErrorInvalidValue;
  hipLaunchKernelGGL(f32b_gemm_kernel, grid, dim3(GB_T), 0, stream, a);
  return hipGetLastError();
}

extern "C" hipError_t st_f32b_gather(const st::F32Batch* r, hipStream_t stream) {
  const long long n = (long long)r->E * r->in_p;
  hipLaunchKernelGGL(st::f32b_gather_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, *r);
  return hipGetLastError();
}

extern "C" hipError_t st_f32b_env(const st::F32Batch* r, hipStream_t stream) {
  hipLaunchKernelGGL(st::f32b_env_kernel, dim3((r->E + 255) / 256), dim3(256), 0, stream, *r);
  return hipGetLastError();
}

extern "C" hipError_t st_f32b_td(const st::F32Batch* r, hipStream_t stream) {
  hipLaunchKernelGGL(st::f32b_td_kernel, dim3((r->E + 255) / 256), dim3(256), 0, stream, *r);
  return hipGetLastError();
}

extern "C" hipError_t st_f32b_colsum(const float* D, long long ld, int E, int N, float* out, hipStream_t stream) {
  if (E <= 0 || N <= 0) return hipErrorInvalidValue;
  dim3 grid((N + 255) / 256, (E + 255) / 256);
  if (grid.y > 65535) return hipErrorInvalidValue;
  hipLaunchKernelGGL(st::f32b_colsum_kernel, grid, dim3(256), 0, stream, D, ld, E, N, out);
  return hipGetLastError();
}
