// Exact-fp32 Q-learning kernels for small batches (the reference-parity path).
//
// The reference runs its 203->200->3 network at batch 1 in fp32 through TF's
// CPU kernels: SelectionAction = 1 forward, UpdateQ = 3 forwards + backward +
// ApplyAdagrad (QDecisionPolicyActor.scala:54-77), ~6 JNI session calls per
// message.  At batch 1..a few hundred these are GEMV-shaped and launch-bound,
// so the design goal is the minimum number of launches, fp32 throughout:
//
//   f32_rows_kernel   one workgroup per row (state):  forward(x) [+ forward(x'),
//                     TD target, dQ, backward-data through every layer]; in
//                     engine mode the row is a vectorised env: the state is
//                     gathered from the HBM price bank, epsilon-greedy (Philox)
//                     and the Buy/Sell/Hold transition run in-kernel too;
//   f32_grad_optim    one thread per parameter: grad = sum_rows dZ[o] * A[i]
//                     (the outer products of the weight gradient), then the
//                     optimizer update (AdaGrad = TF ApplyAdagrad / Adam / SGD).
//
// GEMV work sits on the VALU (a wave per output neuron, lanes split K, wave
// reduction), which is what a batch-1 product is on CDNA: an MFMA tile would be
// >93% padding.  Weights are the flat fp32 layout of sharetrade/models/qnet.py
// (W^T[out_p][in_p] row-major; layer-0 bias folded into column `bias_col`).
#include "common.h"

namespace st {

constexpr int F_NT = 256;
constexpr int F_MAXL = 6;
constexpr int F_MAXW = 1024;     // max padded layer width

struct F32Net {
  int L;                         // layers
  int pd[F_MAXL + 1];            // padded dims: pd[0] = in_p ... pd[L] = 16
  int dims[F_MAXL + 1];          // real dims
  int off_w[F_MAXL];             // W^T_l offset (floats)
  int off_b[F_MAXL];             // b_l offset, -1 for layer 0 (folded)
  int act_off[F_MAXL];           // offset of a_l inside a row's activation record
  int dz_off[F_MAXL];            // offset of dz_l inside a row's dz record
  int act_stride, dz_stride;     // floats per row
  int bias_col, input_dim, output_relu, P;
  int gemv_legacy;               // 1: every layer in the wave-per-neuron form (A/B of the thread-per-neuron form)
};

struct F32Rows {
  const float* params;
  const float* x;                // [B, in_p]  padded states (actor mode)
  const float* xn;               // [B, in_p]  padded next states
  const float* reward;           // [B]
  const int* action;             // [B] taken action or null (compat slot = argmax q')
  float* q_out;                  // [B, 16] q(x)
  float* qn_out;                 // [B, 16] q(x') (may be null)
  float* acts;                   // [B, act_stride] activations a_0..a_{L-1} of x
  float* dz;                     // [B, dz_stride]  dL/dz_l
  float* loss;                   // [B]
  int B, mode;                   // mode 0 = forward only, 1 = TD update rows, 2 = engine step
  float gamma, coef;
  // ---- engine mode (mode 2)
  const float* prices;           // [E, T]
  float* budget; int* shares; float* value; int* pos; int* episodes; float* last_final; float* ret_sum;
  int* actions_out; float* rewards_out;
  const unsigned long long* ctrl;
  int T, H, compat_env, target_compat, feat_mode, s0, env_offset;
  float eps, inv_ramp, b0, inv_b0;
  uint32_t key0, key1;
  int reward_mode;               // engine mode: 1 = reward is the portfolio's one-step return
  float td_clip;                 // > 0: TD error clamped to [-td_clip, td_clip] (Huber loss)
};

// out[n] = act(sum_k W^T[n][k] * in[k] + b[n]) for n < N (padded N); rows of W^T are contiguous.
// Wide layers (N >= 64): a thread per output neuron, 16-byte weight loads along its W^T row (the 64 rows of a
// wave-instruction are distinct L1 lines, each reused by the lane's next 3 loads) against the input vector
// broadcast from LDS, 4 partial sums -- no cross-lane reduction.  The wave-per-neuron form below did ~N/4
// dependent wave reductions per layer and made a batch-1 TD update ~100 us of kernel time.
ST_DEV void gemv_layer(const float* __restrict__ W, const float* __restrict__ b, const float* in, float* out,
                       int N, int K, int nreal, bool relu, bool legacy = false) {
  if (!legacy && N >= 64 && (K & 3) == 0 && (reinterpret_cast<uintptr_t>(W) & 15) == 0 &&
      (reinterpret_cast<uintptr_t>(in) & 15) == 0) {
    const float4* x4 = reinterpret_cast<const float4*>(in);
    for (int n = threadIdx.x; n < N; n += F_NT) {
      float v = 0.f;
      if (n < nreal) {
        const float4* w = reinterpret_cast<const float4*>(W + (size_t)n * K);
        float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
        for (int k = 0; k < (K >> 2); ++k) {
          const float4 a = w[k], x = x4[k];
          s0 = fmaf(a.x, x.x, s0);
          s1 = fmaf(a.y, x.y, s1);
          s2 = fmaf(a.z, x.z, s2);
          s3 = fmaf(a.w, x.w, s3);
        }
        v = ((s0 + s1) + (s2 + s3)) + (b ? b[n] : 0.f);
      }
      out[n] = relu ? fmaxf(v, 0.f) : v;
    }
    return;
  }
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int n = wave; n < N; n += F_NT / 64) {
    float s = 0.f;
    if (n < nreal) {
      const float* w = W + (size_t)n * K;
      for (int k = lane; k < K; k += 64) s = fmaf(w[k], in[k], s);
    }
    s = wave_sum(s);
    if (lane == 0) {
      float v = (n < nreal) ? s + (b ? b[n] : 0.f) : 0.f;
      out[n] = relu ? fmaxf(v, 0.f) : v;
    }
  }
}

// Forward of one row through all layers; hidden activations into `a` (LDS, a_l at aoff[l]),
// q (16 floats) into `q`.  a[aoff[0]...] must hold the padded input.
ST_DEV void forward_row(const F32Net& net, const float* __restrict__ P, float* a, const int* aoff, float* q) {
  for (int l = 0; l < net.L; ++l) {
    const bool last = (l == net.L - 1);
    const float* b = net.off_b[l] >= 0 ? P + net.off_b[l] : nullptr;
    float* out = last ? q : a + aoff[l + 1];
    gemv_layer(P + net.off_w[l], b, a + aoff[l], out, net.pd[l + 1], net.pd[l], net.dims[l + 1],
               last ? (bool)net.output_relu : true, net.gemv_legacy != 0);
    __syncthreads();
  }
}

ST_DEV float feat_p(float w, float inv, int mode) { return mode ? __fsub_rn(__fmul_rn(w, inv), 1.0f) : w; }

__global__ void __launch_bounds__(F_NT) f32_rows_kernel(F32Net net, F32Rows r) {
  // LDS: two activation stacks (x and x') + q buffers + dz scratch
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int tid = threadIdx.x;
  const int row = blockIdx.x;
  if (row >= r.B) return;  // uniform per workgroup
  int aoff[F_MAXL + 1];
  {
    int o = 0;
    for (int l = 0; l < net.L; ++l) { aoff[l] = o; o += net.pd[l]; }
    aoff[net.L] = o;
  }
  const int astack = aoff[net.L];
  float* A = sm;                 // x activations   [astack]
  float* AN = sm + astack;       // x' activations  [astack]
  float* Q = AN + astack;        // [16]
  float* QN = Q + 16;            // [16]
  float* D0 = QN + 16;           // dz scratch [F_MAXW]
  float* D1 = D0 + F_MAXW;       // dz scratch [F_MAXW]
  __shared__ float s_env[8];
  __shared__ int s_envi[4];
  const float* P = r.params;
  const int in_p = net.pd[0];

  // ------------------------------------------------------------ build the input row(s)
  if (r.mode == 2) {
    const int e = row;
    const int ps = r.pos[e];
    const float* pr = r.prices + (size_t)e * r.T + ps;
    const float last = pr[r.H - 1], vnew = pr[r.H];
    const float inv = __fdiv_rn(1.0f, last), invn = __fdiv_rn(1.0f, vnew);
    const float b = r.budget[e];
    const int s = r.shares[e];
    for (int k = tid; k < in_p; k += F_NT) {
      float v = 0.f, vn = 0.f;
      if (k < r.H) {
        v = feat_p(pr[k], inv, r.feat_mode);
        vn = feat_p(pr[k + 1], invn, r.feat_mode);
      } else if (k == r.H) {
        v = r.feat_mode ? __fmul_rn(b, r.inv_b0) : b;
      } else if (k == r.H + 1) {
        v = r.feat_mode ? __fmul_rn(__fmul_rn((float)s, last), r.inv_b0) : (float)s;
      } else if (k == net.bias_col) {
        v = 1.f;
        vn = 1.f;
      }
      A[k] = v;
      AN[k] = vn;  // budget / shares columns of x' are written after the env step
    }
    if (tid == 0) {
      s_env[0] = b;
      s_env[1] = r.value[e];
      s_env[2] = vnew;
      s_envi[0] = ps;
      s_envi[1] = s;
    }
  } else {
    for (int k = tid; k < in_p; k += F_NT) {
      A[k] = r.x[(size_t)row * in_p + k];
      if (r.mode == 1) AN[k] = r.xn[(size_t)row * in_p + k];
    }
  }
  __syncthreads();
  forward_row(net, P, A, aoff, Q);
  if (r.mode == 0) {
    if (tid < 16) r.q_out[(size_t)row * 16 + tid] = Q[tid];
    return;
  }
  // ------------------------------------------------------------ engine: select + env step
  if (r.mode == 2) {
    if (tid == 0) {
      const int e = row;
      const unsigned long long step = r.ctrl[0];
      const float q0 = Q[0], q1 = Q[1], q2 = Q[2];
      int greedy = 0;
      float best = q0;
      if (q1 > best) { best = q1; greedy = 1; }
      if (q2 > best) { best = q2; greedy = 2; }
      const int ps = s_envi[0];
      uint32_t c0 = (uint32_t)(r.env_offset + e), c1 = (uint32_t)(step & 0xFFFFFFFFull),
               c2 = (uint32_t)(step >> 32), c3 = 0u;
      philox4x32(c0, c1, c2, c3, r.key0, r.key1);
      const float u1 = u24(c0), u2 = u24(c1);
      const bool exploit = u1 < fminf(r.eps, __fmul_rn((float)ps, r.inv_ramp));
      int rnd = (int)(u2 * 3.0f);
      rnd = rnd > 2 ? 2 : rnd;
      const int a = exploit ? greedy : rnd;
      const float b = s_env[0], vprev = s_env[1], vnew = s_env[2];
      const int s = s_envi[1];
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
      s_env[3] = b2;
      s_env[4] = rew;
      s_envi[1] = s2;
      s_envi[2] = a;
      AN[r.H] = r.feat_mode ? __fmul_rn(b2, r.inv_b0) : b2;
      AN[r.H + 1] = r.feat_mode ? __fmul_rn(__fmul_rn((float)s2, vnew), r.inv_b0) : (float)s2;
      if (r.actions_out) r.actions_out[e] = a;
      if (r.rewards_out) r.rewards_out[e] = rew;
    }
    __syncthreads();
  }
  forward_row(net, P, AN, aoff, QN);
  // ------------------------------------------------------------ TD target + dQ
  __shared__ int s_slot;
  if (tid == 0) {
    const float n0 = QN[0], n1 = QN[1], n2 = QN[2];
    int am = 0;
    float mx = n0;
    if (n1 > mx) { mx = n1; am = 1; }
    if (n2 > mx) { mx = n2; am = 2; }
    int slot;
    float rew;
    if (r.mode == 2) {
      slot = r.target_compat ? am : s_envi[2];
      rew = s_env[4];
    } else {
      slot = r.action ? r.action[row] : am;
      rew = r.reward[row];
    }
    const float y = __fadd_rn(rew, __fmul_rn(r.gamma, mx));
    const float qs = Q[slot];
    const float diff = __fsub_rn(qs, y);
    float dq = r.coef * (r.td_clip > 0.f ? fminf(fmaxf(diff, -r.td_clip), r.td_clip) : diff);
    if (net.output_relu && !(qs > 0.f)) dq = 0.f;
    s_slot = slot;
    D0[0] = dq;
    r.loss[row] = diff * diff;
    if (r.qn_out) {
      for (int j = 0; j < 16; ++j) r.qn_out[(size_t)row * 16 + j] = QN[j];
    }
    if (r.q_out) {
      for (int j = 0; j < 16; ++j) r.q_out[(size_t)row * 16 + j] = Q[j];
    }
    if (r.mode == 2) {
      // env state write-back
      const int e = row;
      const float b2 = s_env[3], vnew = s_env[2];
      const int s2 = s_envi[1];
      const int np = s_envi[0] + 1;
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
        r.ret_sum[e] = r.ret_sum[e] + s_env[4];
      }
    }
  }
  __syncthreads();
  // ------------------------------------------------------------ backward (data) through every layer
  float* acts_row = r.acts + (size_t)row * net.act_stride;
  float* dz_row = r.dz + (size_t)row * net.dz_stride;
  // activations of x: a_0 .. a_{L-1}
  for (int l = 0; l < net.L; ++l)
    for (int k = tid; k < net.pd[l]; k += F_NT) acts_row[net.act_off[l] + k] = A[aoff[l] + k];
  // dz of the output layer: only the slot entry is non-zero
  {
    const int lo = net.L - 1;
    for (int k = tid; k < net.pd[net.L]; k += F_NT) dz_row[net.dz_off[lo] + k] = (k == s_slot) ? D0[0] : 0.f;
  }
  // dz_{l-1}[i] = (sum_o dz_l[o] * W_l[o][i]) * (a_l[i] > 0); the output layer's dz is one-hot
  float* dcur = D1;
  {
    const int l = net.L - 1;
    const float* W = P + net.off_w[l];
    const float g = D0[0];
    for (int i = tid; i < net.pd[l]; i += F_NT) {
      const float h = A[aoff[l] + i];
      dcur[i] = (h > 0.f) ? g * W[(size_t)s_slot * net.pd[l] + i] : 0.f;
    }
  }
  __syncthreads();
  for (int l = net.L - 1; l >= 1; --l) {
    // dcur = dz_{l-1}, width pd[l]
    for (int k = tid; k < net.pd[l]; k += F_NT) dz_row[net.dz_off[l - 1] + k] = dcur[k];
    if (l == 1) break;
    float* dnext = (dcur == D1) ? D0 : D1;
    const float* W = P + net.off_w[l - 1];   // [pd[l]][pd[l-1]]
    const int N = net.pd[l], K = net.pd[l - 1];
    for (int i = tid; i < K; i += F_NT) {
      float s = 0.f;
      for (int o = 0; o < N; ++o) s = fmaf(dcur[o], W[(size_t)o * K + i], s);
      const float h = A[aoff[l - 1] + i];
      dnext[i] = (h > 0.f) ? s : 0.f;
    }
    __syncthreads();
    dcur = dnext;
  }
}

struct F32Optim {
  float* params;
  const float* mask;
  float* s1;
  float* s2;
  const float* acts;
  const float* dz;
  const unsigned long long* ctrl;  // engine mode: update count t = ctrl[0] + 1 (graph-replay safe)
  float* grad;                     // mode 1: gradient out; mode 2: gradient in (after all-reduce)
  int B, kind, t, mode;            // mode 0 = grad + update, 1 = grad only, 2 = update from grad
  float lr, beta1, beta2, eps, scale;
};

// One thread per parameter of the flat buffer: weight gradient (sum over rows of
// outer products) + optimizer step.
__global__ void __launch_bounds__(256) f32_grad_optim_kernel(F32Net net, F32Optim o) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= net.P) return;
  const float m = o.mask[p];
  float g = 0.f;
  if (o.mode == 2) {
    g = o.grad[p];
  } else {
    if (m == 0.f) {
      if (o.mode == 1) o.grad[p] = 0.f;
      return;
    }
    // locate the segment
    bool found = false;
    for (int l = 0; l < net.L && !found; ++l) {
      const int nw = net.pd[l + 1] * net.pd[l];
      if (p >= net.off_w[l] && p < net.off_w[l] + nw) {
        const int q = p - net.off_w[l];
        const int out = q / net.pd[l], in = q % net.pd[l];
        for (int b = 0; b < o.B; ++b)
          g = fmaf(o.dz[(size_t)b * net.dz_stride + net.dz_off[l] + out],
                   o.acts[(size_t)b * net.act_stride + net.act_off[l] + in], g);
        found = true;
      } else if (net.off_b[l] >= 0 && p >= net.off_b[l] && p < net.off_b[l] + net.pd[l + 1]) {
        const int out = p - net.off_b[l];
        for (int b = 0; b < o.B; ++b) g += o.dz[(size_t)b * net.dz_stride + net.dz_off[l] + out];
        found = true;
      }
    }
    if (o.mode == 1) {
      o.grad[p] = found ? g : 0.f;
      return;
    }
    if (!found) return;
  }
  if (m == 0.f) return;
  g *= m * o.scale;
  const int t = o.ctrl ? (int)(o.ctrl[0] + 1) : o.t;
  float w = o.params[p];
  if (o.kind == 1) {  // AdaGrad (TF ApplyAdagrad: acc += g^2; w -= lr * g * rsqrt(acc))
    const float a = o.s1[p] + g * g;
    o.s1[p] = a;
    w -= o.lr * g / sqrtf(a);
  } else if (o.kind == 2) {  // Adam
    const float c1 = 1.f - powf(o.beta1, (float)t), c2 = 1.f - powf(o.beta2, (float)t);
    const float mm = o.beta1 * o.s1[p] + (1.f - o.beta1) * g;
    const float vv = o.beta2 * o.s2[p] + (1.f - o.beta2) * g * g;
    o.s1[p] = mm;
    o.s2[p] = vv;
    w -= o.lr * (mm / c1) / (sqrtf(vv / c2) + o.eps);
  } else {
    w -= o.lr * g;
  }
  o.params[p] = w;
}

__global__ void f32_advance_kernel(unsigned long long* ctrl) { ctrl[0] += 1; }

}  // namespace st

extern "C" int st_f32_lds_bytes(const st::F32Net* net) {
  int astack = 0;
  for (int l = 0; l < net->L; ++l) astack += net->pd[l];
  return (2 * astack + 32 + 2 * st::F_MAXW) * 4;
}

extern "C" hipError_t st_f32_rows(const st::F32Net* net, const st::F32Rows* rows, hipStream_t stream) {
  if (net->L < 1 || net->L > st::F_MAXL) return hipErrorInvalidValue;
  for (int l = 0; l <= net->L; ++l)
    if (net->pd[l] > st::F_MAXW || net->pd[l] <= 0) return hipErrorInvalidValue;
  const int lds = st_f32_lds_bytes(net);
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)st::f32_rows_kernel,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
    if (e != hipSuccess) return e;
    attr = true;
  }
  if (lds > 65536) return hipErrorInvalidValue;
  hipLaunchKernelGGL(st::f32_rows_kernel, dim3(rows->B), dim3(st::F_NT), lds, stream, *net, *rows);
  return hipGetLastError();
}

extern "C" hipError_t st_f32_grad_optim(const st::F32Net* net, const st::F32Optim* o, hipStream_t stream) {
  hipLaunchKernelGGL(st::f32_grad_optim_kernel, dim3((net->P + 255) / 256), dim3(256), 0, stream, *net, *o);
  return hipGetLastError();
}

extern "C" hipError_t st_f32_advance(unsigned long long* ctrl, hipStream_t stream) {
  hipLaunchKernelGGL(st::f32_advance_kernel, dim3(1), dim3(1), 0, stream, ctrl);
  return hipGetLastError();
}

// struct sizes of this file's launch ABI, for the host mirrors' check (tests/test_abi.py; no HIP call)
extern "C" int st_abi_mlp_f32(int* out, int n) {
  const int sz[] = {(int)sizeof(st::F32Net), (int)sizeof(st::F32Rows), (int)sizeof(st::F32Optim)};
  const int m = (int)(sizeof(sz) / sizeof(sz[0]));
  for (int i = 0; i < n && i < m; ++i) out[i] = sz[i];
  return m;
}
