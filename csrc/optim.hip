// Gradient-slab reduction + optimizer step (SGD / AdaGrad / Adam) over the flat
// fp32 parameter buffer, fused with the fp32 -> bf16 weight refresh the fused
// step kernel consumes.
//
// Reference: `tf.train.AdaGrad(0.01f).minimize(loss)` (QDecisionPolicyActor.scala:50)
// emits ApplyAdagrad on W1/W2 after every UpdateQ; here the update is one
// bandwidth-bound pass over ~50k-3M parameters per engine step.
//
// Step counters live in device memory so that a captured HIP graph replays
// correctly: ctrl[0] = step index read by the fused step kernel, ctrl[1] =
// 1-based update count read here (written by the step kernel's host wrapper
// protocol below):  this kernel reads ctrl[1] and block 0 writes ctrl[0] =
// ctrl[1]; ctrl[1] is advanced by st_advance (1 thread) at step start.
#include "common.h"

namespace st {

struct OptimParams {
  float* params;           // [P] fp32 master
  bf16_t* params_bf;       // [P] bf16 copy (may be null)
  const float* mask;       // [P] trainable mask
  float* s1;               // adagrad acc / adam m
  float* s2;               // adam v
  const float* slab;       // [G][P] partial gradients (fused reduce) or null
  float* grad;             // [P] gradient in (if slab null) / out (reduce-only)
  unsigned long long* ctrl;
  const float* stats;      // [G][nstat] per-workgroup step statistics (or null)
  double* stat_acc;        // [nstat] running fp64 totals
  int G, P, kind, mode;    // mode: 0 = reduce+update, 1 = reduce only, 2 = update only
  int nstat;
  float lr, beta1, beta2, eps, scale;
  int tdelay;              // updates lagging the step counter (overlapped DP applies step t-1's gradient at t)
};

constexpr int RT = 256;   // threads per workgroup
constexpr int CW = 16;    // float4 columns per workgroup (256 B of every slab row)
constexpr int RG = RT / CW;  // row groups per workgroup: 16 independent partial sums per column

__global__ void __launch_bounds__(RT) reduce_optim_kernel(OptimParams p) {
  __shared__ float4 part[RG][CW];
  const int tid = threadIdx.x, rg = tid / CW, c = tid % CW;
  const int col4 = blockIdx.x * CW + c;  // float4 column index
  const int P4 = p.P >> 2;
  if (p.mode != 2 && p.stats && blockIdx.x == gridDim.x - 1) {
    // step statistics folded into this pass (no extra launches): 32 row groups x 8 stats
    __shared__ double sred[RT / 8][8];
    const int j = tid & 7, grp = tid >> 3;
    double acc = 0.0;
    if (j < p.nstat)
      for (int r = grp; r < p.G; r += RT / 8) acc += (double)p.stats[r * p.nstat + j];
    sred[grp][j] = acc;
    __syncthreads();
    if (tid < p.nstat) {
      double t = 0.0;
      for (int k = 0; k < RT / 8; ++k) t += sred[k][tid];
      p.stat_acc[tid] += t;
    }
  }
  float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
  if (p.mode != 2) {
    if (col4 < P4) {
      const float4* s = reinterpret_cast<const float4*>(p.slab) + col4;
#pragma unroll 8
      for (int r = rg; r < p.G; r += RG) {
        const float4 v = s[(size_t)r * P4];
        g.x += v.x; g.y += v.y; g.z += v.z; g.w += v.w;
      }
    }
    part[rg][c] = g;
    __syncthreads();
    if (rg != 0) return;
    for (int k = 1; k < RG; ++k) {
      const float4 v = part[k][c];
      g.x += v.x; g.y += v.y; g.z += v.z; g.w += v.w;
    }
    g.x *= p.scale; g.y *= p.scale; g.z *= p.scale; g.w *= p.scale;
    if (p.mode == 1) {
      if (col4 < P4) reinterpret_cast<float4*>(p.grad)[col4] = g;
      return;
    }
  } else {
    if (rg != 0) return;
    if (col4 < P4) {
      g = reinterpret_cast<const float4*>(p.grad)[col4];
      g.x *= p.scale; g.y *= p.scale; g.z *= p.scale; g.w *= p.scale;
    }
  }
  const unsigned long long tstep = p.ctrl[1];
  if (blockIdx.x == 0 && tid == 0) p.ctrl[0] = tstep;  // next step index (read by the next step kernel)
  const unsigned long long t = tstep - (unsigned long long)p.tdelay;   // 1-based optimizer update count
  if (col4 >= P4) return;
  float gg[4] = {g.x, g.y, g.z, g.w};
  const float4 m4 = reinterpret_cast<const float4*>(p.mask)[col4];
  const float mm[4] = {m4.x, m4.y, m4.z, m4.w};
  float4 w4 = reinterpret_cast<float4*>(p.params)[col4];
  float w[4] = {w4.x, w4.y, w4.z, w4.w};
  if (p.kind == 1) {  // AdaGrad (TF ApplyAdagrad)
    float4 a4 = reinterpret_cast<float4*>(p.s1)[col4];
    float a[4] = {a4.x, a4.y, a4.z, a4.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float gk = gg[k] * mm[k];
      a[k] += gk * gk;
      w[k] -= p.lr * gk * rsqrtf(a[k]);
    }
    reinterpret_cast<float4*>(p.s1)[col4] = make_float4(a[0], a[1], a[2], a[3]);
  } else if (p.kind == 2) {  // Adam
    const float c1 = 1.f - powf(p.beta1, (float)t), c2 = 1.f - powf(p.beta2, (float)t);
    const float ic1 = 1.f / c1, ic2 = 1.f / c2;
    float4 m4v = reinterpret_cast<float4*>(p.s1)[col4];
    float4 v4v = reinterpret_cast<float4*>(p.s2)[col4];
    float m[4] = {m4v.x, m4v.y, m4v.z, m4v.w}, v[4] = {v4v.x, v4v.y, v4v.z, v4v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float gk = gg[k] * mm[k];
      m[k] = p.beta1 * m[k] + (1.f - p.beta1) * gk;
      v[k] = p.beta2 * v[k] + (1.f - p.beta2) * gk * gk;
      w[k] -= p.lr * (m[k] * ic1) / (sqrtf(v[k] * ic2) + p.eps) * mm[k];
    }
    reinterpret_cast<float4*>(p.s1)[col4] = make_float4(m[0], m[1], m[2], m[3]);
    reinterpret_cast<float4*>(p.s2)[col4] = make_float4(v[0], v[1], v[2], v[3]);
  } else {  // SGD
#pragma unroll
    for (int k = 0; k < 4; ++k) w[k] -= p.lr * gg[k] * mm[k];
  }
  reinterpret_cast<float4*>(p.params)[col4] = make_float4(w[0], w[1], w[2], w[3]);
  if (p.params_bf) {
    uint2 o;
    o.x = pack_bf2(w[0], w[1]);
    o.y = pack_bf2(w[2], w[3]);
    reinterpret_cast<uint2*>(p.params_bf)[col4] = o;
  }
}

// ctrl[1] = ctrl[0] + 1 : the 1-based update count of the step about to run.
__global__ void advance_kernel(unsigned long long* ctrl) { ctrl[1] = ctrl[0] + 1; }
// ctrl[0] = ctrl[1] : commit the step index without an optimizer update (first overlapped-DP step)
__global__ void commit_kernel(unsigned long long* ctrl) { ctrl[0] = ctrl[1]; }

__global__ void to_bf16_kernel(const float* __restrict__ in, bf16_t* __restrict__ out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = f2bf(in[i]);
}

}  // namespace st

extern "C" hipError_t st_reduce_optim(const st::OptimParams* p, hipStream_t stream) {
  const int P4 = p->P >> 2;
  const int grid = (P4 + st::CW - 1) / st::CW;   // ~740 workgroups for the 2x128 net: fills 256 CUs
  hipLaunchKernelGGL(st::reduce_optim_kernel, dim3(grid), dim3(st::RT), 0, stream, *p);
  return hipGetLastError();
}

extern "C" hipError_t st_advance(unsigned long long* ctrl, hipStream_t stream) {
  hipLaunchKernelGGL(st::advance_kernel, dim3(1), dim3(1), 0, stream, ctrl);
  return hipGetLastError();
}

extern "C" hipError_t st_commit_step(unsigned long long* ctrl, hipStream_t stream) {
  hipLaunchKernelGGL(st::commit_kernel, dim3(1), dim3(1), 0, stream, ctrl);
  return hipGetLastError();
}

extern "C" hipError_t st_to_bf16(const float* in, bf16_t* out, int n, hipStream_t stream) {
  hipLaunchKernelGGL(st::to_bf16_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, in, out, n);
  return hipGetLastError();
}
