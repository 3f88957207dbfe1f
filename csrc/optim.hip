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
  int slab_bf16;           // slabs are bf16, column-blocked [P/32][G][32] (P % 32 == 0), else fp32 [G][P]
  unsigned* chunk_heads;   // the step kernel's 8 per-XCD chunk-claim heads (stride 32 words) or null:
                           // re-zeroed by the slab pass (it runs after the step kernel, before the next)
  float* ema;              // [P] Polyak average of the parameters (the weights to serve) or null
  float ema_decay;         // ema <- ema + (1 - decay) (w - ema) after every update
  // the ws step kernel's weight images (csrc/qstep_ws.hip QStepParams::wimg) kept current: img_map[i] = bf16
  // element of img (>= 0), -(fp32 word) - 2, or -1 (not in it); both null = no image
  const int* img_map;
  unsigned char* img;
};

// write parameter i (fp32 value w) into the ws weight image
ST_DEV void img_put(unsigned char* img, const int* map, int i, float w) {
  const int d = map[i];
  if (d >= 0) reinterpret_cast<bf16_t*>(img)[d] = f2bf(w);
  else if (d <= -2) reinterpret_cast<float*>(img)[-d - 2] = w;
}

constexpr int CW = 16;    // 16-byte slab columns per workgroup (256 B of every slab row)
constexpr int SLAB_BLK = 128;   // bf16 slabs: parameters per reduce workgroup (= CW x 8) = 4 column blocks
constexpr int SLAB_CB = 32;     // bf16 slabs: parameters per column block of the slab layout

// NV parameters per thread column: 4 (fp32 slabs [G][P], one float4 per row) or 8 (bf16 slabs: the
// step kernel rounds each workgroup's fp32 partial sum once and stores it column-BLOCKED,
// [P/128][G][128], so this workgroup's 128 columns of all G rows are one contiguous 64 KB run
// instead of G strided 256-byte pieces; 8 bf16 = one 16-byte load per row).  The sums are fp32.
// tools/ubench/slab_reduce.hip measured the layouts / shapes (profiles/r1_slab_reduce.md).
template <int NV, int RT>
__global__ void __launch_bounds__(RT) reduce_optim_kernel(OptimParams p) {
  constexpr int NQ = NV / 4;   // float4 groups per thread column
  constexpr int RG = RT / CW;  // row groups per workgroup: independent partial sums per column
  __shared__ float4 part[RG][CW][NQ];
  const int tid = threadIdx.x, rg = tid / CW, c = tid % CW;
  const int colv = blockIdx.x * CW + c;  // NV-parameter column index
  const int PV = p.P / NV;
  if (p.mode != 2 && p.chunk_heads && blockIdx.x == 0 && tid < 8) p.chunk_heads[32 * tid] = 0u;
  if (p.mode != 2 && p.stats && blockIdx.x == 0) {
    // step statistics folded into this pass (no extra launches; block 0 is dispatched first): thread t
    // sums stat (t & 7) over rows t/8, t/8 + RT/8, ...; then a shuffle fold over the 8 lanes of a
    // wave that share the stat, and one LDS slot per wave (all in fp64)
    __shared__ double sred[RT / 64][8];
    const int j = tid & 7, grp = tid >> 3, lane = tid & 63, w = tid >> 6;
    double acc = 0.0;
    if (j < p.nstat)
      for (int r = grp; r < p.G; r += RT / 8) acc += (double)p.stats[r * p.nstat + j];
#pragma unroll
    for (int o = 8; o < 64; o <<= 1) acc += __shfl_xor(acc, o, 64);
    if (lane < 8) sred[w][lane] = acc;
    __syncthreads();
    if (tid < p.nstat) {
      double t = 0.0;
#pragma unroll
      for (int k = 0; k < RT / 64; ++k) t += sred[k][tid];
      p.stat_acc[tid] += t;
    }
  }
  // one thread per parameter of this workgroup's NP = CW * NV columns does the update (was: the 16
  // lanes of row group 0 with NV parameters each -- a one-wave tail per workgroup).  Its operands are
  // fetched BEFORE the slab pass, so their latency hides under it.
  constexpr int NP = CW * NV;
  static_assert(NP <= RT, "one updating thread per parameter");
  const int pidx = blockIdx.x * NP + tid;
  const bool own = tid < NP && pidx < p.P;
  float w = 0.f, mk = 0.f, s1 = 0.f, s2 = 0.f, gsum = 0.f, ema = 0.f;
  if (own) {
    mk = p.mask[pidx];
    if (p.mode != 1) {
      w = p.params[pidx];
      if (p.kind >= 1) s1 = p.s1[pidx];
      if (p.kind == 2) s2 = p.s2[pidx];
      if (p.ema) ema = p.ema[pidx];
    }
  }
  if (p.mode != 2) {
    float4 g[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) g[q] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (colv < PV) {
      if constexpr (NV == 4) {
        const float4* sp = reinterpret_cast<const float4*>(p.slab) + colv;
#pragma unroll 8
        for (int r = rg; r < p.G; r += RG) {
          const float4 v = sp[(size_t)r * PV];
          g[0].x += v.x; g[0].y += v.y; g[0].z += v.z; g[0].w += v.w;
        }
      } else {
        // column c of this workgroup: block 4 * blockIdx.x + c / 4, 16-byte piece c % 4 of its 64-byte rows
        constexpr int PPB = SLAB_CB / 8;   // 16-byte pieces per block row
        const uint4* sp = reinterpret_cast<const uint4*>(p.slab) +
                          (size_t)(blockIdx.x * (CW / PPB) + c / PPB) * p.G * PPB + c % PPB;
#pragma unroll 8
        for (int r = rg; r < p.G; r += RG) {
          const uint4 v = sp[(size_t)r * PPB];
          g[0].x += __uint_as_float(v.x << 16); g[0].y += __uint_as_float(v.x & 0xFFFF0000u);
          g[0].z += __uint_as_float(v.y << 16); g[0].w += __uint_as_float(v.y & 0xFFFF0000u);
          g[1].x += __uint_as_float(v.z << 16); g[1].y += __uint_as_float(v.z & 0xFFFF0000u);
          g[1].z += __uint_as_float(v.w << 16); g[1].w += __uint_as_float(v.w & 0xFFFF0000u);
        }
      }
    }
    // partials [RG][NP] in LDS (part[rg][c][q] as floats: parameter c * NV + 4q + k of row group rg)
#pragma unroll
    for (int q = 0; q < NQ; ++q) part[rg][c][q] = g[q];
    __syncthreads();
    if (!own) return;
    const float* pf = reinterpret_cast<const float*>(&part[0][0][0]);
    float a0 = 0.f, a1 = 0.f;   // two chains: fixed order, deterministic
#pragma unroll
    for (int k = 0; k < RG; k += 2) {
      a0 += pf[k * NP + tid];
      a1 += pf[(k + 1) * NP + tid];
    }
    gsum = (a0 + a1) * p.scale;
    if (p.mode == 1) {
      // masked like the update (padding entries of the 64-env-chunk kernel's slabs are not zero)
      p.grad[pidx] = gsum * mk;
      return;
    }
  } else {
    if (!own) return;
    gsum = p.grad[pidx] * p.scale;
  }
  const unsigned long long tstep = p.ctrl[1];
  if (blockIdx.x == 0 && tid == 0) p.ctrl[0] = tstep;  // next step index (read by the next step kernel)
  const unsigned long long t = tstep - (unsigned long long)p.tdelay;   // 1-based optimizer update count
  const float gk = gsum * mk;
  if (p.kind == 1) {  // AdaGrad (TF ApplyAdagrad)
    s1 += gk * gk;
    w -= p.lr * gk * rsqrtf(s1);
    p.s1[pidx] = s1;
  } else if (p.kind == 2) {  // Adam
    const float ic1 = 1.f / (1.f - powf(p.beta1, (float)t));
    const float ic2 = 1.f / (1.f - powf(p.beta2, (float)t));
    s1 = p.beta1 * s1 + (1.f - p.beta1) * gk;
    s2 = p.beta2 * s2 + (1.f - p.beta2) * gk * gk;
    w -= p.lr * (s1 * ic1) / (sqrtf(s2 * ic2) + p.eps) * mk;
    p.s1[pidx] = s1;
    p.s2[pidx] = s2;
  } else {  // SGD
    w -= p.lr * gk;
  }
  p.params[pidx] = w;
  if (p.params_bf) p.params_bf[pidx] = f2bf(w);
  if (p.img) img_put(p.img, p.img_map, pidx, w);
  if (p.ema) p.ema[pidx] = ema + (1.f - p.ema_decay) * (w - ema);
}

// ctrl[1] = ctrl[0] + 1 : the 1-based update count of the step about to run.
__global__ void advance_kernel(unsigned long long* ctrl) { ctrl[1] = ctrl[0] + 1; }
// ctrl[0] = ctrl[1] : commit the step index without an optimizer update (first overlapped-DP step)
__global__ void commit_kernel(unsigned long long* ctrl) { ctrl[0] = ctrl[1]; }

// the whole ws weight image from the fp32 parameters (after parameters change outside the optimizer pass)
__global__ void img_pack_kernel(const float* __restrict__ params, const int* __restrict__ map, unsigned char* img, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) img_put(img, map, i, params[i]);
}

__global__ void to_bf16_kernel(const float* __restrict__ in, bf16_t* __restrict__ out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = f2bf(in[i]);
}

}  // namespace st

extern "C" hipError_t st_reduce_optim(const st::OptimParams* p, hipStream_t stream) {
  if (p->stats && (p->nstat < 1 || p->nstat > 8)) return hipErrorInvalidValue;
  if (!p->mask || !p->params) return hipErrorInvalidValue;   // every mode reads the trainable mask
  if (p->slab_bf16 && p->mode != 2) {
    if (p->P % st::SLAB_CB != 0) return hipErrorInvalidValue;
    const int grid = (p->P + st::SLAB_BLK - 1) / st::SLAB_BLK;   // 128 parameters (4 column blocks) each
    hipLaunchKernelGGL((st::reduce_optim_kernel<8, 512>), dim3(grid), dim3(512), 0, stream, *p);
  } else {
    if (p->P % 4 != 0) return hipErrorInvalidValue;
    const int grid = (p->P / 4 + st::CW - 1) / st::CW;   // ~740 workgroups for the 2x128 net: fills 256 CUs
    hipLaunchKernelGGL((st::reduce_optim_kernel<4, 256>), dim3(grid), dim3(256), 0, stream, *p);
  }
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

extern "C" hipError_t st_img_pack(const float* params, const int* map, unsigned char* img, int n, hipStream_t stream) {
  if (n <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(st::img_pack_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, params, map, img, n);
  return hipGetLastError();
}

extern "C" hipError_t st_to_bf16(const float* in, bf16_t* out, int n, hipStream_t stream) {
  hipLaunchKernelGGL(st::to_bf16_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, in, out, n);
  return hipGetLastError();
}

// struct sizes of this file's launch ABI, for the host mirrors' check (tests/test_abi.py; no HIP call)
extern "C" int st_abi_optim(int* out, int n) {
  const int sz[] = {(int)sizeof(st::OptimParams)};
  const int m = (int)(sizeof(sz) / sizeof(sz[0]));
  for (int i = 0; i < n && i < m; ++i) out[i] = sz[i];
  return m;
}
