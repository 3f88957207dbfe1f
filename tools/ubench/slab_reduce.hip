// Micro-benchmark: column reduction of G per-workgroup gradient slabs of P parameters (the read side
// of csrc/optim.hip's reduce_optim_kernel): row-major [G][P] vs column-blocked [P/128][G][128] bf16
// slabs, workgroup shapes, serial vs tree fold of the row-group partials.  Run under
//   rocprofv3 --kernel-trace --stats -- tools/ubench/slab_reduce.bin
// (kernel times from the trace; the template arguments name the variant).
#include <hip/hip_runtime.h>
#include <cstdio>

// RT threads = CW 16-byte columns x RG row groups; each thread owns 8 bf16 parameters.
// HALF: the workgroup reads CW=8 of a block's 16 columns (two workgroups per 128-column block).
template <int RT, int CW, bool BLOCKED, bool TREE>
__global__ void __launch_bounds__(RT) red(const uint4* __restrict__ slab, float4* __restrict__ out, int G, int PV) {
  constexpr int RG = RT / CW;
  __shared__ float4 part[RG][CW][2];
  const int tid = threadIdx.x, rg = tid / CW, c = tid % CW;
  const int colv = blockIdx.x * CW + c;
  float4 g0 = make_float4(0.f, 0.f, 0.f, 0.f), g1 = g0;
  const int blk = colv / 16, cin = colv % 16;
  const uint4* sp = BLOCKED ? slab + (size_t)blk * G * 16 + cin : slab + colv;
  const size_t rs = BLOCKED ? 16 : PV;
#pragma unroll 8
  for (int r = rg; r < G; r += RG) {
    const uint4 v = sp[(size_t)r * rs];
    g0.x += __uint_as_float(v.x << 16); g0.y += __uint_as_float(v.x & 0xFFFF0000u);
    g0.z += __uint_as_float(v.y << 16); g0.w += __uint_as_float(v.y & 0xFFFF0000u);
    g1.x += __uint_as_float(v.z << 16); g1.y += __uint_as_float(v.z & 0xFFFF0000u);
    g1.z += __uint_as_float(v.w << 16); g1.w += __uint_as_float(v.w & 0xFFFF0000u);
  }
  part[rg][c][0] = g0;
  part[rg][c][1] = g1;
  __syncthreads();
  if constexpr (TREE) {
#pragma unroll
    for (int s = RG / 2; s > 0; s >>= 1) {
      if (rg < s) {
        const float4 a = part[rg + s][c][0], b = part[rg + s][c][1];
        g0.x += a.x; g0.y += a.y; g0.z += a.z; g0.w += a.w;
        g1.x += b.x; g1.y += b.y; g1.z += b.z; g1.w += b.w;
        part[rg][c][0] = g0;
        part[rg][c][1] = g1;
      }
      __syncthreads();
    }
    if (rg != 0) return;
  } else {
    if (rg != 0) return;
    for (int k = 1; k < RG; ++k) {
      const float4 a = part[k][c][0], b = part[k][c][1];
      g0.x += a.x; g0.y += a.y; g0.z += a.z; g0.w += a.w;
      g1.x += b.x; g1.y += b.y; g1.z += b.z; g1.w += b.w;
    }
  }
  out[2 * colv] = g0;
  out[2 * colv + 1] = g1;
}

template <int RT, int CW, bool BLOCKED, bool TREE>
void run(const uint4* slab, float4* out, int G, int PV) {
  for (int it = 0; it < 30; ++it) red<RT, CW, BLOCKED, TREE><<<PV / CW, RT>>>(slab, out, G, PV);
  (void)hipDeviceSynchronize();
}

int main() {
  const int G = 256, P = 47360;   // 2x128 Q-net parameter count, padded to a multiple of 128
  uint4* slab;
  float4* out;
  (void)hipMalloc(&slab, (size_t)G * P * 2);
  (void)hipMalloc(&out, (size_t)P * 4);
  (void)hipMemset(slab, 0, (size_t)G * P * 2);
  const int PV = P / 8;
  run<512, 16, false, false>(slab, out, G, PV);
  run<512, 16, true, false>(slab, out, G, PV);
  run<512, 16, true, true>(slab, out, G, PV);
  run<256, 16, true, true>(slab, out, G, PV);
  run<256, 8, true, true>(slab, out, G, PV);
  run<512, 8, true, true>(slab, out, G, PV);
  run<1024, 16, true, true>(slab, out, G, PV);
  run<128, 8, true, true>(slab, out, G, PV);
  run<256, 4, true, true>(slab, out, G, PV);
  printf("done\n");
  return 0;
}
