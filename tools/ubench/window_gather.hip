// Micro-benchmark: gathering every env's 202-price window from the HBM bank, as the flagship step
// (csrc/qstep_ws.hip) and the target pass (csrc/qtarget.hip) do, in two access patterns.
//
//   A  operand pattern (the kernels today): a wave owns a 16-env tile; lane (env l16, group g4) loads the
//      float4 pairs of its MFMA B operand -- per instruction 16 rows x 4 scattered 16-byte pieces;
//   B  row pattern: one instruction per env row, lane i loads floats 4i .. 4i + 3 (51 lanes cover the
//      202 floats): every instruction reads one contiguous 816-byte run.
//
// Each wave folds what it loaded into one value per lane (so nothing is dead) and writes it out.  Reports
// useful bytes / kernel time.  One bank row per env, T4 floats apart (as the engine's padded copy), random
// window positions.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench/window_gather.bin tools/ubench/window_gather.hip
//   tools/ubench/window_gather.bin [envs]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int T = 6047, T4 = 6064, H = 201;

__device__ __forceinline__ float4 ldu4(const float* a) {
  float4 v;
  __builtin_memcpy(&v, a, sizeof(v));
  return v;
}

// A: the qtarget / ws operand pattern (13 float4 per lane per tile)
__global__ void __launch_bounds__(512) gather_operand(const float* bank, const int* pos, float* out, int E) {
  const int lane = threadIdx.x & 63, l16 = lane & 15, g4 = lane >> 4;
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, nwaves = (gridDim.x * blockDim.x) >> 6;
  float acc = 0.f;
  for (int t = wave; t < E / 16; t += nwaves) {
    const int e = 16 * t + l16;
    const float* b = bank + (size_t)e * T4 + pos[e];
#pragma unroll
    for (int ks = 0; ks < 6; ++ks) {
      const float4 u = ldu4(b + 1 + 32 * ks + 8 * g4), v = ldu4(b + 5 + 32 * ks + 8 * g4);
      acc += u.x + u.y + u.z + u.w + v.x + v.y + v.z + v.w;
    }
    if (g4 == 1 || g4 == 2) {
      const float4 u = ldu4(b + 193 + 4 * (g4 - 1));
      acc += u.x + u.y + u.z + u.w;
    }
    acc += b[201];
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

// B: one contiguous row per instruction (lanes 0..50 useful)
__global__ void __launch_bounds__(512) gather_rows(const float* bank, const int* pos, float* out, int E) {
  const int lane = threadIdx.x & 63;
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, nwaves = (gridDim.x * blockDim.x) >> 6;
  float acc = 0.f;
  for (int t = wave; t < E / 16; t += nwaves) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int e = 16 * t + r;
      const float* b = bank + (size_t)e * T4 + pos[e];
      if (lane < 51) {
        const float4 u = ldu4(b + 4 * lane);
        acc += u.x + u.y + u.z + u.w;
      }
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main(int argc, char** argv) {
  const int E = argc > 1 ? atoi(argv[1]) : 1835008;
  float* bank;
  int* pos;
  float* out;
  const size_t nb = (size_t)E * T4 + 64;
  if (hipMalloc(&bank, nb * sizeof(float)) != hipSuccess) return 1;
  if (hipMemset(bank, 0, nb * sizeof(float)) != hipSuccess) return 1;
  std::vector<int> hp(E);
  srand(7);
  for (int i = 0; i < E; ++i) hp[i] = rand() % (T - H - 2);
  if (hipMalloc(&pos, E * sizeof(int)) != hipSuccess) return 1;
  if (hipMemcpy(pos, hp.data(), E * sizeof(int), hipMemcpyHostToDevice) != hipSuccess) return 1;
  if (hipMalloc(&out, 1 << 24) != hipSuccess) return 1;
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const double useful = (double)E * 202 * 4;
  printf("| pattern | waves / CU | grid | us | useful GB/s |\n|---|---|---|---|---|\n");
  for (int pat = 0; pat < 2; ++pat)
    for (int wpc : {8, 16, 32}) {
      const int threads = 512, blocks = 256 * wpc / 8;
      for (int rep = 0; rep < 2; ++rep) {   // (first rep warms up)
        (void)hipEventRecord(a, 0);
        for (int i = 0; i < 5; ++i) {
          if (pat == 0)
            hipLaunchKernelGGL(gather_operand, dim3(blocks), dim3(threads), 0, 0, bank, pos, out, E);
          else
            hipLaunchKernelGGL(gather_rows, dim3(blocks), dim3(threads), 0, 0, bank, pos, out, E);
        }
        (void)hipEventRecord(b, 0);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        if (rep == 1)
          printf("| %s | %d | %d | %.1f | %.0f |\n", pat == 0 ? "A operand (today)" : "B row per instruction", wpc,
                 blocks, ms / 5 * 1e3, useful / (ms / 5 * 1e-3) / 1e9);
      }
    }
  return hipFree(bank) == hipSuccess ? 0 : 2;
}
