// Micro-benchmark: gathering every env's 202-price window from the HBM bank, as the flagship step
// (csrc/qstep_ws.hip) and the target pass (csrc/qtarget.hip) do, in two access patterns.
//
//   A  operand pattern (the kernels today): a wave owns a 16-env tile; lane (env l16, group g4) loads the
//      float4 pairs of its MFMA B operand -- per instruction 16 rows x 4 scattered 16-byte pieces;
//   B  row pattern: one instruction per env row, lane i loads floats 4i .. 4i + 3 (51 lanes cover the
//      202 floats): every instruction reads one contiguous 816-byte run;
//   C  pattern A over a 16-bit copy of the bank (u16 ticks of a per-env power-of-two grid): per lane and
//      k-step one 16-byte load of 8 ticks (2-byte aligned) + one 2-byte load, converted to fp32;
//   D  time-major bank (bank[t][env]): lane (env l16, group g4) loads its 9 times per k-step one value per
//      instruction, so each instruction reads 4 time rows x 16 consecutive envs (4 x 64 B);
//   E  as D over u16 ticks (4 x 32 B per instruction);
//   C' as C with the 9th tick of each k-step read by a 4-byte load instead of a 2-byte one.
// argv[2] = "same": every env at the same window position (the engine's lock-step envs), else random.
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

// C: the operand pattern over u16 ticks (half the bytes; one cvt per value)
__device__ __forceinline__ uint4 ldu4h(const unsigned short* a) {
  uint4 v;
  __builtin_memcpy(&v, a, sizeof(v));
  return v;
}
__device__ __forceinline__ float lo16(unsigned x) { return (float)(x & 0xFFFFu); }
__device__ __forceinline__ float hi16(unsigned x) { return (float)(x >> 16); }
template <bool WIDE9>
__global__ void __launch_bounds__(512) gather_u16(const unsigned short* bank, const int* pos, float* out, int E) {
  const int lane = threadIdx.x & 63, l16 = lane & 15, g4 = lane >> 4;
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, nwaves = (gridDim.x * blockDim.x) >> 6;
  float acc = 0.f;
  for (int t = wave; t < E / 16; t += nwaves) {
    const int e = 16 * t + l16;
    const unsigned short* b = bank + (size_t)e * T4 + pos[e];
#pragma unroll
    for (int ks = 0; ks < 6; ++ks) {
      const uint4 u = ldu4h(b + 1 + 32 * ks + 8 * g4);
      acc += lo16(u.x) + hi16(u.x) + lo16(u.y) + hi16(u.y) + lo16(u.z) + hi16(u.z) + lo16(u.w) + hi16(u.w);
      if (WIDE9) {   // the 9th tick through a 4-byte load (2-byte aligned) instead of a 2-byte load
        unsigned w;
        __builtin_memcpy(&w, b + 9 + 32 * ks + 8 * g4, sizeof(w));
        acc += lo16(w);
      } else {
        acc += (float)b[9 + 32 * ks + 8 * g4];
      }
    }
    if (g4 == 1 || g4 == 2) {
      uint2 u;
      __builtin_memcpy(&u, b + 193 + 4 * (g4 - 1), sizeof(u));
      acc += lo16(u.x) + hi16(u.x) + lo16(u.y) + hi16(u.y);
    }
    acc += (float)b[201];
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

// F: the operand pattern over u16 ticks with 4-byte-aligned loads only: per lane and k-step one dwordx4 + one
//    dword from the 4-byte boundary at or below the lane's first tick (20 bytes = 10 ticks cover its 9), the
//    odd-position shift undone by v_alignbyte (per lane: the kernel's envs may sit at different positions);
//    the tail (ticks 193..201) through one dwordx4 + one dword in lanes g4 = 1, 2 -- 14 loads per lane per tile
//    at half the bytes of A, none of them 2-byte
__device__ __forceinline__ unsigned shr16(unsigned lo, unsigned hi, unsigned sh) {   // ({hi, lo} >> sh)[31:0]
  return __builtin_amdgcn_alignbyte(hi, lo, sh);
}
__global__ void __launch_bounds__(512) gather_u16a(const unsigned short* bank, const int* pos, float* out, int E) {
  const int lane = threadIdx.x & 63, l16 = lane & 15, g4 = lane >> 4;
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, nwaves = (gridDim.x * blockDim.x) >> 6;
  float acc = 0.f;
  for (int t = wave; t < E / 16; t += nwaves) {
    const int e = 16 * t + l16;
    const int p0 = pos[e] + 1;
    const unsigned sh = (p0 & 1) * 2;   // bytes
    const unsigned* b = reinterpret_cast<const unsigned*>(bank + (size_t)e * T4) + (p0 >> 1);
#pragma unroll
    for (int ks = 0; ks < 6; ++ks) {
      uint4 u;
      __builtin_memcpy(&u, b + 16 * ks + 4 * g4, sizeof(u));
      const unsigned w = b[16 * ks + 4 * g4 + 4];
      const unsigned x0 = shr16(u.x, u.y, sh), x1 = shr16(u.y, u.z, sh), x2 = shr16(u.z, u.w, sh),
                     x3 = shr16(u.w, w, sh), x4 = shr16(w, 0u, sh);
      acc += lo16(x0) + hi16(x0) + lo16(x1) + hi16(x1) + lo16(x2) + hi16(x2) + lo16(x3) + hi16(x3) + lo16(x4);
    }
    if (g4 == 1 || g4 == 2) {
      uint2 u;
      __builtin_memcpy(&u, b + 96 + 2 * (g4 - 1), sizeof(u));
      const unsigned w = b[98 + 2 * (g4 - 1)];
      const unsigned x0 = shr16(u.x, u.y, sh), x1 = shr16(u.y, w, sh);
      acc += lo16(x0) + hi16(x0) + lo16(x1) + hi16(x1);
    }
    acc += (float)(shr16(b[100], b[101], sh) & 0xFFFFu);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

// D / E: time-major layouts (row t holds every env's price at time t; row stride ET elements)
template <typename TT>
__global__ void __launch_bounds__(512) gather_tm(const TT* bank, size_t ET, const int* pos, float* out, int E) {
  const int lane = threadIdx.x & 63, l16 = lane & 15, g4 = lane >> 4;
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, nwaves = (gridDim.x * blockDim.x) >> 6;
  float acc = 0.f;
  for (int t = wave; t < E / 16; t += nwaves) {
    const int e = 16 * t + l16;
    const TT* b = bank + (size_t)pos[e] * ET + e;
#pragma unroll
    for (int ks = 0; ks < 6; ++ks) {
      float v[9];
#pragma unroll
      for (int j = 0; j < 9; ++j) v[j] = (float)b[(size_t)(1 + 32 * ks + 8 * g4 + j) * ET];
#pragma unroll
      for (int j = 0; j < 9; ++j) acc += v[j];
    }
    if (g4 == 1 || g4 == 2) {
#pragma unroll
      for (int j = 0; j < 5; ++j) acc += (float)b[(size_t)(193 + 4 * (g4 - 1) + j) * ET];
    }
    acc += (float)b[(size_t)201 * ET];
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
  const bool same = argc > 2 && argv[2][0] == 's';
  for (int i = 0; i < E; ++i) hp[i] = same ? 1234 : rand() % (T - H - 2);
  if (hipMalloc(&pos, E * sizeof(int)) != hipSuccess) return 1;
  if (hipMemcpy(pos, hp.data(), E * sizeof(int), hipMemcpyHostToDevice) != hipSuccess) return 1;
  if (hipMalloc(&out, 1 << 24) != hipSuccess) return 1;
  unsigned short* bank16;
  if (hipMalloc(&bank16, nb * sizeof(unsigned short)) != hipSuccess) return 1;
  if (hipMemset(bank16, 0, nb * sizeof(unsigned short)) != hipSuccess) return 1;
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const double useful = (double)E * 202 * 4;   // (fp32-equivalent bytes for C too)
  printf("positions: %s\n\n", same ? "same for every env" : "random per env");
  printf("| pattern | waves / CU | grid | us | useful GB/s |\n|---|---|---|---|---|\n");
  const int pat0 = argc > 3 ? atoi(argv[3]) : 0;
  for (int pat = pat0; pat < 7; ++pat)
    for (int wpc : {8, 16, 32}) {
      const int threads = 512, blocks = 256 * wpc / 8;
      for (int rep = 0; rep < 2; ++rep) {   // (first rep warms up)
        (void)hipEventRecord(a, 0);
        for (int i = 0; i < 5; ++i) {
          if (pat == 0)
            hipLaunchKernelGGL(gather_operand, dim3(blocks), dim3(threads), 0, 0, bank, pos, out, E);
          else if (pat == 3)
            hipLaunchKernelGGL(gather_tm<float>, dim3(blocks), dim3(threads), 0, 0, bank, (size_t)E, pos, out, E);
          else if (pat == 4)
            hipLaunchKernelGGL(gather_tm<unsigned short>, dim3(blocks), dim3(threads), 0, 0, bank16, (size_t)E, pos, out, E);
          else if (pat == 2)
            hipLaunchKernelGGL(gather_u16<false>, dim3(blocks), dim3(threads), 0, 0, bank16, pos, out, E);
          else if (pat == 5)
            hipLaunchKernelGGL(gather_u16<true>, dim3(blocks), dim3(threads), 0, 0, bank16, pos, out, E);
          else if (pat == 6)
            hipLaunchKernelGGL(gather_u16a, dim3(blocks), dim3(threads), 0, 0, bank16, pos, out, E);
          else
            hipLaunchKernelGGL(gather_rows, dim3(blocks), dim3(threads), 0, 0, bank, pos, out, E);
        }
        (void)hipEventRecord(b, 0);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        if (rep == 1)
          printf("| %s | %d | %d | %.1f | %.0f |\n", pat == 0 ? "A operand (today)" : (pat == 1 ? "B row per instruction" : (pat == 2 ? "C operand, u16 ticks" : (pat == 3 ? "D time-major fp32" : (pat == 4 ? "E time-major u16" : (pat == 5 ? "C' as C, 9th tick by a 4-byte load" : "F u16 ticks, 4-B-aligned dwordx4 + dword, alignbyte"))))), wpc,
                 blocks, ms / 5 * 1e3, useful / (ms / 5 * 1e-3) / 1e9);
      }
    }
  (void)hipFree(bank16);
  return hipFree(bank) == hipSuccess ? 0 : 2;
}
