// Micro-benchmark: the ws step kernel's layer-1 loop (csrc/qstep_ws.hip, data wave) in isolation.
//
// The production stamps (profiles/r3_ws_stamps_v8*.md) put layer 1's 96 k-step MFMAs at ~35 s_memtime
// ticks each, with or without the gradient waves working, against ~16 cycles for back-to-back
// v_mfma_f32_16x16x32_bf16.  This program runs the same instruction mix -- W0 fragments from a 128 x 208
// bf16 LDS image (16-byte reads, PD pairs ahead), two MFMAs per fragment into a1[i] / a1n[i] -- and
// variants that drop one ingredient at a time, one data wave per SIMD (4 waves) or with 4 idle waves
// beside them (8 waves, as in the kernel), and prints ticks per MFMA (median over workgroups).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench/l1_loop.bin tools/ubench/l1_loop.hip
//   tools/ubench/l1_loop.bin
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef short s8v __attribute__((ext_vector_type(8)));
typedef float f4v __attribute__((ext_vector_type(4)));
typedef unsigned short bf16_t;

constexpr int KX = 208, HP = 128, REPS = 64;

__device__ __forceinline__ f4v mfma32(s8v a, s8v b, f4v c) { return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0); }

// MODE 0: production mix (LDS fragment reads PD ahead + 2 MFMAs per fragment + 2 VALU mults per pair)
// MODE 1: no VALU filler
// MODE 2: no LDS reads (fragments cycled from registers), no VALU
// MODE 3: one MFMA per fragment (a1 only), LDS reads, no VALU
template <int MODE, int PD, int NWAVE>
__global__ void __launch_bounds__(512) l1(const bf16_t* __restrict__ w0, float* __restrict__ out,
                                         unsigned long long* __restrict__ ticks, unsigned seed) {
  __shared__ __attribute__((aligned(16))) bf16_t W0p[HP * KX];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, l16 = lane & 15, g4 = lane >> 4;
  for (int i = tid; i < HP * KX; i += 64 * NWAVE) W0p[i] = w0[i];
  __syncthreads();
  if (wave >= 4) {   // the idle "gradient" waves of the 8-wave form
    out[blockIdx.x * 1024 + tid] = 0.f;
    return;
  }
  s8v X[6], Xn[6];
#pragma unroll
  for (int k = 0; k < 6; ++k)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      X[k][e] = (short)(0x3C00 + ((seed + lane * 7 + k * 13 + e) & 0x3FF));
      Xn[k][e] = (short)(0x3C00 + ((seed + lane * 5 + k * 11 + e * 3) & 0x3FF));
    }
  f4v a1[8], a1n[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { a1[i] = f4v{0.f, 0.f, 0.f, 0.f}; a1n[i] = a1[i]; }
  unsigned u = seed ^ (unsigned)lane, v = seed * 3u + 1u;
  const bf16_t* w0b = W0p + l16 * KX + 8 * g4;
  unsigned long long t0 = 0, t1 = 0;
  constexpr int NB = PD + 1;
  s8v A[NB];
  if (MODE == 2) {   // fragments read once, then cycled from registers
#pragma unroll
    for (int j = 0; j < NB; ++j) A[j] = *reinterpret_cast<const s8v*>(w0b + (j & 7) * 16 * KX + 32 * (j >> 3));
  }
  for (int rep = 0; rep < REPS; ++rep) {
    if (rep == 8) t0 = __builtin_amdgcn_s_memtime();   // (first reps warm the wave up)
    if (MODE != 2) {
#pragma unroll
      for (int j = 0; j < PD; ++j) A[j] = *reinterpret_cast<const s8v*>(w0b + (j & 7) * 16 * KX + 32 * (j >> 3));
      __builtin_amdgcn_sched_group_barrier(0x100, PD, 0);
    }
#pragma unroll
    for (int j = 0; j < 48; ++j) {
      const int ks = j >> 3, i = j & 7;
      a1[i] = mfma32(A[j % NB], X[ks], a1[i]);
      if (MODE != 3) a1n[i] = mfma32(A[j % NB], Xn[ks], a1n[i]);
      __builtin_amdgcn_sched_group_barrier(0x008, MODE != 3 ? 2 : 1, 0);
      if (j + PD < 48 && MODE != 2) {
        const int jn = j + PD;
        A[jn % NB] = *reinterpret_cast<const s8v*>(w0b + (jn & 7) * 16 * KX + 32 * (jn >> 3));
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      if (MODE == 0) {
        u = __umulhi(u, 0xD2511F53u) ^ v;
        v = v * 0xCD9E8D57u + (unsigned)j;
        __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  t1 = __builtin_amdgcn_s_memtime();
  float s = (float)(u ^ v) * 1e-30f;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += a1[i][0] + a1[i][1] + a1[i][2] + a1[i][3] + a1n[i][0] + a1n[i][3];
  out[blockIdx.x * 1024 + tid] = s;
  if (lane == 0) ticks[blockIdx.x * 4 + wave] = t1 - t0;
}

template <int MODE, int PD, int NWAVE>
static void run(const char* name, const bf16_t* w0, float* out, unsigned long long* ticks, int grid) {
  auto k = l1<MODE, PD, NWAVE>;
  for (int it = 0; it < 3; ++it) hipLaunchKernelGGL(k, dim3(grid), dim3(64 * NWAVE), 0, 0, w0, out, ticks, 12345u + it);
  (void)hipDeviceSynchronize();
  std::vector<unsigned long long> t(grid * 4);
  (void)hipMemcpy(t.data(), ticks, t.size() * 8, hipMemcpyDeviceToHost);
  std::sort(t.begin(), t.end());
  const double mfma = (REPS - 8) * 48.0 * (MODE == 3 ? 1 : 2);
  printf("| %-44s | %d | %d | %.1f | %.1f |\n", name, NWAVE, PD, t[t.size() / 2] / mfma, t[t.size() / 2] / ((REPS - 8) * 48.0));
}

int main() {
  const int grid = 256;
  bf16_t* w0;
  float* out;
  unsigned long long* ticks;
  (void)hipMalloc(&w0, HP * KX * 2);
  (void)hipMalloc(&out, grid * 1024 * 4);
  (void)hipMalloc(&ticks, grid * 4 * 8);
  std::vector<bf16_t> h(HP * KX);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (bf16_t)(0x3C00 + (i * 2654435761u >> 22));
  (void)hipMemcpy(w0, h.data(), h.size() * 2, hipMemcpyHostToDevice);
  printf("| variant | waves / WG | PD | ticks per MFMA | ticks per fragment pair |\n|---|---|---|---|---|\n");
  run<0, 10, 8>("production mix (LDS reads, 2 MFMA / fragment, VALU)", w0, out, ticks, grid);
  run<0, 10, 4>("production mix", w0, out, ticks, grid);
  run<1, 10, 8>("no VALU filler", w0, out, ticks, grid);
  run<1, 10, 4>("no VALU filler", w0, out, ticks, grid);
  run<2, 10, 8>("no LDS reads, no VALU (MFMA only)", w0, out, ticks, grid);
  run<2, 10, 4>("no LDS reads, no VALU (MFMA only)", w0, out, ticks, grid);
  run<3, 10, 8>("1 MFMA per fragment, LDS reads", w0, out, ticks, grid);
  run<1, 6, 8>("no VALU filler", w0, out, ticks, grid);
  run<1, 16, 8>("no VALU filler", w0, out, ticks, grid);
  hipError_t e = hipGetLastError();
  printf("status: %s\n", hipGetErrorString(e));
  return e == hipSuccess ? 0 : 1;
}
