// Synthetic price-bank generation directly in HBM.
//
// The reference "fetches" a single bundled MSFT series (SharePriceGetter.scala:83-102);
// the engine keeps one price series per env resident in HBM ([E, T] fp32,
// ~1.6 GB for 65,536 envs x 6,047 days) and reads state windows from it in place.
// One wave generates one series: Philox normals (Box-Muller) for 64 days at a
// time, a wave-level inclusive scan of the log-returns, coalesced 256-B stores.
#include "common.h"

namespace st {

__global__ void __launch_bounds__(256) random_walk_kernel(float* __restrict__ out, int E, int T, float start_price,
                                                          float vol, float drift, uint32_t key0, uint32_t key1) {
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (wave >= E) return;
  float carry = 0.f;  // log-price at the last day of the previous block
  float* row = out + (size_t)wave * T;
  for (int t0 = 0; t0 < T; t0 += 64) {
    const int t = t0 + lane;
    uint32_t c0 = (uint32_t)wave, c1 = (uint32_t)t, c2 = 0x5EEDu, c3 = 2u;
    philox4x32(c0, c1, c2, c3, key0, key1);
    const float u1 = ((float)(c0 >> 8) + 1.0f) * (1.0f / 16777216.0f);  // (0, 1]
    const float u2 = u24(c1);
    float z = sqrtf(-2.0f * logf(u1)) * cosf(6.283185307179586f * u2);
    float inc = (t == 0 || t >= T) ? 0.f : vol * z + drift;
    // inclusive wave scan
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const float n = __shfl_up(inc, o, 64);
      if (lane >= o) inc += n;
    }
    const float lp = carry + inc;
    if (t < T) row[t] = start_price * expf(lp);
    carry = __shfl(lp, 63, 64);
  }
}

// 4-way shifted replicas of the price bank: dst[s][e][i] = src[e][i + s] (0 past the end).
// A window starting at ANY day ps is then one run of 16-byte-aligned float4s in replica
// ps & 3 — the fused step kernel's gather becomes one global_load_dwordx4 per lane per row
// with no realignment.  4 x 1.6 GB for 65,536 envs: cheap on 288 GB of HBM3E.
__global__ void __launch_bounds__(256) replicate4_kernel(const float* __restrict__ src, float* __restrict__ dst,
                                                         int E, int T, int T4, int reps) {
  const size_t n = (size_t)reps * E * T4;
  for (size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x; idx < n; idx += (size_t)gridDim.x * blockDim.x) {
    const int i = (int)(idx % T4);
    const size_t se = idx / T4;
    const int e = (int)(se % E), sft = (int)(se / E);
    dst[idx] = (i + sft < T) ? src[(size_t)e * T + i + sft] : 0.f;
  }
}

// 16-bit tick banks.  Every env's series on its own power-of-two grid: price = tick * 2^x_e with 0 < tick <=
// 65535, x_e the smallest exponent that fits the series' largest price.  The flagship step reads windows as u16
// ticks (half the bytes of fp32, 4-byte-aligned dwordx4 loads: profiles/r6_window_gather_ubench.md) and gets
// bit-identical features: w / last - 1 = fma(tick_w, rn(1 / tick_last), -1) exactly (the powers of two cancel),
// and prices for the env step as tick * 2^x_e (exact in fp32).
//   mode 0 (quantize): bank[e][t] := tick * 2^x_e in place (synthetic banks are generated on the grid);
//   mode 1 (check):    the bank is left alone; bad[0] |= 1 where a value is not exactly tick * 2^x_e with a
//                      tick in [1, 65535] (the engine then keeps its fp32 window path).
// Both write ticks[e][0 .. T16) (zero past T) and scale[e] = 2^x_e (mode 0: either may be null).  One wave per env.
__global__ void __launch_bounds__(256) tick16_kernel(float* __restrict__ bank, int E, int T, unsigned short* __restrict__ ticks,
                                                     int T16, float* __restrict__ scale, int mode, unsigned* bad) {
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (wave >= E) return;
  float* row = bank + (size_t)wave * T;
  float m = 0.f;
  bool ok = true;
  for (int t = lane; t < T; t += 64) {
    const float v = row[t];
    ok = ok && (v > 0.f) && (v <= 3.0e38f);
    m = fmaxf(m, v);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  // smallest x with m * 2^-x <= 65535 (ldexpf is exact away from the subnormal range)
  int x;
  (void)frexpf(m, &x);   // m = f 2^x, f in [0.5, 1)
  x -= 16;
  while (x > -126 && ldexpf(m, -(x - 1)) <= 65535.f) --x;
  while (ldexpf(m, -x) > 65535.f) ++x;
  const float sc = ldexpf(1.0f, x);
  unsigned short* trow = ticks ? ticks + (size_t)wave * T16 : nullptr;
  const int tend = trow ? T16 : T;
  for (int t = lane; t < tend; t += 64) {
    unsigned tk = 0u;
    if (t < T) {
      const float v = row[t];
      const float q = rintf(ldexpf(v, -x));
      tk = (unsigned)fminf(fmaxf(q, 1.0f), 65535.0f);
      const float back = ldexpf((float)tk, x);
      if (mode == 0)
        row[t] = back;
      else if (back != v)
        ok = false;
    }
    if (trow) trow[t] = (unsigned short)tk;
  }
  if (lane == 0 && scale) scale[wave] = sc;
  if (mode == 1 && __any(!ok) && lane == 0) atomicOr(bad, 1u);
}

// Weight initialisation on the device (tf.RandomNormalInitializer, QDecisionPolicyActor.scala:41,45,
// 80-81): W[r][c] = std * N(0,1) for r < rows, c < cols of a row-major [.., ld] block, one Philox4x32-10
// counter per element -- (c0, c1, c2, c3) = (r * cols + c, 0, stream, 0x1417) -- and one Box-Muller
// normal from its first two words.  Counter-based, so the values depend only on (key, stream, index):
// sharetrade/models/qnet.py mirrors it on the host (same formula in fp32; libm vs device ulps).
__global__ void __launch_bounds__(256) init_normal_kernel(float* __restrict__ out, int rows, int cols, int ld,
                                                          float std, uint32_t key0, uint32_t key1, uint32_t stream) {
  const long n = (long)rows * cols;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    uint32_t c0 = (uint32_t)i, c1 = 0u, c2 = stream, c3 = 0x1417u;
    philox4x32(c0, c1, c2, c3, key0, key1);
    const float u1 = ((float)(c0 >> 8) + 1.0f) * (1.0f / 16777216.0f);   // (0, 1]
    const float u2 = u24(c1);
    const float z = sqrtf(-2.0f * logf(u1)) * cosf(6.283185307179586f * u2);
    const int r = (int)(i / cols), c = (int)(i % cols);
    out[(size_t)r * ld + c] = std * z;
  }
}

}  // namespace st

extern "C" hipError_t st_init_normal(float* out, int rows, int cols, int ld, float std, uint32_t key0, uint32_t key1,
                                     uint32_t stream, hipStream_t s) {
  if (rows < 0 || cols < 0 || ld < cols) return hipErrorInvalidValue;
  const long n = (long)rows * cols;
  if (n == 0) return hipSuccess;
  const int grid = (int)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096);
  hipLaunchKernelGGL(st::init_normal_kernel, dim3(grid), dim3(256), 0, s, out, rows, cols, ld, std, key0, key1, stream);
  return hipGetLastError();
}

// reps shifted copies (replica s = row shifted left by s): 4 for the 16-B-aligned window gathers of
// qstep_wide / fused / pair, 1 (a padded copy) for qstep_ws, whose 4-B-aligned dwordx4 reads measured as
// fast (profiles/r3_ws_ab.md)
extern "C" hipError_t st_replicate4(const float* src, float* dst, int E, int T, int T4, int reps, hipStream_t stream) {
  if (T4 % 4 != 0 || T4 < T || reps < 1 || reps > 4) return hipErrorInvalidValue;
  hipLaunchKernelGGL(st::replicate4_kernel, dim3(4096), dim3(256), 0, stream, src, dst, E, T, T4, reps);
  return hipGetLastError();
}

extern "C" hipError_t st_random_walk(float* out, int E, int T, float start_price, float vol, float drift,
                                     uint32_t key0, uint32_t key1, hipStream_t stream) {
  const int threads = 256;
  const long waves = E;
  const int grid = (int)((waves * 64 + threads - 1) / threads);
  hipLaunchKernelGGL(st::random_walk_kernel, dim3(grid), dim3(threads), 0, stream, out, E, T, start_price, vol,
                     drift, key0, key1);
  return hipGetLastError();
}

// 16-bit tick bank of an [E][T] fp32 bank (tick16_kernel): ticks [E][T16] (T16 >= T + 8, a multiple of 8),
// scale [E]; mode 0 quantizes the bank in place, mode 1 only checks it (*bad set when not on a tick grid)
extern "C" hipError_t st_tick16(float* bank, int E, int T, unsigned short* ticks, int T16, float* scale, int mode,
                                unsigned* bad, hipStream_t stream) {
  if (E <= 0 || T <= 0 || (mode != 0 && mode != 1) || (mode == 1 && (bad == nullptr || ticks == nullptr)))
    return hipErrorInvalidValue;
  if (ticks != nullptr && (T16 < T + 8 || T16 % 8)) return hipErrorInvalidValue;
  const long waves = E;
  const int grid = (int)((waves * 64 + 255) / 256);
  hipLaunchKernelGGL(st::tick16_kernel, dim3(grid), dim3(256), 0, stream, bank, E, T, ticks, T16, scale, mode, bad);
  return hipGetLastError();
}
