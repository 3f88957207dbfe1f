// Shared pieces of the GRU(256) recurrent Q-net kernels (BASELINE config 5):
// actor (gru.hip) and fused learner (gru_learn.hip).
#pragma once
#include "common.h"

namespace st {

typedef int i8v __attribute__((ext_vector_type(8)));   // 32 fp8 bytes: one MX A/B fragment

constexpr int RH = 256;            // hidden units
constexpr int RG = 3 * RH;         // gate rows
constexpr int RF = 32;             // actor x width (bf16, one K=32 MFMA step)
constexpr int RFL = 64;            // learner x width (GEMM K multiple of 64)
constexpr int RMF = 8;             // market features per bar
constexpr int RW = 8;              // waves per actor workgroup
constexpr int RN = 32;             // envs per actor chunk
constexpr int RT = RW * 64;
constexpr int XS = RF + 8;         // sX row stride (bf16) = 80 B: conflict-free ds_read_b128
constexpr int HS = RH + 16;        // sH8 row stride (bytes) = 272 B
constexpr int SCS = 9;             // scale row stride (ints)

// ---------------------------------------------------------------- MX-fp8 helpers
ST_DEV f4v mx_mfma(const i8v& a, const i8v& b, f4v c, int sa, int sb) {
  // fmt 0/0 = e4m3 x e4m3; scales are E8M0 bytes (byte 0 of sa / sb)
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, sa, 0, sb);
}
// same, with the A scale taken from byte SEL of a packed register (op_sel), 4 scales per VGPR
template <int SEL>
ST_DEV f4v mx_mfma_sel(const i8v& a, const i8v& b, f4v c, int sa4, int sb) {
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, SEL, sa4, 0, sb);
}
// smallest e with amax / 2^e <= 448 (e4m3 max): e = ceil(log2(amax / 448))
ST_DEV int mx_exp(float amax) {
  if (!(amax > 0.f)) return -127;
  int e;
  const float m = frexpf(amax * (1.0f / 448.0f), &e);
  if (m == 0.5f) e -= 1;
  if (ldexpf(amax, -e) > 448.f) e += 1;
  return e < -127 ? -127 : (e > 127 ? 127 : e);
}
ST_DEV uint32_t fp8x4(float a, float b, float c, float d) {
  int v = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  v = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, v, true);
  return (uint32_t)v;
}
// raw v_exp_f32 / v_rcp_f32 (1 ulp): __frcp_rn would expand to the IEEE division sequence
ST_DEV float sigm(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }
// actor epilogue forms: exp2 with the log2(e) scale folded, explicit FMAs (the build keeps
// -ffp-contract=off for the bit-exact env arithmetic, so contraction is spelled out here)
ST_DEV float sigm2(float x) { return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(x * -1.44269504f)); }
ST_DEV float tanh2(float x) {
  return __builtin_fmaf(2.f, __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(x * -2.88539008f)), -1.f);
}
ST_DEV float tanh_f(float x) { return 2.f * sigm(2.f * x) - 1.f; }
// gate pre-activations arrive pre-scaled (gru_pack_kernel folds -log2(e) into the r / z rows of W_hh, W_ih and
// their biases, -2 log2(e) into the n rows): sigmoid / tanh are then exp2 + add + rcp with no scaling
// multiply -- 48 fewer VALU per wave-step of the actor (profiles/r4_gru_prescale.md)
constexpr float GS_RZ = -1.44269504f;
constexpr float GS_N = -2.88539008f;
ST_DEV float sigm_ps(float y) { return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(y)); }
ST_DEV float tanh_ps(float y) { return __builtin_fmaf(2.f, __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(y)), -1.f); }

// max over the 4 rows of 16 lanes (lanes l, l^16, l^32, l^48) of a non-negative value: two VALU
// row swaps (v_permlane16/32_swap) instead of two LDS round trips (ds_bpermute); unsigned max of
// the bit patterns == float max for non-negative finite values, without NaN canonicalisation
ST_DEV float rowmax4(float v) {
  uint32_t b = __float_as_uint(v);
  const auto r16 = __builtin_amdgcn_permlane16_swap(b, b, false, false);
  b = max((uint32_t)r16[0], (uint32_t)r16[1]);
  const auto r32 = __builtin_amdgcn_permlane32_swap(b, b, false, false);
  b = max((uint32_t)r32[0], (uint32_t)r32[1]);
  return __uint_as_float(b);
}

// quantize the lane's h values (units of this wave, 2 env tiles) into an LDS fp8 tile
ST_DEV void quant_h(const float (&hr)[2][2][4], unsigned char* sH8, int* sSc, int wave, int l16, int g4) {
#pragma unroll
  for (int n = 0; n < 2; ++n) {
    float amax = 0.f;
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int i = 0; i < 4; ++i) amax = fmaxf(amax, fabsf(hr[m][n][i]));
    amax = rowmax4(amax);
    const int e = mx_exp(amax);
    const int row = 16 * n + l16;
#pragma unroll
    for (int m = 0; m < 2; ++m)
      *reinterpret_cast<uint32_t*>(sH8 + row * HS + 32 * wave + 16 * m + 4 * g4) =
          fp8x4(ldexpf(hr[m][n][0], -e), ldexpf(hr[m][n][1], -e), ldexpf(hr[m][n][2], -e), ldexpf(hr[m][n][3], -e));
    if (g4 == 0) sSc[row * SCS + wave] = e + 127;
  }
}

}  // namespace st
