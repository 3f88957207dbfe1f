// Shared device helpers for the sharetrade CDNA4 (gfx950) kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef short s8v __attribute__((ext_vector_type(8)));
typedef short s4v __attribute__((ext_vector_type(4)));
typedef float f4v __attribute__((ext_vector_type(4)));
typedef unsigned short bf16_t;

#define ST_DEV __device__ __forceinline__

// ----------------------------------------------------------------- bf16
ST_DEV bf16_t f2bf(float x) {
  __bf16 h = (__bf16)x;  // v_cvt_pk_bf16_f32 (RNE, NaN-preserving) on gfx950
  return __builtin_bit_cast(bf16_t, h);
}
ST_DEV float bf2f(bf16_t h) { return __uint_as_float(((uint32_t)h) << 16); }
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
// one v_cvt_pk_bf16_f32 (RNE) for two values
ST_DEV uint32_t pack_bf2(float lo, float hi) {
  f32x2_t v = {lo, hi};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
}

// ----------------------------------------------------------------- LDS fragment loads
// 8 contiguous bf16 (16 B) -> ds_read_b128.  p must be 16-byte aligned.
ST_DEV s8v lds_ld8(const bf16_t* p) { return *reinterpret_cast<const s8v*>(p); }
ST_DEV s4v lds_ld4(const bf16_t* p) { return *reinterpret_cast<const s4v*>(p); }
// ds_read_b64_tr_b16: per 16-lane group, a 4-row x 16-col block delivered column-major.
ST_DEV s4v lds_tr4(const bf16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4v*)(p));
}
ST_DEV void lds_st4(bf16_t* p, float a, float b, float c, float d) {
  uint2 v;
  v.x = pack_bf2(a, b);
  v.y = pack_bf2(c, d);
  *reinterpret_cast<uint2*>(p) = v;
}

ST_DEV f4v mfma32(s8v a, s8v b, f4v c) { return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0); }
ST_DEV f4v mfma16(s4v a, s4v b, f4v c) { return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0); }

ST_DEV f4v zero4() { f4v z = {0.f, 0.f, 0.f, 0.f}; return z; }

// ----------------------------------------------------------------- Philox4x32-10
// Bit-identical to sharetrade/utils/rng.py::philox4x32.
ST_DEV void philox4x32(uint32_t& c0, uint32_t& c1, uint32_t& c2, uint32_t& c3, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
    const uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
}
ST_DEV float u24(uint32_t x) { return (float)(x >> 8) * (1.0f / 16777216.0f); }

// ----------------------------------------------------------------- wave reductions
ST_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
