// Target-network values of the three candidate next states of every env, for the flagship bf16 step kernels
// (agent.target_every / agent.double_dqn on csrc/qstep_ws.hip; the learning-quality knobs of the torch oracle,
// sharetrade/env/trading.py engine_step_ref: `qt = forward(target_params, x2)`).
//
// The next state x' of an env depends on the action the step kernel has not drawn yet, but only through its
// last three features (budget, shares after Buy / Sell / Hold: TrainerChildActor.scala:118-146); the price
// window of x' is fixed.  So this pass, run before the step kernel, evaluates the target net on all three
// candidates: layer 1 of the shared window once, then for each candidate its 3-feature tail, layer 2 and the
// output layer.  QT[e][a][0..2] = Q_target(x' after action a)[0..2] (output ReLU applied when the model has
// it); the step kernel reads the row of the action it takes.
//
// MFMA layout (TPW 16-env tiles per wave, NWV waves per workgroup, one workgroup per CU, grid-stride; each
// weight fragment read from LDS feeds the TPW tiles' MFMAs): the target weights
// are converted to bf16 into LDS once per workgroup (fp32 master copy of the target net: no second bf16
// image to keep in sync); x' features are built in registers as B operands (the ws kernel's slot order: the
// last 16-wide k-step carries budget, shares, 1, fxn(vnew) in lane group 0); hidden activations stay in
// registers (layer-1 / layer-2 accumulator tiles re-packed as the next layer's B operand, the hidden-unit
// permutation absorbed by the column order of the W1 / W2 images).  Numerics: bf16 operands, fp32
// accumulation, the rounding points of the step kernel.
#include "qstep.h"

namespace st {
namespace qtgt {

constexpr int INP = 224, HP = 128, KX = 208, HWIN = 201;

constexpr int KS = 208;                        // W0 image row stride (bf16): 416-byte rows are conflict-free
                                               // for the 16-row b128 fragment reads (tools/lds_bank_sim.py;
                                               // 216 would be 2-way)
constexpr int oW0 = 0;                         // W0 [128][KS] bf16 (slot order)
constexpr int oW1 = oW0 + HP * KS * 2;         // W1 [128][128] bf16, columns in pi order, 16-B chunks
                                               // XOR-swizzled by the row (w1_off): conflict-free fragments
constexpr int oW2 = oW1 + HP * HP * 2;         // W2 [4][128] bf16, columns in pi order (row 3 zero)
constexpr int oB1 = oW2 + 4 * HP * 2;          // b1 [128] f32
constexpr int LDS_BYTES = oB1 + HP * 4;

ST_DEV int slot_col(int s) {
  if (s < 192) return s;
  const int t = s - 192, g = t >> 2, j = t & 3;
  if (g == 0) return j < 3 ? 201 + j : 200;
  if (g == 1) return 192 + j;
  if (g == 2) return 196 + j;
  return 204 + j;
}
// position s of a B operand built from accumulator tiles 2 ks, 2 ks + 1 -> hidden unit (qstep_ws.hip's pi)
ST_DEV int pi_unit(int s) {
  const int ks = s >> 5, g = (s >> 3) & 3, j = s & 7;
  return 32 * ks + 16 * (j >> 2) + 4 * g + (j & 3);
}
// W1 image: 16-byte chunk c / 8 of row r stored at chunk (c / 8) ^ (r & 15).  The fragment read of unit tile
// i, k-step ks (lane (l16, g4): row 16 i + l16, chunk 4 ks + g4) then hits 16 different chunks per lane group
// instead of one bank group 16 times (256-byte rows)
ST_DEV int w1_off(int r, int c) { return r * HP + ((((c >> 3) ^ (r & 15))) << 3) + (c & 7); }
ST_DEV s8v cat8(s4v a, s4v b) {
  s8v r;
  r[0] = a[0]; r[1] = a[1]; r[2] = a[2]; r[3] = a[3];
  r[4] = b[0]; r[5] = b[1]; r[6] = b[2]; r[7] = b[3];
  return r;
}
ST_DEV s4v pk4(float a, float b, float c, float d) {
  uint2 v;
  v.x = pack_bf2(a, b);
  v.y = pack_bf2(c, d);
  return __builtin_bit_cast(s4v, v);
}
typedef short s2v __attribute__((ext_vector_type(2)));
ST_DEV s4v relu_bf(f4v v) {
  const s2v z = {0, 0};
  const s2v a = __builtin_elementwise_max(__builtin_bit_cast(s2v, pack_bf2(v[0], v[1])), z);
  const s2v b = __builtin_elementwise_max(__builtin_bit_cast(s2v, pack_bf2(v[2], v[3])), z);
  s4v r = {a[0], a[1], b[0], b[1]};
  return r;
}
// a 16-wide k-step as a 16x16x32 MFMA with the upper halves of both operands zero (same cost on gfx950).  Not
// v_mfma_f32_16x16x16_bf16: reading a 16x16x32 result as its accumulator needs >= 4 wait states on MI355X
// (tools/ubench/mfma_raw_gen.py), hipcc (ROCm 7.2) emitted that pair with 1 here and the 16x16x16 MFMA saw the
// accumulator without the last 16x16x32 k-step (2 % error in QT; tools/debug/qt_colprobe.py,
// tools/mfma_hazard_scan.py)
ST_DEV f4v mfma32z(s4v a, s4v b, f4v c) {
  const s4v z = {0, 0, 0, 0};
  return mfma32(cat8(a, z), cat8(b, z), c);
}
ST_DEV float4 ldu4(const float* a) {
  float4 v;
  __builtin_memcpy(&v, a, sizeof(v));
  return v;
}

struct QTargetParams {
  const float* prices4;   // one padded copy of the bank [E][T4]
  const int* env;         // env state rows (qstep.h EnvRow)
  const float* wt;        // fp32 flat target params (engine layout)
  float* qt;              // [E][3][4] out
  int T, E, T4;
  int off_w0, off_w1, off_b1, off_w2, off_b2;
  float b0, inv_b0;
  int s0, compat_env, output_relu, feat_mode;
  const unsigned char* wimg;   // the weight images in LDS byte order (refreshed with the target copy), or null
  const unsigned short* ticks; // the 16-bit tick bank [E][T16] (csrc/series.hip tick16) read instead of prices4
  const float* tscale;         // when non-null (relative features only): price = tick * tscale[e]
  int T16;
};

// TPW 16-env tiles per wave (each weight fragment read from LDS feeds TPW MFMAs), NWV waves per workgroup (one
// workgroup per CU: the weight images take 87.5 KB of LDS)
template <int FEAT, int TPW, int NWV, bool U16 = false>
__global__ void __launch_bounds__(64 * NWV, 1) qtarget_kernel(QTargetParams p) {
  static_assert(!U16 || FEAT, "the tick bank serves the relative features only");
  constexpr int NW = NWV, NT = 64 * NWV;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* W0 = reinterpret_cast<bf16_t*>(smem + oW0);
  bf16_t* W1 = reinterpret_cast<bf16_t*>(smem + oW1);
  bf16_t* W2 = reinterpret_cast<bf16_t*>(smem + oW2);
  float* B1 = reinterpret_cast<float*>(smem + oB1);
  const int tid = threadIdx.x, lane = tid & 63, l16 = lane & 15, g4 = lane >> 4;
  const int w = tid >> 6;
  if (p.wimg != nullptr) {
    // the images as one run (packed from the target net right before the pass): 16 bytes per lane and LDS-DMA
    // instruction (the element-wise gather + conversion below cost ~10 us per launch in the step kernel's
    // equivalent, profiles/r5_ws_prologue.md)
    constexpr int NCH = LDS_BYTES / 16;
    const int lane_ = tid & 63;
    for (int j = tid >> 6; j * 64 < NCH; j += NW) {
      const int c = j * 64 + lane_;
      if (c < NCH)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(p.wimg + 16 * c),
                                         (__attribute__((address_space(3))) void*)(smem + 1024 * j), 16, 0, 0);
    }
    __builtin_amdgcn_s_waitcnt(0xF70);   // vmcnt(0)
  } else {
  for (int i = tid; i < HP * KX; i += NT) {
    const int r = i / KX, s = i % KX;
    W0[r * KS + s] = f2bf(p.wt[p.off_w0 + r * INP + slot_col(s)]);
  }
  for (int i = tid; i < HP * HP; i += NT) {
    const int r = i / HP, s = i % HP;
    W1[w1_off(r, s)] = f2bf(p.wt[p.off_w1 + r * HP + pi_unit(s)]);
  }
  for (int i = tid; i < 4 * HP; i += NT) {
    const int a = i / HP, s = i % HP;
    W2[i] = a < 3 ? f2bf(p.wt[p.off_w2 + a * HP + pi_unit(s)]) : (bf16_t)0;
  }
  for (int i = tid; i < HP; i += NT) B1[i] = p.wt[p.off_b1 + i];
  }
  __syncthreads();
  const float b2v[3] = {p.wt[p.off_b2], p.wt[p.off_b2 + 1], p.wt[p.off_b2 + 2]};
  const size_t E = (size_t)p.E;
  const int ntiles = p.E / 16;
  // the tail A fragments (input slots 192..207 of every unit tile): read once
  s4v w0t[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) w0t[i] = lds_ld4(W0 + (16 * i + l16) * KS + 192 + 4 * g4);
  for (int t0 = (blockIdx.x * NW + w) * TPW; t0 < ntiles; t0 += gridDim.x * NW * TPW) {
    // an opaque zero offset per iteration: the weight-fragment LDS reads are loop-invariant, and hoisted out of
    // the loops they would pin ~400 registers (W0 / W1 / W2 fragments) and spill
    int zo = 0;
    asm volatile("" : "+s"(zo));
    const bf16_t* W0i = W0 + zo;
    // ---------------------------------------------------------------- x' features of the wave's TPW env tiles
    float vnew[TPW], invn[TPW], bd[TPW], vnw[TPW];   // vnw: vnew in the window's units (U16: the tick)
    int sd[TPW];
    s8v X[TPW][6];
    s4v Xw[TPW];
#pragma unroll
    for (int q = 0; q < TPW; ++q) {
      const int e = 16 * (t0 + q) + l16;
      const int pos = p.env[ER_POS * E + e];
      const float bud = __int_as_float(p.env[ER_BUDGET * E + e]);
      const int sh = p.env[ER_SHARES * E + e];
      const int pc = min(max(pos, 0), p.T - HWIN - 1);
      if (U16) {
        // x' starts at tick pc + 1: per k-step a dwordx4 + a dword from the 4-byte boundary at or below the lane's
        // first tick, the odd start dropped by v_alignbyte; features from ticks are the fp32 prices' bit for bit
        const unsigned* b = reinterpret_cast<const unsigned*>(p.ticks + (size_t)e * p.T16) + ((pc + 1) >> 1);
        const unsigned shb = (unsigned)((pc + 1) & 1) * 2u;
        const unsigned tv = __builtin_amdgcn_alignbyte(0u, b[100], shb);   // tick pc + 201
        const float vw = (float)(tv & 0xFFFFu);
        vnew[q] = __fmul_rn(vw, p.tscale[e]);
        invn[q] = __fdiv_rn(1.0f, vw);
        vnw[q] = vw;
        const float iv = invn[q];
        auto fxn = [&](float v) { return __fmaf_rn(v, iv, -1.0f); };
        auto lo16f = [](unsigned v) { return (float)(v & 0xFFFFu); };
        auto hi16f = [](unsigned v) { return (float)(v >> 16); };
#pragma unroll
        for (int ks = 0; ks < 6; ++ks) {
          uint4 u;
          __builtin_memcpy(&u, b + 16 * ks + 4 * g4, sizeof(u));
          const unsigned t4 = b[16 * ks + 4 * g4 + 4];
          const unsigned w0 = __builtin_amdgcn_alignbyte(u.y, u.x, shb), w1 = __builtin_amdgcn_alignbyte(u.z, u.y, shb),
                         w2 = __builtin_amdgcn_alignbyte(u.w, u.z, shb), w3 = __builtin_amdgcn_alignbyte(t4, u.w, shb);
          X[q][ks] = cat8(pk4(fxn(lo16f(w0)), fxn(hi16f(w0)), fxn(lo16f(w1)), fxn(hi16f(w1))),
                          pk4(fxn(lo16f(w2)), fxn(hi16f(w2)), fxn(lo16f(w3)), fxn(hi16f(w3))));
        }
        Xw[q] = s4v{0, 0, 0, 0};
        if (g4 == 1 || g4 == 2) {
          uint2 u;
          __builtin_memcpy(&u, b + 96 + 2 * (g4 - 1), sizeof(u));
          const unsigned t2 = b[98 + 2 * (g4 - 1)];
          const unsigned w0 = __builtin_amdgcn_alignbyte(u.y, u.x, shb), w1 = __builtin_amdgcn_alignbyte(t2, u.y, shb);
          Xw[q] = pk4(fxn(lo16f(w0)), fxn(hi16f(w0)), fxn(lo16f(w1)), fxn(hi16f(w1)));
        }
      } else {
      const float* b = p.prices4 + (size_t)e * p.T4 + (size_t)pc;
      vnew[q] = b[201];
      vnw[q] = vnew[q];
      invn[q] = FEAT ? __fdiv_rn(1.0f, vnew[q]) : 0.f;
      const float iv = invn[q];
      auto fxn = [&](float v) { return FEAT ? __fmaf_rn(v, iv, -1.0f) : v; };
      // x' window B operands: k-step ks, lane group g4: x'[32 ks + 8 g4 + j] = p[pos + 1 + 32 ks + 8 g4 + j]
#pragma unroll
      for (int ks = 0; ks < 6; ++ks) {
        const float4 u = ldu4(b + 1 + 32 * ks + 8 * g4), v = ldu4(b + 5 + 32 * ks + 8 * g4);
        X[q][ks] = cat8(pk4(fxn(u.x), fxn(u.y), fxn(u.z), fxn(u.w)), pk4(fxn(v.x), fxn(v.y), fxn(v.z), fxn(v.w)));
      }
      // the last 16-wide k-step: lane groups 1, 2 window columns 192..199 of x' (p[pos + 193 ..]); group 0 the
      // candidate's tail (below); group 3 pads
      Xw[q] = s4v{0, 0, 0, 0};
      if (g4 == 1 || g4 == 2) {
        const float4 u = ldu4(b + 193 + 4 * (g4 - 1));
        Xw[q] = pk4(fxn(u.x), fxn(u.y), fxn(u.z), fxn(u.w));
      }
      }
      // the three candidates: Buy, Sell, Hold from (bd, sd) -- the env's own transition
      bd[q] = p.compat_env ? p.b0 : bud;
      sd[q] = p.compat_env ? p.s0 : sh;
    }
    // ---------------------------------------------------------------- layer 1 over the window (shared by the
    // candidates): one W0 fragment read per (unit tile, k-step) feeds the TPW env tiles' MFMAs
    f4v a1[TPW][8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
#pragma unroll
      for (int q = 0; q < TPW; ++q) a1[q][i] = f4v{0.f, 0.f, 0.f, 0.f};
      const bf16_t* wr = W0i + (16 * i + l16) * KS + 8 * g4;
#pragma unroll
      for (int ks = 0; ks < 6; ++ks) {
        const s8v A = lds_ld8(wr + 32 * ks);
#pragma unroll
        for (int q = 0; q < TPW; ++q) a1[q][i] = mfma32(A, X[q][ks], a1[q][i]);
      }
#pragma unroll
      for (int q = 0; q < TPW; ++q) a1[q][i] = mfma32z(w0t[i], Xw[q], a1[q][i]);
    }
#pragma unroll 1
    for (int a = 0; a < 3; ++a) {
      int za = 0;
      asm volatile("" : "+s"(za));
      const bf16_t* W1a = W1 + za;
      const bf16_t* W2a = W2 + za;
      s8v H1[TPW][4];
#pragma unroll
      for (int q = 0; q < TPW; ++q) {
        const bool buy = a == 0 && bd[q] >= vnew[q], sell = a == 1 && sd[q] > 0;
        const float b2 = buy ? __fsub_rn(bd[q], vnew[q]) : (sell ? __fadd_rn(bd[q], vnew[q]) : bd[q]);
        const int s2 = buy ? sd[q] + 1 : (sell ? sd[q] - 1 : sd[q]);
        const float fvn = FEAT ? __fmaf_rn(vnw[q], invn[q], -1.0f) : vnew[q];
        const s4v tl = g4 == 0 ? pk4(feat_budget(b2, p.inv_b0, FEAT), feat_shares(s2, vnew[q], p.inv_b0, FEAT),
                                     1.0f, fvn)
                               : s4v{0, 0, 0, 0};
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
          const f4v z0 = mfma32z(w0t[2 * ks], tl, a1[q][2 * ks]);
          const f4v z1 = mfma32z(w0t[2 * ks + 1], tl, a1[q][2 * ks + 1]);
          H1[q][ks] = cat8(relu_bf(z0), relu_bf(z1));
        }
      }
      // layer 2: one W1 fragment read per (unit tile, k-step) for the TPW env tiles; each pair of unit tiles
      // (one k-step of the output layer) goes into the output MFMA as soon as it is done
      f4v qo[TPW];
#pragma unroll
      for (int q = 0; q < TPW; ++q) qo[q] = f4v{0.f, 0.f, 0.f, 0.f};
      const bf16_t* w2r = W2a + min(l16, 3) * HP + 8 * g4;
#pragma unroll
      for (int ks2 = 0; ks2 < 4; ++ks2) {
        f4v z[TPW][2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int i = 2 * ks2 + h;
          const f4v bias = *reinterpret_cast<const f4v*>(B1 + 16 * i + 4 * g4);
#pragma unroll
          for (int q = 0; q < TPW; ++q) z[q][h] = bias;
#pragma unroll
          for (int ks = 0; ks < 4; ++ks) {
            const s8v A = lds_ld8(W1a + w1_off(16 * i + l16, 32 * ks + 8 * g4));
#pragma unroll
            for (int q = 0; q < TPW; ++q) z[q][h] = mfma32(A, H1[q][ks], z[q][h]);
          }
        }
        const s8v A2 = lds_ld8(w2r + 32 * ks2);
#pragma unroll
        for (int q = 0; q < TPW; ++q) qo[q] = mfma32(A2, cat8(relu_bf(z[q][0]), relu_bf(z[q][1])), qo[q]);
      }
      if (g4 == 0) {
#pragma unroll
        for (int q = 0; q < TPW; ++q) {
          float o[3];
#pragma unroll
          for (int j = 0; j < 3; ++j) {
            o[j] = qo[q][j] + b2v[j];
            if (p.output_relu) o[j] = fmaxf(o[j], 0.f);
          }
          const int e = 16 * (t0 + q) + l16;
          *reinterpret_cast<float4*>(p.qt + ((size_t)e * 3 + a) * 4) = make_float4(o[0], o[1], o[2], 0.f);
        }
      }
    }
  }
}

// the prologue's image entries, inverted (map[parameter] = bf16 element (>= 0), -(fp32 word) - 2, or -1 (host
// fill)): the same index math as the gather above
__global__ void __launch_bounds__(256) qt_img_map_kernel(int* map, int off_w0, int off_w1, int off_w2, int off_b1) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < HP * KX) map[off_w0 + (i / KX) * INP + slot_col(i % KX)] = oW0 / 2 + (i / KX) * KS + i % KX;
  if (i < HP * HP) map[off_w1 + (i / HP) * HP + pi_unit(i % HP)] = oW1 / 2 + w1_off(i / HP, i % HP);
  if (i < 3 * HP) map[off_w2 + (i / HP) * HP + pi_unit(i % HP)] = oW2 / 2 + i;
  if (i < HP) map[off_b1 + i] = -(oB1 / 4 + i) - 2;
}

}  // namespace qtgt
}  // namespace st

extern "C" int st_qtarget_img_bytes() { return st::qtgt::LDS_BYTES; }

extern "C" hipError_t st_qtarget_img_map(int* map, int off_w0, int off_w1, int off_w2, int off_b1, hipStream_t stream) {
  using namespace st::qtgt;
  static_assert(LDS_BYTES % 16 == 0 && oW0 == 0, "image run");
  hipLaunchKernelGGL(qt_img_map_kernel, dim3((HP * KX + 255) / 256), dim3(256), 0, stream, map, off_w0, off_w1, off_w2,
                     off_b1);
  return hipGetLastError();
}


namespace {
template <int TPW, int NWV>
hipError_t launch_qt(const st::qtgt::QTargetParams* p, int grid, hipStream_t stream) {
  using namespace st::qtgt;
  if (p->E % (16 * TPW) != 0) return hipErrorInvalidValue;
  static bool attr[3] = {false, false, false};
  const bool u16 = p->ticks != nullptr;
  if (u16 && (!p->feat_mode || p->tscale == nullptr || p->T16 < p->T + 8 || p->T16 % 8)) return hipErrorInvalidValue;
  const int f = u16 ? 2 : (p->feat_mode ? 1 : 0);
  const void* fn = f == 2 ? (const void*)qtarget_kernel<1, TPW, NWV, true>
                          : (f ? (const void*)qtarget_kernel<1, TPW, NWV> : (const void*)qtarget_kernel<0, TPW, NWV>);
  if (!attr[f]) {
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    if (e != hipSuccess) return e;
    attr[f] = true;
  }
  if (f == 2)
    hipLaunchKernelGGL((qtarget_kernel<1, TPW, NWV, true>), dim3(grid), dim3(64 * NWV), LDS_BYTES, stream, *p);
  else if (f)
    hipLaunchKernelGGL((qtarget_kernel<1, TPW, NWV>), dim3(grid), dim3(64 * NWV), LDS_BYTES, stream, *p);
  else
    hipLaunchKernelGGL((qtarget_kernel<0, TPW, NWV>), dim3(grid), dim3(64 * NWV), LDS_BYTES, stream, *p);
  return hipGetLastError();
}
}  // namespace

// variant (tiles per wave, waves per workgroup): 0 = (4, 4), 1 = (2, 8), 2 = (1, 8), 3 = (1, 16).  At 1.835 M
// envs (tools/bench_qtarget.py, profiles/r5_ws_knobs_cost.md): 629 / 447 / 568 / 442 us with the conflict-free
// weight images (658 / 489 / 779 / 703 before: the 256-byte W1 rows put every fragment read 16-way on one bank
// group; W0 rows at 216 bf16 were measured too, 2-way per the bank model and no faster).  The pass streams every env's 202-price x' window from HBM (1.47 GB, 300 us alone at ~5 TB/s);
// variant 1 keeps two waves per SIMD and feeds each weight fragment to two MFMAs; the engine uses it
extern "C" hipError_t st_qtarget_launch_v(const st::qtgt::QTargetParams* p, int grid, int variant, hipStream_t stream) {
  using namespace st::qtgt;
  if (grid < 1 || p->T < HWIN + 2 || p->T4 < p->T + 4) return hipErrorInvalidValue;
  switch (variant) {
    case 0: return launch_qt<4, 4>(p, grid, stream);
    case 1: return launch_qt<2, 8>(p, grid, stream);
    case 2: return launch_qt<1, 8>(p, grid, stream);
    case 3: return launch_qt<1, 16>(p, grid, stream);
    default: return hipErrorInvalidValue;
  }
}
extern "C" hipError_t st_qtarget_launch(const st::qtgt::QTargetParams* p, int grid, hipStream_t stream) {
  return st_qtarget_launch_v(p, grid, 1, stream);
}

// struct sizes of this file's launch ABI, for the host mirrors' check (tests/test_abi.py; no HIP call)
extern "C" int st_abi_qtarget(int* out, int n) {
  const int sz[] = {(int)sizeof(st::QStepParams), (int)sizeof(st::qtgt::QTargetParams)};
  const int m = (int)(sizeof(sz) / sizeof(sz[0]));
  for (int i = 0; i < n && i < m; ++i) out[i] = sz[i];
  return m;
}
