// Shared definitions of the fused online-DQN step kernels (qstep_fused.hip: 32-env chunks,
// weights resident in LDS; qstep_wide.hip: 64-env chunks, layer-1 weights resident in VGPRs).
#pragma once
#include "common.h"

namespace st {

constexpr int OUTP = 16;    // padded action dimension
constexpr int NSTAT = 8;

struct QStepParams {
  const float* prices;      // [E, T] env-major
  const float* prices4;     // [4][E][T4] shifted replicas (series.hip: replicate4)
  // env state + per-step outputs as ONE struct-of-arrays buffer [ENV_ROWS][E] of 4-byte
  // words (rows below): one base pointer instead of nine keeps the kernel's scalar
  // registers from spilling across the chunk loop
  int* env;
  const bf16_t* wq;         // bf16 flat params (kernel layout)
  const float* wf;          // fp32 flat params (biases read from here)
  float* slab;              // [G][P] per-workgroup partial gradients
  float* stats;             // [G][NSTAT]
  unsigned long long* ctrl;   // ctrl[0] = step index (read), ctrl[1] = step+1 (written by block 0)
  int T, E, H, P, T4;
  int off_w0, off_w1, off_b1, off_w2, off_b2;
  float eps, inv_ramp, gamma, loss_coef, b0, inv_b0;
  int s0, compat_env, target_compat, output_relu, feat_mode;
  uint32_t key0, key1;
  int env_offset;
  unsigned long long* stamps;  // debug: s_memtime per phase of workgroup 0 ([iter][16]) or null
  int slab_bf16;            // slabs written as bf16, column-blocked [P/32][slab_rows][32]
                            // (64-env-chunk kernel only; csrc/optim.hip reads them)
  int slab_rows;            // G: workgroups of the launch (= slab rows)
  // dynamic chunk schedule (64-env-chunk kernel): 8 per-XCD claim heads, one per 128-byte line
  // (heads[32 * x]), zero at launch; null = static schedule.  csrc/optim.hip re-zeroes them.
  unsigned* chunk_heads;
  int reward_mode;          // 0: reward = change of portfolio value; 1: its one-step return (change / previous)
  float td_clip;            // > 0: the TD error fed back is clamped to [-td_clip, td_clip] (Huber loss)
  unsigned* err;            // csrc/qstep_ws.hip: bit 0 = a ring wait gave up (bounded spin), or null
  // learning-quality knobs of the torch oracle (sharetrade/env/trading.py engine_step_ref), ws / pipe kernels:
  float reward_scale;       // the reward in the TD target is multiplied by this (1: the reference)
  int ramp_global;          // 1: the exploit ramp runs over the step count instead of the episode position
  const float* qt;          // target net (csrc/qtarget.hip): [E][3][4] Q_target(x' after action a), or null
  int double_dqn;           // with qt: the next action is the online net's argmax, valued by the target
  // csrc/qstep_ws.hip: the workgroup's weight images in LDS byte order (kept current by the optimizer pass,
  // csrc/optim.hip img / img_map), copied into LDS by DMA in the prologue; null = gather them from wq / wf
  const unsigned char* wimg;
  // csrc/qstep_ws.hip / csrc/qtarget.hip: the bank as 16-bit ticks (csrc/series.hip tick16: [E][T16], price =
  // tick * tscale[e], a power of two per env) -- read instead of prices4 when non-null (relative features only)
  const unsigned short* ticks;
  const float* tscale;
  int T16;
};

// rows of QStepParams::env
enum EnvRow : int { ER_POS = 0, ER_BUDGET, ER_SHARES, ER_VALUE, ER_RET_SUM, ER_EPISODES, ER_LAST_FINAL,
                    ER_ACTION, ER_REWARD, ENV_ROWS };
#define ENV_I(R, e) (p.env[(size_t)(R) * p.E + (e)])
#define ENV_F(R, e) (reinterpret_cast<float*>(p.env)[(size_t)(R) * p.E + (e)])

// A/B fragment from a row-major image: rows r0 + l16, k = k0 + 8*g4 .. +7
ST_DEV s8v frag_row(const bf16_t* img, int S, int r0, int k0, int l16, int g4) {
  return lds_ld8(img + (r0 + l16) * S + k0 + 8 * g4);
}
// Fragment with k running down the image rows (hardware transpose read):
// element j of lane (g4, l16) = img[k0 + 8*g4 + j][c0 + l16]
ST_DEV s8v frag_tr(const bf16_t* img, int S, int k0, int c0, int l16, int g4) {
  const bf16_t* p = img + (k0 + 8 * g4 + (l16 >> 2)) * S + c0 + 4 * (l16 & 3);
  s4v lo = lds_tr4(p);
  s4v hi = lds_tr4(p + 4 * S);
  s8v r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}

// frag_tr with the k (row) order permuted for bank-conflict-free reads: lane (g4, l16) element j =
// img[k0 + 4*g4 + j][c0 + l16] for j < 4 and img[k0 + 16 + 4*g4 + j - 4][c0 + l16] for j >= 4, so
// each ds_read_b64_tr_b16 lane group of 32 reads 8 consecutive rows (one 8-dword bank window per row
// when the row stride is an odd multiple of 8 dwords: 144 / 240 bf16).  Valid wherever BOTH operands
// of the MFMA are read with it (k runs over a sum index, e.g. envs in a weight gradient).
ST_DEV s8v frag_trp(const bf16_t* img, int S, int k0, int c0, int l16, int g4) {
  const bf16_t* p = img + (k0 + 4 * g4 + (l16 >> 2)) * S + c0 + 4 * (l16 & 3);
  s4v lo = lds_tr4(p);
  s4v hi = lds_tr4(p + 16 * S);
  s8v r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}

// inclusive sum over each 16-lane DPP row (lane 15 of a row holds the row total): 4 row_shr adds
ST_DEV float row16_sum(float v) {
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x111, 0xF, 0xF, true));
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x112, 0xF, 0xF, true));
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x114, 0xF, 0xF, true));
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x118, 0xF, 0xF, true));
  return v;
}

// value of lane+1 (lane 63 gets 0): DPP wave_shl:1 — one VALU op instead of a ds_bpermute
ST_DEV float dpp_next_lane(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x130, 0xF, 0xF, true));
}

ST_DEV float feat_price(float w, float inv, int mode) {
  return mode ? __fsub_rn(__fmul_rn(w, inv), 1.0f) : w;
}
ST_DEV float feat_budget(float b, float inv_b0, int mode) { return mode ? __fmul_rn(b, inv_b0) : b; }
ST_DEV float feat_shares(int s, float last, float inv_b0, int mode) {
  return mode ? __fmul_rn(__fmul_rn((float)s, last), inv_b0) : (float)s;
}

}  // namespace st
