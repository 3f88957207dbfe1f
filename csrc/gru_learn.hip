// Fused learner of the GRU(256) recurrent Q-net (BASELINE config 5).
//
// Replaces a per-time-step chain of GEMM + elementwise launches (~130 kernels per update)
// with two persistent kernels; a workgroup owns 32 sampled sequences for all time steps,
// wave w owns hidden units 32w..32w+31 of all three gates (the actor's tiling, gru.hip):
//
//   gru_seq_fwd_kernel  (grid B/32 x 2: online and target net in one launch)
//     S+1 steps of the recurrence on-chip, exactly the actor's arithmetic: W_hh as MX-fp8
//     fragments resident in VGPRs (v_mfma_scale_f32_16x16x128_f8f6f4), W_ih bf16 in LDS,
//     h fp32 in registers, re-quantized per step; Q head as one bf16 MFMA per tile.
//     The online net saves r, z, n, gh_n, h_prev (bf16, in the lanes' own accumulator
//     order -> one 16-byte store / load per quantity and tile) and the masked h rows the
//     weight-gradient GEMM needs.
//   gru_seq_bwd_kernel  (grid B/32)
//     backward through time: the recurrent gradient dL/dh stays in registers; per step
//     the fused GRU backward writes dGx / dGh (bf16) and the dGh tile to LDS, then
//     dh_{t-1} = dGh . W_hh is one 32x256x768 product per workgroup on bf16 MFMAs with
//     W_hh^T streamed from L2 (384 KB shared by all workgroups) through a register ring.
//     Bias and W_q gradients are reduced in registers and added once per workgroup.
// The forward uses the quantized W_hh, the backward the bf16 master copy (straight-through,
// the usual fp8-training split); weight gradients dW_hh / dW_ih stay split-K GEMMs.
#include "gru_common.h"

namespace st {

constexpr int LB = 32;      // sequences per workgroup
constexpr int NSV = 5;      // saved quantities: r, z, n, gh_n, h_prev

// ---------------------------------------------------------------- sequence gather
struct GruGather {
  const bf16_t* rx;
  const unsigned char* ra;
  const float* rr;
  const unsigned char* rd;
  const bf16_t* rh0;
  const unsigned long long* rctrl;
  int cap, S, B;
  uint32_t key0, key1;
  const unsigned long long* step;   // update counter (device, graph-replay safe)
  bf16_t* X;         // [(S+1)B][RFL] time-major rows t*B + b (columns >= RF zero)
  float* H0;         // [B][RH]
  int* A;            // [S][B]
  float* R;
  float* D;
};

// one wave per sampled segment (uniform over the filled ring, Philox counter = (row, update))
__global__ void __launch_bounds__(256) gru_gather_kernel(GruGather g) {
  const int b = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, lane = threadIdx.x & 63;
  if (b >= g.B) return;
  const unsigned long long sz = g.rctrl[1], st = g.step[0];
  uint32_t c0 = (uint32_t)b, c1 = (uint32_t)(st & 0xFFFFFFFFull), c2 = (uint32_t)(st >> 32), c3 = 0x53455131u;
  philox4x32(c0, c1, c2, c3, g.key0, g.key1);
  const size_t idx = (size_t)(((((unsigned long long)c0) << 32) | c1) % (sz ? sz : 1ull));
  const int S = g.S;
  const uint4 z = {0u, 0u, 0u, 0u};
  // every load of the segment is issued before the first store (the stores could alias the later
  // loads as far as the compiler knows, which would otherwise make each a dependent round trip)
  constexpr int XP = 3;   // x pieces per lane held at once: (S + 1) * 8 <= 192 covers S <= 23 in one pass
  for (int j0 = 0; j0 < (S + 1) * 8; j0 += 64 * XP) {
    uint4 v[XP];
#pragma unroll
    for (int k = 0; k < XP; ++k) {
      const int j = j0 + 64 * k + lane, t = j >> 3, c = j & 7;
      v[k] = z;
      if (j < (S + 1) * 8 && c < RF / 8) v[k] = reinterpret_cast<const uint4*>(g.rx + (idx * (size_t)(S + 1) + t) * RF)[c];
      if (c == RF / 8) v[k].x = 0x3F80u;   // column RF = 1.0: the dW_ih GEMM's column RF is then db_ih
    }
    const s4v hv = *reinterpret_cast<const s4v*>(g.rh0 + idx * RH + 4 * lane);
    unsigned char a = 0, d = 0;
    float r = 0.f;
    if (j0 == 0 && lane < S) {
      a = g.ra[idx * S + lane];
      r = g.rr[idx * S + lane];
      d = g.rd[idx * S + lane];
    }
#pragma unroll
    for (int k = 0; k < XP; ++k) {
      const int j = j0 + 64 * k + lane, t = j >> 3, c = j & 7;
      if (j < (S + 1) * 8) reinterpret_cast<uint4*>(g.X + ((size_t)t * g.B + b) * RFL)[c] = v[k];
    }
    if (j0 == 0) {
      *reinterpret_cast<float4*>(g.H0 + (size_t)b * RH + 4 * lane) =
          make_float4(bf2f((bf16_t)hv[0]), bf2f((bf16_t)hv[1]), bf2f((bf16_t)hv[2]), bf2f((bf16_t)hv[3]));
      if (lane < S) {
        g.A[(size_t)lane * g.B + b] = a;
        g.R[(size_t)lane * g.B + b] = r;
        g.D[(size_t)lane * g.B + b] = (float)d;
      }
    }
  }
}

// ---------------------------------------------------------------- fused forward
struct GruNetW {
  const i8v* whh8;
  const int* whhs;
  const s8v* wih;
  const float* bias4;
  const float* wq;
};

struct GruSeqFwd {
  GruNetW on, tg;       // online / target packed weights (gru_pack_kernel layout)
  const bf16_t* X;      // [(S+1)B][RFL]
  const float* H0;      // [B][RH]
  const float* D;       // [S][B]
  float* Q;             // [(S+1)B][4] online
  float* Qt;            // [(S+1)B][4] target
  bf16_t* HT;           // online: h_{t-1}^T (masked) for the dW_hh GEMM, [RH][ldht], column t*B + b
  int ldht;
  uint4* sv;            // online saves [S][B/LB][RW][NSV][2][64] x 16 B
  int B, S;
};

struct FwdLds {
  static constexpr int WX = 0;                          // RW*6*64 s8v
  static constexpr int X = WX + RW * 6 * 64 * 16;       // [2][LB*XS] bf16
  static constexpr int H8 = X + 2 * LB * XS * 2;        // [2][LB*HS] bytes
  static constexpr int SC = H8 + 2 * LB * HS;           // [2][LB*SCS] int
  static constexpr int B = SC + 2 * LB * SCS * 4;       // [4*RH] float
  static constexpr int WQ = B + 4 * RH * 4;             // [4*RH] float
  static constexpr int QP = WQ + 4 * RH * 4;            // [2][RW][3][LB] float
  static constexpr int HT = QP + 2 * RW * 3 * LB * 4;    // [2][RH][LB] bf16: h^T staging
  static constexpr int BYTES = HT + 2 * RH * LB * 2;
};
static_assert(FwdLds::BYTES <= 160 * 1024, "fwd LDS");

ST_DEV uint4 pack8_bf(const float (&v)[8]) {
  uint4 r;
  r.x = pack_bf2(v[0], v[1]);
  r.y = pack_bf2(v[2], v[3]);
  r.z = pack_bf2(v[4], v[5]);
  r.w = pack_bf2(v[6], v[7]);
  return r;
}
ST_DEV void unpack8_bf(uint4 u, float (&v)[8]) {
  v[0] = __uint_as_float(u.x << 16); v[1] = __uint_as_float(u.x & 0xFFFF0000u);
  v[2] = __uint_as_float(u.y << 16); v[3] = __uint_as_float(u.y & 0xFFFF0000u);
  v[4] = __uint_as_float(u.z << 16); v[5] = __uint_as_float(u.z & 0xFFFF0000u);
  v[6] = __uint_as_float(u.w << 16); v[7] = __uint_as_float(u.w & 0xFFFF0000u);
}

__global__ void __launch_bounds__(RT, 1) gru_seq_fwd_kernel(GruSeqFwd p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  bf16_t* sX = reinterpret_cast<bf16_t*>(lds + FwdLds::X);
  unsigned char* sH8 = lds + FwdLds::H8;
  int* sSc = reinterpret_cast<int*>(lds + FwdLds::SC);
  float* sB = reinterpret_cast<float*>(lds + FwdLds::B);
  float* sWq = reinterpret_cast<float*>(lds + FwdLds::WQ);
  float* sQp = reinterpret_cast<float*>(lds + FwdLds::QP);
  bf16_t* sHT = reinterpret_cast<bf16_t*>(lds + FwdLds::HT);
  const int tid = threadIdx.x, lane = tid & 63, l16 = lane & 15, g4 = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool online = blockIdx.y == 0;
  // h (masked) -> transposed staging [unit][seq] (bf16), then 64-B rows of HT after the next barrier
  auto stage_h = [&](bf16_t* st, const float (&h)[2][2][4]) {
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int i = 0; i < 4; ++i) st[(32 * wave + 16 * m + 4 * g4 + i) * LB + 16 * n + l16] = f2bf(h[m][n][i]);
  };
  auto flush_h = [&](const bf16_t* st, int blk) {
    for (int c = tid; c < RH * (LB / 8); c += RT) {
      const int u = c / (LB / 8), j = c % (LB / 8);
      *reinterpret_cast<uint4*>(p.HT + (size_t)u * p.ldht + (size_t)blk * p.B + blockIdx.x * LB + 8 * j) =
          *reinterpret_cast<const uint4*>(st + u * LB + 8 * j);
    }
  };
  const i8v* whh8 = online ? p.on.whh8 : p.tg.whh8;
  const int* whhs = online ? p.on.whhs : p.tg.whhs;
  const s8v* wih = online ? p.on.wih : p.tg.wih;
  const float* bias4 = online ? p.on.bias4 : p.tg.bias4;
  const float* wq = online ? p.on.wq : p.tg.wq;
  float* Qout = online ? p.Q : p.Qt;
  const int B = p.B, S = p.S, b0 = blockIdx.x * LB;

  for (int i = tid; i < RW * 6 * 64; i += RT) reinterpret_cast<s8v*>(lds + FwdLds::WX)[i] = wih[i];
  for (int i = tid; i < 4 * RH; i += RT) {
    sB[i] = bias4[i];
    sWq[i] = wq[i];
  }
  i8v Wh[3][2][2];
  int Ws4[3] = {0, 0, 0};
#pragma unroll
  for (int g = 0; g < 3; ++g)
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int idx = (((wave * 3 + g) * 2 + m) * 2 + ks) * 64 + lane;
        Wh[g][m][ks] = whh8[idx];
        Ws4[g] |= (whhs[idx] & 0xFF) << (8 * (2 * m + ks));
      }
  const s8v* myWx = reinterpret_cast<const s8v*>(lds + FwdLds::WX) + wave * 6 * 64 + lane;
  s8v WqA;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int u = 32 * wave + (j < 4 ? 4 * g4 + j : 16 + 4 * g4 + j - 4);
    WqA[j] = (short)f2bf(l16 < 3 ? wq[l16 * RH + u] : 0.f);
  }
  // h0 and x_0
  float hr[2][2][4];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      const int b = b0 + 16 * n + l16, u0 = 32 * wave + 16 * m + 4 * g4;
      const float4 v = *reinterpret_cast<const float4*>(p.H0 + (size_t)b * RH + u0);
      hr[m][n][0] = v.x; hr[m][n][1] = v.y; hr[m][n][2] = v.z; hr[m][n][3] = v.w;
    }
  if (online) stage_h(sHT + RH * LB, hr);   // block 0 = h0, staged in buffer 1
  quant_h(hr, sH8, sSc, wave, l16, g4);
  // x rows: thread tid < LB*4 moves 16 B (row tid/4, chunk tid%4); x_{t+1} is prefetched a step ahead
  const int xr = tid >> 2, xc = tid & 3;
  const bool xmover = tid < LB * 4;
  uint4 xnext = {0u, 0u, 0u, 0u};
  if (xmover) {
    reinterpret_cast<uint4*>(sX + xr * XS)[xc] = reinterpret_cast<const uint4*>(p.X + (size_t)(b0 + xr) * RFL)[xc];
    xnext = reinterpret_cast<const uint4*>(p.X + ((size_t)B + b0 + xr) * RFL)[xc];
  }
  __syncthreads();
  if (online) flush_h(sHT + RH * LB, 0);
  const size_t nblk = (size_t)(B / LB);

  for (int t = 0; t <= S; ++t) {
    const int cur = t & 1, nxt = cur ^ 1;
    const bf16_t* cX = sX + cur * LB * XS;
    const unsigned char* cH = sH8 + cur * LB * HS;
    const int* cS = sSc + cur * LB * SCS;
    float* qp = sQp + cur * RW * 3 * LB;
    const bool save = online && t < S;
    float keep[2] = {1.f, 1.f};
    if (t < S) {
      keep[0] = 1.f - p.D[(size_t)t * B + b0 + l16];
      keep[1] = 1.f - p.D[(size_t)t * B + b0 + 16 + l16];
    }
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      f4v ar[2], az[2], anx[2], anh[2];
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const int u0 = 32 * wave + 16 * m + 4 * g4;
        ar[m] = *reinterpret_cast<const f4v*>(sB + u0);
        az[m] = *reinterpret_cast<const f4v*>(sB + RH + u0);
        anx[m] = *reinterpret_cast<const f4v*>(sB + 2 * RH + u0);
        anh[m] = *reinterpret_cast<const f4v*>(sB + 3 * RH + u0);
      }
      const int row = 16 * n + l16;
      {
        const s8v xb = lds_ld8(cX + row * XS + 8 * g4);
#pragma unroll
        for (int m = 0; m < 2; ++m) {
          ar[m] = mfma32(myWx[(0 * 2 + m) * 64], xb, ar[m]);
          az[m] = mfma32(myWx[(1 * 2 + m) * 64], xb, az[m]);
          anx[m] = mfma32(myWx[(2 * 2 + m) * 64], xb, anx[m]);
        }
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const uint4 h0 = *reinterpret_cast<const uint4*>(cH + row * HS + 128 * ks + 16 * g4);
        const uint4 h1 = *reinterpret_cast<const uint4*>(cH + row * HS + 128 * ks + 64 + 16 * g4);
        i8v hb;
        hb[0] = (int)h0.x; hb[1] = (int)h0.y; hb[2] = (int)h0.z; hb[3] = (int)h0.w;
        hb[4] = (int)h1.x; hb[5] = (int)h1.y; hb[6] = (int)h1.z; hb[7] = (int)h1.w;
        const int sc = cS[row * SCS + 4 * ks + g4];
#define ST_MX3(M, KS)                                                              \
  ar[M] = mx_mfma_sel<2 * (M) + (KS)>(Wh[0][M][KS], hb, ar[M], Ws4[0], sc);          \
  az[M] = mx_mfma_sel<2 * (M) + (KS)>(Wh[1][M][KS], hb, az[M], Ws4[1], sc);          \
  anh[M] = mx_mfma_sel<2 * (M) + (KS)>(Wh[2][M][KS], hb, anh[M], Ws4[2], sc);
        if (ks == 0) { ST_MX3(0, 0) ST_MX3(1, 0) } else { ST_MX3(0, 1) ST_MX3(1, 1) }
#undef ST_MX3
      }
      float vr[8], vz[8], vn[8], vg[8], vh[8];
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float r = sigm_ps(ar[m][i]);
          const float z = sigm_ps(az[m][i]);
          const float nn = tanh_ps(__builtin_fmaf(r, anh[m][i], anx[m][i]));
          // gh_n un-scaled for the backward (the packed weights are pre-scaled, gru_common.h)
          vr[4 * m + i] = r; vz[4 * m + i] = z; vn[4 * m + i] = nn; vg[4 * m + i] = anh[m][i] * (1.f / GS_N);
          vh[4 * m + i] = hr[m][n][i];
          hr[m][n][i] = __builtin_fmaf(z, hr[m][n][i] - nn, nn);
        }
      if (save) {
        uint4* sv = p.sv + ((((size_t)t * nblk + blockIdx.x) * RW + wave) * NSV * 2) * 64 + lane;
        sv[(0 * 2 + n) * 64] = pack8_bf(vr);
        sv[(1 * 2 + n) * 64] = pack8_bf(vz);
        sv[(2 * 2 + n) * 64] = pack8_bf(vn);
        sv[(3 * 2 + n) * 64] = pack8_bf(vg);
        sv[(4 * 2 + n) * 64] = pack8_bf(vh);
      }
      {
        s8v hb;
        const uint32_t p0 = pack_bf2(hr[0][n][0], hr[0][n][1]), p1 = pack_bf2(hr[0][n][2], hr[0][n][3]);
        const uint32_t p2 = pack_bf2(hr[1][n][0], hr[1][n][1]), p3 = pack_bf2(hr[1][n][2], hr[1][n][3]);
        hb[0] = (short)(p0 & 0xFFFF); hb[1] = (short)(p0 >> 16); hb[2] = (short)(p1 & 0xFFFF); hb[3] = (short)(p1 >> 16);
        hb[4] = (short)(p2 & 0xFFFF); hb[5] = (short)(p2 >> 16); hb[6] = (short)(p3 & 0xFFFF); hb[7] = (short)(p3 >> 16);
        const f4v q = mfma32(WqA, hb, zero4());
        if (g4 == 0) {
          qp[(wave * 3 + 0) * LB + row] = q[0];
          qp[(wave * 3 + 1) * LB + row] = q[1];
          qp[(wave * 3 + 2) * LB + row] = q[2];
        }
      }
    }
    if (t < S) {
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
          for (int i = 0; i < 4; ++i) hr[m][n][i] *= keep[n];
      if (online && t + 1 < S) stage_h(sHT + cur * RH * LB, hr);   // HT block t+1 = masked h_t
      quant_h(hr, sH8 + nxt * LB * HS, sSc + nxt * LB * SCS, wave, l16, g4);
      if (xmover) {
        reinterpret_cast<uint4*>(sX + nxt * LB * XS + xr * XS)[xc] = xnext;
        if (t + 2 <= S) xnext = reinterpret_cast<const uint4*>(p.X + ((size_t)(t + 2) * B + b0 + xr) * RFL)[xc];
      }
    }
    __syncthreads();
    if (online && t + 1 < S) flush_h(sHT + cur * RH * LB, t + 1);
    if (wave == 0 && lane < LB) {
      float q[3];
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        float v = sWq[3 * RH + a];
#pragma unroll
        for (int w = 0; w < RW; ++w) v += qp[(w * 3 + a) * LB + lane];
        q[a] = v;
      }
      *reinterpret_cast<float4*>(Qout + ((size_t)t * B + b0 + lane) * 4) = make_float4(q[0], q[1], q[2], 0.f);
    }
  }
}

// ---------------------------------------------------------------- TD targets (double DQN)
struct GruTD {
  const float* Q;     // [(S+1)B][4] online
  const float* Qt;    // [(S+1)B][4] target net
  const int* A;
  const float* R;
  const float* D;     // [S][B]
  float* dQ;          // [S*B][4]
  float* loss;        // [1] (atomic)
  int B, S, burn;
  float gamma, coef;
};

__global__ void __launch_bounds__(256) gru_td_kernel(GruTD p) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  float l = 0.f;
  if (i < p.S * p.B) {
    const int t = i / p.B;
    const float* qn = p.Q + ((size_t)i + p.B) * 4;
    int as = 0;
    if (qn[1] > qn[as]) as = 1;
    if (qn[2] > qn[as]) as = 2;
    const float y = p.R[i] + p.gamma * (1.f - p.D[i]) * p.Qt[((size_t)i + p.B) * 4 + as];
    const int a = p.A[i];
    const float d = p.Q[(size_t)i * 4 + a] - y;
    float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
    if (t >= p.burn) {
      const float v = p.coef * d;
      if (a == 0) g.x = v; else if (a == 1) g.y = v; else g.z = v;
      l = d * d;
    }
    *reinterpret_cast<float4*>(p.dQ + (size_t)i * 4) = g;
  }
  l = wave_sum(l);
  if ((threadIdx.x & 63) == 0) atomicAdd(p.loss, l);
}

// ---------------------------------------------------------------- fused backward through time
struct GruSeqBwd {
  const uint4* sv;      // forward saves
  const float* dQ;      // [S*B][4]
  const float* D;       // [S][B]
  const i8v* whhT8;     // W_hh^T MX-fp8 A fragments [RW][2][6][64] (gru_pack_kernel, online net)
  const int* whhTs;     // their E8M0 scales
  const float* wq;      // [3][RH] online fp32
  bf16_t* dGxT;         // [RG][S*B]: weight-gradient GEMM operands, written transposed (staged in LDS)
  bf16_t* dGhT;         // [RG][S*B]
  float* gwq;           // [3][RH]   (+= ; zeroed by the host each update)
  float* gbq;           // [3]
  int B, S;
};

constexpr int GQS = RG + 16;      // dGh fp8 tile row stride (bytes): 784, conflict-free b128 reads
constexpr int GSC = RG / 32 + 1;  // scale row stride (ints): 24 K-blocks + pad

constexpr int LBB = 16;          // sequences per backward workgroup (one MFMA env tile: register budget)

struct BwdLds {
  // [2 buffers][hi, lo][LBB][GQS] bytes, then scales [2][hi, lo][LBB][GSC] ints, then W_q
  static constexpr int G8 = 0;
  static constexpr int SC = G8 + 2 * 2 * LBB * GQS;
  static constexpr int WQ = SC + 2 * 2 * LBB * GSC * 4;
  static constexpr int TR = WQ + 3 * RH * 4;                 // [2 buffers][dGh, dGx][RG][LBB] bf16
  static constexpr int BYTES = TR + 2 * 2 * RG * LBB * 2;
};
static_assert(BwdLds::BYTES <= 160 * 1024, "bwd LDS");

ST_DEV float row16_sum(float v) {   // sum over the 16 lanes of a row (same lane group)
  v += __shfl_xor(v, 1, 64);
  v += __shfl_xor(v, 2, 64);
  v += __shfl_xor(v, 4, 64);
  v += __shfl_xor(v, 8, 64);
  return v;
}
template <int BYTE>
ST_DEV float fp8_to_f32(uint32_t word) {
  return __builtin_amdgcn_cvt_f32_fp8((int)word, BYTE);
}

// dGh of one gate for this lane's (m, i) units of env tile n, as an MX-fp8 hi/lo pair:
// hi = q(x), lo = q(x - deq(hi)), each with its own E8M0 scale per (seq, 32-unit block = this
// wave's units): ~bf16-level precision for the recurrent GEMM's B operand.
ST_DEV void quant_hilo(const float (&x)[8], unsigned char* hiRow, unsigned char* loRow, int* scHi, int* scLo,
                       int off, int blk, int g4) {
  float amax = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) amax = fmaxf(amax, fabsf(x[k]));
  amax = rowmax4(amax);
  const int eh = mx_exp(amax);
  uint32_t hw[2];
  float res[8];
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    hw[m] = fp8x4(ldexpf(x[4 * m], -eh), ldexpf(x[4 * m + 1], -eh), ldexpf(x[4 * m + 2], -eh),
                  ldexpf(x[4 * m + 3], -eh));
    res[4 * m + 0] = x[4 * m + 0] - ldexpf(fp8_to_f32<0>(hw[m]), eh);
    res[4 * m + 1] = x[4 * m + 1] - ldexpf(fp8_to_f32<1>(hw[m]), eh);
    res[4 * m + 2] = x[4 * m + 2] - ldexpf(fp8_to_f32<2>(hw[m]), eh);
    res[4 * m + 3] = x[4 * m + 3] - ldexpf(fp8_to_f32<3>(hw[m]), eh);
  }
  float rmax = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) rmax = fmaxf(rmax, fabsf(res[k]));
  rmax = rowmax4(rmax);
  const int el = mx_exp(rmax);
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    *reinterpret_cast<uint32_t*>(hiRow + off + 16 * m) = hw[m];
    *reinterpret_cast<uint32_t*>(loRow + off + 16 * m) =
        fp8x4(ldexpf(res[4 * m], -el), ldexpf(res[4 * m + 1], -el), ldexpf(res[4 * m + 2], -el),
              ldexpf(res[4 * m + 3], -el));
  }
  if (g4 == 0) {
    scHi[blk] = eh + 127;
    scLo[blk] = el + 127;
  }
}

__global__ void __launch_bounds__(RT, 1) gru_seq_bwd_kernel(GruSeqBwd p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  int* sSc = reinterpret_cast<int*>(lds + BwdLds::SC);
  float* sWq = reinterpret_cast<float*>(lds + BwdLds::WQ);
  bf16_t* sT = reinterpret_cast<bf16_t*>(lds + BwdLds::TR);
  const size_t RS = (size_t)p.S * p.B;
  const int tid = threadIdx.x, lane = tid & 63, l16 = lane & 15, g4 = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int B = p.B, S = p.S, b0 = blockIdx.x * LBB;
  const size_t nblk = (size_t)(B / LB);
  const int fblk = blockIdx.x >> 1, fn = blockIdx.x & 1;   // forward block / env tile of the saves
  for (int i = tid; i < 3 * RH; i += RT) sWq[i] = p.wq[i];
  // resident W_hh^T (this wave's 32 units x 768 gates) as MX-fp8: 96 VGPRs + 3 packed scale regs
  i8v Wt[2][6];
  int Wts4[3] = {0, 0, 0};   // (m, ks) -> reg (6m + ks) >> 2, byte (6m + ks) & 3
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int ks = 0; ks < 6; ++ks) {
      const int idx = ((wave * 2 + m) * 6 + ks) * 64 + lane;
      const int q = 6 * m + ks;
      Wt[m][ks] = p.whhT8[idx];
      Wts4[q >> 2] |= (p.whhTs[idx] & 0xFF) << (8 * (q & 3));
    }

  float rec[2][4];           // dL/d(masked h_t) arriving from step t+1 (direct + GEMM)
  float gq[3][2][4];         // W_q gradient partials (units m, i), summed over this lane's steps
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      rec[m][i] = 0.f;
      gq[0][m][i] = gq[1][m][i] = gq[2][m][i] = 0.f;
    }
  float gbq0 = 0.f, gbq1 = 0.f, gbq2 = 0.f;
  // step inputs (saves, dQ rows, done flags) are loaded one step ahead
  uint4 pf[NSV];
  float4 pdq;
  float pkeep;
  auto load_step = [&](int tt) {
    const uint4* sv = p.sv + ((((size_t)tt * nblk + fblk) * RW + wave) * NSV * 2) * 64 + lane;
#pragma unroll
    for (int q = 0; q < NSV; ++q) pf[q] = sv[(q * 2 + fn) * 64];
    const int b = b0 + l16;
    pdq = *reinterpret_cast<const float4*>(p.dQ + ((size_t)tt * B + b) * 4);
    pkeep = (tt < S - 1) ? 1.f - p.D[(size_t)tt * B + b] : 0.f;
  };
  load_step(S - 1);
  __syncthreads();

  for (int t = S - 1; t >= 0; --t) {
    const int cur = t & 1;
    unsigned char* gHi = lds + BwdLds::G8 + (cur * 2 + 0) * LBB * GQS;
    unsigned char* gLo = lds + BwdLds::G8 + (cur * 2 + 1) * LBB * GQS;
    int* sHi = sSc + (cur * 2 + 0) * LBB * GSC;
    int* sLo = sSc + (cur * 2 + 1) * LBB * GSC;
    const int row = l16;
    float nrec[2][4];
    float dghv[3][8];      // dGh per gate (r, z, n_h), (m, i)
    {
      const float4 dq = pdq;
      const float keep = pkeep;
      float vr[8], vz[8], vn[8], vg[8], vh[8];
      unpack8_bf(pf[0], vr);
      unpack8_bf(pf[1], vz);
      unpack8_bf(pf[2], vn);
      unpack8_bf(pf[3], vg);
      unpack8_bf(pf[4], vh);
      if (wave == 0 && g4 == 0) { gbq0 += dq.x; gbq1 += dq.y; gbq2 += dq.z; }
      float dan[8];
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const int u0 = 32 * wave + 16 * m + 4 * g4;
        const f4v w0 = *reinterpret_cast<const f4v*>(sWq + u0);
        const f4v w1 = *reinterpret_cast<const f4v*>(sWq + RH + u0);
        const f4v w2 = *reinterpret_cast<const f4v*>(sWq + 2 * RH + u0);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int k = 4 * m + i;
          const float r = vr[k], z = vz[k], nn = vn[k], gh = vg[k], hp = vh[k];
          float dh = keep * rec[m][i];
          dh = __builtin_fmaf(dq.x, w0[i], dh);
          dh = __builtin_fmaf(dq.y, w1[i], dh);
          dh = __builtin_fmaf(dq.z, w2[i], dh);
          const float h = __builtin_fmaf(z, hp - nn, nn);      // unmasked h_t (Q input)
          gq[0][m][i] = __builtin_fmaf(dq.x, h, gq[0][m][i]);
          gq[1][m][i] = __builtin_fmaf(dq.y, h, gq[1][m][i]);
          gq[2][m][i] = __builtin_fmaf(dq.z, h, gq[2][m][i]);
          const float dn = dh * (1.f - z);
          const float dz = dh * (hp - nn);
          nrec[m][i] = dh * z;                                  // direct path into h_{t-1}
          const float a_n = dn * (1.f - nn * nn);
          dghv[0][k] = a_n * gh * r * (1.f - r);
          dghv[1][k] = dz * z * (1.f - z);
          dghv[2][k] = a_n * r;
          dan[k] = a_n;
        }
      }
      // transposed staging [gate row][seq] (dGh, dGx share the r / z rows; n differs)
      bf16_t* th = sT + (cur * 2 + 0) * RG * LBB;
      bf16_t* tx = sT + (cur * 2 + 1) * RG * LBB;
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int u = 32 * wave + 16 * m + 4 * g4 + i, k = 4 * m + i;
          const bf16_t vr_ = f2bf(dghv[0][k]), vz_ = f2bf(dghv[1][k]);
          th[(0 * RH + u) * LBB + row] = vr_;
          th[(1 * RH + u) * LBB + row] = vz_;
          th[(2 * RH + u) * LBB + row] = f2bf(dghv[2][k]);
          tx[(0 * RH + u) * LBB + row] = vr_;
          tx[(1 * RH + u) * LBB + row] = vz_;
          tx[(2 * RH + u) * LBB + row] = f2bf(dan[k]);
        }
    }
    if (t > 0) {
      load_step(t - 1);          // next step's inputs land during the quantization + GEMM
      // dGh -> MX-fp8 hi/lo tiles [seq][gate row] (+ scales per (seq, 32-row block = gate*8 + wave))
#pragma unroll
      for (int gt = 0; gt < 3; ++gt)
        quant_hilo(dghv[gt], gHi + row * GQS, gLo + row * GQS, sHi + row * GSC, sLo + row * GSC,
                   gt * RH + 32 * wave + 4 * g4, gt * 8 + wave, g4);
    }
    __syncthreads();
    // dGh^T / dGx^T rows of this step: 32 B per gate row (16 sequences), written as 16-B pieces
    for (int c = tid; c < 2 * RG * 2; c += RT) {
      const int mat = c / (RG * 2), rem = c % (RG * 2), gr = rem >> 1, half = rem & 1;
      const uint4 v = *reinterpret_cast<const uint4*>(sT + ((cur * 2 + mat) * RG + gr) * LBB + 8 * half);
      bf16_t* dst = (mat ? p.dGxT : p.dGhT) + (size_t)gr * RS + (size_t)t * B + b0 + 8 * half;
      *reinterpret_cast<uint4*>(dst) = v;
    }
    if (t == 0) break;
    // dh_{t-1} (through the recurrence) = direct + dGh_t . W_hh  (D[unit][seq], K = 768 gate rows)
    f4v acc[2];
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      acc[m][0] = nrec[m][0]; acc[m][1] = nrec[m][1]; acc[m][2] = nrec[m][2]; acc[m][3] = nrec[m][3];
    }
#define BW_KS(KS)                                                                                        \
    {                                                                                                    \
      i8v bh, bl;                                                                                        \
      const uint4 h0 = *reinterpret_cast<const uint4*>(gHi + row * GQS + 128 * (KS) + 16 * g4);          \
      const uint4 h1 = *reinterpret_cast<const uint4*>(gHi + row * GQS + 128 * (KS) + 64 + 16 * g4);     \
      bh[0] = (int)h0.x; bh[1] = (int)h0.y; bh[2] = (int)h0.z; bh[3] = (int)h0.w;                        \
      bh[4] = (int)h1.x; bh[5] = (int)h1.y; bh[6] = (int)h1.z; bh[7] = (int)h1.w;                        \
      const uint4 l0 = *reinterpret_cast<const uint4*>(gLo + row * GQS + 128 * (KS) + 16 * g4);          \
      const uint4 l1 = *reinterpret_cast<const uint4*>(gLo + row * GQS + 128 * (KS) + 64 + 16 * g4);     \
      bl[0] = (int)l0.x; bl[1] = (int)l0.y; bl[2] = (int)l0.z; bl[3] = (int)l0.w;                        \
      bl[4] = (int)l1.x; bl[5] = (int)l1.y; bl[6] = (int)l1.z; bl[7] = (int)l1.w;                        \
      const int sch = sHi[row * GSC + 4 * (KS) + g4], scl = sLo[row * GSC + 4 * (KS) + g4];             \
      acc[0] = mx_mfma_sel<(KS) & 3>(Wt[0][KS], bh, acc[0], Wts4[(KS) >> 2], sch);                       \
      acc[0] = mx_mfma_sel<(KS) & 3>(Wt[0][KS], bl, acc[0], Wts4[(KS) >> 2], scl);                       \
      acc[1] = mx_mfma_sel<(6 + (KS)) & 3>(Wt[1][KS], bh, acc[1], Wts4[(6 + (KS)) >> 2], sch);           \
      acc[1] = mx_mfma_sel<(6 + (KS)) & 3>(Wt[1][KS], bl, acc[1], Wts4[(6 + (KS)) >> 2], scl);           \
    }
    BW_KS(0) BW_KS(1) BW_KS(2) BW_KS(3) BW_KS(4) BW_KS(5)
#undef BW_KS
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int i = 0; i < 4; ++i) rec[m][i] = acc[m][i];
  }
  // W_q / b_q gradients: reduce the per-lane partials over the 16 sequences of a lane group
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int u = 32 * wave + 16 * m + 4 * g4 + i;
      const float v0 = row16_sum(gq[0][m][i]), v1 = row16_sum(gq[1][m][i]), v2 = row16_sum(gq[2][m][i]);
      if (l16 == 0) {
        atomicAdd(p.gwq + u, v0);
        atomicAdd(p.gwq + RH + u, v1);
        atomicAdd(p.gwq + 2 * RH + u, v2);
      }
    }
  if (wave == 0) {
    gbq0 = wave_sum(gbq0);
    gbq1 = wave_sum(gbq1);
    gbq2 = wave_sum(gbq2);
    if (lane == 0) {
      atomicAdd(p.gbq + 0, gbq0);
      atomicAdd(p.gbq + 1, gbq1);
      atomicAdd(p.gbq + 2, gbq2);
    }
  }
}

// Gradient fix-up after the weight-gradient GEMMs (one launch instead of four strided copies):
// dW_hh <- ext[:, :RH], db_hh <- ext[:, RH] (ones row of h^T), db_ih <- dW_ih[:, RF] (ones column
// of x), dW_ih[:, RF] <- 0.
__global__ void __launch_bounds__(256) gru_grad_fixup_kernel(const float* __restrict__ ext, int ldx, float* dwhh,
                                                             float* dbhh, float* dwih, float* dbih) {
  const int g = blockIdx.x;   // gate row
  const float* e = ext + (size_t)g * ldx;
  for (int u = threadIdx.x; u < RH; u += blockDim.x) dwhh[(size_t)g * RH + u] = e[u];
  if (threadIdx.x == 0) {
    dbhh[g] = e[RH];
    dbih[g] = dwih[(size_t)g * RFL + RF];
    dwih[(size_t)g * RFL + RF] = 0.f;
  }
}

}  // namespace st

extern "C" hipError_t st_gru_gather(const st::GruGather* g, hipStream_t s) {
  if (g->S > 64 || g->S <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(st::gru_gather_kernel, dim3((g->B + 3) / 4), dim3(256), 0, s, *g);
  return hipGetLastError();
}

extern "C" hipError_t st_gru_seq_fwd(const st::GruSeqFwd* p, hipStream_t s) {
  if (p->B % st::LB || p->S <= 0 || p->S > 64) return hipErrorInvalidValue;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)st::gru_seq_fwd_kernel,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, st::FwdLds::BYTES);
    if (e != hipSuccess) return e;
    attr = true;
  }
  hipLaunchKernelGGL(st::gru_seq_fwd_kernel, dim3(p->B / st::LB, 2), dim3(st::RT), st::FwdLds::BYTES, s, *p);
  return hipGetLastError();
}

extern "C" hipError_t st_gru_td(const st::GruTD* p, hipStream_t s) {
  hipLaunchKernelGGL(st::gru_td_kernel, dim3((p->S * p->B + 255) / 256), dim3(256), 0, s, *p);
  return hipGetLastError();
}

extern "C" hipError_t st_gru_seq_bwd(const st::GruSeqBwd* p, hipStream_t s) {
  if (p->B % st::LB || p->S <= 0 || p->S > 64) return hipErrorInvalidValue;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)st::gru_seq_bwd_kernel,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, st::BwdLds::BYTES);
    if (e != hipSuccess) return e;
    attr = true;
  }
  hipLaunchKernelGGL(st::gru_seq_bwd_kernel, dim3(p->B / st::LBB), dim3(st::RT), st::BwdLds::BYTES, s, *p);
  return hipGetLastError();
}

extern "C" hipError_t st_gru_grad_fixup(const float* ext, int ldx, float* dwhh, float* dbhh, float* dwih, float* dbih,
                                        hipStream_t s) {
  hipLaunchKernelGGL(st::gru_grad_fixup_kernel, dim3(st::RG), dim3(256), 0, s, ext, ldx, dwhh, dbhh, dwih, dbih);
  return hipGetLastError();
}

// struct sizes of this file's launch ABI, for the host mirrors' check (tests/test_abi.py; no HIP call)
extern "C" int st_abi_gru_learn(int* out, int n) {
  const int sz[] = {(int)sizeof(st::GruGather), (int)sizeof(st::GruNetW), (int)sizeof(st::GruSeqFwd), (int)sizeof(st::GruTD), (int)sizeof(st::GruSeqBwd)};
  const int m = (int)(sizeof(sz) / sizeof(sz[0]));
  for (int i = 0; i < n && i < m; ++i) out[i] = sz[i];
  return m;
}
