// bf16 MFMA GEMM with fused epilogues for the deep-MLP learner (BASELINE config 4:
// 4x1024 MLP Q-net, batch 4096 from an HBM replay buffer).
//
//   C[M,N] = A[M,K] . B[N,K]^T      A, B bf16, K-contiguous rows (lda, ldb elements)
//
// Every product of the MLP is put in this "NT" form by keeping the operands the
// next product needs in the right layout: the forward epilogue writes each hidden
// activation both row-major H[m][n] and transposed H^T[n][m], the optimizer keeps bf16
// copies of every weight as W[o][i] and W^T[i][o], so
//   forward   H   = act(X . W^T + b)          -> gemm(A=X,    B=W)
//   bwd-data  dH  = dZ . W     (masked)       -> gemm(A=dZ,   B=W^T)
//   bwd-wgrad dW  = dZ^T . X                  -> gemm(A=dZ^T, B=X^T)
//
// Kernel: 256 threads (2x2 waves), BM x BN block tile, BK = 64, double-buffered LDS
// filled by global_load_lds_dwordx4 (LDS-DMA, 1 KiB per wave-instruction) with the
// XOR-(row&7) chunk swizzle applied on the global SOURCE address, so the 16x16x32
// fragment reads (ds_read_b128) are bank-conflict-free; one barrier per K-tile
// (cdna_hip_programming.md T2, T3+T4 minimum 2-phase form).  Epilogues are staged
// through the (then idle) LDS buffers so that C and C^T leave in 16-byte stores.
#include "common.h"

#include <type_traits>

namespace st {

constexpr int GT = 256;   // threads
constexpr int GBK = 64;   // K tile

enum GemmEpi : int {
  EPI_BF16 = 0,      // out = act(alpha*acc + bias) as bf16 [M][N] (+ optional outT [N][M])
  EPI_RELU_GRAD = 1, // out = acc * (auxT[n][m] > 0) as bf16 [M][N] (+ outT)
  EPI_F32 = 2,       // out = alpha*acc (+ bias[n]) (+ out if accumulate) as fp32 [M][N]
  EPI_BF16_QH = 3,   // (internal) EPI_BF16 with the qpart head: its own instantiation, so the plain bf16
                     // epilogue keeps its registers (the launcher picks it when a problem sets qpart)
};

struct GemmArgs {
  const bf16_t* A;
  const bf16_t* B;
  void* out;
  bf16_t* outT;          // optional transposed bf16 output
  const float* bias;     // [N] or null
  const bf16_t* auxT;    // [N][M] activations (relu-grad mask), EPI_RELU_GRAD
  int M, N, K;
  int lda, ldb, ldo, ldoT, ldaux;
  int relu, accumulate;
  float alpha;
  int splitk;            // EPI_F32 only: K split over splitk workgroups per tile, atomically
                         // added into out (which then holds the prior value / zeros)
  // EPI_RELU_GRAD (2-stage gemm_body tiles) only, optional: column sums of the bf16 output over each wave's
  // rows, colpart[(M / WM) rows][ldcp] fp32 with partial row tm * NWM + wm -- the bias gradient's partials
  // (plain stores, no atomics; the optimizer sums the M / WM rows)
  float* colpart;
  int ldcp;
  // EPI_BF16 (2-stage gemm_body tiles) only, optional: the next layer's output head folded into this epilogue --
  // per row m and head row a < nq, the fp32 sum over each wave's WN columns of the stored (bf16) value times
  // qw[a][n]: qpart[(part * M + m) * 4 + a], part = n / WN (N / WN parts, plain stores; the consumer sums the
  // parts in a fixed order).  The update's Q(x) / Q_target(x') head without an output-layer launch.
  const bf16_t* qw;      // [nq][ldqw] bf16 head rows
  float* qpart;
  int ldqw, nq;
  int nqp;               // parts qpart holds (checked: N / WN of the launch's tile)
};

// a group of up to 4 products with one epilogue / tile in one launch (e.g. the online and target
// networks' forward of one layer): consecutive workgroup ranges compute problems 0, 1, ...
constexpr int GEMM_MAXB = 4;
struct GemmBatch {
  GemmArgs a[GEMM_MAXB];
  int n;
};

template <int BM, int BN, int S = 2>
struct GemmGeo {
  static constexpr int A_EL = BM * GBK, B_EL = BN * GBK;
  static constexpr int BUF_EL = A_EL + B_EL;
  static constexpr int KLOOP_BYTES = S * BUF_EL * 2;   // S-stage LDS ring
  // 256 x 256 tiles stage only C for the epilogue (C and C^T would need 270 KB): no transposed output
  static constexpr bool HAS_T = !(BM >= 256 && BN >= 256);
  static constexpr int EPI_BYTES = (BM * (BN + 8) + (HAS_T ? BN * (BM + 8) : 0)) * 2;
  static constexpr int LDS_BYTES = KLOOP_BYTES > EPI_BYTES ? KLOOP_BYTES : EPI_BYTES;
  // waves: 2 x 2 (256 threads, two blocks per CU); for 256 x 128, 4 x 2 (512 threads, one block per
  // CU: 1.33x fewer L2 bytes per MFMA than 128 x 128); for 256 x 256, 2 x 2 waves of 128 x 128 each
  // (one block per CU, 256 accumulator registers per lane: half the LDS fragment bytes per MFMA of
  // the 64 x 64 wave tiles)
  static constexpr int NWM = (BM >= 256 && BN < 256) ? 4 : 2, NWN = 2, NT = 64 * NWM * NWN;
  static constexpr int MINB = (NT > 256 || S > 2 || BM * BN >= 256 * 256) ? 1 : 2;
  // LDS-DMA instructions per wave per K-tile (vmcnt budget of the S-stage ring)
  static constexpr int LPT = (BM / 8 + NT / 64 - 1) / (NT / 64) + (BN / 8 + NT / 64 - 1) / (NT / 64);
  static constexpr int WM = BM / NWM, WN = BN / NWN;    // per-wave output tile
  static constexpr int TM = WM / 16, TN = WN / 16;  // 16x16 MFMA tiles per wave
  static_assert(BM % 32 == 0 && BN % 32 == 0, "tile");
  static_assert(LDS_BYTES * MINB <= 163840, "LDS per CU");
};

// stage one operand tile (ROWS x 64 bf16) of K-tile k0 into a linear LDS image with the
// chunk swizzle moved to the source address.  ROWS*8 16-B pieces, 64 per wave-instruction.
template <int ROWS, int NWAVE = GT / 64>
ST_DEV void stage_tile(const bf16_t* __restrict__ G, int ld, int row0, int k0, bf16_t* lds, int wave, int lane) {
  constexpr int INSTR = ROWS / 8;        // wave-instructions per tile
#pragma unroll
  for (int j = wave; j < INSTR; j += NWAVE) {
    const int r = j * 8 + (lane >> 3);
    const int c = lane & 7;
    const int g = c ^ (r & 7);
    const bf16_t* src = G + (size_t)(row0 + r) * ld + k0 + g * 8;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)(lds + j * 512), 16, 0, 0);
  }
}

// fragment (8 bf16) of row r, global chunk g of a staged tile
ST_DEV s8v frag_sw(const bf16_t* lds, int r, int g) {
  return lds_ld8(lds + r * GBK + ((g ^ (r & 7)) << 3));
}

template <int BM, int BN> constexpr int gemm_threads() { return (BM >= 256 && BN < 256) ? 512 : 256; }
template <int BM, int BN, int S> constexpr int gemm_min_blocks() {
  return ((BM >= 256 && BN < 256) || S > 2 || BM * BN >= 256 * 256) ? 1 : 2;
}

// s_waitcnt immediate: vmcnt = N (gfx9 split field), expcnt / lgkmcnt not waited on
template <int N>
ST_DEV void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 0xF) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}

// one reduce-scatter step of the qpart head sums (see gemm_body's epilogue): lanes l and l ^ H swap halves
template <int H>
ST_DEV void qh_step(float* x, int l16) {
  const bool up = (l16 & H) != 0;
#pragma unroll
  for (int k = 0; k < H; ++k) {
    const float keep = up ? x[k + H] : x[k], send = up ? x[k] : x[k + H];
    x[k] = keep + __shfl_xor(send, H);
  }
}

// workgroups of one problem: tiles x K-splits
template <int BM, int BN>
ST_DEV int gemm_blocks(const GemmArgs& p) {
  return (p.N / BN) * (p.M / BM) * (p.splitk > 1 ? p.splitk : 1);
}
ST_DEV int xcd_remap(int bid, int all) {   // neighbouring ids on one XCD's L2 (bijective)
  const int xcd = bid % 8, q = all / 8, r = all % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
}

// one workgroup's tile (and K split) of product p; bid = its index within p's blocks
template <int BM, int BN, int EPI, int S>
ST_DEV void gemm_body(const GemmArgs& p, int bid, char* gsm) {
  using G = GemmGeo<BM, BN, S>;
  constexpr int NW = G::NT / 64;
  bf16_t* buf = reinterpret_cast<bf16_t*>(gsm);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, l16 = lane & 15, g4 = lane >> 4;
  const int ntn = p.N / BN, ntm = p.M / BM, nwg = ntn * ntm;
  const int nsplit = p.splitk > 1 ? p.splitk : 1;
  const int ks = bid / nwg;   // K split (split-major: one split's tiles stay on one XCD's L2)
  bid -= ks * nwg;
  const int tm = bid / ntn, tn = bid % ntn;
  const int m0 = tm * BM, n0 = tn * BN;
  const int wm = wave / G::NWN, wn = wave % G::NWN;

  f4v acc[G::TM][G::TN];
#pragma unroll
  for (int i = 0; i < G::TM; ++i)
#pragma unroll
    for (int j = 0; j < G::TN; ++j) acc[i][j] = zero4();
  // EPI_BF16 head (qpart): qw[a][this lane's column of j] (0 for a >= nq), loaded under the K loop
  const bool qh = EPI == EPI_BF16_QH && p.qpart != nullptr;
  float qwv[G::TN][4];
  if (qh) {
#pragma unroll
    for (int j = 0; j < G::TN; ++j)
#pragma unroll
      for (int a = 0; a < 4; ++a)
        qwv[j][a] = a < p.nq ? bf2f(p.qw[(size_t)a * p.ldqw + n0 + wn * G::WN + 16 * j + l16]) : 0.f;
  }

  const int nk = p.K / GBK / nsplit;
  const int kb = ks * nk * GBK;
  if constexpr (S > 2) {
    // S-stage ring: tiles t+1 .. t+S-2 stay in flight while tile t is multiplied; one barrier per
    // K-tile (it also retires every wave's reads of tile t-1, whose buffer the next load refills)
#pragma unroll
    for (int s0 = 0; s0 < S - 1; ++s0)
      if (s0 < nk) {
        stage_tile<BM, NW>(p.A, p.lda, m0, kb + s0 * GBK, buf + s0 * G::BUF_EL, wave, lane);
        stage_tile<BN, NW>(p.B, p.ldb, n0, kb + s0 * GBK, buf + s0 * G::BUF_EL + G::A_EL, wave, lane);
      }
    int slot = 0;
    for (int t = 0; t < nk; ++t) {
      if (t + S - 2 < nk) wait_vmcnt<(S - 2) * G::LPT>();   // tile t landed, later ones may fly
      else __builtin_amdgcn_s_waitcnt(0);
      __syncthreads();
      if (t + S - 1 < nk) {
        const int ls = slot == 0 ? S - 1 : slot - 1;        // (t + S - 1) % S: tile t-1's buffer
        stage_tile<BM, NW>(p.A, p.lda, m0, kb + (t + S - 1) * GBK, buf + ls * G::BUF_EL, wave, lane);
        stage_tile<BN, NW>(p.B, p.ldb, n0, kb + (t + S - 1) * GBK, buf + ls * G::BUF_EL + G::A_EL, wave, lane);
      }
      const bf16_t* cA = buf + slot * G::BUF_EL;
      const bf16_t* cB = cA + G::A_EL;
#pragma unroll
      for (int kk = 0; kk < GBK / 32; ++kk) {
        s8v a[G::TM], b[G::TN];
#pragma unroll
        for (int i = 0; i < G::TM; ++i) a[i] = frag_sw(cA, wm * G::WM + 16 * i + l16, kk * 4 + g4);
#pragma unroll
        for (int j = 0; j < G::TN; ++j) b[j] = frag_sw(cB, wn * G::WN + 16 * j + l16, kk * 4 + g4);
#pragma unroll
        for (int i = 0; i < G::TM; ++i)
#pragma unroll
          for (int j = 0; j < G::TN; ++j) acc[i][j] = mfma32(a[i], b[j], acc[i][j]);
      }
      slot = slot == S - 1 ? 0 : slot + 1;
    }
    __syncthreads();   // every wave's last reads retired before the epilogue reuses the ring
  } else {
  stage_tile<BM, NW>(p.A, p.lda, m0, kb, buf, wave, lane);
  stage_tile<BN, NW>(p.B, p.ldb, n0, kb, buf + G::A_EL, wave, lane);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  for (int t = 0; t < nk; ++t) {
    bf16_t* cur = buf + (t & 1) * G::BUF_EL;
    if (t + 1 < nk) {
      bf16_t* nxt = buf + ((t + 1) & 1) * G::BUF_EL;
      stage_tile<BM, NW>(p.A, p.lda, m0, kb + (t + 1) * GBK, nxt, wave, lane);
      stage_tile<BN, NW>(p.B, p.ldb, n0, kb + (t + 1) * GBK, nxt + G::A_EL, wave, lane);
    }
    const bf16_t* cA = cur;
    const bf16_t* cB = cur + G::A_EL;
#pragma unroll
    for (int kk = 0; kk < GBK / 32; ++kk) {
      s8v a[G::TM], b[G::TN];
#pragma unroll
      for (int i = 0; i < G::TM; ++i) a[i] = frag_sw(cA, wm * G::WM + 16 * i + l16, kk * 4 + g4);
#pragma unroll
      for (int j = 0; j < G::TN; ++j) b[j] = frag_sw(cB, wn * G::WN + 16 * j + l16, kk * 4 + g4);
#pragma unroll
      for (int i = 0; i < G::TM; ++i)
#pragma unroll
        for (int j = 0; j < G::TN; ++j) acc[i][j] = mfma32(a[i], b[j], acc[i][j]);
    }
    __builtin_amdgcn_s_waitcnt(0);   // next tile landed (and this tile's reads retired)
    __syncthreads();
  }
  }

  // ------------------------------------------------------------------ epilogues
  if constexpr (EPI == EPI_F32) {
    float* out = reinterpret_cast<float*>(p.out);
#pragma unroll
    for (int i = 0; i < G::TM; ++i)
#pragma unroll
      for (int j = 0; j < G::TN; ++j) {
        const int n = n0 + wn * G::WN + 16 * j + l16;
        const float bb = (p.bias && ks == 0) ? p.bias[n] : 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * G::WM + 16 * i + 4 * g4 + r;
          float v = p.alpha * acc[i][j][r] + bb;
          float* o = out + (size_t)m * p.ldo + n;
          if (nsplit > 1) {
            atomicAdd(o, v);   // fp32 L2 atomic; the host zeroed out unless accumulating
          } else {
            if (p.accumulate) v += *o;
            *o = v;
          }
        }
      }
    return;
  } else {
    // stage C [BM][BN+8] and C^T [BN][BM+8] in LDS (the K-loop buffers are idle now)
    constexpr int SC = BN + 8, SCT = BM + 8;
    bf16_t* sC = buf;
    bf16_t* sCT = buf + BM * SC;   // (only with G::HAS_T)
    float csum[G::TN];   // EPI_RELU_GRAD: this lane's column sums over its TM x 4 rows
#pragma unroll
    for (int j = 0; j < G::TN; ++j) csum[j] = 0.f;
#pragma unroll
    for (int i = 0; i < G::TM; ++i) {
      float qs[4][4];   // [r][a]: this lane's head sums of rows 16 i + 4 g4 + r over its TN columns
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int a = 0; a < 4; ++a) qs[r][a] = 0.f;
#pragma unroll
      for (int j = 0; j < G::TN; ++j) {
        const int nl = wn * G::WN + 16 * j + l16;          // local col
        const int ml = wm * G::WM + 16 * i + 4 * g4;       // local row of r = 0
        float v[4];
        if constexpr (EPI == EPI_BF16 || EPI == EPI_BF16_QH) {
          const float bb = p.bias ? p.bias[n0 + nl] : 0.f;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float x = p.alpha * acc[i][j][r] + bb;
            v[r] = p.relu ? fmaxf(x, 0.f) : x;
          }
          if (qh) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float hv = bf2f(f2bf(v[r]));   // the stored value
#pragma unroll
              for (int a = 0; a < 4; ++a) qs[r][a] = fmaf(hv, qwv[j][a], qs[r][a]);
            }
          }
        } else {  // EPI_RELU_GRAD: mask by the forward activation (read from its transposed copy)
          const s4v h = *reinterpret_cast<const s4v*>(p.auxT + (size_t)(n0 + nl) * p.ldaux + m0 + ml);
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = (bf2f((bf16_t)h[r]) > 0.f) ? acc[i][j][r] : 0.f;
          if constexpr (EPI == EPI_RELU_GRAD) {
#pragma unroll
            for (int r = 0; r < 4; ++r) csum[j] += bf2f(f2bf(v[r]));   // the stored (bf16) values
          }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) sC[(ml + r) * SC + nl] = f2bf(v[r]);
        if constexpr (G::HAS_T) lds_st4(sCT + nl * SCT + ml, v[0], v[1], v[2], v[3]);
      }
      if (qh) {
        // sum the 16 values k = 4 r + a over the 16 lanes of the row group (its 16 columns per j) by a
        // reduce-scatter: at each step a lane keeps the half of its values selected by one bit of l16 and adds the
        // partner's copy of it (8 + 4 + 2 + 1 shuffles instead of 64); lane l16 ends with the sum of k = l16
        float x[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) x[k] = qs[k >> 2][k & 3];
        qh_step<8>(x, l16);   // (one template step each: constant indices, so x stays in registers)
        qh_step<4>(x, l16);
        qh_step<2>(x, l16);
        qh_step<1>(x, l16);
        const int part = (n0 + wn * G::WN) / G::WN;
        const int m = m0 + wm * G::WM + 16 * i + 4 * g4 + (l16 >> 2);
        p.qpart[((size_t)part * p.M + m) * 4 + (l16 & 3)] = x[0];
      }
    }
    if (EPI == EPI_RELU_GRAD && p.colpart) {
      // the 4 lane groups (rows 4 g4 ..) of each column, then one store per column of the wave's WM rows
#pragma unroll
      for (int j = 0; j < G::TN; ++j) {
        float x = csum[j];
        x += __shfl_xor(x, 16);
        x += __shfl_xor(x, 32);
        if (g4 == 0) p.colpart[(size_t)(tm * G::NWM + wm) * p.ldcp + n0 + wn * G::WN + 16 * j + l16] = x;
      }
    }
    __syncthreads();
    bf16_t* out = reinterpret_cast<bf16_t*>(p.out);
    constexpr int CPR = BN / 8;   // 16-byte chunks per C row
    for (int c = tid; c < BM * CPR; c += G::NT) {
      const int r = c / CPR, k = (c % CPR) * 8;
      *reinterpret_cast<uint4*>(out + (size_t)(m0 + r) * p.ldo + n0 + k) =
          *reinterpret_cast<const uint4*>(sC + r * SC + k);
    }
    if (G::HAS_T && p.outT) {
      constexpr int CPRT = BM / 8;
      for (int c = tid; c < BN * CPRT; c += G::NT) {
        const int r = c / CPRT, k = (c % CPRT) * 8;
        *reinterpret_cast<uint4*>(p.outT + (size_t)(n0 + r) * p.ldoT + m0 + k) =
            *reinterpret_cast<const uint4*>(sCT + r * SCT + k);
      }
    }
  }
}

// a batch of same-shape products (one problem per range of workgroups)
template <int BM, int BN, int EPI, int S = 2>
__global__ void __launch_bounds__((gemm_threads<BM, BN>()), (gemm_min_blocks<BM, BN, S>())) gemm_nt_kernel(GemmBatch batch) {
  using G = GemmGeo<BM, BN, S>;
  static_assert(G::NT == gemm_threads<BM, BN>() && G::MINB == gemm_min_blocks<BM, BN, S>(), "launch bounds");
  extern __shared__ __attribute__((aligned(16))) char gsm[];
  // problems may differ in shape (grouped GEMM): workgroup ranges in problem order
  int all = 0;
  for (int i = 0; i < batch.n; ++i) all += gemm_blocks<BM, BN>(batch.a[i]);
  int bid = xcd_remap(blockIdx.x, all), pi = 0;
  for (; pi + 1 < batch.n; ++pi) {
    const int nb = gemm_blocks<BM, BN>(batch.a[pi]);
    if (bid < nb) break;
    bid -= nb;
  }
  pi = __builtin_amdgcn_readfirstlane(pi);
  gemm_body<BM, BN, EPI, S>(batch.a[pi], bid, gsm);
}

// two products of any shapes and epilogues in one grid (e.g. a layer's data gradient beside the
// next layer's split-K weight gradient): no fork / join of streams between them
template <int BM, int BN, int EPI0, int EPI1, int S = 2>
__global__ void __launch_bounds__((gemm_threads<BM, BN>()), (gemm_min_blocks<BM, BN, S>())) gemm_dual_kernel(GemmArgs a0,
                                                                                                          GemmArgs a1) {
  extern __shared__ __attribute__((aligned(16))) char gsm[];
  const int n0 = gemm_blocks<BM, BN>(a0), n1 = gemm_blocks<BM, BN>(a1);
  const int bid = xcd_remap(blockIdx.x, n0 + n1);
  if (bid < n0) gemm_body<BM, BN, EPI0, S>(a0, bid, gsm);
  else gemm_body<BM, BN, EPI1, S>(a1, bid - n0, gsm);
}

template <int EPI0, int EPI1>
static hipError_t launch_dual(const GemmArgs& a0, const GemmArgs& a1, hipStream_t s) {
  using G = GemmGeo<128, 128, 2>;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)gemm_dual_kernel<128, 128, EPI0, EPI1, 2>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS_BYTES);
    if (e != hipSuccess) return e;
    attr = true;
  }
  const int nwg = (a0.M / 128) * (a0.N / 128) * (a0.splitk > 1 ? a0.splitk : 1) +
                  (a1.M / 128) * (a1.N / 128) * (a1.splitk > 1 ? a1.splitk : 1);
  hipLaunchKernelGGL((gemm_dual_kernel<128, 128, EPI0, EPI1, 2>), dim3(nwg), dim3(G::NT), G::LDS_BYTES, s, a0, a1);
  return hipGetLastError();
}

template <int BM, int BN, int EPI, int S = 2>
static hipError_t launch_gemm(const GemmBatch& p, hipStream_t s) {
  using G = GemmGeo<BM, BN, S>;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)gemm_nt_kernel<BM, BN, EPI, S>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS_BYTES);
    if (e != hipSuccess) return e;
    attr = true;
  }
  int nwg = 0;
  for (int i = 0; i < p.n; ++i) nwg += (p.a[i].M / BM) * (p.a[i].N / BN) * (p.a[i].splitk > 1 ? p.a[i].splitk : 1);
  hipLaunchKernelGGL((gemm_nt_kernel<BM, BN, EPI, S>), dim3(nwg), dim3(G::NT), G::LDS_BYTES, s, p);
  return hipGetLastError();
}

// ---------------------------------------------------------------- 256x256 ping-pong kernel
// 8 waves = 2 groups (wr = M half) x 4 (wc = 64-column quarter); waves w and w + 4 share a SIMD, one
// from each group.  The groups run one barrier interval apart: while one group issues the 64 MFMAs
// of a K-tile (C segment) the other reads all its fragments of its next K-tile from LDS (L segment:
// 16 A + 8 B ds_read_b128), so each SIMD's MFMA pipe is fed by one wave while the other loads.
// Interval 2t: G0 = L(t), G1 = C(t-1); interval 2t+1: G0 = C(t), G1 = L(t).
// LDS (160 KB): A in 2 buffers (K-tile parity; A0 = rows 0-127 read only by G0's L, A1 = rows 128-255
// only by G1's L), B in 3 (t mod 3; B0 / B1 = columns 0-127 / 128-255, read by both groups' L), so a
// half-tile can be restaged one interval after its last read and lands 3 intervals before it is read.
// global_load_lds staging (2 per thread per half-tile), 4 per thread per interval:
//   interval 2t:   A1(t+1), B0(t+2)
//   interval 2t+1: A0(t+2), B1(t+2)
// Every interval ends with lgkmcnt(0) (its fragment reads retired) + a counted vmcnt + a raw
// s_barrier (a __syncthreads() fence would add vmcnt(0) and drain the staging): vmcnt(10) after even
// intervals (A1(t) landed for G1's L(t)), vmcnt(8) after odd ones (A0(t+1), B(t+1) landed for G0's
// L(t+1)); vmcnt(0) in the last two K-tiles, where stages are skipped.  The two groups' loops are
// written out separately with the same stages, waits and barrier count (one loop with a role branch
// per interval made the register allocator keep both roles' values live: 500 VGPRs of spills).
// Epilogues: EPI_BF16 (bias / relu; no C^T) and EPI_F32 (alpha, bias, accumulate; no split-K).
namespace pp {
constexpr int NT = 512, HT = 128 * GBK;     // threads, elements per half-tile
constexpr int AB = 2 * HT, BB = 2 * HT;     // one K-tile of A (A0 A1) / of B (B0 B1)
constexpr int A_OFF = 0, B_OFF = 2 * AB;    // 2 A buffers, then 3 B buffers
constexpr int KLOOP_BYTES = (2 * AB + 3 * BB) * 2;   // 160 KB
constexpr int SC = 256 + 8;                 // epilogue C staging row stride (bf16)
constexpr int EPI_BYTES = 256 * SC * 2;
constexpr int LDS_BYTES = KLOOP_BYTES > EPI_BYTES ? KLOOP_BYTES : EPI_BYTES;
static_assert(LDS_BYTES <= 163840, "LDS");

template <int N>
ST_DEV void wait_vm_lgkm0() {   // vmcnt = N, lgkmcnt = 0, expcnt not waited on
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 0xF) | ((N >> 4) << 14) | (0x7 << 4));
}
// raw barrier that is also a compiler memory barrier (no LDS access moves across it) and emits no
// wait of its own
ST_DEV void barrier() { asm volatile("s_barrier" ::: "memory"); }
}  // namespace pp

// ABL (tools/ubench/gemm_lab.hip ablations only; wrong results by design): 1 no staging in the K-loop,
// 2 neither staging nor fragment reads (fragments of K-tile 0 reused), 3 no MFMAs.  GROUPED = 0: the
// round-5 tile order (one tile row per XCD wave), kept for the lab's A/B (profiles/r6_gemm_ablation.md)
template <int EPI, int PRIO = 0, int ABL = 0, int GROUPED = 1>
__global__ void __launch_bounds__(512, 1) gemm_pp_kernel(GemmArgs p) {
  extern __shared__ __attribute__((aligned(16))) char gsm[];
  bf16_t* buf = reinterpret_cast<bf16_t*>(gsm);
  const int tid = threadIdx.x, lane = tid & 63, l16 = lane & 15, g4 = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int ntn = p.N / 256, ntm = p.M / 256, nwg = ntn * ntm;
  int bid = blockIdx.x;
  {
    const int xcd = bid % 8, q = nwg / 8, r = nwg % 8;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
  }
  // tile order within an XCD's range: groups of 8 tile rows walked column by column, so the ~32
  // workgroups one XCD runs at a time cover an 8 x 4 block of C (12 operand tiles per K-tile through its
  // L2) instead of one tile row (1 + ntn); the same order as before when ntn <= 4
  int tm, tn;
  {
    const int gsz = 8 * ntn, g = bid / gsz, r = bid % gsz;
    const int gm = ntm - 8 * g < 8 ? ntm - 8 * g : 8;
    tm = 8 * g + r % gm;
    tn = r / gm;
  }
  const int m0 = (GROUPED ? tm : bid / ntn) * 256, n0 = (GROUPED ? tn : bid % ntn) * 256;
  const int nk = p.K / GBK;

  // Half-tile staging = stage_tile<128, 8>'s pieces (rows 8 wave + lane / 8 and 64 below them, swizzled
  // chunk (lane & 7) ^ (lane / 8)), addressed as a uniform base (SGPRs: tile row, K-tile, wave) plus ONE
  // loop-invariant 32-bit lane offset per operand: per-piece 64-bit lane addresses kept group 0's loop 2
  // VGPRs over the 256 budget, and the spill's reload put a vmcnt(0) -- a drain of the staging -- in
  // every K-tile.
  const uint32_t sw8 = (uint32_t)(((lane & 7) ^ (lane >> 3)) << 3);
  const uint32_t offA = ((uint32_t)(lane >> 3) * (uint32_t)p.lda + sw8) * 2u;
  const uint32_t offB = ((uint32_t)(lane >> 3) * (uint32_t)p.ldb + sw8) * 2u;
  auto glds = [&](const bf16_t* base, uint32_t off, bf16_t* lds) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(reinterpret_cast<const char*>(base) + off),
                                     (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
  };
  bool in_loop = false;   // ABL 1 / 2: no staging once the K-loop starts
  auto stAq = [&](int half, int kt, int q) {   // piece q (rows + 64 q) of A half-tile (rows m0 + 128 half ..)
    if ((ABL == 1 || ABL == 2) && in_loop) return;
    if (kt < nk)
      glds(p.A + (size_t)(m0 + 128 * half + 8 * wave + 64 * q) * p.lda + kt * GBK, offA,
           buf + pp::A_OFF + (kt & 1) * pp::AB + half * pp::HT + (wave + 8 * q) * 512);
  };
  auto stBq = [&](int half, int kt, int q) {
    if ((ABL == 1 || ABL == 2) && in_loop) return;
    if (kt < nk)
      glds(p.B + (size_t)(n0 + 128 * half + 8 * wave + 64 * q) * p.ldb + kt * GBK, offB,
           buf + pp::B_OFF + (kt % 3) * pp::BB + half * pp::HT + (wave + 8 * q) * 512);
  };
  auto stA = [&](int half, int kt) { stAq(half, kt, 0); stAq(half, kt, 1); };
  auto stB = [&](int half, int kt) { stBq(half, kt, 0); stBq(half, kt, 1); };

  f4v acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = zero4();
  s8v fa[8][2], fb[4][2];
  auto load = [&](int kt) {   // L segment: every fragment of K-tile kt this wave multiplies
    if constexpr (ABL == 2) {
      if (kt > 0) return;
    }
    const bf16_t* bA = buf + pp::A_OFF + (kt & 1) * pp::AB + wr * pp::HT;
    const bf16_t* bB = buf + pp::B_OFF + (kt % 3) * pp::BB + (wc >> 1) * pp::HT;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j][kk] = frag_sw(bB, (wc & 1) * 64 + 16 * j + l16, kk * 4 + g4);
#pragma unroll
      for (int i = 0; i < 8; ++i) fa[i][kk] = frag_sw(bA, 16 * i + l16, kk * 4 + g4);
    }
  };
  auto compute = [&]() {      // C segment: 64 MFMAs, no LDS access
    if constexpr (ABL == 3) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
        for (int i = 0; i < 8; ++i) asm volatile("" ::"v"(fa[i][kk]));
#pragma unroll
        for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(fb[j][kk]));
      }
      return;
    }
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);   // the MFMA wave first when both can issue
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma32(fa[i][kk], fb[j][kk], acc[i][j]);
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
  };
  auto even_end = [&](int t) {   // end of interval 2t
    if (t + 2 < nk) pp::wait_vm_lgkm0<10>(); else pp::wait_vm_lgkm0<0>();
    pp::barrier();
  };
  auto odd_end = [&](int t) {    // end of interval 2t+1
    if (t + 2 < nk) pp::wait_vm_lgkm0<8>(); else pp::wait_vm_lgkm0<0>();
    pp::barrier();
  };
  auto stage_even = [&](int t) {
    stA(1, t + 1);
    stB(0, t + 2);
  };
  auto stage_odd = [&](int t) {
    stA(0, t + 2);
    stB(1, t + 2);
  };

  // prologue: K-tile 0 whole, then what intervals -2 / -1 would have staged: A1(0) B0(1), A0(1) B1(1)
  stA(0, 0);
  stB(0, 0);
  stB(1, 0);
  stA(1, 0);
  stB(0, 1);
  stA(0, 1);
  stB(1, 1);
  if (nk > 1) pp::wait_vm_lgkm0<6>(); else pp::wait_vm_lgkm0<0>();
  pp::barrier();
  in_loop = true;
  if (wr == 0) {
    for (int t = 0; t < nk; ++t) {
      stage_even(t);
      load(t);                     // interval 2t
      even_end(t);
      stage_odd(t);
      compute();                   // interval 2t+1
      odd_end(t);
    }
  } else {
    stage_even(0);                 // interval 0: nothing to multiply yet
    even_end(0);
    stage_odd(0);
    load(0);                       // interval 1
    odd_end(0);
    for (int t = 1; t < nk; ++t) {
      stage_even(t);
      compute();                   // interval 2t
      even_end(t);
      stage_odd(t);
      load(t);                     // interval 2t+1
      odd_end(t);
    }
    compute();                     // interval 2nk
  }
  pp::wait_vm_lgkm0<0>();
  pp::barrier();   // every wave is done with the K-loop buffers

  // ------------------------------------------------------------------ epilogues
  const int wm0 = wr * 128, wn0 = wc * 64;   // this wave's block of the tile
  float bj[4];                                // bias of this lane's 4 columns: loaded once
#pragma unroll
  for (int j = 0; j < 4; ++j) bj[j] = 0.f;
  if (p.bias) {
#pragma unroll
    for (int j = 0; j < 4; ++j) bj[j] = p.bias[n0 + wn0 + 16 * j + l16];
  }
  if constexpr (EPI == EPI_F32) {
    float* out = reinterpret_cast<float*>(p.out);
    auto store = [&](auto accumulate) {   // the accumulate branch hoisted out of the element loops
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int n = n0 + wn0 + 16 * j + l16;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int m = m0 + wm0 + 16 * i + 4 * g4 + r;
            float* o = out + (size_t)m * p.ldo + n;
            const float v = p.alpha * acc[i][j][r] + bj[j];
            if constexpr (decltype(accumulate)::value) *o += v; else *o = v;
          }
        }
    };
    if (p.accumulate) store(std::true_type{}); else store(std::false_type{});
  } else {
    bf16_t* sC = buf;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int nl = wn0 + 16 * j + l16, ml = wm0 + 16 * i + 4 * g4;
        const float bb = bj[j];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float x = p.alpha * acc[i][j][r] + bb;
          sC[(ml + r) * pp::SC + nl] = f2bf(p.relu ? fmaxf(x, 0.f) : x);
        }
      }
    __syncthreads();
    bf16_t* out = reinterpret_cast<bf16_t*>(p.out);
    for (int c = tid; c < 256 * 32; c += pp::NT) {
      const int r = c >> 5, k = (c & 31) * 8;
      *reinterpret_cast<uint4*>(out + (size_t)(m0 + r) * p.ldo + n0 + k) = *reinterpret_cast<const uint4*>(sC + r * pp::SC + k);
    }
  }
}

template <int EPI, int PRIO = 0, int ABL = 0, int GROUPED = 1>
static hipError_t launch_gemm_pp(const GemmArgs& p, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)gemm_pp_kernel<EPI, PRIO, ABL, GROUPED>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, pp::LDS_BYTES);
    if (e != hipSuccess) return e;
    attr = true;
  }
  hipLaunchKernelGGL((gemm_pp_kernel<EPI, PRIO, ABL, GROUPED>), dim3((p.M / 256) * (p.N / 256)), dim3(pp::NT), pp::LDS_BYTES, s, p);
  return hipGetLastError();
}

// ---------------------------------------------------------------- 256x256, 4 waves of 128x128
// One wave per SIMD, each with a 128x128 accumulator block (256 AGPRs) -- 4 MFMAs per fragment read
// (the ping-pong kernel's 8 waves of 128x64 get 2.7) -- and two fragment register sets, so every
// LDS read is issued a whole 64-MFMA k-step ahead of its use.  Per K-tile t (BK = 64, LDS buffer
// t & 1, 2 x 64 KB):
//   phase X(t): 64 MFMAs on F0 = k-step 0 of tile t;  read F1 = k-step 1 of tile t
//   -- vmcnt(0) (tile t+1 landed) + lgkmcnt(0) + raw s_barrier --
//   phase Y(t): stage tile t+2 into buffer t & 1 (its last reads, F1(t), retired before the barrier);
//               64 MFMAs on F1;  read F0 = k-step 0 of tile t+1 (landed and visible since the barrier)
// One barrier per K-tile; a tile is staged 2 phases (one K-tile) before the wait that retires it,
// and no wave ever waits on an LDS read: the barrier is passed with X(t)'s MFMAs still in the pipe.
#ifndef ST_W4_ASM
#define ST_W4_ASM 1
#endif
namespace w4 {
constexpr int NT = 256;
constexpr int TILE = 256 * GBK;                         // one operand of one K-tile (elements)
constexpr int BUF = 2 * TILE;                           // A + B
constexpr int KLOOP_BYTES = 2 * BUF * 2;                // 128 KB
constexpr int SC = 256 + 8;
constexpr int EPI_BYTES = 256 * SC * 2;
constexpr int LDS_BYTES = KLOOP_BYTES > EPI_BYTES ? KLOOP_BYTES : EPI_BYTES;
static_assert(LDS_BYTES <= 163840, "LDS");
}  // namespace w4

template <int EPI>
__global__ void __launch_bounds__(256, 1) gemm_w4_kernel(GemmArgs p) {
  extern __shared__ __attribute__((aligned(16))) char gsm[];
  bf16_t* buf = reinterpret_cast<bf16_t*>(gsm);
  const int tid = threadIdx.x, lane = tid & 63, l16 = lane & 15, g4 = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  const int ntn = p.N / 256, ntm = p.M / 256;
  const int bid = xcd_remap(blockIdx.x, ntn * ntm);
  const int m0 = (bid / ntn) * 256, n0 = (bid % ntn) * 256;
  const int nk = p.K / GBK;

  auto stage = [&](int kt) {   // both operands of K-tile kt (8 + 8 global_load_lds per thread)
    if (kt < nk) {
      bf16_t* b = buf + (kt & 1) * w4::BUF;
      stage_tile<256, 4>(p.A, p.lda, m0, kt * GBK, b, wave, lane);
      stage_tile<256, 4>(p.B, p.ldb, n0, kt * GBK, b + w4::TILE, wave, lane);
    }
  };
  s8v F0a[8], F0b[8], F1a[8], F1b[8];
  auto read = [&](s8v (&fa)[8], s8v (&fb)[8], int kt, int kk) {
    const bf16_t* bA = buf + (kt & 1) * w4::BUF;
    const bf16_t* bB = bA + w4::TILE;
#pragma unroll
    for (int i = 0; i < 8; ++i) fa[i] = frag_sw(bA, wr * 128 + 16 * i + l16, kk * 4 + g4);
#pragma unroll
    for (int j = 0; j < 8; ++j) fb[j] = frag_sw(bB, wc * 128 + 16 * j + l16, kk * 4 + g4);
  };
  f4v acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = zero4();
  auto mma = [&](const s8v (&fa)[8], const s8v (&fb)[8]) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
#if ST_W4_ASM
        // accumulators pinned to AGPRs ("+a"): the builtin left the allocator free to move them
        // between the VGPR and AGPR files (~940 v_accvgpr_* per kernel)
        asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[i][j]) : "v"(fa[i]), "v"(fb[j]));
#else
        acc[i][j] = mfma32(fa[i], fb[j], acc[i][j]);
#endif
      }
  };

  // prologue: tiles 0 and 1 staged, tile 0 landed; F0 = k-step 0 of tile 0
  stage(0);
  stage(1);
  if (nk > 1) pp::wait_vm_lgkm0<16>(); else pp::wait_vm_lgkm0<0>();
  pp::barrier();
  read(F0a, F0b, 0, 0);
  for (int t = 0; t + 1 < nk; ++t) {   // (the last K-tile is peeled: no conditional fragment read in
                                      // the loop, which made the allocator shuffle accumulators)
    // ---- X(t)
    read(F1a, F1b, t, 1);
    mma(F0a, F0b);
    pp::wait_vm_lgkm0<0>();          // tile t+1 landed (this wave's part); F1 read retired
    pp::barrier();
    // ---- Y(t)
    stage(t + 2);
    read(F0a, F0b, t + 1, 0);
    mma(F1a, F1b);
  }
  read(F1a, F1b, nk - 1, 1);          // X(nk-1), Y(nk-1)
  mma(F0a, F0b);
  mma(F1a, F1b);
#if ST_W4_ASM
  // the hazard recognizer does not see through the asm MFMAs: cover the last MFMAs' result latency before
  // the epilogue's accumulator reads.  The accumulators the last eight MFMAs wrote are operands of the nop
  // block, so the compiler cannot schedule a read of them above it (a plain volatile asm does not order
  // register reads; profiles/r5_gemm_w4k.md)
  asm volatile("s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7"
               : "+a"(acc[7][7]), "+a"(acc[7][6]), "+a"(acc[7][5]), "+a"(acc[7][4]), "+a"(acc[7][3]),
                 "+a"(acc[7][2]), "+a"(acc[7][1]), "+a"(acc[7][0])::"memory");
#endif
  pp::wait_vm_lgkm0<0>();
  pp::barrier();   // every wave is done with the K-loop buffers

  // ------------------------------------------------------------------ epilogues
  const int wm0 = wr * 128, wn0 = wc * 128;
  float bj[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) bj[j] = 0.f;
  if (p.bias) {
#pragma unroll
    for (int j = 0; j < 8; ++j) bj[j] = p.bias[n0 + wn0 + 16 * j + l16];
  }
  if constexpr (EPI == EPI_F32) {
    float* out = reinterpret_cast<float*>(p.out);
    auto store = [&](auto accumulate) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int n = n0 + wn0 + 16 * j + l16;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int m = m0 + wm0 + 16 * i + 4 * g4 + r;
            float* o = out + (size_t)m * p.ldo + n;
            const float v = p.alpha * acc[i][j][r] + bj[j];
            if constexpr (decltype(accumulate)::value) *o += v; else *o = v;
          }
        }
    };
    if (p.accumulate) store(std::true_type{}); else store(std::false_type{});
  } else {
    bf16_t* sC = buf;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int nl = wn0 + 16 * j + l16, ml = wm0 + 16 * i + 4 * g4;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float x = p.alpha * acc[i][j][r] + bj[j];
          sC[(ml + r) * w4::SC + nl] = f2bf(p.relu ? fmaxf(x, 0.f) : x);
        }
      }
    __syncthreads();
    bf16_t* out = reinterpret_cast<bf16_t*>(p.out);
    for (int c = tid; c < 256 * 32; c += w4::NT) {
      const int r = c >> 5, k = (c & 31) * 8;
      *reinterpret_cast<uint4*>(out + (size_t)(m0 + r) * p.ldo + n0 + k) = *reinterpret_cast<const uint4*>(sC + r * w4::SC + k);
    }
  }
}

template <int EPI>
static hipError_t launch_gemm_w4(const GemmArgs& p, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)gemm_w4_kernel<EPI>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       w4::LDS_BYTES);
    if (e != hipSuccess) return e;
    attr = true;
  }
  hipLaunchKernelGGL((gemm_w4_kernel<EPI>), dim3((p.M / 256) * (p.N / 256)), dim3(w4::NT), w4::LDS_BYTES, s, p);
  return hipGetLastError();
}

}  // namespace st

// tile: 0 = 128x128, 1 = 64x64, 2 = 128x64, 3 = 256x128 (BM x BN; 3 runs 8 waves),
//       4 / 5 = 128x128 with a 3- / 4-stage LDS ring (one block per CU),
//       6 = 256x256 (4 waves of 128x128, one block per CU; no transposed output)
// shape / stride / epilogue checks of one product for a BM x BN tile (the kernel assumes whole tiles)
static bool gemm_args_ok(const st::GemmArgs* p, int epi, int bm, int bn, bool has_t) {
  if (!has_t && p->outT) return false;
  if (p->M % bm || p->N % bn || p->K % st::GBK || p->M <= 0 || p->N <= 0 || p->K <= 0) return false;
  if (p->lda % 8 || p->ldb % 8 || (epi != st::EPI_F32 && p->ldo % 8)) return false;
  if (p->outT && (p->ldoT % 8 || epi == st::EPI_F32)) return false;
  if (epi == st::EPI_RELU_GRAD && (!p->auxT || p->ldaux % 4)) return false;
  if (p->splitk > 1 && (epi != st::EPI_F32 || (p->K / st::GBK) % p->splitk)) return false;
  if (p->colpart && (epi != st::EPI_RELU_GRAD || p->ldcp < p->N)) return false;
  if (p->qpart && (epi != st::EPI_BF16 || !p->qw || p->nq < 1 || p->nq > 4 || p->ldqw < p->N || p->splitk > 1 ||
                   p->nqp != p->N / (bn / 2)))   // (every gemm_body tile has 2 wave columns: WN = BN / 2)
    return false;
  return true;
}

// n products (any shapes; same tile and epilogue) in one launch; st_gemm_nt = n 1
extern "C" hipError_t st_gemm_nt_batched(const st::GemmArgs* ps, int n, int epi, int tile, hipStream_t stream) {
  if (tile < 0 || tile > 6 || n < 1 || n > st::GEMM_MAXB) return hipErrorInvalidValue;
  const int bm = (tile == 3 || tile == 6) ? 256 : (tile == 1 ? 64 : 128);
  const int bn = (tile == 1 || tile == 2) ? 64 : (tile == 6 ? 256 : 128);
  st::GemmBatch b;
  b.n = n;
  bool qh = false;
  for (int i = 0; i < n; ++i) {
    const st::GemmArgs* p = ps + i;
    if (!gemm_args_ok(p, epi, bm, bn, tile != 6)) return hipErrorInvalidValue;
    b.a[i] = *p;
    qh = qh || p->qpart;
  }
  if (qh) epi = st::EPI_BF16_QH;   // (gemm_args_ok: qpart only with EPI_BF16)
#define ST_G(BM_, BN_, S_)                                                               \
  switch (epi) {                                                                         \
    case 0: return st::launch_gemm<BM_, BN_, 0, S_>(b, stream);                          \
    case 1: return st::launch_gemm<BM_, BN_, 1, S_>(b, stream);                          \
    case 2: return st::launch_gemm<BM_, BN_, 2, S_>(b, stream);                          \
    case 3: return st::launch_gemm<BM_, BN_, 3, S_>(b, stream);                          \
    default: return hipErrorInvalidValue;                                                \
  }
  if (tile == 0) { ST_G(128, 128, 2) }
  if (tile == 1) { ST_G(64, 64, 2) }
  if (tile == 2) { ST_G(128, 64, 2) }
  if (tile == 3) { ST_G(256, 128, 2) }
  if (tile == 4) { ST_G(128, 128, 3) }
  if (tile == 5) { ST_G(128, 128, 4) }
  if (tile == 6) { ST_G(256, 256, 2) }
#undef ST_G
  return hipErrorInvalidValue;
}

// two products of any shapes / epilogues on 128x128 tiles in one launch (epi pairs: relu-grad + f32,
// f32 + f32, bf16 + f32)
// struct sizes of this file's launch ABI, for the host mirror's check (tests/test_abi.py; no HIP call)
extern "C" int st_gemm_abi(int* out, int n) {
  const int sz[] = {(int)sizeof(st::GemmArgs), (int)sizeof(st::GemmBatch)};
  for (int i = 0; i < n && i < 2; ++i) out[i] = sz[i];
  return 2;
}

extern "C" hipError_t st_gemm_dual(const st::GemmArgs* a0, int epi0, const st::GemmArgs* a1, int epi1, hipStream_t stream) {
  if (!gemm_args_ok(a0, epi0, 128, 128, true) || !gemm_args_ok(a1, epi1, 128, 128, true)) return hipErrorInvalidValue;
  if (epi0 == st::EPI_RELU_GRAD && epi1 == st::EPI_F32) return st::launch_dual<1, 2>(*a0, *a1, stream);
  if (epi0 == st::EPI_F32 && epi1 == st::EPI_F32) return st::launch_dual<2, 2>(*a0, *a1, stream);
  if (epi0 == st::EPI_BF16 && epi1 == st::EPI_F32) return st::launch_dual<0, 2>(*a0, *a1, stream);
  return hipErrorInvalidValue;
}

extern "C" hipError_t st_gemm_nt(const st::GemmArgs* p, int epi, int tile, hipStream_t stream) {
  if ((p->colpart || p->qpart) && tile >= 7) return hipErrorInvalidValue;   // 2-stage gemm_body tiles only
  if (tile == 9) {   // 256x256, 4 waves of 128x128 (bf16 / fp32 epilogues, no C^T, no split-K)
    if (p->M % 256 || p->N % 256 || p->K % st::GBK || p->M <= 0 || p->N <= 0 || p->K <= 0) return hipErrorInvalidValue;
    if (p->lda % 8 || p->ldb % 8 || (epi != st::EPI_F32 && p->ldo % 8) || p->outT || p->splitk > 1)
      return hipErrorInvalidValue;
    if (epi == st::EPI_BF16) return st::launch_gemm_w4<st::EPI_BF16>(*p, stream);
    if (epi == st::EPI_F32) return st::launch_gemm_w4<st::EPI_F32>(*p, stream);
    return hipErrorInvalidValue;
  }
  if (tile == 7 || tile == 8) {   // 256x256 ping-pong (8: with s_setprio); one product per launch,
                                 // bf16 / fp32 epilogues, no C^T, no split-K
    if (p->M % 256 || p->N % 256 || p->K % st::GBK || p->M <= 0 || p->N <= 0 || p->K <= 0) return hipErrorInvalidValue;
    if (p->lda % 8 || p->ldb % 8 || (epi != st::EPI_F32 && p->ldo % 8) || p->outT || p->splitk > 1)
      return hipErrorInvalidValue;
    if (tile == 8) {
      if (epi == st::EPI_BF16) return st::launch_gemm_pp<st::EPI_BF16, 1>(*p, stream);
      if (epi == st::EPI_F32) return st::launch_gemm_pp<st::EPI_F32, 1>(*p, stream);
      return hipErrorInvalidValue;
    }
    if (epi == st::EPI_BF16) return st::launch_gemm_pp<st::EPI_BF16>(*p, stream);
    if (epi == st::EPI_F32) return st::launch_gemm_pp<st::EPI_F32>(*p, stream);
    return hipErrorInvalidValue;
  }
  return st_gemm_nt_batched(p, 1, epi, tile, stream);
}
