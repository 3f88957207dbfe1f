// Kernels of the deep-MLP replay learner (BASELINE config 4: 4x1024 MLP Q-net,
// 1M-transition replay buffer resident in HBM, batch 4096).  The GEMMs are in
// gemm_bf16.hip; these are the gather / env / TD / optimizer pieces around them.
//
// Replay layout (MI355X-first): a transition is NOT stored as two 203-float states
// (1M x 1.6 KB = 1.6 GB of mostly duplicated price windows) but as the indices that
// regenerate them from the HBM-resident price bank: {env, pos, budget, shares,
// action, reward, budget', shares', done} = 36 B -> 36 MB for 1M transitions; states
// are rebuilt by deep_gather directly into the bf16 GEMM operand (Hankel addressing).
#include "common.h"

namespace st {

struct Replay {
  int* env;
  int* pos;
  float* budget;
  int* shares;
  int* action;
  float* reward;
  float* budget2;
  int* shares2;
  int* done;
  unsigned long long* ctrl;   // [0] = write cursor (monotonic), [1] = size (min(cursor, cap))
  int cap;
};

struct DeepGather {
  const float* prices;        // [E, T]
  int T, H, in_p, feat_mode;
  float inv_b0;
  // mode 0: rows = current env states; mode 1: rows = sampled transitions (x and x')
  int mode, B;
  // env mode
  const int* pos;
  const float* budget;
  const int* shares;
  // replay mode
  Replay rp;
  uint32_t key0, key1;
  const unsigned long long* step;   // sampling counter (device, graph-safe)
  // outputs
  bf16_t* X;                  // [B, in_p]
  bf16_t* Xn;                 // [B, in_p] (replay mode)
  float* r_out;               // [B]
  int* a_out;                 // [B]
  float* done_out;            // [B]
  // replay mode: fp32 buffers zeroed on the way (split-K weight-gradient outputs, accumulated with
  // atomics later in the same update) -- replaces two fill launches
  float* zero0;
  int zero0_n;
  float* zero1;
  int zero1_n;
  // replay mode, optional: X transposed [in_p][ldxt] as well (the layer-0 weight gradient's operand),
  // written from LDS 16 rows at a time -- replaces a transpose launch in the update
  bf16_t* XT;
  int ldxt;
};

ST_DEV float dfeat_price(float w, float inv, int mode) { return mode ? (w * inv - 1.0f) : w; }

// One wave per row: lane L owns columns 4L..4L+3 (in_p <= 256).
// One gathered row (one wave, lane L owns columns 4L..4L+3): x (and x' in replay mode) as bf16 to X / Xn,
// the sampled reward / action / done; returns the row's x values in xv.
ST_DEV void gather_row(const DeepGather& g, int row, int lane, float (&xv)[4]) {
  int e, ps, s, s2 = 0;
  float b, b2 = 0.f;
  if (g.mode == 0) {
    e = row;
    ps = g.pos[e];
    b = g.budget[e];
    s = g.shares[e];
  } else {
    // uniform sample over the filled part of the ring (Philox, counter = (row, step))
    const unsigned long long sz = g.rp.ctrl[1];
    const unsigned long long st = g.step[0];
    uint32_t c0 = (uint32_t)row, c1 = (uint32_t)(st & 0xFFFFFFFFull), c2 = (uint32_t)(st >> 32), c3 = 7u;
    philox4x32(c0, c1, c2, c3, g.key0, g.key1);
    const unsigned long long idx = ((((unsigned long long)c0) << 32) | c1) % (sz ? sz : 1ull);
    e = g.rp.env[idx];
    ps = g.rp.pos[idx];
    b = g.rp.budget[idx];
    s = g.rp.shares[idx];
    b2 = g.rp.budget2[idx];
    s2 = g.rp.shares2[idx];
    if (lane == 0) {
      g.r_out[row] = g.rp.reward[idx];
      g.a_out[row] = g.rp.action[idx];
      g.done_out[row] = (float)g.rp.done[idx];
    }
  }
  const float* pr = g.prices + (size_t)e * g.T + ps;
  const int H = g.H;
  const float last = pr[H - 1], vnew = pr[H];
  const float inv = 1.0f / last, invn = 1.0f / vnew;
  float xnv[4];
  // the lane's 4 window prices (and the 4 shifted by one for x') as 16-byte loads from 4-byte-aligned
  // addresses where all 4 are window columns; scalar loads on the boundary lane
  float wv[4], wnv[4];
  if (4 * lane + 3 < H) {
    float4 a4;
    __builtin_memcpy(&a4, pr + 4 * lane, sizeof(a4));
    wv[0] = a4.x; wv[1] = a4.y; wv[2] = a4.z; wv[3] = a4.w;
    if (g.mode == 1) {   // x' window = the same prices shifted by one: one more scalar (pr[4 L + 4] <= pr[H])
      wnv[0] = a4.y; wnv[1] = a4.z; wnv[2] = a4.w; wnv[3] = pr[4 * lane + 4];
    } else {
      wnv[0] = wnv[1] = wnv[2] = wnv[3] = 0.f;
    }
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = 4 * lane + j;
      wv[j] = pr[k < H ? k : H - 1];
      wnv[j] = pr[k < H ? k + 1 : H];
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int k = 4 * lane + j;
    const float w = wv[j];
    const float wn = wnv[j];
    float fb = g.feat_mode ? b * g.inv_b0 : b;
    float fs = g.feat_mode ? (float)s * last * g.inv_b0 : (float)s;
    float fb2 = g.feat_mode ? b2 * g.inv_b0 : b2;
    float fs2 = g.feat_mode ? (float)s2 * vnew * g.inv_b0 : (float)s2;
    xv[j] = k < H ? dfeat_price(w, inv, g.feat_mode) : (k == H ? fb : (k == H + 1 ? fs : 0.f));
    xnv[j] = k < H ? dfeat_price(wn, invn, g.feat_mode) : (k == H ? fb2 : (k == H + 1 ? fs2 : 0.f));
  }
  if (4 * lane < g.in_p) {
    lds_st4(g.X + (size_t)row * g.in_p + 4 * lane, xv[0], xv[1], xv[2], xv[3]);  // 8-byte global store
    if (g.mode == 1) lds_st4(g.Xn + (size_t)row * g.in_p + 4 * lane, xnv[0], xnv[1], xnv[2], xnv[3]);
  }
}

constexpr int GT_ROWS = 16;   // rows per block of the transposed-copy path

__global__ void __launch_bounds__(1024) deep_gather_kernel(DeepGather g) {
  const int lane = threadIdx.x & 63;
  if (g.mode == 1) {
    // 16-byte stores where the span allows (the spans start 16-byte aligned: checked on the host)
    const int gid = blockIdx.x * blockDim.x + threadIdx.x, gs = gridDim.x * blockDim.x;
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int i = gid; i < g.zero0_n / 4; i += gs) reinterpret_cast<float4*>(g.zero0)[i] = z4;
    for (int i = (g.zero0_n & ~3) + gid; i < g.zero0_n; i += gs) g.zero0[i] = 0.f;
    for (int i = gid; i < g.zero1_n / 4; i += gs) reinterpret_cast<float4*>(g.zero1)[i] = z4;
    for (int i = (g.zero1_n & ~3) + gid; i < g.zero1_n; i += gs) g.zero1[i] = 0.f;
  }
  if (!g.XT) {
    const int row = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (row >= g.B) return;
    float xv[4];
    gather_row(g, row, lane, xv);
    return;
  }
  // transposed copy as well: 16 waves per block, wave w gathers row r0 + w (one row per wave, as
  // above) into an LDS tile, then thread c < in_p writes column c of the 16 rows to XT as two 16-byte
  // stores (B % 16 == 0, checked on the host)
  __shared__ __attribute__((aligned(16))) bf16_t t[GT_ROWS][256 + 8];
  const int r0 = blockIdx.x * GT_ROWS, wave = threadIdx.x >> 6;
  {
    float xv[4];
    gather_row(g, r0 + wave, lane, xv);
    if (4 * lane < g.in_p) lds_st4(&t[wave][4 * lane], xv[0], xv[1], xv[2], xv[3]);
  }
  __syncthreads();
  const int c = threadIdx.x;
  if (c < g.in_p) {
    uint32_t u[GT_ROWS / 2];
#pragma unroll
    for (int r = 0; r < GT_ROWS / 2; ++r)
      u[r] = (uint32_t)t[2 * r][c] | ((uint32_t)t[2 * r + 1][c] << 16);
    uint4* o = reinterpret_cast<uint4*>(g.XT + (size_t)c * g.ldxt + r0);
    o[0] = make_uint4(u[0], u[1], u[2], u[3]);
    o[1] = make_uint4(u[4], u[5], u[6], u[7]);
  }
}

struct DeepEnv {
  const float* prices;
  int T, H, E, compat_env, s0, n_actions;
  float b0, eps, inv_ramp;
  float* budget;
  int* shares;
  float* value;
  int* pos;
  int* episodes;
  float* last_final;
  const float* q;             // [E, ldq] fp32 Q(x)
  int ldq;
  uint32_t key0, key1;
  unsigned long long* ctrl;   // [0] = env step counter, [1] = finished blocks of the running env step
  Replay rp;
  float* stats;               // [4]: reward sum, explore count, episodes done, final sum (atomics)
};

// epsilon-greedy + Buy/Sell/Hold transition + replay insert of env e (greedy: argmax of its Q row)
ST_DEV void deep_env_one(const DeepEnv& p, int e, int greedy, unsigned long long step, float& r_, float& x_) {
  const int ps = p.pos[e];
  uint32_t c0 = (uint32_t)e, c1 = (uint32_t)(step & 0xFFFFFFFFull), c2 = (uint32_t)(step >> 32), c3 = 0u;
  philox4x32(c0, c1, c2, c3, p.key0, p.key1);
  const float u1 = u24(c0), u2 = u24(c1);
  const bool exploit = u1 < fminf(p.eps, (float)ps * p.inv_ramp);
  int rnd = (int)(u2 * 3.0f);
  rnd = rnd > 2 ? 2 : rnd;
  const int a = exploit ? greedy : rnd;
  const float* pr = p.prices + (size_t)e * p.T + ps;
  const float vnew = pr[p.H];
  const float b = p.budget[e], vprev = p.value[e];
  const int s = p.shares[e];
  const float bd = p.compat_env ? p.b0 : b;
  const int sd = p.compat_env ? p.s0 : s;
  const bool buy = (a == 0) && (bd >= vnew);
  const bool sell = (a == 1) && (sd > 0);
  const float b2 = buy ? bd - vnew : (sell ? bd + vnew : bd);
  const int s2 = buy ? sd + 1 : (sell ? sd - 1 : sd);
  const float rew = (b2 + (float)s2 * vnew) - (b + (float)s * vprev);
  const int np = ps + 1;
  const bool done = np >= p.T - p.H;
  // replay insert (ring)
  const unsigned long long slot = (p.rp.ctrl[0] + (unsigned long long)e) % (unsigned long long)p.rp.cap;
  p.rp.env[slot] = e;
  p.rp.pos[slot] = ps;
  p.rp.budget[slot] = b;
  p.rp.shares[slot] = s;
  p.rp.action[slot] = a;
  p.rp.reward[slot] = rew;
  p.rp.budget2[slot] = b2;
  p.rp.shares2[slot] = s2;
  p.rp.done[slot] = done ? 1 : 0;
  if (done) {
    const float fin = b2 + (float)s2 * vnew;
    p.last_final[e] = fin;
    p.episodes[e] += 1;
    p.budget[e] = p.b0;
    p.shares[e] = p.s0;
    p.value[e] = 0.f;
    p.pos[e] = 0;
    atomicAdd(p.stats + 2, 1.f);
    atomicAdd(p.stats + 3, fin);
  } else {
    p.budget[e] = b2;
    p.shares[e] = s2;
    p.value[e] = vnew;
    p.pos[e] = np;
  }
  r_ = rew;
  x_ = exploit ? 0.f : 1.f;
}

// the launch's statistics (every thread of every block takes part) and, in its last block, the ring cursor /
// step counter advance (every thread read them before; ctrl[1] counts finished blocks, 0 between launches)
ST_DEV void deep_env_finish(const DeepEnv& p, unsigned long long step, float r_, float x_) {
  // block sums first: one pair of stats atomics per block (per-wave atomics on two addresses serialise)
  __shared__ float red[16][2];
  r_ = wave_sum(r_);
  x_ = wave_sum(x_);
  const int nw = blockDim.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[threadIdx.x >> 6][0] = r_;
    red[threadIdx.x >> 6][1] = x_;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float rs = 0.f, xs = 0.f;
    for (int w = 0; w < nw; ++w) {
      rs += red[w][0];
      xs += red[w][1];
    }
    atomicAdd(p.stats + 0, rs);
    atomicAdd(p.stats + 1, xs);
  }
  if (threadIdx.x == 0) {
    __threadfence();
    unsigned* done_blocks = reinterpret_cast<unsigned*>(p.ctrl + 1);
    if (atomicAdd(done_blocks, 1u) == gridDim.x - 1) {
      const unsigned long long w = p.rp.ctrl[0] + (unsigned long long)p.E;
      p.rp.ctrl[0] = w;
      p.rp.ctrl[1] = w < (unsigned long long)p.rp.cap ? w : (unsigned long long)p.rp.cap;
      p.ctrl[0] = step + 1;
      *done_blocks = 0u;
      __threadfence();
    }
  }
}

// one thread per env: greedy action from the Q rows the output-layer GEMM wrote
__global__ void __launch_bounds__(256) deep_env_step_kernel(DeepEnv p) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  const unsigned long long step = p.ctrl[0];
  float r_ = 0.f, x_ = 0.f;
  if (e < p.E) {
    const float* q = p.q + (size_t)e * p.ldq;
    int greedy = 0;
    float best = q[0];
    for (int a = 1; a < p.n_actions; ++a)
      if (q[a] > best) { best = q[a]; greedy = a; }
    deep_env_one(p, e, greedy, step, r_, x_);
  }
  deep_env_finish(p, step, r_, x_);
}

struct DeepTD {
  const float* q;       // [B, ldq] Q(x) online
  const float* qt;      // [B, ldq] Q(x') target net
  const float* r;
  const int* a;
  const float* done;
  bf16_t* dq;           // [B, ldq] bf16
  bf16_t* dqT;          // [ldq, B]
  float* loss;          // [1] (atomic)
  int B, ldq, n_actions;
  float gamma, coef;
  unsigned long long* t;   // update counter: advanced here (after this update's replay gather read it,
                           // before its Adam reads it as the 1-based step)
};

__global__ void __launch_bounds__(256) deep_td_kernel(DeepTD p) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  float l = 0.f;
  if (b < p.B) {
    const float* qt = p.qt + (size_t)b * p.ldq;
    float mx = qt[0];
    for (int a = 1; a < p.n_actions; ++a) mx = fmaxf(mx, qt[a]);
    const float y = p.r[b] + p.gamma * (1.0f - p.done[b]) * mx;
    const int a = p.a[b];
    const float diff = p.q[(size_t)b * p.ldq + a] - y;
    l = diff * diff;
    // only the n_actions real columns: the padding columns j >= n_actions of dq / dqT are zero from
    // allocation and nothing else writes them
    for (int j = 0; j < p.n_actions; ++j) {
      const float v = (j == a) ? p.coef * diff : 0.f;
      p.dq[(size_t)b * p.ldq + j] = f2bf(v);
      p.dqT[(size_t)j * p.B + b] = f2bf(v);
    }
  }
  l = wave_sum(l);
  if ((threadIdx.x & 63) == 0) atomicAdd(p.loss, l);
  if (p.t && blockIdx.x == 0 && threadIdx.x == 0) p.t[0] += 1ull;
}

// TD + the output layer's backward in one launch (replaces deep_td_kernel, the G_{L-2} = (dq . W_{L-1}) *
// (A > 0) GEMM and the dW_{L-1} = dq^T . A split-K GEMM of the update chain).  dq has ONE nonzero per row
// (coef * diff at the taken action a), so (dq . W)[m][n] = dq[m][a_m] * W[a_m][n]: the product of two bf16
// values, exact in fp32 -- bit-identical to the GEMM's EPI_RELU_GRAD output -- and dW_{L-1}[a][n] is a sum
// over the rows that took a.  Block (column block of 256, row block of 64), 256 threads:
//   threads 0-63: TD of row m0 + t (dq, dqT, loss written by column block 0 only);
//   thread (rg = t / 32, cc = t % 32): rows m0 + 8 rg .. +7, columns n0 + 8 cc .. +7 -- 16-byte loads of A
//   and stores of G, G^T through an LDS transpose (8 rows of a column = one 16-byte LDS store), dW partials
//   reduced over the 8 row groups in LDS, then one fp32 atomic per (action, column) per block (dW prezeroed).
// With ``qp`` set the output layer's forward comes from the batched forward's last hidden-layer launch: its
// epilogue leaves fp32 partial head sums per row and 64-column group (GemmArgs::qpart), summed here in a fixed
// order + bias -- Q(x) and Q_target(x') without an output-layer launch.  Column block 0 writes them to q / qt.
struct DeepHead {
  DeepTD td;
  const bf16_t* A;      // [B, H] last hidden activation (row-major)
  const bf16_t* W;      // [ldq, H] output weights, bf16 copy
  bf16_t* G;            // [B, H]
  bf16_t* GT;           // [H, B]
  float* dW;            // [ldq, H] fp32, zeroed before the launch
  int H;
  float* gpart;         // optional: column sums of G over each 64-row block [B / 64][ldgp] (bias partials)
  int ldgp;
  const float* qp;      // optional: Q(x) partials [nqp][B][4] from the last hidden layer's GEMM epilogue (qpart)
  const float* qpt;     // the same for Q_target(x')
  int nqp;
  const float* bq;      // [>= n_actions] online output bias
  const float* bqt;     // [>= n_actions] target output bias
};
constexpr int HEAD_MAXA = 4;

__global__ void __launch_bounds__(256) deep_head_kernel(DeepHead p) {
  __shared__ float s_g[64];
  __shared__ int s_a[64];
  __shared__ __attribute__((aligned(16))) bf16_t sT[256][72];
  __shared__ float red[8][HEAD_MAXA][256];
  __shared__ float gred[8][256];
  __shared__ float s_q[2][64][HEAD_MAXA];
  const DeepTD& q = p.td;
  // 1-D grid, XCD-aware: workgroup L runs on XCD L % 8, and the nx column blocks of a row block share an XCD
  // (its L2 holds the row block's A rows once for all of them); plain row-major order when ny % 8 != 0
  const int nx = p.H / 256, ny = p.td.B / 64, L = blockIdx.x;
  int bx, by;
  if (ny % 8 == 0) {
    const int xcd = L % 8, slot = L / 8;
    by = xcd * (ny / 8) + slot / nx;
    bx = slot % nx;
  } else {
    by = L / nx;
    bx = L % nx;
  }
  const int tid = threadIdx.x, m0 = by * 64, n0 = bx * 256;
  const int nact = q.n_actions;
  if (p.qp) {
    // Q(x), Q_target(x') of the block's rows from the last hidden layer's epilogue partials (fixed order)
    const int rl = tid >> 2, a = tid & 3;
    float v0 = 0.f, v1 = 0.f;
#pragma unroll 16
    for (int part = 0; part < p.nqp; ++part) {
      v0 += p.qp[((size_t)part * q.B + m0 + rl) * 4 + a];
      v1 += p.qpt[((size_t)part * q.B + m0 + rl) * 4 + a];
    }
    if (a < nact) {
      s_q[0][rl][a] = v0 + p.bq[a];
      s_q[1][rl][a] = v1 + p.bqt[a];
    }
    __syncthreads();
  }
  if (tid < 64) {
    const int b = m0 + tid;
    const bool qf = p.qp != nullptr;
    const float* qt = q.qt + (size_t)b * q.ldq;
    float mx = qf ? s_q[1][tid][0] : qt[0];
    for (int a = 1; a < nact; ++a) mx = fmaxf(mx, qf ? s_q[1][tid][a] : qt[a]);
    const float y = q.r[b] + q.gamma * (1.0f - q.done[b]) * mx;
    const int a = q.a[b];
    const float diff = (qf ? s_q[0][tid][a] : q.q[(size_t)b * q.ldq + a]) - y;
    if (qf && bx == 0)
      for (int j = 0; j < nact; ++j) {
        const_cast<float*>(q.q)[(size_t)b * q.ldq + j] = s_q[0][tid][j];
        const_cast<float*>(q.qt)[(size_t)b * q.ldq + j] = s_q[1][tid][j];
      }
    const bf16_t dqv = f2bf(q.coef * diff);
    s_g[tid] = bf2f(dqv);
    s_a[tid] = a;
    if (bx == 0) {
      for (int j = 0; j < nact; ++j) {
        const bf16_t v = (j == a) ? dqv : (bf16_t)0;
        q.dq[(size_t)b * q.ldq + j] = v;
        q.dqT[(size_t)j * q.B + b] = v;
      }
      const float l = wave_sum(diff * diff);
      if (tid == 0) {
        atomicAdd(q.loss, l);
        if (q.t && by == 0) q.t[0] += 1ull;
      }
    }
  }
  __syncthreads();
  const int rg = tid >> 5, cc = tid & 31, n = n0 + 8 * cc;
  float wv[HEAD_MAXA][8];
#pragma unroll
  for (int a = 0; a < HEAD_MAXA; ++a) {
    if (a < nact) {
      const uint4 w4 = *reinterpret_cast<const uint4*>(p.W + (size_t)a * p.H + n);
      const uint32_t u[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        wv[a][2 * k] = bf2f((bf16_t)(u[k] & 0xFFFF));
        wv[a][2 * k + 1] = bf2f((bf16_t)(u[k] >> 16));
      }
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) wv[a][k] = 0.f;
    }
  }
  float acc[HEAD_MAXA][8];
#pragma unroll
  for (int a = 0; a < HEAD_MAXA; ++a)
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[a][k] = 0.f;
  bf16_t gcol[8][8];   // [column k][row r]
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    const int ml = 8 * rg + r, m = m0 + ml;
    const int am = s_a[ml];
    const float g = s_g[ml];
    const uint4 x4 = *reinterpret_cast<const uint4*>(p.A + (size_t)m * p.H + n);
    const uint32_t u[4] = {x4.x, x4.y, x4.z, x4.w};
    uint32_t o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      bf16_t h[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int c = 2 * k + e;
        const float av = bf2f((bf16_t)(e ? (u[k] >> 16) : (u[k] & 0xFFFF)));
        float w = 0.f;
#pragma unroll
        for (int a = 0; a < HEAD_MAXA; ++a) {
          if (a == am) w = wv[a][c];
          acc[a][c] += (a == am) ? g * av : 0.f;
        }
        h[e] = (av > 0.f) ? f2bf(__fadd_rn(__fmul_rn(g, w), 0.f)) : (bf16_t)0;
        gcol[c][r] = h[e];
      }
      o[k] = (uint32_t)h[0] | ((uint32_t)h[1] << 16);
    }
    *reinterpret_cast<uint4*>(p.G + (size_t)m * p.H + n) = make_uint4(o[0], o[1], o[2], o[3]);
  }
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    uint32_t o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) o[k] = (uint32_t)gcol[c][2 * k] | ((uint32_t)gcol[c][2 * k + 1] << 16);
    *reinterpret_cast<uint4*>(&sT[8 * cc + c][8 * rg]) = make_uint4(o[0], o[1], o[2], o[3]);
  }
#pragma unroll
  for (int a = 0; a < HEAD_MAXA; ++a)
    if (a < nact)
#pragma unroll
      for (int c = 0; c < 8; ++c) red[rg][a][8 * cc + c] = acc[a][c];
  if (p.gpart) {   // G's column sums over the thread's 8 rows (the stored bf16 values)
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      float cs = 0.f;
#pragma unroll
      for (int r = 0; r < 8; ++r) cs += bf2f(gcol[c][r]);
      gred[rg][8 * cc + c] = cs;
    }
  }
  __syncthreads();
  if (p.gpart) {
    float cs = 0.f;
#pragma unroll
    for (int g = 0; g < 8; ++g) cs += gred[g][tid];
    p.gpart[(size_t)by * p.ldgp + n0 + tid] = cs;
  }
#pragma unroll
  for (int i = tid; i < 256 * 8; i += 256) {
    const int nl = i >> 3, ch = i & 7;
    *reinterpret_cast<uint4*>(p.GT + (size_t)(n0 + nl) * q.B + m0 + 8 * ch) = *reinterpret_cast<const uint4*>(&sT[nl][8 * ch]);
  }
  for (int a = 0; a < nact; ++a) {
    float sacc = 0.f;
#pragma unroll
    for (int g = 0; g < 8; ++g) sacc += red[g][a][tid];
    atomicAdd(p.dW + (size_t)a * p.H + n0 + tid, sacc);
  }
}

// Output layer of the act step: Q[r][a] = A[r] . W[a] + bias[a] for the n_actions (<= 4) real rows of W -- a few
// outputs per 2 KB row, so no GEMM tile: 16 lanes per row, each with its 8 (H = 1024) 16-byte units of the row in
// flight at once, packed bf16 pairs into v_dot2c_f32_bf16 against W staged in LDS, a butterfly over the 16 lanes
// (fixed order).  Replaces the 64-wide padded EPI_F32 GEMM launch (13.3 us at 16,384 x 1024).
struct QHead {
  const bf16_t* A;      // [R][lda] bf16
  const bf16_t* W;      // [>= nact][ldw] bf16
  const float* bias;    // [>= nact]
  float* Q;             // [R][ldq] fp32: columns < nact written
  int R, H, lda, ldw, ldq, nact;
};
constexpr int QHEAD_MAXH = 1024;
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

__global__ void __launch_bounds__(256) qhead_kernel(QHead p) {
  __shared__ uint4 sW[HEAD_MAXA][QHEAD_MAXH / 8];
  const int tid = threadIdx.x, l16 = tid & 15, r = blockIdx.x * 16 + (tid >> 4), hc = p.H / 8;
  uint4 xs[QHEAD_MAXH / 128];
  const bf16_t* Ar = p.A + (size_t)r * p.lda;
#pragma unroll
  for (int i = 0; i < QHEAD_MAXH / 128; ++i) {   // issued before the W staging barrier
    const int c = l16 + 16 * i;
    xs[i] = c < hc ? *reinterpret_cast<const uint4*>(Ar + 8 * c) : make_uint4(0u, 0u, 0u, 0u);
  }
  for (int i = tid; i < p.nact * hc; i += 256)
    sW[i / hc][i % hc] = *reinterpret_cast<const uint4*>(p.W + (size_t)(i / hc) * p.ldw + 8 * (i % hc));
  __syncthreads();
  float acc[HEAD_MAXA] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < QHEAD_MAXH / 128; ++i) {
    const int c = l16 + 16 * i;
    if (c >= hc) break;
    const uint32_t u[4] = {xs[i].x, xs[i].y, xs[i].z, xs[i].w};
#pragma unroll
    for (int a = 0; a < HEAD_MAXA; ++a) {
      if (a >= p.nact) break;
      const uint4 w4 = sW[a][c];
      const uint32_t w[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
      for (int k = 0; k < 4; ++k)
        acc[a] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, u[k]), __builtin_bit_cast(bf16x2_t, w[k]),
                                                 acc[a], false);
    }
  }
#pragma unroll
  for (int a = 0; a < HEAD_MAXA; ++a) {
    float v = acc[a];
    v += __shfl_xor(v, 1);
    v += __shfl_xor(v, 2);
    v += __shfl_xor(v, 4);
    v += __shfl_xor(v, 8);
    if (l16 == 0 && a < p.nact) p.Q[(size_t)r * p.ldq + a] = v + p.bias[a];
  }
}

// bias gradient: db[o] = sum_b dZT[o][b]  (one workgroup per output row)
__global__ void __launch_bounds__(256) row_sum_bf16_kernel(const bf16_t* __restrict__ X, int ld, int n, float* out) {
  __shared__ float red[4];
  const int r = blockIdx.x;
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) s += bf2f(X[(size_t)r * ld + i]);
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) out[r] = red[0] + red[1] + red[2] + red[3];
}

// bf16 transpose through LDS: out[c][r] = in[r][c], 64x64 tiles
__global__ void __launch_bounds__(256) transpose_bf16_kernel(const bf16_t* __restrict__ in, int ldi, bf16_t* __restrict__ out,
                                                             int ldo, int R, int Ccols) {
  // 16-byte loads and stores (8 bf16; R, Ccols, ldi, ldo multiples of 8, checked on the host)
  __shared__ __attribute__((aligned(16))) bf16_t t[64][72];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
#pragma unroll
  for (int i = threadIdx.x; i < 64 * 8; i += 256) {
    const int r = i >> 3, c = (i & 7) * 8;
    if (r0 + r < R && c0 + c < Ccols)
      *reinterpret_cast<uint4*>(&t[r][c]) = *reinterpret_cast<const uint4*>(in + (size_t)(r0 + r) * ldi + c0 + c);
  }
  __syncthreads();
#pragma unroll
  for (int i = threadIdx.x; i < 64 * 8; i += 256) {
    const int c = i >> 3, r = (i & 7) * 8;
    if (r0 + r < R && c0 + c < Ccols) {
      uint32_t w[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) w[k] = (uint32_t)t[r + 2 * k][c] | ((uint32_t)t[r + 2 * k + 1][c] << 16);
      *reinterpret_cast<uint4*>(out + (size_t)(c0 + c) * ldo + r0 + r) = make_uint4(w[0], w[1], w[2], w[3]);
    }
  }
}

struct AdamLayer {
  float* w;             // [O, I] fp32 master
  const float* g;       // [O, I] grad
  float* m;
  float* v;
  const float* mask;    // [O, I] trainable mask (null = all trainable)
  bf16_t* wb;           // [O, I] bf16 copy
  bf16_t* wbT;          // [I, O] bf16 transposed copy
  const unsigned long long* t;   // device update counter, already advanced by deep_td (1-based t = *t)
  int O, I;
  float lr, beta1, beta2, eps;
};

// Adam over one weight matrix in 32x32 tiles; writes the bf16 copy and, through LDS,
// the transposed bf16 copy with coalesced stores.
__global__ void __launch_bounds__(256) adam_tile_kernel(AdamLayer p) {
  __shared__ bf16_t t[32][34];
  const int o0 = blockIdx.y * 32, i0 = blockIdx.x * 32;
  const float tt = (float)(*p.t);
  const float c1 = 1.f / (1.f - powf(p.beta1, tt)), c2 = 1.f / (1.f - powf(p.beta2, tt));
  for (int k = threadIdx.x; k < 32 * 32; k += 256) {
    const int oo = k / 32, ii = k % 32;
    const int o = o0 + oo, i = i0 + ii;
    bf16_t wb = 0;
    if (o < p.O && i < p.I) {
      const size_t idx = (size_t)o * p.I + i;
      float w = p.w[idx];
      const float mk = p.mask ? p.mask[idx] : 1.f;
      if (mk != 0.f) {
        const float g = p.g[idx] * mk;
        const float m = p.beta1 * p.m[idx] + (1.f - p.beta1) * g;
        const float v = p.beta2 * p.v[idx] + (1.f - p.beta2) * g * g;
        p.m[idx] = m;
        p.v[idx] = v;
        w -= p.lr * (m * c1) / (sqrtf(v * c2) + p.eps);
        p.w[idx] = w;
      }
      wb = f2bf(w);
      p.wb[idx] = wb;
    }
    t[oo][ii] = wb;
  }
  __syncthreads();
  for (int k = threadIdx.x; k < 32 * 32; k += 256) {
    const int ii = k / 32, oo = k % 32;
    const int o = o0 + oo, i = i0 + ii;
    if (p.wbT && o < p.O && i < p.I) p.wbT[(size_t)i * p.O + o] = t[oo][ii];
  }
}

// ---------------------------------------------------------------- multi-tensor Adam (one launch)
// Every weight matrix and bias of the MLP in one launch: weight segments in 64x64 tiles (the bf16
// copy and, through LDS, its transpose, with 16-byte vector accesses); bias segments in blocks of 32 entries
// whose gradient is reduced here from the transposed layer gradient GT [O][B] (bf16) -- the bias
// gradient row sums need no launch of their own.  The update counter was advanced by deep_td (a
// last-block counter here cost ~40 us: 3.5k device-scope atomics on one word).  Replaces 2L Adam +
// L row-sum + 1 counter launches.
constexpr int ADAM_MAX_SEG = 16;
struct AdamSeg {
  float* w;
  float* g;              // weights: gradient (read); biases: gradient (written here, from gT)
  float* m;
  float* v;
  const float* mask;     // trainable mask (null = all trainable)
  bf16_t* wb;            // weights: bf16 copy [O][I]
  bf16_t* wbT;           // weights: bf16 transposed copy [I][O]
  const bf16_t* gT;      // biases: layer gradient transposed [I][ldg] (bf16); row sums over nb columns --
                         // or null: the bias gradient is already in g (data parallel: summed over ranks)
  int O, I;              // weights: [O][I]; biases: O = 1, I = n
  int ldg, nb;
  int bias;
  int blocks;            // tiles (weights), 4-row blocks (biases from gT) or 32-entry blocks (biases from g / gP)
  const float* gP;       // biases, instead of gT: fp32 partial column sums [np][ldp] (the backward GEMM epilogue's /
                         // the head kernel's), summed over np here -- 1 / 64 of gT's bytes
  int np, ldp;
};
struct AdamMulti {
  AdamSeg seg[ADAM_MAX_SEG];
  int nseg;
  const unsigned long long* t;   // update counter, already advanced by deep_td (1-based t = *t)
  int total;
  float lr, beta1, beta2, eps;
  int grads_only;        // bias segments only: write the reduced gradients to g, no update (data parallel:
                         // the gradients are all-reduced, then a second launch with gT = null updates)
};

__global__ void __launch_bounds__(256) adam_multi_kernel(AdamMulti p) {
  __shared__ __attribute__((aligned(16))) bf16_t tl[64][72];   // 144-byte rows: 16-byte aligned chunks
  int b = blockIdx.x, si = 0;
  while (si + 1 < p.nseg && b >= p.seg[si].blocks) b -= p.seg[si++].blocks;
  const AdamSeg& S = p.seg[si];
  const float tt = (float)(*p.t);
  const float c1 = 1.f / (1.f - powf(p.beta1, tt)), c2 = 1.f / (1.f - powf(p.beta2, tt));
  auto upd = [&](size_t idx, float g) {
    float w = S.w[idx];
    const float mk = S.mask ? S.mask[idx] : 1.f;
    if (mk != 0.f) {
      g *= mk;
      const float m = p.beta1 * S.m[idx] + (1.f - p.beta1) * g;
      const float v = p.beta2 * S.v[idx] + (1.f - p.beta2) * g * g;
      S.m[idx] = m;
      S.v[idx] = v;
      w -= p.lr * (m * c1) / (sqrtf(v * c2) + p.eps);
      S.w[idx] = w;
    }
    if (S.wb) S.wb[idx] = f2bf(w);   // biases: optional bf16 copy (the library act-step epilogue's operand)
    return w;
  };
  if (S.bias && S.gP) {
    // 32 entries per block, 8 threads per entry (a stride-8 share of the np partial rows each), combined by
    // shuffles in a fixed order
    const int i = b * 32 + (threadIdx.x >> 3), part = threadIdx.x & 7;
    float acc = 0.f;
    if (i < S.I)
      for (int r = part; r < S.np; r += 8) acc += S.gP[(size_t)r * S.ldp + i];
    acc += __shfl_xor(acc, 1);
    acc += __shfl_xor(acc, 2);
    acc += __shfl_xor(acc, 4);
    if (part == 0 && i < S.I) {
      S.g[i] = acc;
      if (!p.grads_only) upd((size_t)i, acc);
    }
  } else if (S.bias && !S.gT) {
    if (threadIdx.x < 32) {
      const int i = b * 32 + threadIdx.x;
      if (i < S.I) upd((size_t)i, S.g[i]);
    }
  } else if (S.bias) {
    // 4 entries per block, one row of gT per wave (nb bf16, 16-byte loads, up to 8 in flight per lane): the
    // reduction spreads over ~1,000 short blocks instead of 130 long ones (32 rows each), which left a ~9 us tail
    // behind the weight tiles (tools/bench_adam_bias.py).  Per row the same summation order as before.
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, i = b * 4 + wave;
    float acc = 0.f;
    if (i < S.I) {
      const bf16_t* row = S.gT + (size_t)i * S.ldg;
#pragma unroll 8
      for (int c = 8 * lane; c < S.nb; c += 512) {
        const uint4 q = *reinterpret_cast<const uint4*>(row + c);
        const uint32_t u[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) acc += bf2f((bf16_t)(u[k] & 0xFFFF)) + bf2f((bf16_t)(u[k] >> 16));
      }
    }
    const float g = wave_sum(acc);
    if (lane == 0 && i < S.I) {
      S.g[i] = g;
      if (!p.grads_only) upd((size_t)i, g);
    }
  } else {
    // 64 x 64 tile: thread t owns columns i0 + 4 (t % 16) .. +3 of rows o0 + t / 16 + 16 r (r < 4) --
    // float4 loads / stores of w, g, m, v, mask and an 8-byte store of the bf16 copy; the transposed
    // copy leaves through LDS as 16-byte stores of 8 consecutive o of one i (I % 4 == 0 and O % 8 == 0,
    // checked on the host).  Same per-element arithmetic as upd(); a masked element keeps w, m, v.
    const int tiles_i = (S.I + 63) / 64;
    const int o0 = (b / tiles_i) * 64, i0 = (b % tiles_i) * 64;
    const int ic = 4 * (threadIdx.x & 15), orow = threadIdx.x >> 4, i = i0 + ic;
    // all 4 rows' loads are issued before any store (20 float4 in flight per lane): the stores could
    // alias the later loads as far as the compiler knows, which would otherwise serialize the rows
    float4 W[4], G[4], M[4], V[4], K[4];
    bool ok[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int o = o0 + orow + 16 * r;
      ok[r] = o < S.O && i < S.I;
      const size_t idx = ok[r] ? (size_t)o * S.I + i : 0;
      W[r] = *reinterpret_cast<const float4*>(S.w + idx);
      G[r] = *reinterpret_cast<const float4*>(S.g + idx);
      M[r] = *reinterpret_cast<const float4*>(S.m + idx);
      V[r] = *reinterpret_cast<const float4*>(S.v + idx);
      K[r] = S.mask ? *reinterpret_cast<const float4*>(S.mask + idx) : make_float4(1.f, 1.f, 1.f, 1.f);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int ol = orow + 16 * r, o = o0 + ol;
      uint32_t lo = 0, hi = 0;
      if (ok[r]) {
        const size_t idx = (size_t)o * S.I + i;
        float4 w = W[r];
        const float4 g4 = G[r];
        float4 m = M[r];
        float4 v = V[r];
        const float4 mk = K[r];
        auto one = [&](float& wv, float& mv, float& vv, float g, float k) {
          if (k != 0.f) {
            g *= k;
            const float mn = p.beta1 * mv + (1.f - p.beta1) * g;
            const float vn = p.beta2 * vv + (1.f - p.beta2) * g * g;
            mv = mn;
            vv = vn;
            wv -= p.lr * (mn * c1) / (sqrtf(vn * c2) + p.eps);
          }
        };
        one(w.x, m.x, v.x, g4.x, mk.x);
        one(w.y, m.y, v.y, g4.y, mk.y);
        one(w.z, m.z, v.z, g4.z, mk.z);
        one(w.w, m.w, v.w, g4.w, mk.w);
        *reinterpret_cast<float4*>(S.w + idx) = w;
        *reinterpret_cast<float4*>(S.m + idx) = m;
        *reinterpret_cast<float4*>(S.v + idx) = v;
        lo = (uint32_t)f2bf(w.x) | ((uint32_t)f2bf(w.y) << 16);
        hi = (uint32_t)f2bf(w.z) | ((uint32_t)f2bf(w.w) << 16);
        *reinterpret_cast<uint2*>(S.wb + idx) = make_uint2(lo, hi);
      }
      tl[ic + 0][ol] = (bf16_t)(lo & 0xFFFF);
      tl[ic + 1][ol] = (bf16_t)(lo >> 16);
      tl[ic + 2][ol] = (bf16_t)(hi & 0xFFFF);
      tl[ic + 3][ol] = (bf16_t)(hi >> 16);
    }
    __syncthreads();
    if (S.wbT) {
#pragma unroll
      for (int c = threadIdx.x; c < 64 * 8; c += 256) {
        const int il = c >> 3, oc = (c & 7) * 8, ii = i0 + il, o = o0 + oc;
        if (ii < S.I && o < S.O)
          *reinterpret_cast<uint4*>(S.wbT + (size_t)ii * S.O + o) = *reinterpret_cast<const uint4*>(&tl[il][oc]);
      }
    }
  }
}

}  // namespace st

extern "C" hipError_t st_adam_multi(const st::AdamMulti* p, hipStream_t s) {
  if (p->nseg < 1 || p->nseg > st::ADAM_MAX_SEG) return hipErrorInvalidValue;
  int total = 0;
  for (int i = 0; i < p->nseg; ++i) {
    const st::AdamSeg& g = p->seg[i];
    const int want = g.bias ? ((g.gT && !g.gP) ? (g.I + 3) / 4 : (g.I + 31) / 32) : ((g.I + 63) / 64) * ((g.O + 63) / 64);
    if (g.bias && g.gP && (g.np < 1 || g.ldp < g.I)) return hipErrorInvalidValue;
    if (g.blocks != want || (g.bias && g.gT && (g.nb % 8 || g.ldg % 8))) return hipErrorInvalidValue;
    if (!g.bias && (g.I % 4 || g.O % 8)) return hipErrorInvalidValue;   // vector paths of the weight tiles
    if (p->grads_only && !(g.bias && (g.gT || g.gP))) return hipErrorInvalidValue;
    total += g.blocks;
  }
  if (total != p->total) return hipErrorInvalidValue;
  hipLaunchKernelGGL(st::adam_multi_kernel, dim3(total), dim3(256), 0, s, *p);
  return hipGetLastError();
}

extern "C" hipError_t st_deep_gather(const st::DeepGather* g, hipStream_t s) {
  if ((reinterpret_cast<uintptr_t>(g->zero0) & 15) || (reinterpret_cast<uintptr_t>(g->zero1) & 15)) return hipErrorInvalidValue;
  if (g->in_p > 256 || g->in_p % 4 || g->H + 2 > g->in_p) return hipErrorInvalidValue;
  if (g->XT) {
    if (g->mode != 1 || g->B % st::GT_ROWS || g->ldxt < g->B || g->ldxt % 8 ||
        (reinterpret_cast<uintptr_t>(g->XT) & 15))
      return hipErrorInvalidValue;
    hipLaunchKernelGGL(st::deep_gather_kernel, dim3(g->B / st::GT_ROWS), dim3(64 * st::GT_ROWS), 0, s, *g);
    return hipGetLastError();
  }
  const int waves = g->B, per = 4;
  hipLaunchKernelGGL(st::deep_gather_kernel, dim3((waves + per - 1) / per), dim3(256), 0, s, *g);
  return hipGetLastError();
}

extern "C" hipError_t st_deep_env_step(const st::DeepEnv* p, hipStream_t s) {
  hipLaunchKernelGGL(st::deep_env_step_kernel, dim3((p->E + 255) / 256), dim3(256), 0, s, *p);   // (advances too)
  return hipGetLastError();
}

// struct sizes of this file's launch ABI, for the host mirrors' check (tests/test_abi.py; no HIP call)
extern "C" int st_deep_abi(int* out, int n) {
  const int sz[] = {(int)sizeof(st::Replay), (int)sizeof(st::DeepGather), (int)sizeof(st::DeepEnv), (int)sizeof(st::DeepTD),
                    (int)sizeof(st::DeepHead), (int)sizeof(st::QHead), (int)sizeof(st::AdamLayer),
                    (int)sizeof(st::AdamSeg), (int)sizeof(st::AdamMulti)};
  const int m = (int)(sizeof(sz) / sizeof(sz[0]));
  for (int i = 0; i < n && i < m; ++i) out[i] = sz[i];
  return m;
}

extern "C" hipError_t st_qhead(const st::QHead* p, hipStream_t s) {
  if (p->R % 16 || p->R <= 0 || p->H % 8 || p->H <= 0 || p->H > st::QHEAD_MAXH || p->nact < 1 || p->nact > st::HEAD_MAXA ||
      p->lda % 8 || p->ldw % 8 || p->ldw < p->H || p->lda < p->H || p->ldq < p->nact || !p->A || !p->W || !p->bias || !p->Q)
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(st::qhead_kernel, dim3(p->R / 16), dim3(256), 0, s, *p);
  return hipGetLastError();
}

extern "C" hipError_t st_deep_td(const st::DeepTD* p, hipStream_t s) {
  hipLaunchKernelGGL(st::deep_td_kernel, dim3((p->B + 63) / 64), dim3(64), 0, s, *p);
  return hipGetLastError();
}

extern "C" hipError_t st_deep_head(const st::DeepHead* p, hipStream_t s) {
  const st::DeepTD& q = p->td;
  if (q.n_actions < 1 || q.n_actions > st::HEAD_MAXA || q.n_actions > q.ldq || q.B % 64 || p->H % 256 || q.B <= 0 ||
      (p->gpart && p->ldgp < p->H))
    return hipErrorInvalidValue;
  if (p->qp && (!p->qpt || p->nqp < 1 || !p->bq || !p->bqt)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(st::deep_head_kernel, dim3((p->H / 256) * (q.B / 64)), dim3(256), 0, s, *p);
  return hipGetLastError();
}

extern "C" hipError_t st_row_sum_bf16(const bf16_t* X, int ld, int rows, int n, float* out, hipStream_t s) {
  hipLaunchKernelGGL(st::row_sum_bf16_kernel, dim3(rows), dim3(256), 0, s, X, ld, n, out);
  return hipGetLastError();
}

extern "C" hipError_t st_transpose_bf16(const bf16_t* in, int ldi, bf16_t* out, int ldo, int R, int Cc, hipStream_t s) {
  if (R % 8 || Cc % 8 || ldi % 8 || ldo % 8) return hipErrorInvalidValue;
  hipLaunchKernelGGL(st::transpose_bf16_kernel, dim3((Cc + 63) / 64, (R + 63) / 64), dim3(256), 0, s, in, ldi, out, ldo,
                     R, Cc);
  return hipGetLastError();
}

__global__ void st_counter_inc_kernel(unsigned long long* c) { c[0] += 1; }

extern "C" hipError_t st_counter_inc(unsigned long long* c, hipStream_t s) {
  hipLaunchKernelGGL(st_counter_inc_kernel, dim3(1), dim3(1), 0, s, c);
  return hipGetLastError();
}

extern "C" hipError_t st_adam_tile(const st::AdamLayer* p, hipStream_t s) {
  hipLaunchKernelGGL(st::adam_tile_kernel, dim3((p->I + 31) / 32, (p->O + 31) / 32), dim3(256), 0, s, *p);
  return hipGetLastError();
}
