// One recurrent step of a (Zoneout)LSTM, forward and backward.
//
// Replaces, per decoder / encoder time step, TF LSTMCell + the ext tacotron2 ZoneoutLSTMCell
// (used at modules/module.py:93-108 in ZoneoutCBHG, :1522-1540 in DualSourceTransformerDecoder).
// The input projection x @ W_x + b of every step is hoisted out of the recurrence into one big
// MFMA GEMM over all steps (sat_gemm); the step kernel only does the recurrent product
// rin @ W_r, the gate nonlinearities and zoneout.
//
// Weight layout (MI355X-first): gate-interleaved [K][U][4] (i, j, f, o of one unit adjacent), so
// a workgroup owning a tile of units reads contiguous rows and one float4 per (k, unit).
//
// Tiling: a 256-thread workgroup owns UT=4 units x BT=8 batch rows; the reduction K is split
// over 8 lanes of a wave (k-slices) and combined with 3 xor-shuffles -- no LDS, no barrier.
// For U=256, B=32: 64 x 4 = 256 workgroups, one per CU.
#include "sat_common.h"

#include <algorithm>

namespace sat {
namespace {

constexpr int UT = 4, BT = 8, KS = 8;

struct LstmFwdP {
  int B, U, K;
  const float* xproj; int64_t xproj_sb;
  const float* bias;
  const float* rin; int64_t rin_sb;
  const float* W;
  const float* c_prev;
  const float* h_prev; int64_t h_prev_sb;
  const float* mask_c; const float* mask_h;
  float zc, zh;
  const int64_t* lengths; int t;
  float* h_raw; int64_t h_raw_sb;
  float* c_out;
  float* h_out; int64_t h_out_sb;
  float* gates;
  const float* rin1; int64_t rin1_sb;   // optional input segments: row = [rin | rin1 | rin2]
  const float* rin2; int64_t rin2_sb;
  int K1, K2;
};

// Forward step.  Every global load is issued up front: the workgroup's weight slice
// W[:, u0:u0+4, :] (K x 16 floats) and its 8 input rows go global -> LDS in one burst of
// 16-byte loads, the pointwise operands (xproj, c, h, masks) are prefetched into registers,
// then the K-split dot products run out of LDS.
// UT_ units x BT_ = 256 / KS_ / UT_ batch rows per workgroup, K split over KS_ lanes.  The
// training fallback uses <4, 8> (U = 256, B = 32: 256 workgroups); the free-running decode at
// batch <= 8 uses <1, 32>: one unit per workgroup, so U = 256 still gives 256 workgroups and
// each streams K x 4 weights instead of K x 16 (inference.py's per-step launches).
template <int UT_, int KS_>
__device__ __forceinline__ void lstm_fwd_block(const LstmFwdP& p, int bx, int by, float* smem) {
  constexpr int BT_ = 256 / KS_ / UT_;
  const int K = p.K;
  float4* Ws = reinterpret_cast<float4*>(smem);          // [K][UT_]
  float* xs = smem + (size_t)K * UT_ * 4;                 // [BT_][K + 4]
  const int xld = K + 4;
  const int tid = threadIdx.x;
  const int ks = tid & (KS_ - 1), pair = tid / KS_;
  const int u0 = bx * UT_, b0 = by * BT_;
  const int u = u0 + (pair % UT_);
  const int bl = pair / UT_;
  const int b = b0 + bl;
  const bool active = (u < p.U) && (b < p.B);
  // prefetch the pointwise operands of this (b, u)
  const int64_t bu = (int64_t)b * p.U + u;
  float4 xp = make_float4(0.f, 0.f, 0.f, 0.f);
  float cp = 0.f, hp = 0.f, mc = 0.f, mh = 0.f;
  bool valid = true;
  if (active && ks == 0) {
    if (p.xproj) xp = reinterpret_cast<const float4*>(p.xproj + (int64_t)b * p.xproj_sb)[u];
    else if (p.bias) xp = reinterpret_cast<const float4*>(p.bias)[u];
    cp = p.c_prev ? p.c_prev[bu] : 0.f;
    hp = p.h_prev ? p.h_prev[(int64_t)b * p.h_prev_sb + u] : 0.f;
    if (p.mask_c) { mc = p.mask_c[bu]; mh = p.mask_h[bu]; }
    valid = p.lengths ? (p.t < p.lengths[b]) : true;
  }
  // weights: K rows x UT float4 (rows are UT*16 contiguous bytes at stride U*16)
  const float4* W4 = reinterpret_cast<const float4*>(p.W);
  const int nu = min(UT_, p.U - u0);
  for (int i = tid; i < K * UT_; i += 256) {
    const int k = i / UT_, j = i - k * UT_;
    Ws[i] = j < nu ? W4[(int64_t)k * p.U + u0 + j] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  const int kq = K >> 2, k0q = (K - p.K1 - p.K2) >> 2, k1q = k0q + (p.K1 >> 2);
  for (int i = tid; i < BT_ * kq; i += 256) {
    const int r = i / kq, c = i - r * kq;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (b0 + r < p.B) {
      const int64_t br = b0 + r;
      v = c < k0q ? reinterpret_cast<const float4*>(p.rin + br * p.rin_sb)[c]
        : c < k1q ? reinterpret_cast<const float4*>(p.rin1 + br * p.rin1_sb)[c - k0q]
                  : reinterpret_cast<const float4*>(p.rin2 + br * p.rin2_sb)[c - k1q];
    }
    *reinterpret_cast<float4*>(xs + r * xld + 4 * c) = v;
  }
  __syncthreads();
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  const float* xr = xs + bl * xld;
  const int ul = pair % UT_;
#pragma unroll 4
  for (int k = ks; k < K; k += KS_) {
    const float xv = xr[k];
    const float4 w = Ws[k * UT_ + ul];
    acc[0] = fmaf(xv, w.x, acc[0]);
    acc[1] = fmaf(xv, w.y, acc[1]);
    acc[2] = fmaf(xv, w.z, acc[2]);
    acc[3] = fmaf(xv, w.w, acc[3]);
  }
#pragma unroll
  for (int o = 1; o < KS_; o <<= 1)
#pragma unroll
    for (int g = 0; g < 4; ++g) acc[g] += __shfl_xor(acc[g], o, 64);
  if (!active || ks != 0) return;
  if (!valid) {  // bidirectional_dynamic_rnn(sequence_length): state copied, output 0
    p.c_out[bu] = cp;
    p.h_out[(int64_t)b * p.h_out_sb + u] = hp;
    if (p.h_raw) p.h_raw[(int64_t)b * p.h_raw_sb + u] = 0.f;
    if (p.gates) reinterpret_cast<float4*>(p.gates)[bu] = make_float4(0.f, 0.f, 0.f, 0.f);
    return;
  }
  // activations formed as in every LSTM kernel (sat_common.h sigmoid_fast / tanh_lstm)
  const float gi = sigmoid_fast(acc[0] + xp.x);
  const float gj = tanh_lstm(acc[1] + xp.y);
  const float gf = sigmoid_fast(acc[2] + xp.z + 1.0f);   // forget_bias = 1.0
  const float go = sigmoid_fast(acc[3] + xp.w);
  const float cn = gf * cp + gi * gj;
  const float hn = go * tanh_lstm(cn);
  float c2, h2;
  if (p.mask_c) {
    c2 = mc * cn + (1.f - mc) * cp;
    h2 = mh * hn + (1.f - mh) * hp;
  } else {
    c2 = (1.f - p.zc) * cn + p.zc * cp;
    h2 = (1.f - p.zh) * hn + p.zh * hp;
  }
  p.c_out[bu] = c2;
  p.h_out[(int64_t)b * p.h_out_sb + u] = h2;
  if (p.h_raw) p.h_raw[(int64_t)b * p.h_raw_sb + u] = hn;
  if (p.gates) reinterpret_cast<float4*>(p.gates)[bu] = make_float4(gi, gj, gf, go);
}

// Up to kMaxProblems independent steps (e.g. the attention RNN at t, decoder LSTM1 at t - C,
// LSTM2 at t - 2C) in ONE launch: disjoint workgroup ranges, dynamic LDS = the largest need.
constexpr int kMaxProblems = 4;

struct LstmFwdMulti {
  LstmFwdP p[kMaxProblems];
  int first[kMaxProblems + 1];   // first workgroup of each problem (prefix sums)
  int gx[kMaxProblems];          // unit tiles per problem
  int n;
};

__global__ void __launch_bounds__(256) lstm_fwd_kernel(LstmFwdMulti m) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  int i = 0;
#pragma unroll
  for (int j = 1; j < kMaxProblems; ++j)
    if (j < m.n && (int)blockIdx.x >= m.first[j]) i = j;
  const int local = blockIdx.x - m.first[i];
  const int by = local / m.gx[i], bx = local - by * m.gx[i];
  lstm_fwd_block<UT, KS>(m.p[i], bx, by, smem);
}

// One step at batch <= 8 (the free-running decoder, inference.py): one unit per workgroup,
// thread = (batch row b < 8, k-slice ks < 32); every thread loads its k-slice of the input row
// and the unit's 4 gate weights straight into registers -- all loads in flight at once, no LDS
// staging, no barrier -- then 5 xor-shuffles sum the slices.  Same cell as lstm_fwd_block.
__global__ void __launch_bounds__(256) lstm_fwd_small_kernel(LstmFwdP p) {
  constexpr int KS_ = 32, KMAX = 1024 / KS_;   // K <= 1024
  const int tid = threadIdx.x, ks = tid & (KS_ - 1), b = tid / KS_;
  const int u = blockIdx.x, K = p.K;
  const bool active = b < p.B;
  const int k0 = K - p.K1 - p.K2, k1 = k0 + p.K1;
  const int64_t br = active ? b : 0;
  const float4* W4 = reinterpret_cast<const float4*>(p.W);
  float xv[KMAX];
  float4 wv[KMAX];
#pragma unroll
  for (int i = 0; i < KMAX; ++i) {
    const int k = ks + KS_ * i;
    xv[i] = 0.f;
    wv[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (k < K) {
      wv[i] = W4[(int64_t)k * p.U + u];
      if (active)
        xv[i] = k < k0 ? p.rin[br * p.rin_sb + k]
              : k < k1 ? p.rin1[br * p.rin1_sb + (k - k0)] : p.rin2[br * p.rin2_sb + (k - k1)];
    }
  }
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < KMAX; ++i) {
    acc[0] = fmaf(xv[i], wv[i].x, acc[0]);
    acc[1] = fmaf(xv[i], wv[i].y, acc[1]);
    acc[2] = fmaf(xv[i], wv[i].z, acc[2]);
    acc[3] = fmaf(xv[i], wv[i].w, acc[3]);
  }
#pragma unroll
  for (int o = 1; o < KS_; o <<= 1)
#pragma unroll
    for (int g = 0; g < 4; ++g) acc[g] += __shfl_xor(acc[g], o, 64);
  if (!active || ks != 0) return;
  const int64_t bu = (int64_t)b * p.U + u;
  const float4 xp = p.xproj ? reinterpret_cast<const float4*>(p.xproj + (int64_t)b * p.xproj_sb)[u]
                  : p.bias ? reinterpret_cast<const float4*>(p.bias)[u] : make_float4(0.f, 0.f, 0.f, 0.f);
  const float cp = p.c_prev ? p.c_prev[bu] : 0.f;
  const float hp = p.h_prev ? p.h_prev[(int64_t)b * p.h_prev_sb + u] : 0.f;
  const float gi = sigmoid_fast(acc[0] + xp.x);
  const float gj = tanh_lstm(acc[1] + xp.y);
  const float gf = sigmoid_fast(acc[2] + xp.z + 1.0f);   // forget_bias = 1.0
  const float go = sigmoid_fast(acc[3] + xp.w);
  const float cn = gf * cp + gi * gj;
  const float hn = go * tanh_lstm(cn);
  float c2, h2;
  if (p.mask_c) {
    const float mc = p.mask_c[bu], mh = p.mask_h[bu];
    c2 = mc * cn + (1.f - mc) * cp;
    h2 = mh * hn + (1.f - mh) * hp;
  } else {
    c2 = (1.f - p.zc) * cn + p.zc * cp;
    h2 = (1.f - p.zh) * hn + p.zh * hp;
  }
  p.c_out[bu] = c2;
  p.h_out[(int64_t)b * p.h_out_sb + u] = h2;
  if (p.h_raw) p.h_raw[(int64_t)b * p.h_raw_sb + u] = hn;
  if (p.gates) reinterpret_cast<float4*>(p.gates)[bu] = make_float4(gi, gj, gf, go);
}

struct LstmBwdP {
  int B, U, K, hoff;
  const float* W;                       // [K][U][4]
  const float* dgates_next;             // [B][U][4] at t+1 (null at the last step)
  const float* gates;                   // [B][U][4] at t (activated)
  const float* c_prev;                  // c_{t-1} [B][U] (null = zeros)
  const float* dy; int64_t dy_sb;       // dL/dh'_t (raw output), nullable
  const float* dq0; const float* wq0; int dq0_n;   // optional extra dy += dq0[b] . wq0[u]
  const float* dq1; const float* wq1; int dq1_n;
  int dq_parts; int64_t dq_pstride, dq_bstride;     // dq0/dq1 rows are sums of dq_parts partials
  const float* dh_carry;                // [B][U] (1-m_h(t+1)) dh_{t+1}, or full dh_t if t+1 invalid
  const float* dc_carry;                // [B][U] dL/dc_t
  const float* mask_c; const float* mask_h;
  float zc, zh;
  const int64_t* lengths; int t;
  float* dgates;                        // [B][U][4]
  float* dh_carry_out;                  // [B][U]
  float* dc_carry_out;                  // [B][U]
  const float* rec; int64_t rec_sb;     // precomputed recurrent product [B][U] (nullable)
};

// dL/dh_t = dh_carry + sum_g dgates_{t+1}[b, g] * W[hoff + u, g]  (the recurrent product)
// plus, for the attention RNN, the query-gradient term sum_d dq[b, d] wq[u, d] where dq is the
// sum of `dq_parts` per-tile partials.  Both are ONE dot product of length 4U + DQ:
//   row b:  [dgates_{t+1}[b] (4U) | dq[b] (DQ)]         (partials summed while staging)
//   row u:  [W[hoff + u] (4U) | wq0[u] (D0) | wq1[u] (D1)]
// staged global -> LDS in one burst of 16-byte loads (all independent), then 8 k-slices per
// (b, u) and 3 xor-shuffles.
constexpr int kMaxDq = 320;

__device__ __forceinline__ void lstm_bwd_block(const LstmBwdP& p, int bx, int by, float* smem) {
  // with a precomputed recurrent product (p.rec) only the query term is a dot here
  const int G = p.rec ? 0 : 4 * p.U;
  const int D0 = p.dq0 ? p.dq0_n : 0, D1 = p.dq1 ? p.dq1_n : 0, DQ = D0 + D1;
  const int L = G + DQ;                                // dot length
  const int ld = L + 4;
  float* dgs = smem;                                   // [BT][ld]
  float* wrs = dgs + (size_t)BT * ld;                  // [UT][ld]
  const int tid = threadIdx.x;
  const int ks = tid & (KS - 1), pair = tid >> 3;
  const int u0 = bx * UT, b0 = by * BT;
  const int ul = pair & (UT - 1), bl = pair >> 2;
  const int u = u0 + ul, b = b0 + bl;
  const bool active = (u < p.U) && (b < p.B);
  const int64_t bu = (int64_t)b * p.U + u;
  // prefetch the pointwise operands
  float4 g4 = make_float4(0.f, 0.f, 0.f, 0.f);
  float cp = 0.f, dyv = 0.f, dhc = 0.f, dcc = 0.f, mc = 0.f, mh = 0.f;
  bool valid = true;
  if (active && ks == 0) {
    g4 = reinterpret_cast<const float4*>(p.gates)[bu];
    cp = p.c_prev ? p.c_prev[bu] : 0.f;
    dyv = p.dy ? p.dy[(int64_t)b * p.dy_sb + u] : 0.f;
    dhc = p.dh_carry ? p.dh_carry[bu] : 0.f;
    dcc = p.dc_carry ? p.dc_carry[bu] : 0.f;
    if (p.rec) dhc += p.rec[(int64_t)b * p.rec_sb + u];
    if (p.mask_c) { mc = p.mask_c[bu]; mh = p.mask_h[bu]; }
    valid = p.lengths ? (p.t < p.lengths[b]) : true;
  }
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  const int gq = G >> 2, lq = L >> 2, q0 = D0 >> 2;
  // batch rows: dgates_{t+1} then the summed query gradient
  for (int i = tid; i < BT * lq; i += 256) {
    const int r = i / lq, c = i - r * lq;
    const int bb = b0 + r;
    float4 v = z4;
    if (bb < p.B) {
      if (c < gq) {
        if (p.dgates_next) v = reinterpret_cast<const float4*>(p.dgates_next + (int64_t)bb * 4 * p.U)[c];
      } else {
        const int dc = c - gq;
        const float* src = dc < q0 ? p.dq0 + 4 * dc : p.dq1 + 4 * (dc - q0);
        src += (int64_t)bb * p.dq_bstride;
        for (int part = 0; part < p.dq_parts; ++part) {
          const float4 w = *reinterpret_cast<const float4*>(src + (int64_t)part * p.dq_pstride);
          v.x += w.x; v.y += w.y; v.z += w.z; v.w += w.w;
        }
      }
    }
    *reinterpret_cast<float4*>(dgs + r * ld + 4 * c) = v;
  }
  // unit rows: recurrent weights then the query-layer weights of this unit
  for (int i = tid; i < UT * lq; i += 256) {
    const int r = i / lq, c = i - r * lq;
    const int uu = u0 + r;
    float4 v = z4;
    if (uu < p.U) {
      if (c < gq) v = reinterpret_cast<const float4*>(p.W + (int64_t)(p.hoff + uu) * 4 * p.U)[c];
      else if (c - gq < q0) v = reinterpret_cast<const float4*>(p.wq0 + (int64_t)uu * D0)[c - gq];
      else v = reinterpret_cast<const float4*>(p.wq1 + (int64_t)uu * D1)[c - gq - q0];
    }
    *reinterpret_cast<float4*>(wrs + r * ld + 4 * c) = v;
  }
  __syncthreads();
  // the recurrent term belongs to dL/dh_t (the zoneout-blended state), the query term to
  // dL/dh'_t (it enters through the raw output h'): two accumulators, G % 32 == 0 so every
  // 32-float stride of the k-slices lies on one side of the split
  float rec = 0.f, qterm = 0.f;
  if (active) {
    const float* dg = dgs + bl * ld;
    const float* wr = wrs + ul * ld;
    if (p.dgates_next && G > 0) {
#pragma unroll 4
      for (int v = 4 * ks; v < G; v += 4 * KS) {
        const float4 g = *reinterpret_cast<const float4*>(dg + v);
        const float4 w = *reinterpret_cast<const float4*>(wr + v);
        rec += g.x * w.x + g.y * w.y + g.z * w.z + g.w * w.w;
      }
    }
    for (int v = G + 4 * ks; v < L; v += 4 * KS) {
      const float4 g = *reinterpret_cast<const float4*>(dg + v);
      const float4 w = *reinterpret_cast<const float4*>(wr + v);
      qterm += g.x * w.x + g.y * w.y + g.z * w.z + g.w * w.w;
    }
  }
#pragma unroll
  for (int o = 1; o < KS; o <<= 1) {
    rec += __shfl_xor(rec, o, 64);
    qterm += __shfl_xor(qterm, o, 64);
  }
  if (!active || ks != 0) return;
  const float dh_t = rec + dhc;
  const float dc_t = dcc;
  if (!valid) {
    reinterpret_cast<float4*>(p.dgates)[bu] = make_float4(0.f, 0.f, 0.f, 0.f);
    p.dh_carry_out[bu] = dh_t;
    p.dc_carry_out[bu] = dc_t;
    return;
  }
  const float gi = g4.x, gj = g4.y, gf = g4.z, go = g4.w;
  const float cn = gf * cp + gi * gj;
  const float tc = tanh_lstm(cn);
  if (!p.mask_c) { mc = 1.f - p.zc; mh = 1.f - p.zh; }
  const float dy = dyv + qterm;
  const float dhn = dy + mh * dh_t;                 // dL/dh'
  const float dcn = mc * dc_t + dhn * go * (1.f - tc * tc);
  const float d_o = dhn * tc * go * (1.f - go);
  const float d_f = dcn * cp * gf * (1.f - gf);
  const float d_i = dcn * gj * gi * (1.f - gi);
  const float d_j = dcn * gi * (1.f - gj * gj);
  reinterpret_cast<float4*>(p.dgates)[bu] = make_float4(d_i, d_j, d_f, d_o);
  p.dc_carry_out[bu] = dcn * gf + (1.f - mc) * dc_t;
  p.dh_carry_out[bu] = (1.f - mh) * dh_t;
}

struct LstmBwdMulti {
  LstmBwdP p[kMaxProblems];
  int first[kMaxProblems + 1];
  int gx[kMaxProblems];
  int n;
};

__global__ void __launch_bounds__(256) lstm_bwd_kernel(LstmBwdMulti m) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  int i = 0;
#pragma unroll
  for (int j = 1; j < kMaxProblems; ++j)
    if (j < m.n && (int)blockIdx.x >= m.first[j]) i = j;
  const int local = blockIdx.x - m.first[i];
  const int by = local / m.gx[i], bx = local - by * m.gx[i];
  lstm_bwd_block(m.p[i], bx, by, smem);
}

}  // namespace
}  // namespace sat

using namespace sat;


static int check_fwd(const SatLstmFwd* a, LstmFwdP& p, size_t& shm) {
  SAT_CHECK_ARG(a && a->B > 0 && a->U > 0 && a->K >= 0, "sat_lstm_step_fwd: bad sizes");
  SAT_CHECK_ARG(a->K % 4 == 0 && a->rin_sb % 4 == 0, "sat_lstm_step_fwd: K and rin stride must be multiples of 4");
  SAT_CHECK_ARG((a->K == 0 || a->rin) && a->W && a->c_out && a->h_out, "sat_lstm_step_fwd: null pointer");
  SAT_CHECK_ARG((a->mask_c == nullptr) == (a->mask_h == nullptr), "sat_lstm_step_fwd: masks come in pairs");
  SAT_CHECK_ARG(a->K1 >= 0 && a->K2 >= 0 && a->K1 % 4 == 0 && a->K2 % 4 == 0 &&
                a->K1 + a->K2 <= a->K && (a->K1 == 0 || (a->rin1 && a->rin1_sb % 4 == 0 && aligned16(a->rin1))) &&
                (a->K2 == 0 || (a->rin2 && a->rin2_sb % 4 == 0 && aligned16(a->rin2))),
                "sat_lstm_step_fwd: input segments need K1, K2, strides % 4 and 16-byte alignment");
  p.B = a->B; p.U = a->U; p.K = a->K;
  p.xproj = a->xproj; p.xproj_sb = a->xproj_sb; p.bias = a->bias;
  p.rin = a->rin; p.rin_sb = a->rin_sb; p.W = a->W;
  p.c_prev = a->c_prev; p.h_prev = a->h_prev; p.h_prev_sb = a->h_prev_sb;
  p.mask_c = a->mask_c; p.mask_h = a->mask_h; p.zc = a->zc; p.zh = a->zh;
  p.lengths = a->lengths; p.t = a->t;
  p.h_raw = a->h_raw; p.h_raw_sb = a->h_raw_sb;
  p.c_out = a->c_out; p.h_out = a->h_out; p.h_out_sb = a->h_out_sb; p.gates = a->gates;
  p.rin1 = a->rin1; p.rin1_sb = a->rin1_sb; p.rin2 = a->rin2; p.rin2_sb = a->rin2_sb;
  p.K1 = a->K1; p.K2 = a->K2;
  shm = ((size_t)a->K * UT * 4 + (size_t)BT * (a->K + 4)) * sizeof(float);
  SAT_CHECK_ARG(shm <= 160 * 1024, "sat_lstm_step_fwd: K too large for the LDS-staged step");
  return SAT_OK;
}

extern "C" int sat_lstm_steps_fwd(const SatLstmFwd* steps, int32_t n, void* stream) {
  SAT_CHECK_ARG(steps && n >= 1 && n <= kMaxProblems, "sat_lstm_steps_fwd: 1..4 steps");
  LstmFwdMulti m;
  m.n = n;
  m.first[0] = 0;
  size_t shm = 0;
  for (int i = 0; i < n; ++i) {
    size_t s_i = 0;
    const int rc = check_fwd(steps + i, m.p[i], s_i);
    if (rc != SAT_OK) return rc;
    shm = std::max(shm, s_i);
    m.gx[i] = ceil_div(steps[i].U, UT);
    m.first[i + 1] = m.first[i] + m.gx[i] * ceil_div(steps[i].B, BT);
  }
  for (int i = n; i < kMaxProblems; ++i) { m.gx[i] = 1; m.first[i + 1] = m.first[n]; }
  hipLaunchKernelGGL(lstm_fwd_kernel, dim3(m.first[n]), dim3(256), shm, as_stream(stream), m);
  SAT_LAUNCH_CHECK("sat_lstm_steps_fwd");
  return SAT_OK;
}

extern "C" int sat_lstm_step_fwd(const SatLstmFwd* a, void* stream) {
  if (a && a->B > 0 && a->B <= 8 && a->U >= 64 && a->K <= 1024 && !a->lengths) {
    LstmFwdP p;
    size_t shm = 0;
    const int rc = check_fwd(a, p, shm);
    if (rc != SAT_OK) return rc;
    hipLaunchKernelGGL(lstm_fwd_small_kernel, dim3(a->U), dim3(256), 0, as_stream(stream), p);
    SAT_LAUNCH_CHECK("sat_lstm_step_fwd");
    return SAT_OK;
  }
  return sat_lstm_steps_fwd(a, 1, stream);
}

static int check_bwd(const SatLstmBwd* a, LstmBwdP& p, size_t& shm) {
  SAT_CHECK_ARG(a && a->B > 0 && a->U > 0, "sat_lstm_step_bwd: bad sizes");
  SAT_CHECK_ARG(a->W && a->gates && a->dgates && a->dh_carry_out && a->dc_carry_out,
                "sat_lstm_step_bwd: null pointer");
  SAT_CHECK_ARG(a->hoff >= 0 && a->hoff + a->U <= a->K, "sat_lstm_step_bwd: hoff out of range");
  SAT_CHECK_ARG((a->dq0 ? a->dq0_n : 0) + (a->dq1 ? a->dq1_n : 0) <= kMaxDq,
                "sat_lstm_step_bwd: query width > 320");
  SAT_CHECK_ARG((!a->dq0 || (a->wq0 && a->dq0_n % 4 == 0 && aligned16(a->dq0) && aligned16(a->wq0))) &&
                (!a->dq1 || (a->wq1 && a->dq1_n % 4 == 0 && aligned16(a->dq1) && aligned16(a->wq1))) &&
                a->dq_pstride % 4 == 0 && a->dq_bstride % 4 == 0 && aligned16(a->W) &&
                aligned16(a->dgates_next),
                "sat_lstm_step_bwd: query-gradient operands must be 16-byte aligned, widths % 4");
  p.B = a->B; p.U = a->U; p.K = a->K; p.hoff = a->hoff;
  p.W = a->W; p.dgates_next = a->dgates_next; p.gates = a->gates; p.c_prev = a->c_prev;
  p.dy = a->dy; p.dy_sb = a->dy_sb;
  p.dq0 = a->dq0; p.wq0 = a->wq0; p.dq0_n = a->dq0_n;
  p.dq1 = a->dq1; p.wq1 = a->wq1; p.dq1_n = a->dq1_n;
  p.dq_parts = a->dq_parts > 0 ? a->dq_parts : 1;
  p.dq_pstride = a->dq_pstride;
  p.dq_bstride = a->dq_bstride > 0 ? a->dq_bstride : a->dq0_n;
  p.dh_carry = a->dh_carry; p.dc_carry = a->dc_carry;
  p.mask_c = a->mask_c; p.mask_h = a->mask_h; p.zc = a->zc; p.zh = a->zh;
  p.lengths = a->lengths; p.t = a->t;
  p.dgates = a->dgates; p.dh_carry_out = a->dh_carry_out; p.dc_carry_out = a->dc_carry_out;
  p.rec = a->rec; p.rec_sb = a->rec_sb;
  const int DQ = (a->dq0 ? a->dq0_n : 0) + (a->dq1 ? a->dq1_n : 0);
  shm = (size_t)(BT + UT) * ((a->rec ? 0 : 4 * a->U) + DQ + 4) * sizeof(float);
  SAT_CHECK_ARG(shm <= 160 * 1024, "sat_lstm_step_bwd: U too large for the LDS-staged step");
  return SAT_OK;
}

extern "C" int sat_lstm_steps_bwd(const SatLstmBwd* steps, int32_t n, void* stream) {
  SAT_CHECK_ARG(steps && n >= 1 && n <= kMaxProblems, "sat_lstm_steps_bwd: 1..4 steps");
  LstmBwdMulti m;
  m.n = n;
  m.first[0] = 0;
  size_t shm = 0;
  for (int i = 0; i < n; ++i) {
    size_t s_i = 0;
    const int rc = check_bwd(steps + i, m.p[i], s_i);
    if (rc != SAT_OK) return rc;
    shm = std::max(shm, s_i);
    m.gx[i] = ceil_div(steps[i].U, UT);
    m.first[i + 1] = m.first[i] + m.gx[i] * ceil_div(steps[i].B, BT);
  }
  for (int i = n; i < kMaxProblems; ++i) { m.gx[i] = 1; m.first[i + 1] = m.first[n]; }
  hipLaunchKernelGGL(lstm_bwd_kernel, dim3(m.first[n]), dim3(256), shm, as_stream(stream), m);
  SAT_LAUNCH_CHECK("sat_lstm_steps_bwd");
  return SAT_OK;
}

extern "C" int sat_lstm_step_bwd(const SatLstmBwd* a, void* stream) {
  return sat_lstm_steps_bwd(a, 1, stream);
}
