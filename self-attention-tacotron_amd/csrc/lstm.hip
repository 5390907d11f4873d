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
};

__global__ void __launch_bounds__(256) lstm_fwd_kernel(LstmFwdP p) {
  const int tid = threadIdx.x;
  const int ks = tid & (KS - 1), pair = tid >> 3;
  const int u = blockIdx.x * UT + (pair & (UT - 1));
  const int b = blockIdx.y * BT + (pair >> 2);
  const bool active = (u < p.U) && (b < p.B);
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  if (active) {
    const float* rin = p.rin + (int64_t)b * p.rin_sb;
    const float4* W4 = reinterpret_cast<const float4*>(p.W);
    const int nchunk = p.K >> 2;
#pragma unroll 4
    for (int c = ks; c < nchunk; c += KS) {
      const float4 x = *reinterpret_cast<const float4*>(rin + 4 * c);
      const float xs[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float4 w = W4[(int64_t)(4 * c + r) * p.U + u];
        acc[0] = fmaf(xs[r], w.x, acc[0]);
        acc[1] = fmaf(xs[r], w.y, acc[1]);
        acc[2] = fmaf(xs[r], w.z, acc[2]);
        acc[3] = fmaf(xs[r], w.w, acc[3]);
      }
    }
  }
#pragma unroll
  for (int o = 1; o < KS; o <<= 1)
#pragma unroll
    for (int g = 0; g < 4; ++g) acc[g] += __shfl_xor(acc[g], o, 64);
  if (!active || ks != 0) return;

  const int64_t bu = (int64_t)b * p.U + u;
  const float cp = p.c_prev ? p.c_prev[bu] : 0.f;
  const float hp = p.h_prev ? p.h_prev[(int64_t)b * p.h_prev_sb + u] : 0.f;
  const bool valid = p.lengths ? (p.t < p.lengths[b]) : true;
  if (!valid) {  // bidirectional_dynamic_rnn(sequence_length): state copied, output 0
    p.c_out[bu] = cp;
    p.h_out[(int64_t)b * p.h_out_sb + u] = hp;
    if (p.h_raw) p.h_raw[(int64_t)b * p.h_raw_sb + u] = 0.f;
    if (p.gates) reinterpret_cast<float4*>(p.gates)[bu] = make_float4(0.f, 0.f, 0.f, 0.f);
    return;
  }
  float4 xp;
  if (p.xproj) xp = reinterpret_cast<const float4*>(p.xproj + (int64_t)b * p.xproj_sb)[u];
  else if (p.bias) xp = reinterpret_cast<const float4*>(p.bias)[u];
  else xp = make_float4(0.f, 0.f, 0.f, 0.f);
  const float gi = sigmf(acc[0] + xp.x);
  const float gj = tanhf(acc[1] + xp.y);
  const float gf = sigmf(acc[2] + xp.z + 1.0f);   // forget_bias = 1.0
  const float go = sigmf(acc[3] + xp.w);
  const float cn = gf * cp + gi * gj;
  const float hn = go * tanhf(cn);
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
};

// dL/dh_t = dh_carry + sum_g dgates_{t+1}[b, g] * W[hoff + u, g]  (the recurrent product)
// The optional query-gradient term sum_d dq[b, d] wq[u, d] reads dq as `dq_parts` per-tile
// partials: the workgroup first sums them for its 8 batch rows into LDS (all 256 threads, loads
// independent), then every (b, u) group dots the LDS row with wq's row.
constexpr int kMaxDq = 320;

__global__ void __launch_bounds__(256) lstm_bwd_kernel(LstmBwdP p) {
  __shared__ float dqs[BT][kMaxDq];
  const int tid = threadIdx.x;
  const int ks = tid & (KS - 1), pair = tid >> 3;
  const int u = blockIdx.x * UT + (pair & (UT - 1));
  const int bl = pair >> 2;
  const int b = blockIdx.y * BT + bl;
  const bool active = (u < p.U) && (b < p.B);
  const int D0 = p.dq0 ? p.dq0_n : 0, D1 = p.dq1 ? p.dq1_n : 0;
  if (D0 + D1 > 0) {
    for (int i = tid; i < BT * (D0 + D1); i += 256) {
      const int r = i / (D0 + D1), d = i - r * (D0 + D1);
      const int bb = blockIdx.y * BT + r;
      float g = 0.f;
      if (bb < p.B) {
        const float* src = d < D0 ? p.dq0 + d : p.dq1 + (d - D0);
        for (int part = 0; part < p.dq_parts; ++part)
          g += src[(int64_t)bb * p.dq_bstride + part * p.dq_pstride];
      }
      dqs[r][d] = g;
    }
    __syncthreads();
  }
  float rec = 0.f, extra = 0.f;
  if (active && p.dgates_next) {
    const float4* dg = reinterpret_cast<const float4*>(p.dgates_next + (int64_t)b * p.U * 4);
    const float4* wr = reinterpret_cast<const float4*>(p.W + (int64_t)(p.hoff + u) * p.U * 4);
#pragma unroll 8
    for (int v = ks; v < p.U; v += KS) {
      const float4 g = dg[v], w = wr[v];
      rec += g.x * w.x + g.y * w.y + g.z * w.z + g.w * w.w;
    }
  }
  if (active && D0 > 0) {
    const float* w0 = p.wq0 + (int64_t)u * D0;
    for (int d = ks; d < D0; d += KS) extra = fmaf(dqs[bl][d], w0[d], extra);
  }
  if (active && D1 > 0) {
    const float* w1 = p.wq1 + (int64_t)u * D1;
    for (int d = ks; d < D1; d += KS) extra = fmaf(dqs[bl][D0 + d], w1[d], extra);
  }
#pragma unroll
  for (int o = 1; o < KS; o <<= 1) {
    rec += __shfl_xor(rec, o, 64);
    extra += __shfl_xor(extra, o, 64);
  }
  if (!active || ks != 0) return;
  const int64_t bu = (int64_t)b * p.U + u;
  const float dh_t = rec + (p.dh_carry ? p.dh_carry[bu] : 0.f);
  const float dc_t = p.dc_carry ? p.dc_carry[bu] : 0.f;
  const bool valid = p.lengths ? (p.t < p.lengths[b]) : true;
  if (!valid) {
    reinterpret_cast<float4*>(p.dgates)[bu] = make_float4(0.f, 0.f, 0.f, 0.f);
    p.dh_carry_out[bu] = dh_t;
    p.dc_carry_out[bu] = dc_t;
    return;
  }
  const float4 g = reinterpret_cast<const float4*>(p.gates)[bu];
  const float gi = g.x, gj = g.y, gf = g.z, go = g.w;
  const float cp = p.c_prev ? p.c_prev[bu] : 0.f;
  const float cn = gf * cp + gi * gj;
  const float tc = tanhf(cn);
  float mc, mh;
  if (p.mask_c) { mc = p.mask_c[bu]; mh = p.mask_h[bu]; }
  else { mc = 1.f - p.zc; mh = 1.f - p.zh; }
  const float dy = (p.dy ? p.dy[(int64_t)b * p.dy_sb + u] : 0.f) + extra;
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

}  // namespace
}  // namespace sat

using namespace sat;

extern "C" int sat_lstm_step_fwd(const SatLstmFwd* a, void* stream) {
  SAT_CHECK_ARG(a && a->B > 0 && a->U > 0 && a->K >= 0, "sat_lstm_step_fwd: bad sizes");
  SAT_CHECK_ARG(a->K % 4 == 0 && a->rin_sb % 4 == 0, "sat_lstm_step_fwd: K and rin stride must be multiples of 4");
  SAT_CHECK_ARG((a->K == 0 || a->rin) && a->W && a->c_out && a->h_out, "sat_lstm_step_fwd: null pointer");
  SAT_CHECK_ARG((a->mask_c == nullptr) == (a->mask_h == nullptr), "sat_lstm_step_fwd: masks come in pairs");
  LstmFwdP p;
  p.B = a->B; p.U = a->U; p.K = a->K;
  p.xproj = a->xproj; p.xproj_sb = a->xproj_sb; p.bias = a->bias;
  p.rin = a->rin; p.rin_sb = a->rin_sb; p.W = a->W;
  p.c_prev = a->c_prev; p.h_prev = a->h_prev; p.h_prev_sb = a->h_prev_sb;
  p.mask_c = a->mask_c; p.mask_h = a->mask_h; p.zc = a->zc; p.zh = a->zh;
  p.lengths = a->lengths; p.t = a->t;
  p.h_raw = a->h_raw; p.h_raw_sb = a->h_raw_sb;
  p.c_out = a->c_out; p.h_out = a->h_out; p.h_out_sb = a->h_out_sb; p.gates = a->gates;
  dim3 grid(ceil_div(a->U, UT), ceil_div(a->B, BT));
  hipLaunchKernelGGL(lstm_fwd_kernel, grid, dim3(256), 0, as_stream(stream), p);
  SAT_LAUNCH_CHECK("sat_lstm_step_fwd");
  return SAT_OK;
}

extern "C" int sat_lstm_step_bwd(const SatLstmBwd* a, void* stream) {
  SAT_CHECK_ARG(a && a->B > 0 && a->U > 0, "sat_lstm_step_bwd: bad sizes");
  SAT_CHECK_ARG(a->W && a->gates && a->dgates && a->dh_carry_out && a->dc_carry_out,
                "sat_lstm_step_bwd: null pointer");
  SAT_CHECK_ARG(a->hoff >= 0 && a->hoff + a->U <= a->K, "sat_lstm_step_bwd: hoff out of range");
  SAT_CHECK_ARG((a->dq0 ? a->dq0_n : 0) + (a->dq1 ? a->dq1_n : 0) <= kMaxDq,
                "sat_lstm_step_bwd: query width > 320");
  LstmBwdP p;
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
  dim3 grid(ceil_div(a->U, UT), ceil_div(a->B, BT));
  hipLaunchKernelGGL(lstm_bwd_kernel, grid, dim3(256), 0, as_stream(stream), p);
  SAT_LAUNCH_CHECK("sat_lstm_step_bwd");
  return SAT_OK;
}
