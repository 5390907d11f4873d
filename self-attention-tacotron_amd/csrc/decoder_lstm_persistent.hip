// Persistent decoder LSTM stack: ALL T' steps of DecoderRNNV2's two ZoneoutLSTM(256) layers
// (ext tacotron2 DecoderRNNV2, built at modules/module.py:1531-1540: MultiRNNCell([attention
// cell, ZoneoutLSTM, ZoneoutLSTM])) in ONE launch, forward and backward.  The arithmetic is
// lstm.hip's step (TF LSTMCell gate order i, j, f, o, forget_bias 1.0; zoneout masks as inputs)
// restated; only the schedule differs.
//
// Why: after the persistent attention chain (decoder_persistent.hip) the two decoder LSTMs were
// a launch-per-step wavefront -- ~740 launches per direction per training step, each paying a
// kernel boundary plus a cold reload of its recurrent weights from MALL.  Here every workgroup
// keeps its weight columns in registers for the whole sequence, and one step costs one in-kernel
// hand-off plus on-chip arithmetic.
//
// Layout: 16 groups x 16 workgroups of 512 threads (256, one per CU).  Group g = blockIdx % 16
// owns utterances b = g + 16*ub (ub < 2, b < B); workgroup j = blockIdx / 16 owns units
// [16j, 16j+16) of BOTH layers, wave w of it units 16j + 2w, +1.  The LSTMs couple units, never
// utterances, so a group's hand-offs never leave the group, and blocks g, g+16, ... share an XCD
// under the observed round-robin placement (speed only).  A step's hand-off is an all-gather of
// the group's rows, so two utterances per group (not four over 32 workgroups) halve the bytes
// every workgroup must pull per step; the weights per workgroup double (96 floats per thread at
// 512 threads).
//   forward, iteration i (0..T'):   LSTM1 step i  and  LSTM2 step i-1
//     LSTM1 step i   needs h1_{i-1} (all units)
//     LSTM2 step i-1 needs h1'_{i-1} (raw output, its input) and h2_{i-2}
//   backward, iteration j (0..T'):  LSTM2 step T'-1-j  and  LSTM1 step T'-j
//     LSTM2 step t   needs dgates2_{t+1} (its recurrent product)
//     LSTM1 step t+1 needs dgates2_{t+1} (its output gradient through LSTM2's input rows)
//                    and  dgates1_{t+2} (its recurrent product)
// Every spin is bounded and a timeout raises err[0] so the grid always drains.
#include "sat_common.h"
#include "persistent.h"

namespace sat {
namespace {

constexpr int kG = 16;             // groups
constexpr int kGW = 16;            // workgroups per group
constexpr int kU = 256;            // units per layer
constexpr int kUW = kU / kGW;      // units per workgroup per layer (16)
constexpr int kUBmax = 2;          // utterances per group
constexpr int kThreads = 512;      // 8 waves, 2 units each
constexpr int kX = 3 * kU;         // forward staging row: [h1_{i-1} | h1'_{i-1} | h2_{i-2}]
static_assert(kUW == 2 * (kThreads / 64), "two units per wave");

struct DecLstmFwdP {
  int B, T, flags;
  float zc, zh;
  const float* X1;                                    // [T][B][4U]
  const float* W1r;                                   // [U][U][4]
  const float* W2;                                    // [2U][U][4]
  const float* b2;                                    // [4U]
  const float* m1c; const float* m1h; const float* m2c; const float* m2h;   // [T][B][U] | null
  float* H1RAW; float* C1S; float* H1S; float* G1;
  float* H2RAW; float* C2S; float* H2S; float* G2;
  float* xch;                                         // hand-off granules (zeroed per call)
  int* err;
  long long* prof;                                    // [256][4] segment clocks (nullable)
};

__device__ __forceinline__ unsigned tag_of(float x) { return __float_as_uint(x); }

// Forward.  Dot role: wave w owns units 2w, 2w+1 of the workgroup in both layers (8 gate
// columns each), lane = k-slice ks: LSTM1's recurrent rows 4ks..4ks+3 and LSTM2's [input |
// recurrent] rows 8ks..8ks+7 of those 8 columns live in registers (96 floats), so each staged
// float4 of the input rows feeds 8 columns.  The 32 partial sums per lane (layer x utterance x
// column) are transpose-reduced across the wave; the 4 gate sums of a (layer, utterance, unit)
// then sit in lanes l, l+2, l+4, l+6 and lane l runs the cell with its (c, h) state in registers.
// Hand-off (MI355X_MICROARCH.md / cdna_hip_programming.md Guideline 16, R2: the data IS the
// flag): every published value travels in an 8-byte {value, tag} granule, two per 16-byte sc1
// store; a consumer re-loads (sc1) the granules whose tag is not yet the step's epoch.  No group
// barrier, no drain.  Slots alternate by step parity: a producer can only reach step i+2 after
// every workgroup of its group has consumed step i.
//   XA[par][b][u]     = {h1_i, tag, h1'_i, tag}                  (LSTM1 step i)
//   XB[par][b][u/2]   = {h2_{i-1}[u], tag, h2_{i-1}[u+1], tag}   (LSTM2 step i-1)
// both published at iteration i with tag i+1 and consumed at iteration i+1.
__global__ void __launch_bounds__(kThreads) dec_lstm_fwd_kernel(DecLstmFwdP p) {
  __shared__ __attribute__((aligned(16))) float xs[kUBmax][kX];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = blockIdx.x % kG, j = blockIdx.x / kG;
  const int u0 = j * kUW;
  const int B = p.B, T = p.T;

  // ---- weights: 8 columns (units u0+2w, u0+2w+1, gates i j f o) x my k rows
  float w1[4][8], w2[8][8];
  {
    const int ucol = u0 + 2 * w;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4* src = reinterpret_cast<const float4*>(p.W1r + ((int64_t)(4 * lane + q) * kU + ucol) * 4);
      const float4 a = src[0], b = src[1];
      w1[q][0] = a.x; w1[q][1] = a.y; w1[q][2] = a.z; w1[q][3] = a.w;
      w1[q][4] = b.x; w1[q][5] = b.y; w1[q][6] = b.z; w1[q][7] = b.w;
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float4* src = reinterpret_cast<const float4*>(p.W2 + ((int64_t)(8 * lane + q) * kU + ucol) * 4);
      const float4 a = src[0], b = src[1];
      w2[q][0] = a.x; w2[q][1] = a.y; w2[q][2] = a.z; w2[q][3] = a.w;
      w2[q][4] = b.x; w2[q][5] = b.y; w2[q][6] = b.z; w2[q][7] = b.w;
    }
  }
  bool uvalid[kUBmax];
#pragma unroll
  for (int ub = 0; ub < kUBmax; ++ub) uvalid[ub] = g + kG * ub < B;
  // ---- cell role: output m = lane >> 1 = layer*16 + ub*8 + uu*4 + gate; lanes with gate 0
  const int m = lane >> 1;
  const int layer = m >> 4, pub = (m >> 3) & 1, puu = (m >> 2) & 1;
  const int pu = u0 + 2 * w + puu;
  const int pb = g + kG * pub;
  const bool cell = (lane & 7) == 0 && pb < B;
  float cst = 0.f, hst = 0.f;
  float4 bias2 = make_float4(0.f, 0.f, 0.f, 0.f);
  if (cell) {
    const int64_t i0 = (int64_t)pb * kU + pu;
    cst = layer == 0 ? p.C1S[i0] : p.C2S[i0];
    hst = layer == 0 ? p.H1S[i0] : p.H2S[i0];
    if (layer == 1) bias2 = reinterpret_cast<const float4*>(p.b2)[pu];
  }
  const bool masked = p.m1c != nullptr;
  float* XA = p.xch;                                   // [2][B][U] x 4
  float* XBb = p.xch + (size_t)8 * B * kU;              // [2][B][U/2] x 4
  const auto rXA = rsrc(XA), rXB = rsrc(XBb);
  // hand-off granules this thread consumes: XA (ub = tid / 256, u = tid % 256), XB (tid < 256)
  const int aub = tid >> 8, au = tid & (kU - 1);
  const int ab = g + kG * aub;
  const bool a_on = ab < B;
  const int bub = tid >> 7, bu2 = tid & (kU / 2 - 1);
  const int bb = g + kG * bub;
  const bool b_on = tid < kUBmax * (kU / 2) && bb < B;

  // cell operands of iteration ii (forward inputs, plain loads), prefetched one iteration
  // ahead so their HBM latency hides behind the hand-off wait.  Branch-free (clamped in-range
  // address, raw values; defaults applied at the use) so no vmcnt wait lands before the wait.
  auto ops_on = [&](int ii) {
    const int tt = layer == 0 ? ii : ii - 1;
    return cell && tt >= 0 && tt < T;
  };
  // this lane's mask pointers, selected once and kept opaque: selected inside the step loop,
  // the per-lane choice between two adjacent kernel-argument fields compiled to a per-lane
  // global load of the pointer from the argument block -- a dependent load, and a vmcnt wait
  // for it (behind every older memory operation of the wave), in every step
  uint64_t mc_addr = (uint64_t)(masked ? (layer == 0 ? p.m1c : p.m2c) : p.X1);
  uint64_t mh_addr = (uint64_t)(masked ? (layer == 0 ? p.m1h : p.m2h) : p.X1);
  asm volatile("" : "+v"(mc_addr), "+v"(mh_addr));
  auto load_ops = [&](int ii, float4& xp_, float& mc_, float& mh_) {
    const int tt = layer == 0 ? ii : ii - 1;
    const int64_t bu = ops_on(ii) ? ((int64_t)tt * B + pb) * kU + pu : 0;
    // (global address space: a generic pointer would compile to flat loads, which the waitcnt
    // pass must treat as out of order)
    typedef const __attribute__((address_space(1))) float* gptr;
    const gptr Mc = reinterpret_cast<gptr>(mc_addr);
    const gptr Mh = reinterpret_cast<gptr>(mh_addr);
    xp_ = reinterpret_cast<const float4*>(p.X1)[bu];
    mc_ = Mc[bu];
    mh_ = Mh[bu];
  };
  float4 xpn;
  float mcn, mhn;
  load_ops(0, xpn, mcn, mhn);

  // optional segment clocks (thread 0): hand-off wait, staging, dots, cell + publish
  // hand-off store policy (persistent.h xcd_local_group): plain stores iff the group is on one XCD
  const bool xl = (p.flags & 1) ? xcd_local_group(reinterpret_cast<unsigned*>(p.xch + (size_t)12 * B * kU), g, kG, kGW, p.err) : false;
  long long tp[4] = {0, 0, 0, 0};
  long long t0 = wall_clock64();
  auto tick = [&](int seg) {
    if (p.prof) {
      const long long t1 = wall_clock64();
      tp[seg] += t1 - t0;
      t0 = t1;
    }
  };

  for (int i = 0; i <= T; ++i) {
    const bool do1 = i < T, do2 = i >= 1;
    const int t = layer == 0 ? i : i - 1;
    const bool cell_step = cell && (layer == 0 ? do1 : do2);
    // ---- consume: h1_{i-1}, h1'_{i-1} (XA) and h2_{i-2} (XB) of the group's utterances
    if (i == 0) {
      xs[aub][au] = a_on ? p.H1S[(int64_t)ab * kU + au] : 0.f;
    } else {
      const unsigned ep = (unsigned)i;
      const int par = i & 1;
      float4 ga = make_float4(0.f, 0.f, 0.f, 0.f), gb = ga;
      bool oka = !a_on, okb = !b_on;
      for (unsigned spins = 0;; ++spins) {
        if (!oka) {
          ga = ldc4(rXA, (par * B + ab) * kU + au);
          oka = tag_of(ga.y) == ep && tag_of(ga.w) == ep;
        }
        if (!okb) {
          gb = ldc4(rXB, (par * B + bb) * (kU / 2) + bu2);
          okb = tag_of(gb.y) == ep && tag_of(gb.w) == ep;
        }
        if (oka && okb) break;
        if ((spins & 255u) == 255u) {
          if (__hip_atomic_load(p.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) break;
          if (spins > (1u << 20)) {   // a producer never published (not co-resident?)
            __hip_atomic_store(p.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
          }
        }
        __builtin_amdgcn_s_sleep(1);
      }
      tick(0);
      xs[aub][au] = ga.x;
      xs[aub][kU + au] = ga.z;
      if (tid < kUBmax * (kU / 2)) {
        xs[bub][2 * kU + 2 * bu2] = gb.x;
        xs[bub][2 * kU + 2 * bu2 + 1] = gb.z;
      }
    }
    // this iteration's prefetched operands (waited for only now, after the hand-off), then
    // the next iteration's prefetch
    const bool on_i = ops_on(i);
    const float4 xp = (layer == 0 && on_i) ? xpn : bias2;
    const float mc = (masked && on_i) ? mcn : 1.f - p.zc;
    const float mh = (masked && on_i) ? mhn : 1.f - p.zh;
    if (i < T) load_ops(i + 1, xpn, mcn, mhn);
    lds_barrier();   // LDS staging only: a __syncthreads would drain the prefetch just issued
    tick(1);
    // ---- dots: v[layer*16 + ub*8 + column]
    float v[32];
#pragma unroll
    for (int ub = 0; ub < kUBmax; ++ub) {
      float a1[8], a2[8];
#pragma unroll
      for (int cc = 0; cc < 8; ++cc) { a1[cc] = 0.f; a2[cc] = 0.f; }
      if (uvalid[ub]) {
        const float4* x4 = reinterpret_cast<const float4*>(xs[ub]);
        if (do1) {
          const float4 x = x4[lane];
          const float xv[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
          for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int cc = 0; cc < 8; ++cc) a1[cc] = fmaf(xv[q], w1[q][cc], a1[cc]);
        }
        if (do2) {
          const float4 xa = x4[kU / 4 + 2 * lane], xb = x4[kU / 4 + 2 * lane + 1];
          const float xv[8] = {xa.x, xa.y, xa.z, xa.w, xb.x, xb.y, xb.z, xb.w};
#pragma unroll
          for (int q = 0; q < 8; ++q)
#pragma unroll
            for (int cc = 0; cc < 8; ++cc) a2[cc] = fmaf(xv[q], w2[q][cc], a2[cc]);
        }
      }
#pragma unroll
      for (int cc = 0; cc < 8; ++cc) {
        v[ub * 8 + cc] = a1[cc];
        v[16 + ub * 8 + cc] = a2[cc];
      }
    }
    transpose_reduce32(v, lane);
    // gates of (layer, ub, unit): i at lane l, j at l+2, f at l+4, o at l+6 (l % 8 == 0)
    const float gj_ = dpp_mov<0x102>(v[0]);
    const float gf_ = dpp_mov<0x104>(v[0]);
    const float go_ = dpp_mov<0x106>(v[0]);
    tick(2);
    float hpub = hst;                                   // value published by LSTM2 lanes
    if (cell_step) {
      // one v_exp + one v_rcp per activation (the libm tanhf / IEEE-division logistic cost
      // ~5x the instructions on the step's critical path; <= 2 ulp apart)
      const float gi = sigmoid_fast(v[0] + xp.x);
      const float gj = tanh_lstm(gj_ + xp.y);
      const float gf = sigmoid_fast(gf_ + xp.z + 1.0f);   // forget_bias = 1.0
      const float go = sigmoid_fast(go_ + xp.w);
      const float cn = gf * cst + gi * gj;
      const float hn = go * tanh_lstm(cn);
      const float c2 = mc * cn + (1.f - mc) * cst;
      const float h2 = mh * hn + (1.f - mh) * hst;
      cst = c2;
      hst = h2;
      hpub = h2;
      const int64_t bu = ((int64_t)t * B + pb) * kU + pu;
      const int64_t bn = bu + (int64_t)B * kU;       // [t + 1]
      if (layer == 0) {
        if (i < T) {
          const float tg = __uint_as_float((unsigned)(i + 1));
          stc4x(xl, rXA, ((((i + 1) & 1) * B + pb) * kU + pu), make_float4(h2, tg, hn, tg));
        }
        p.H1RAW[bu] = hn;
        p.H1S[bn] = h2;
        p.C1S[bn] = c2;
        reinterpret_cast<float4*>(p.G1)[bu] = make_float4(gi, gj, gf, go);
      } else {
        p.H2RAW[bu] = hn;
        p.H2S[bn] = h2;
        p.C2S[bn] = c2;
        reinterpret_cast<float4*>(p.G2)[bu] = make_float4(gi, gj, gf, go);
      }
    }
    // LSTM2 lanes publish h2 (at i == 0: the initial state) in unit pairs: the uu = 1 partner
    // sits 8 lanes up
    const float hpart = dpp_mov<0x108>(hpub);
    if (cell && layer == 1 && puu == 0 && i < T) {
      const float tg = __uint_as_float((unsigned)(i + 1));
      stc4x(xl, rXB, ((((i + 1) & 1) * B + pb) * (kU / 2) + (pu >> 1)), make_float4(hpub, tg, hpart, tg));
    }
    tick(3);
  }
  if (p.prof && tid == 0)
    for (int i = 0; i < 4; ++i) p.prof[blockIdx.x * 4 + i] = tp[i];
}

struct DecLstmBwdP {
  int B, T, flags;
  float zc, zh;
  const float* W1r;                                   // [U][U][4]
  const float* W2;                                    // [2U][U][4]
  const float* G1; const float* C1S; const float* G2; const float* C2S;
  const float* DH2;                                   // [T][B][U]
  const float* m1c; const float* m1h; const float* m2c; const float* m2h;
  float* DG1; float* DG2;                             // [T][B][4U]
  unsigned* ctr;   // XG [2 slots][2 streams][B][4U] tagged gate gradients, then XID [256]
  int* err;
  long long* prof;                                    // [256][4] segment clocks (nullable)
};

// TF LSTMCell + zoneout backward of one (utterance, unit) (lstm.hip lstm_bwd_block's pointwise):
// returns dgates and updates the (dh, dc) carries.
__device__ __forceinline__ float4 lstm_cell_bwd(float4 g4, float cp, float dy, float rec,
                                                float mc, float mh, float& dhc, float& dcc) {
  const float gi = g4.x, gj = g4.y, gf = g4.z, go = g4.w;
  const float cn = gf * cp + gi * gj;
  const float tc = tanh_lstm(cn);   // formed exactly as the forward formed it
  const float dh_t = rec + dhc;
  const float dc_t = dcc;
  const float dhn = dy + mh * dh_t;                 // dL/dh'
  const float dcn = mc * dc_t + dhn * go * (1.f - tc * tc);
  const float d_o = dhn * tc * go * (1.f - go);
  const float d_f = dcn * cp * gf * (1.f - gf);
  const float d_i = dcn * gj * gi * (1.f - gi);
  const float d_j = dcn * gi * (1.f - gj * gj);
  dcc = dcn * gf + (1.f - mc) * dc_t;
  dhc = (1.f - mh) * dh_t;
  return make_float4(d_i, d_j, d_f, d_o);
}

// Backward.  Dot role: wave w owns units u = 2w, 2w+1 of the workgroup; lane = k-slice of 16 of
// the 4U-long gate-gradient rows.  Its weights are those 16 entries of three rows per unit:
// LSTM2's recurrent row W2[U+u], LSTM2's input row W2[u] (LSTM1's output gradient) and LSTM1's
// recurrent row W1r[u] (96 floats).  The 16 partial sums per lane (utterance x unit x
// {r2, y1, r1, pad}) are transpose-reduced across the wave (permlane swaps + DPP), after which
// lanes 4m..4m+3 hold output m.  Cells: the lane holding r2 runs LSTM2's cell, the lane holding
// r1 LSTM1's (y1 comes from 4 lanes below by DPP); carries stay in their registers.  Hand-off:
// data-tagged gate gradients, no barrier (persistent.h lsb_tag rule): each cell writes its
// tagged dgates to the history (for the weight-gradient GEMMs) and to exchange slot q & 1 of its
// stream (LSTM2: q = jj, LSTM1: q = jj - 1, so every slot's first occupant is written at q = 0
// or 1), and the next iteration's staging polls the group's rows of that slot until every word
// carries bit lsb_tag(q).  A workgroup reaches iteration jj + 2 (overwriting slot q) only after
// staging every workgroup's iteration jj + 1 rows, which their makers wrote after consuming
// iteration jj's -- so no slot is overwritten before it is read.  (Replaced a drained store + an
// agent-scope counter barrier + a reload: 1.06 + 0.99 us of the 3.2 us step.)  Cell operands
// (forward histories, the head's gradient) are prefetched one iteration ahead.
__global__ void __launch_bounds__(kThreads) dec_lstm_bwd_kernel(DecLstmBwdP p) {
  __shared__ __attribute__((aligned(16))) float dg2s[kUBmax][4 * kU];
  __shared__ __attribute__((aligned(16))) float dg1s[kUBmax][4 * kU];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = blockIdx.x % kG, j = blockIdx.x / kG;
  const int u0 = j * kUW;
  const int B = p.B, T = p.T;
  float* XG = reinterpret_cast<float*>(p.ctr);          // [2][2][B][4U]
  unsigned* XID = p.ctr + (size_t)16 * B * kU;

  float4 wa[2][4], wb[2][4], wc[2][4];
#pragma unroll
  for (int uu = 0; uu < 2; ++uu) {
    const int u = u0 + 2 * w + uu;
    const float4* ra = reinterpret_cast<const float4*>(p.W2 + (int64_t)(kU + u) * 4 * kU) + 4 * lane;
    const float4* rb = reinterpret_cast<const float4*>(p.W2 + (int64_t)u * 4 * kU) + 4 * lane;
    const float4* rc = reinterpret_cast<const float4*>(p.W1r + (int64_t)u * 4 * kU) + 4 * lane;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      wa[uu][q] = ra[q];
      wb[uu][q] = rb[q];
      wc[uu][q] = rc[q];
    }
  }
  bool uvalid[kUBmax];
#pragma unroll
  for (int ub = 0; ub < kUBmax; ++ub) uvalid[ub] = g + kG * ub < B;
  // cell role: output m = lane >> 2 = ub*8 + uu*4 + prod (prod 0: r2 -> LSTM2, 2: r1 -> LSTM1)
  const int m = lane >> 2, prod = m & 3, puu = (m >> 2) & 1, pub = m >> 3;
  const int pu = u0 + 2 * w + puu, pb = g + kG * pub;
  const bool cell = (lane & 3) == 0 && (prod == 0 || prod == 2) && pb < B;
  const int layer = prod == 0 ? 2 : 1;
  float dhc = 0.f, dcc = 0.f;
  const bool masked = p.m1c != nullptr;
  const auto rXG = rsrc(XG);

  // cell operands of iteration jj (plain loads of read-only inputs).  Branch-free: every lane
  // loads from a clamped in-range address and only cell lanes of live steps use the values, so
  // the loads stay in flight across the barrier (a conditional load into a defaulted register
  // forces a vmcnt(0) at the join).
  auto load_ops = [&](int jj, float4& g4, float& cp, float& dyv, float& mc, float& mh) {
    const int t = layer == 2 ? T - 1 - jj : T - jj;
    const bool on = cell && t >= 0 && t < T;
    const int64_t bu = on ? ((int64_t)t * B + pb) * kU + pu : 0;
    const float* Gp = layer == 2 ? p.G2 : p.G1;
    const float* Cs = layer == 2 ? p.C2S : p.C1S;
    const float* Mc = masked ? (layer == 2 ? p.m2c : p.m1c) : Cs;
    const float* Mh = masked ? (layer == 2 ? p.m2h : p.m1h) : Cs;
    g4 = reinterpret_cast<const float4*>(Gp)[bu];
    cp = Cs[bu];
    dyv = p.DH2[bu];
    mc = Mc[bu];
    mh = Mh[bu];
  };
  float4 g4n;
  float cpn, dyn, mcn, mhn;
  load_ops(0, g4n, cpn, dyn, mcn, mhn);

  // optional segment clocks (thread 0): barrier wait, staging loads, dots, cells + stores
  // hand-off store policy (persistent.h xcd_local_group): plain stores iff the group is on one XCD
  const bool xl = (p.flags & 1) ? xcd_local_group(XID, g, kG, kGW, p.err) : false;
  bool gave_up = false;
  long long tp[4] = {0, 0, 0, 0};
  long long t0 = wall_clock64();
  auto tick = [&](int seg) {
    if (p.prof) {
      const long long t1 = wall_clock64();
      tp[seg] += t1 - t0;
      t0 = t1;
    }
  };

  for (int jj = 0; jj <= T; ++jj) {
    const int t2 = T - 1 - jj, t1 = T - jj;
    const bool has2 = t2 >= 0, has1 = jj >= 1;
    const bool stage2 = jj >= 1, stage1 = jj >= 2;   // DG2[t2+1] and DG1[t1+1] exist
    const int t = layer == 2 ? t2 : t1;
    const bool cell_step = cell && (layer == 2 ? has2 : has1);
    const float4 g4 = g4n;
    const float cp = cpn, dyv = dyn;
    const float mc = masked ? mcn : 1.f - p.zc, mh = masked ? mhn : 1.f - p.zh;
    // stage dgates2_{t2+1} (stream 0, q = jj - 1) and dgates1_{t1+1} (stream 1, q = jj - 2) of
    // the group's utterances from their exchange slots: thread = (utterance slot tid / U, float4
    // column tid % U); sc1 polls until every word carries the step's tag
    {
      static_assert(kUBmax * kU == kThreads, "staging map");
      const int ub = tid / kU, q = tid - ub * kU, b = g + kG * ub;
      const bool bo = b < B;
      const int bb = bo ? b : 0;
      const int q2 = jj - 1, q1 = jj - 2;
      const int i2 = ((((q2 & 1) * 2 + 0) * B + bb) * kU) + q;
      const int i1 = ((((q1 & 1) * 2 + 1) * B + bb) * kU) + q;
      const unsigned w2 = lsb_tag(q2), w1 = lsb_tag(q1);
      float4 v2 = make_float4(0.f, 0.f, 0.f, 0.f), v1 = v2;
      bool ok2 = !(stage2 && bo), ok1 = !(stage1 && bo);
      // first attempt branch-free (every thread issues both loads; slots of steps not yet
      // staged are in-range addresses whose values are discarded), the retry loop only on a
      // miss: 2.55 -> 2.50-2.52 us/step (round 6, two A/B rounds; the same change in the
      // forward's granule poll measured 2.61 -> 2.72, not made there)
      {
        const float4 f2 = ldc4(rXG, i2), f1 = ldc4(rXG, i1);
        if (!ok2) { v2 = f2; ok2 = tag_ok4(v2, w2); }
        if (!ok1) { v1 = f1; ok1 = tag_ok4(v1, w1); }
      }
      if (__builtin_amdgcn_ballot_w64(!(ok1 && ok2)) != 0 && !gave_up)
      for (unsigned spins = 0;; ++spins) {
        if (!ok2) v2 = ldc4(rXG, i2);
        if (!ok1) v1 = ldc4(rXG, i1);
        ok2 = ok2 || tag_ok4(v2, w2);
        ok1 = ok1 || tag_ok4(v1, w1);
        if (__builtin_amdgcn_ballot_w64(!(ok1 && ok2)) == 0 || gave_up) break;
        if (poll_give_up(spins, p.err)) { gave_up = true; break; }
        __builtin_amdgcn_s_sleep(1);
      }
      *reinterpret_cast<float4*>(&dg2s[ub][4 * q]) = v2;
      *reinterpret_cast<float4*>(&dg1s[ub][4 * q]) = v1;
    }
    if (jj < T) load_ops(jj + 1, g4n, cpn, dyn, mcn, mhn);   // in flight across the barrier
    lds_barrier();   // (a __syncthreads would drain them: its release fence waits on vmcnt)
    tick(1);
    float v[16];
#pragma unroll
    for (int ub = 0; ub < kUBmax; ++ub) {
      float r2[2] = {0.f, 0.f}, y1[2] = {0.f, 0.f}, r1[2] = {0.f, 0.f};
      if (uvalid[ub]) {
        const float4* d2 = reinterpret_cast<const float4*>(dg2s[ub]) + 4 * lane;
        const float4* d1 = reinterpret_cast<const float4*>(dg1s[ub]) + 4 * lane;
        if (stage2) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float4 x = d2[q];
#pragma unroll
            for (int uu = 0; uu < 2; ++uu) {
              r2[uu] = dot4(x, wa[uu][q], r2[uu]);
              y1[uu] = dot4(x, wb[uu][q], y1[uu]);
            }
          }
        }
        if (stage1) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float4 x = d1[q];
#pragma unroll
            for (int uu = 0; uu < 2; ++uu) r1[uu] = dot4(x, wc[uu][q], r1[uu]);
          }
        }
      }
#pragma unroll
      for (int uu = 0; uu < 2; ++uu) {
        v[ub * 8 + uu * 4 + 0] = r2[uu];
        v[ub * 8 + uu * 4 + 1] = y1[uu];
        v[ub * 8 + uu * 4 + 2] = r1[uu];
        v[ub * 8 + uu * 4 + 3] = 0.f;
      }
    }
    transpose_reduce16(v, lane);
    const float y1v = dpp_mov<0x114>(v[0]);     // row_shr:4: y1 sits one output (4 lanes) below
    tick(2);
    if (cell_step) {
      const float rec = layer == 2 ? (stage2 ? v[0] : 0.f) : (stage1 ? v[0] : 0.f);
      const float dy = layer == 2 ? dyv : y1v;
      const int qs = layer == 2 ? jj : jj - 1;            // the stream's sequence number
      const float4 dg = tagf4(lstm_cell_bwd(g4, cp, dy, rec, mc, mh, dhc, dcc), lsb_tag(qs));
      const int64_t bu = ((int64_t)t * B + pb) * kU + pu;
      reinterpret_cast<float4*>(layer == 2 ? p.DG2 : p.DG1)[bu] = dg;   // history (GEMMs)
      stc4x(xl, rXG, ((((qs & 1) * 2 + (layer == 2 ? 0 : 1)) * B + pb) * kU) + pu, dg);
    }
    tick(3);
    tick(0);
  }
  if (p.prof && tid == 0)
    for (int i = 0; i < 4; ++i) p.prof[blockIdx.x * 4 + i] = tp[i];
}

int check_coresident(const void* kernel, const char* name) {
  int dev = 0, cus = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kThreads, 0) != hipSuccess) {
    set_error("%s: device query failed", name);
    return SAT_ERR_HIP;
  }
  SAT_CHECK_ARG((int64_t)cus * per_cu >= kG * kGW,
                "%s: fewer than 256 co-resident workgroups on this device", name);
  return SAT_OK;
}

}  // namespace
}  // namespace sat

using namespace sat;

extern "C" int64_t sat_decoder_lstms_scratch(int32_t B) {
  return (int64_t)12 * B * kU + kG * kGW;   // XA [2][B][U] + XB [2][B][U/2] granule pairs + XID
}

extern "C" int64_t sat_decoder_lstms_bwd_scratch(int32_t B) {
  return (int64_t)16 * B * kU + kG * kGW;   // XG [2][2][B][4U] tagged gate gradients + XID
}

extern "C" int sat_decoder_lstms_fwd(const SatDecLstmFwd* a, void* stream) {
  const char* nm = "sat_decoder_lstms_fwd";
  SAT_CHECK_ARG(a && a->B > 0 && a->T > 0, "%s: bad sizes", nm);
  SAT_CHECK_ARG(a->U == kU, "%s: compiled for U=256 (the self-attention-tacotron configs)", nm);
  SAT_CHECK_ARG(a->B <= kG * kUBmax, "%s: B <= 32", nm);
  SAT_CHECK_ARG(a->X1 && a->W1r && a->W2 && a->b2 && a->H1RAW && a->C1S && a->H1S && a->G1 &&
                a->H2RAW && a->C2S && a->H2S && a->G2 && a->xch && a->err, "%s: null pointer", nm);
  SAT_CHECK_ARG((a->mask1_c == nullptr) == (a->mask1_h == nullptr) &&
                (a->mask1_c == nullptr) == (a->mask2_c == nullptr) &&
                (a->mask2_c == nullptr) == (a->mask2_h == nullptr),
                "%s: the four zoneout masks are all given or all NULL", nm);
  SAT_CHECK_ARG(aligned16(a->X1) && aligned16(a->b2) && aligned16(a->G1) && aligned16(a->G2) &&
                aligned16(a->W1r) && aligned16(a->W2) && aligned16(a->xch),
                "%s: 16-byte aligned operands", nm);
  SAT_CHECK_ARG((int64_t)(a->T + 1) * a->B * 4 * kU < (1ll << 29), "%s: histories too long", nm);
  int rc = check_coresident(reinterpret_cast<const void*>(dec_lstm_fwd_kernel), nm);
  if (rc != SAT_OK) return rc;
  DecLstmFwdP p;
  p.B = a->B; p.T = a->T; p.zc = a->zc; p.zh = a->zh;
  p.X1 = a->X1; p.W1r = a->W1r; p.W2 = a->W2; p.b2 = a->b2;
  p.m1c = a->mask1_c; p.m1h = a->mask1_h; p.m2c = a->mask2_c; p.m2h = a->mask2_h;
  p.H1RAW = a->H1RAW; p.C1S = a->C1S; p.H1S = a->H1S; p.G1 = a->G1;
  p.H2RAW = a->H2RAW; p.C2S = a->C2S; p.H2S = a->H2S; p.G2 = a->G2;
  p.xch = a->xch; p.err = a->err; p.flags = xcd_local_env();
  p.prof = reinterpret_cast<long long*>(a->prof);
  hipStream_t s = as_stream(stream);
  if (zero_ranges(s, a->xch, sat_decoder_lstms_scratch(a->B), a->err, 2) != hipSuccess) {
    set_error("%s: memset failed", nm);
    return SAT_ERR_HIP;
  }
  hipLaunchKernelGGL(dec_lstm_fwd_kernel, dim3(kG * kGW), dim3(kThreads), 0, s, p);
  SAT_LAUNCH_CHECK(nm);
  return SAT_OK;
}

extern "C" int sat_decoder_lstms_bwd(const SatDecLstmBwd* a, void* stream) {
  const char* nm = "sat_decoder_lstms_bwd";
  SAT_CHECK_ARG(a && a->B > 0 && a->T > 0, "%s: bad sizes", nm);
  SAT_CHECK_ARG(a->U == kU, "%s: compiled for U=256 (the self-attention-tacotron configs)", nm);
  SAT_CHECK_ARG(a->B <= kG * kUBmax, "%s: B <= 32", nm);
  SAT_CHECK_ARG(a->W1r && a->W2 && a->G1 && a->C1S && a->G2 && a->C2S && a->DH2 && a->DG1 &&
                a->DG2 && a->ctr && a->err, "%s: null pointer", nm);
  SAT_CHECK_ARG((a->mask1_c == nullptr) == (a->mask1_h == nullptr) &&
                (a->mask1_c == nullptr) == (a->mask2_c == nullptr) &&
                (a->mask2_c == nullptr) == (a->mask2_h == nullptr),
                "%s: the four zoneout masks are all given or all NULL", nm);
  SAT_CHECK_ARG(aligned16(a->W1r) && aligned16(a->W2) && aligned16(a->G1) && aligned16(a->G2) &&
                aligned16(a->DG1) && aligned16(a->DG2), "%s: 16-byte aligned operands", nm);
  SAT_CHECK_ARG((int64_t)a->T * a->B * 4 * kU < (1ll << 29), "%s: histories too long", nm);
  int rc = check_coresident(reinterpret_cast<const void*>(dec_lstm_bwd_kernel), nm);
  if (rc != SAT_OK) return rc;
  DecLstmBwdP p;
  p.B = a->B; p.T = a->T; p.zc = a->zc; p.zh = a->zh;
  p.W1r = a->W1r; p.W2 = a->W2; p.G1 = a->G1; p.C1S = a->C1S; p.G2 = a->G2; p.C2S = a->C2S;
  p.DH2 = a->DH2;
  p.m1c = a->mask1_c; p.m1h = a->mask1_h; p.m2c = a->mask2_c; p.m2h = a->mask2_h;
  p.DG1 = a->DG1; p.DG2 = a->DG2; p.ctr = a->ctr; p.err = a->err; p.flags = xcd_local_env();
  p.prof = reinterpret_cast<long long*>(a->prof);
  hipStream_t s = as_stream(stream);
  SAT_CHECK_ARG(aligned16(a->ctr), "%s: 16-byte aligned scratch", nm);
  if (zero_ranges(s, a->ctr, sat_decoder_lstms_bwd_scratch(a->B), a->err, 2) != hipSuccess) {
    set_error("%s: memset failed", nm);
    return SAT_ERR_HIP;
  }
  hipLaunchKernelGGL(dec_lstm_bwd_kernel, dim3(kG * kGW), dim3(kThreads), 0, s, p);
  SAT_LAUNCH_CHECK(nm);
  return SAT_OK;
}
