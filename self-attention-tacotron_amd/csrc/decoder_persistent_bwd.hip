// Persistent BPTT of the decoder's attention chain: ALL T' reverse steps of
//   dual-source attention backward  ->  attention-RNN (ZoneoutLSTM 256) backward
// in ONE launch -- the reverse of decoder_persistent.hip, and the per-step kernels'
// arithmetic (attention.hip attn_bwd_kernel, lstm.hip lstm_bwd_block) restated.
//
// Same layout as the forward: 8 groups x 32 workgroups; group g owns utterances g + 8*ub; its
// workgroup j owns LSTM units [8j, 8j+8) and, if j < UB*ntiles, one (utterance, 32-position
// tile) whose K1/V1/K2/V2 slice stays in LDS.  512 threads (8 waves) per workgroup.
// Per reverse step t, two phases separated by group barriers:
//   Y (tile workgroups): dL/dctx_t = (LSTM1's part, precomputed) + sum of the 32 row-dot
//      partials of the attention RNN's input gradient; the attention backward of the tile
//      (utterance-wide sums as dots with the forward context -- see attention.hip); publishes
//      the tile's query-gradient partial, Y_t and dL/df_t for step t-1.
//   Z (every workgroup): its 8 units' reverse LSTM step: dh_t = recurrent product (sum of the
//      32 partials) + carry, dy += dq_t . Wq[unit] (dq_t = sum of the tile partials), gates
//      gradient DG0[t]; then its 32 gate columns' share of the next row-dot,
//      partial[j][k] = sum_c DG0[t][c] W0r[k][32j + c] for all 544 inputs k (the context and
//      recurrent gradients of step t-1), so no workgroup ever needs all 1024 gate gradients.
// Hand-offs and bounded spins: persistent.h.  Outputs are the per-step histories the
// launch-based BPTT writes (DG0, DE1/DE2, DFH, DQP, the full dL/dctx into RD), so the
// post-loop parameter-gradient GEMMs and sat_attn_param_grads are unchanged.
#include "sat_common.h"
#include "persistent.h"

namespace sat {
namespace {

constexpr int kG = 8, kGW = 32, kPN = 32, kUBmax = 4;
constexpr int kU = 256, kM1 = 256, kM2 = 32, kD1 = 224, kD2 = 32, kF = 5, kKW = 10;
constexpr int kK0 = kM1 + kM2 + kU;          // 544: [c1 | c2 | h0] inputs of the attention RNN
constexpr int kC = kM1 + kM2;                // 288 context dims
constexpr int kQ = kD1 + kD2;                // 256 query dims
constexpr int kUW = kU / kGW;                // 8 units per workgroup
constexpr int kNmax = 8 * kPN;               // 256 memory positions
constexpr int kTh = 512, kWv = 8;            // threads, waves
constexpr int kPPW = kPN / kWv;              // 4 tile positions per wave

struct DecAttnBwdP {
  int B, N, T, ntiles, UB;
  float u, zc, zh;
  const float* REC0; const float* C0; const float* G0; const float* Q;
  const float* S1; const float* AL1; const float* S2; const float* ST; const float* LOC;
  const float* K1; const float* V1; const float* K2; const float* V2;
  const float* v1; const float* b1; const float* convW; const float* locW; const float* v2;
  const float* W0r; const float* Wq1; const float* Wq2;
  const float* mask_c; const float* mask_h;
  const float* DH0;          // [T][B][U]     dL/dh0'_t from LSTM1 (precomputed)
  float* RD;                 // [T][B][K0]    in: [:, :C] LSTM1's dL/dctx_t; out: full dL/dctx_t
  float* DG0;                // [T][B][4U]
  float* DE1; float* DE2;    // [T][B][N]
  float* DFH;                // [T][B][N][F]
  float* DQP;                // [T][B][ntiles][Q]
  float* RDP;                // [2][B][kGW][K0]  row-dot partials (scratch)
  float* YA;                 // [2][B][N]        alignment-recursion gradient (scratch)
  unsigned* ctr; int* err;
};

__global__ void __launch_bounds__(kTh) dec_attn_bwd_kernel(DecAttnBwdP p) {
  __shared__ __attribute__((aligned(16))) float k1s[kPN][kD1];
  __shared__ __attribute__((aligned(16))) float v1s[kPN][kM1];
  __shared__ __attribute__((aligned(16))) float k2s[kPN][kD2];
  __shared__ __attribute__((aligned(16))) float v2s[kPN][kM2];
  __shared__ __attribute__((aligned(16))) float qb[kD1];
  __shared__ __attribute__((aligned(16))) float vv[kD1];
  __shared__ __attribute__((aligned(16))) float locw[kF][kD1];
  __shared__ float q2s[kD2], vv2[kD2];
  __shared__ float cw[kKW * kF];
  __shared__ float dc[kC];
  __shared__ __attribute__((aligned(16))) float4 dcred[kWv][kC / 4];
  __shared__ float dfall[kNmax * kF];
  __shared__ float fs[kPN][kF], dfs[kPN][kF];
  __shared__ float dsn_t[kPN], dan_t[kPN], stv[kPN], s2v[kPN], apv[kPN + 1];
  __shared__ float de1[kPN], de2[kPN];
  __shared__ float red[3 * kWv];
  __shared__ float dqred[kWv][kQ + 32];
  // phase Z
  __shared__ __attribute__((aligned(16))) float dqs[kUBmax][kQ];
  __shared__ float recs[kUBmax][kUW];
  __shared__ float qt[kUBmax][kUW];
  __shared__ float dgs[kUBmax][32];
  __shared__ float wtail[kK0 - kTh][33];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = blockIdx.x % kG, j = blockIdx.x / kG;
  const int B = p.B, N = p.N, T = p.T, UB = p.UB, ntiles = p.ntiles;
  unsigned* ctr = p.ctr + 64 * g;
  unsigned phase = 0;
  const bool tile_wg = j < UB * ntiles;
  const int tub = tile_wg ? j / ntiles : 0, tile = tile_wg ? j % ntiles : 0;
  const int tb = g + kG * tub;
  const int n0 = tile * kPN, nt = tile_wg ? min(kPN, N - n0) : 0;
  const int64_t trb = (int64_t)tb * N;
  const int padl = (kKW - 1) / 2;
  const float u = p.u;
  const auto rRDP = rsrc(p.RDP), rYA = rsrc(p.YA), rDF = rsrc(p.DFH), rDQ = rsrc(p.DQP);

  // ---------------- prologue: resident operands
  // row-dot: thread k holds W0r[k][32j .. 32j+32) for k < 512; the last 32 rows sit in LDS
  float wr0[32];
#pragma unroll
  for (int c = 0; c < 32; ++c) wr0[c] = p.W0r[(int64_t)tid * (4 * kU) + 32 * j + c];
  for (int i = tid; i < (kK0 - kTh) * 32; i += kTh) {
    const int r = i >> 5, c = i & 31;
    wtail[r][c] = p.W0r[(int64_t)(kTh + r) * (4 * kU) + 32 * j + c];
  }
  // query term: wave = unit uu, lane covers d = lane + 64 i of Wq[8j + uu][:]
  float wq[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int d = lane + 64 * i, k = kUW * j + wave;
    wq[i] = d < kD1 ? p.Wq1[k * kD1 + d] : p.Wq2[k * kD2 + (d - kD1)];
  }
  if (tile_wg) {
    for (int i = tid; i < kPN * kD1 / 4; i += kTh) {
      const int r = i / (kD1 / 4), c4 = i - r * (kD1 / 4), n = n0 + r;
      reinterpret_cast<float4*>(&k1s[r][0])[c4] = n < N
          ? reinterpret_cast<const float4*>(p.K1 + (trb + n) * kD1)[c4] : make_float4(0, 0, 0, 0);
    }
    for (int i = tid; i < kPN * kM1 / 4; i += kTh) {
      const int r = i / (kM1 / 4), c4 = i - r * (kM1 / 4), n = n0 + r;
      reinterpret_cast<float4*>(&v1s[r][0])[c4] = n < N
          ? reinterpret_cast<const float4*>(p.V1 + (trb + n) * kM1)[c4] : make_float4(0, 0, 0, 0);
    }
    for (int i = tid; i < kPN * kD2; i += kTh) {
      const int r = i / kD2, c = i - r * kD2, n = n0 + r;
      k2s[r][c] = n < N ? p.K2[(trb + n) * kD2 + c] : 0.f;
      v2s[r][c] = n < N ? p.V2[(trb + n) * kM2 + c] : 0.f;
    }
    for (int d = tid; d < kD1; d += kTh) {
      vv[d] = p.v1[d];
#pragma unroll
      for (int f = 0; f < kF; ++f) locw[f][d] = p.locW[f * kD1 + d];
    }
    if (tid < kD2) vv2[tid] = p.v2[tid];
    if (tid < kKW * kF) cw[tid] = p.convW[tid];
  }
  float dh_c = 0.f, dc_c = 0.f;     // carries of lane tid < UB*8: (ub = tid >> 3, unit 8j + (tid & 7))
  __syncthreads();

  for (int t = T - 1; t >= 0; --t) {
    const bool last = t == T - 1;
    const int slot = t & 1, nslot = (t + 1) & 1;
    // ===================== phase Y: attention backward of the tile
    if (tile_wg) {
      // ---- batch of loads
      // dctx partials: wave w sums rows 4w..4w+3; lane covers float4 columns lane, lane+64
      float4 pr[2][4];
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int c4 = min(lane + 64 * h, kC / 4 - 1);
          pr[h][r] = last ? make_float4(0.f, 0.f, 0.f, 0.f)
                          : ldc4(rRDP, (((slot * B + tb) * kGW + 4 * wave + r) * kK0) / 4 + c4);
        }
      float yn0 = 0.f, yn1 = 0.f, rat = 0.f, rst = 0.f;
      const int n = tid;
      if (n < N) {
        if (!last) {
          yn0 = ldc(rYA, nslot * B * N + tb * N + n);
          yn1 = n + 1 < N ? ldc(rYA, nslot * B * N + tb * N + n + 1) : 0.f;
        }
        rat = p.AL1[((int64_t)(t + 1) * B + tb) * N + n];
        rst = p.S1[((int64_t)(t + 1) * B + tb) * N + n];
      }
      float dfv[3] = {0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const int e = tid + kTh * i;
        if (!last && e < N * kF) dfv[i] = ldc(rDF, ((t + 1) * B + tb) * N * kF + e);
      }
      const float* ctxf = p.REC0 + ((int64_t)(t + 1) * B + tb) * kK0;       // [c1 | c2] of step t
      const float* dl1 = p.RD + ((int64_t)t * B + tb) * kK0;                 // LSTM1's dL/dctx_t
      float cv = 0.f, dv = 0.f;
      if (tid < kC) { cv = ctxf[tid]; dv = dl1[tid]; }
      const float* q = p.Q + ((int64_t)t * B + tb) * kQ;
      if (tid < kD1) qb[tid] = q[tid] + p.b1[tid];
      else if (tid < kQ) q2s[tid - kD1] = q[tid];
      // ---- reduce the dctx partials: per wave over 4 rows, then over the 8 waves
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int c4 = lane + 64 * h;
        if (c4 < kC / 4) {
          float4 a = pr[h][0];
#pragma unroll
          for (int r = 1; r < 4; ++r) { a.x += pr[h][r].x; a.y += pr[h][r].y; a.z += pr[h][r].z; a.w += pr[h][r].w; }
          dcred[wave][c4] = a;
        }
      }
      for (int i = 0; i < 3; ++i) {
        const int e = tid + kTh * i;
        if (e < N * kF) dfall[e] = dfv[i];
      }
      if (tid < nt) {
        const int nn = n0 + tid;
        stv[tid] = p.S1[((int64_t)(t + 1) * B + tb) * N + nn];
        s2v[tid] = p.S2[((int64_t)t * B + tb) * N + nn];
#pragma unroll
        for (int f = 0; f < kF; ++f) fs[tid][f] = p.LOC[(((int64_t)t * B + tb) * N + nn) * kF + f];
      }
      if (tid <= nt) {
        const int nn = n0 - 1 + tid;
        apv[tid] = (nn >= 0 && nn < N) ? p.AL1[((int64_t)t * B + tb) * N + nn] : 0.f;
      }
      __syncthreads();
      float dcc1 = 0.f, dcc2 = 0.f;
      if (tid < kC) {
        const int c4 = tid >> 2, cmp = tid & 3;
        float a = 0.f;
#pragma unroll
        for (int w = 0; w < kWv; ++w) {
          const float4 v = dcred[w][c4];
          a += cmp == 0 ? v.x : cmp == 1 ? v.y : cmp == 2 ? v.z : v.w;
        }
        const float full = dv + a;
        dc[tid] = full;
        if (tile == 0) p.RD[((int64_t)t * B + tb) * kK0 + tid] = full;   // full dL/dctx_t
        if (tid < kM1) dcc1 = full * cv;
        else dcc2 = full * cv;
      }
      // ---- utterance-wide sums s1 = dc1.c1 + sum dalpha_next alpha, s3 = dc2.c2, s2sum
      float s1 = dcc1, s3 = dcc2, s2 = 0.f;
      if (n < N) {
        const float dan = (1.f - u) * yn0 + u * yn1;
        s1 = fmaf(dan, rat, s1);
        float dsn = 0.f;
        if (!last) {
#pragma unroll
          for (int jj = 0; jj < kKW; ++jj) {
            const int m = n - jj + padl;
            if (m < 0 || m >= N) continue;
#pragma unroll
            for (int f = 0; f < kF; ++f) dsn = fmaf(dfall[m * kF + f], cw[jj * kF + f], dsn);
          }
          s2 = rst * dsn;
        }
        const int r = n - n0;
        if (r >= 0 && r < nt) { dsn_t[r] = dsn; dan_t[r] = dan; }
      }
      s1 = wave_sum_dpp(s1);
      s3 = wave_sum_dpp(s3);
      s2 = wave_sum_dpp(s2);
      if (lane == 0) { red[wave] = s1; red[kWv + wave] = s3; red[2 * kWv + wave] = s2; }
      __syncthreads();
      s1 = 0.f; s3 = 0.f; s2 = 0.f;
#pragma unroll
      for (int w = 0; w < kWv; ++w) { s1 += red[w]; s3 += red[kWv + w]; s2 += red[2 * kWv + w]; }
      const float Sa = p.ST[((int64_t)t * B + tb) * 4 + 2];
      const float rSa = 1.f / Sa;
      // ---- tile: DA, DS2 (wave per position, lanes over the value dims) -> de, de2, Y
#pragma unroll
      for (int i = 0; i < kPPW; ++i) {
        const int nl = wave + kWv * i;
        if (nl >= nt) break;
        float a = 0.f;
#pragma unroll
        for (int sdx = 0; sdx < 4; ++sdx) {
          const int d = lane + 64 * sdx;
          a = fmaf(dc[d], v1s[nl][d], a);
        }
        float c = lane < kM2 ? dc[kM1 + lane] * v2s[nl][lane] : 0.f;
        a = wave_sum(a);
        c = wave_sum(c);
        if (lane == 0) {
          const int nn = n0 + nl;
          const float DA = a + dan_t[nl];
          const float st = stv[nl];
          const float da = (DA - s1) * rSa;
          const float prior = (1.f - u) * apv[nl + 1] + u * apv[nl] + 1e-7f;
          const float ds = dsn_t[nl] + da * prior;
          stc(rYA, slot * B * N + tb * N + nn, st * da);
          const float e1v = st * (ds - s2), e2v = s2v[nl] * (c - s3);
          de1[nl] = e1v;
          de2[nl] = e2v;
          p.DE1[((int64_t)t * B + tb) * N + nn] = e1v;
          p.DE2[((int64_t)t * B + tb) * N + nn] = e2v;
        }
      }
      __syncthreads();
      // ---- recompute the tile's energies, back-propagate through tanh
      float aq[4] = {0.f, 0.f, 0.f, 0.f};
      float aq2 = 0.f;
      const float q2 = lane < kD2 ? q2s[lane] : 0.f, v2w = lane < kD2 ? vv2[lane] : 0.f;
#pragma unroll
      for (int i = 0; i < kPPW; ++i) {
        const int nl = wave + kWv * i;
        if (nl >= nt) break;
        const float e = de1[nl];
        float fl[kF], dfp[kF];
#pragma unroll
        for (int f = 0; f < kF; ++f) { fl[f] = fs[nl][f]; dfp[f] = 0.f; }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int d = lane + 64 * k;
          if (d < kD1) {
            float pre = k1s[nl][d] + qb[d];
            float lw[kF];
#pragma unroll
            for (int f = 0; f < kF; ++f) { lw[f] = locw[f][d]; pre = fmaf(fl[f], lw[f], pre); }
            const float z = tanh_fast(pre);
            const float dp = e * vv[d] * (1.f - z * z);
            aq[k] += dp;
#pragma unroll
            for (int f = 0; f < kF; ++f) dfp[f] = fmaf(dp, lw[f], dfp[f]);
          }
        }
#pragma unroll
        for (int f = 0; f < kF; ++f) {
          const float sdf = wave_sum_dpp(dfp[f]);
          if (lane == 0) dfs[nl][f] = sdf;
        }
        if (lane < kD2) {
          const float z = tanh_fast(k2s[nl][lane] + q2);
          aq2 = fmaf(de2[nl] * v2w, 1.f - z * z, aq2);
        }
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) dqred[wave][lane + 64 * k] = aq[k];
      if (lane < 32) dqred[wave][kQ + lane] = aq2;
      __syncthreads();
      if (tid < nt * kF) {
        const int nl = tid / kF, f = tid - nl * kF;
        stc(rDF, ((t * B + tb) * N + n0 + nl) * kF + f, dfs[nl][f]);
      }
      if (tid < kQ) {
        const int o = tid < kD1 ? tid : kQ + (tid - kD1);
        float acc = 0.f;
#pragma unroll
        for (int w = 0; w < kWv; ++w) acc += dqred[w][o];
        stc(rDQ, ((t * B + tb) * ntiles + tile) * kQ + tid, acc);
      }
    }
    group_barrier(ctr, (++phase) * kGW, p.err);

    // ===================== phase Z: the attention RNN's reverse step t for the 8 units
    {
      // ---- batch of loads: recurrent-product partials (own units), dq tile partials
      float rv[2] = {0.f, 0.f};
      const int zub = tid >> 7, zr = (tid >> 2) & 31, zq = tid & 3;
      if (!last && zub < UB) {
        const int base = ((slot * B + g + kG * zub) * kGW + zr) * kK0 + kC + kUW * j + 2 * zq;
        rv[0] = ldc(rRDP, base);
        rv[1] = ldc(rRDP, base + 1);
      }
      // dq_t of utterance (ub = tid >> 6): lane sums float4 column (tid & 63) over the tiles
      float4 dqv[8];
      const int qub = tid >> 6, qc4 = tid & 63;
#pragma unroll
      for (int tl = 0; tl < 8; ++tl) {
        dqv[tl] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (qub < UB && tl < ntiles)
          dqv[tl] = ldc4(rDQ, ((t * B + g + kG * qub) * ntiles + tl) * (kQ / 4) + qc4);
      }
      // pointwise operands of lane tid < UB*8
      const int pub = tid >> 3, puu = tid & 7, punit = kUW * j + puu, pb = g + kG * pub;
      const bool pw = tid < UB * 8;
      float4 g4 = make_float4(0.f, 0.f, 0.f, 0.f);
      float cp = 0.f, dyv = 0.f, mc = 1.f - p.zc, mh = 1.f - p.zh;
      if (pw) {
        const int64_t tbu = ((int64_t)t * B + pb) * kU + punit;
        g4 = reinterpret_cast<const float4*>(p.G0 + ((int64_t)t * B + pb) * 4 * kU)[punit];
        cp = p.C0[((int64_t)t * B + pb) * kU + punit];
        dyv = p.DH0[tbu];
        if (p.mask_c) { mc = p.mask_c[tbu]; mh = p.mask_h[tbu]; }
      }
      // ---- reduce: rec over the 32 partial rows (staged in the dead dq flush buffer), dq over
      //      the tiles (in registers)
      float* rst8 = &dqred[0][0];                       // [UB][32 rows][8 units]
      if (zub < UB) {
        rst8[(zub * 32 + zr) * kUW + 2 * zq] = rv[0];
        rst8[(zub * 32 + zr) * kUW + 2 * zq + 1] = rv[1];
      }
      if (qub < UB) {
        float4 a = dqv[0];
#pragma unroll
        for (int tl = 1; tl < 8; ++tl) {
          a.x += dqv[tl].x; a.y += dqv[tl].y; a.z += dqv[tl].z; a.w += dqv[tl].w;
        }
        reinterpret_cast<float4*>(&dqs[qub][0])[qc4] = a;
      }
      __syncthreads();
      if (tid < UB * kUW) {
        const int ub = tid >> 3, uu = tid & 7;
        float a = 0.f;
#pragma unroll 8
        for (int r = 0; r < kGW; ++r) a += rst8[(ub * 32 + r) * kUW + uu];
        recs[ub][uu] = a;
      }
      __syncthreads();
      // ---- query term dq . Wq[unit]: wave = unit, lanes over d
#pragma unroll
      for (int ub = 0; ub < kUBmax; ++ub) {
        if (ub >= UB) break;
        float a = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) a = fmaf(dqs[ub][lane + 64 * i], wq[i], a);
        a = wave_sum_dpp(a);
        if (lane == 0) qt[ub][wave] = a;
      }
      __syncthreads();
      // ---- pointwise reverse step (lstm.hip lstm_bwd_block, zoneout masks or eval blend)
      if (pw) {
        const float dh_t = recs[pub][puu] + dh_c;
        const float dc_t = dc_c;
        const float gi = g4.x, gj = g4.y, gf = g4.z, go = g4.w;
        const float cn = gf * cp + gi * gj;
        const float tc = tanhf(cn);
        const float dy = dyv + qt[pub][puu];
        const float dhn = dy + mh * dh_t;
        const float dcn = mc * dc_t + dhn * go * (1.f - tc * tc);
        const float d_o = dhn * tc * go * (1.f - go);
        const float d_f = dcn * cp * gf * (1.f - gf);
        const float d_i = dcn * gj * gi * (1.f - gi);
        const float d_j = dcn * gi * (1.f - gj * gj);
        reinterpret_cast<float4*>(p.DG0 + ((int64_t)t * B + pb) * 4 * kU)[punit] =
            make_float4(d_i, d_j, d_f, d_o);
        dgs[pub][4 * puu] = d_i; dgs[pub][4 * puu + 1] = d_j;
        dgs[pub][4 * puu + 2] = d_f; dgs[pub][4 * puu + 3] = d_o;
        dc_c = dcn * gf + (1.f - mc) * dc_t;
        dh_c = (1.f - mh) * dh_t;
      }
      __syncthreads();
      // ---- this workgroup's share of step t-1's input gradients: k = tid (and tid + 512)
      if (t > 0) {
        const int oslot = (t - 1) & 1;
#pragma unroll
        for (int ub = 0; ub < kUBmax; ++ub) {
          if (ub >= UB) break;
          float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
#pragma unroll
          for (int c = 0; c < 32; c += 4) {
            a0 = fmaf(dgs[ub][c], wr0[c], a0);
            a1 = fmaf(dgs[ub][c + 1], wr0[c + 1], a1);
            a2 = fmaf(dgs[ub][c + 2], wr0[c + 2], a2);
            a3 = fmaf(dgs[ub][c + 3], wr0[c + 3], a3);
          }
          const int base = ((oslot * B + g + kG * ub) * kGW + j) * kK0;
          stc(rRDP, base + tid, (a0 + a1) + (a2 + a3));
          if (tid < kK0 - kTh) {
            float a = 0.f;
#pragma unroll 8
            for (int c = 0; c < 32; ++c) a = fmaf(dgs[ub][c], wtail[tid][c], a);
            stc(rRDP, base + kTh + tid, a);
          }
        }
      }
    }
    group_barrier(ctr, (++phase) * kGW, p.err);
  }
}

}  // namespace
}  // namespace sat

using namespace sat;

extern "C" int sat_decoder_attention_bwd(const SatDecAttnBwd* a, void* stream) {
  SAT_CHECK_ARG(a && a->B > 0 && a->N > 0 && a->T > 0, "sat_decoder_attention_bwd: bad sizes");
  SAT_CHECK_ARG(a->U == kU && a->M1 == kM1 && a->M2 == kM2 && a->D1 == kD1 && a->D2 == kD2 &&
                a->F == kF && a->KW == kKW,
                "sat_decoder_attention_bwd: compiled for the self-attention-tacotron shapes");
  SAT_CHECK_ARG(a->B % kG == 0 && a->B / kG <= kUBmax, "sat_decoder_attention_bwd: B in {8,16,24,32}");
  const int ntiles = ceil_div(a->N, kPN);
  SAT_CHECK_ARG((a->B / kG) * ntiles <= kGW && ntiles <= 8,
                "sat_decoder_attention_bwd: (B/8) * ceil(N/32) must be <= 32");
  SAT_CHECK_ARG(a->REC0 && a->C0 && a->G0 && a->Q && a->S1 && a->AL1 && a->S2 && a->ST &&
                a->LOC && a->K1 && a->V1 && a->K2 && a->V2 && a->v1 && a->b1 && a->convW &&
                a->locW && a->v2 && a->W0r && a->Wq1 && a->Wq2 && a->DH0 && a->RD && a->DG0 &&
                a->DE1 && a->DE2 && a->DFH && a->DQP && a->RDP && a->YA && a->ctr && a->err,
                "sat_decoder_attention_bwd: null pointer");
  SAT_CHECK_ARG((a->mask_c == nullptr) == (a->mask_h == nullptr), "sat_decoder_attention_bwd: masks come in pairs");
  int dev = 0, cus = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, dec_attn_bwd_kernel, kTh, 0) != hipSuccess) {
    set_error("sat_decoder_attention_bwd: device query failed");
    return SAT_ERR_HIP;
  }
  SAT_CHECK_ARG((int64_t)cus * per_cu >= kG * kGW,
                "sat_decoder_attention_bwd: fewer than 256 co-resident workgroups on this device");
  DecAttnBwdP p;
  p.B = a->B; p.N = a->N; p.T = a->T; p.ntiles = ntiles; p.UB = a->B / kG;
  p.u = a->u; p.zc = a->zc; p.zh = a->zh;
  p.REC0 = a->REC0; p.C0 = a->C0; p.G0 = a->G0; p.Q = a->Q; p.S1 = a->S1; p.AL1 = a->AL1;
  p.S2 = a->S2; p.ST = a->ST; p.LOC = a->LOC;
  p.K1 = a->K1; p.V1 = a->V1; p.K2 = a->K2; p.V2 = a->V2;
  p.v1 = a->v1; p.b1 = a->b1; p.convW = a->convW; p.locW = a->locW; p.v2 = a->v2;
  p.W0r = a->W0r; p.Wq1 = a->Wq1; p.Wq2 = a->Wq2; p.mask_c = a->mask_c; p.mask_h = a->mask_h;
  p.DH0 = a->DH0; p.RD = a->RD; p.DG0 = a->DG0; p.DE1 = a->DE1; p.DE2 = a->DE2;
  p.DFH = a->DFH; p.DQP = a->DQP; p.RDP = a->RDP; p.YA = a->YA; p.ctr = a->ctr; p.err = a->err;
  hipStream_t s = as_stream(stream);
  if (hipMemsetAsync(a->ctr, 0, kG * 64 * sizeof(unsigned), s) != hipSuccess ||
      hipMemsetAsync(a->err, 0, 2 * sizeof(int), s) != hipSuccess) {
    set_error("sat_decoder_attention_bwd: memset failed");
    return SAT_ERR_HIP;
  }
  hipLaunchKernelGGL(dec_attn_bwd_kernel, dim3(kG * kGW), dim3(kTh), 0, s, p);
  SAT_LAUNCH_CHECK("sat_decoder_attention_bwd");
  return SAT_OK;
}

extern "C" int64_t sat_decoder_attention_bwd_scratch(int32_t B, int32_t N, int64_t* rdp_floats,
                                                     int64_t* ya_floats) {
  if (rdp_floats) *rdp_floats = (int64_t)2 * B * kGW * kK0;
  if (ya_floats) *ya_floats = (int64_t)2 * B * N;
  return kG * 64;
}
