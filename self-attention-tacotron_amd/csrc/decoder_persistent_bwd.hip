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
constexpr int kTh = 512, kWv = 8;            // threads, waves
constexpr int kPadL = (kKW - 1) / 2;         // 4: SAME padding of the location convolution
constexpr int kHL = kKW - 1 - kPadL;         // 5: left halo of the transposed convolution
constexpr int kHalo = kPN + kKW - 1;         // 41 positions of dL/df_{t+1} a tile needs
constexpr int kJF = kKW * kF;                // 50 taps of the location convolution

struct DecAttnBwdP {
  int B, N, T, ntiles, UB, flags;
  float u, zc, zh;
  const float* REC0; const float* C0; const float* G0;
  const float* S1; const float* AL1; const float* S2; const float* ST; const float* LOC;
  const float* V1; const float* V2;
  const float* v1; const float* convW; const float* convb; const float* locW;
  const float* v2;
  const float* W0r; const float* Wq1; const float* Wq2;
  const float* mask_c; const float* mask_h;
  const float* DH0;          // [T][B][U]     dL/dh0'_t from LSTM1 (precomputed)
  const float* ZH;           // [T][B][N][Q]  tanh of the energy pre-activations (forward)
  float* RD;                 // [T][B][K0]    in: [:, :C] LSTM1's dL/dctx_t; out: full dL/dctx_t
  float* DG0;                // [T][B][4U]
  float* DE1; float* DE2;    // [T][B][N]
  float* DFH;                // [T][B][N][F]
  float* DQP;                // [T][B][ntiles][Q]
  float* RDP;                // [2][B][kGW][K0]  row-dot partials (scratch)
  float* YA;                 // [2][B][N] alignment-recursion gradient, then [2][B][8][2] tile sums
  unsigned* ctr; int* err;
  long long* prof;           // [256][16] segment clocks (nullable)
};

// sum over the 4 rows (16-lane groups) of a wave, every lane gets the total (gfx950 swaps)
__device__ __forceinline__ float rows4_sum(float v) {
  const unsigned x = __float_as_uint(v);
  const auto a = __builtin_amdgcn_permlane16_swap(x, x, false, false);
  const float s = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  const unsigned y = __float_as_uint(s);
  const auto b = __builtin_amdgcn_permlane32_swap(y, y, false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

__global__ void __launch_bounds__(kTh) dec_attn_bwd_kernel(DecAttnBwdP p) {
  // resident tile of the memories and the attention parameters
  __shared__ __attribute__((aligned(16))) float v1s[kPN][kM1];
  __shared__ __attribute__((aligned(16))) float v2s[kPN][kM2];
  __shared__ __attribute__((aligned(16))) float vv[kD1];
  __shared__ __attribute__((aligned(16))) float locw[kF][kD1];
  __shared__ __attribute__((aligned(16))) float vv2[kD2];
  __shared__ float cw[kJF], cb[kF];
  // per step
  __shared__ __attribute__((aligned(16))) float dc[kC];
  __shared__ __attribute__((aligned(16))) float4 dcred[kWv][kC / 4];
  __shared__ float ysh[kPN + 1], dfsh[kHalo * kF], pps[16];
  __shared__ float fs[kPN][kF], stv[kPN], s2v[kPN], apv[kPN + 1];
  __shared__ float red[8], red2[kWv][2];
  __shared__ __attribute__((aligned(16))) float dqred[kWv][kQ];
  __shared__ __attribute__((aligned(16))) float dqs[kUBmax][kQ];
  __shared__ __attribute__((aligned(16))) float dgs[kUBmax][32];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = blockIdx.x % kG, j = blockIdx.x / kG;
  const int B = p.B, N = p.N, T = p.T, ntiles = p.ntiles;
  // utterances of this group (b = g + 8 ub < B); a group without any has no hand-off partner
  // outside itself, so it leaves at once
  const int UB = g < B ? (B - 1 - g) / kG + 1 : 0;
  if (UB == 0) return;
  unsigned* ctr = p.ctr + 64 * g;
  unsigned phase = 0;
  const bool tile_wg = j < UB * ntiles;
  const int tub = tile_wg ? j / ntiles : 0, tile = tile_wg ? j % ntiles : 0;
  const int tb = g + kG * tub;
  const int n0 = tile * kPN, nt = tile_wg ? min(kPN, N - n0) : 0;
  const int64_t trb = (int64_t)tb * N;
  const float u = p.u;
  float* PS = p.YA + 2 * B * N;              // [2][B][8][2] tile sums (s1, s2 of step t-1)
  const auto rRDP = rsrc(p.RDP), rYA = rsrc(p.YA), rPS = rsrc(PS), rDF = rsrc(p.DFH),
             rDQ = rsrc(p.DQP);
  // hand-off store policy (persistent.h xcd_local_group): plain stores iff the group is on one XCD
  const bool xl = (p.flags & 1) ? xcd_local_group(p.ctr + kG * 64, g, kG, kGW, p.err) : false;
  // LPP-16 layout of the tile work: 16 lanes per memory position
  const int pl = tid >> 4, part = tid & 15;
  // unit layout of phase Z: (utterance zu, unit 8j + zuu, 16-lane part)
  const int zu = tid >> 7, zuu = (tid >> 4) & 7, zunit = kUW * j + zuu, zb = g + kG * zu;
  const bool zown = zu < UB;                  // this lane group has an utterance
  const bool zlead = zown && part == 0;       // ... and owns its carries / pointwise step

  // ---------------- prologue: resident operands
  // row-dot partials of DG0[t] x W0r[k][32j .. 32j+32), split by consumer:
  //   part A (k < 288: dL/dctx_{t-1}, read by Y(t-1)) right after the pointwise step in Z(t):
  //     waves 4-7, lane (kq, cg) rows 4kq..4kq+3 < 256, cols 8cg..8cg+7; rows 256..287 by
  //     waves 0-3, lane (r = tid >> 3, c8 = tid & 7) cols 4c8..4c8+3 (scalar stores);
  //   part B (k >= 288: the recurrent product of step t-1, read by Z(t-1)) in the shadow of
  //     Y(t-1)'s loads: waves 0-3, lane (kq, cg) rows 288 + 4kq ..
  // A quad's 4 row sums leave as one 16-byte store (scalar write-through stores cost ~6x).
  const int kq = (tid >> 2) & 63, cg = tid & 3;
  const int wrow = tid < 256 ? kC + 4 * kq : 4 * kq;
  float wr[32];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int cc = 0; cc < 8; ++cc)
      wr[r * 8 + cc] = p.W0r[(int64_t)(wrow + r) * (4 * kU) + 32 * j + 8 * cg + cc];
  const int tr = (tid >> 3) & 31, c8 = tid & 7;
  float wt[4];
#pragma unroll
  for (int cc = 0; cc < 4; ++cc) wt[cc] = p.W0r[(int64_t)(256 + tr) * (4 * kU) + 32 * j + 4 * c8 + cc];
  // query term: lane (zuu, part) holds Wq[8j + zuu][16 part .. 16 part + 16)
  float wq[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int d = 16 * part + i;
    wq[i] = d < kD1 ? p.Wq1[zunit * kD1 + d] : p.Wq2[zunit * kD2 + (d - kD1)];
  }
  if (tile_wg) {
    for (int i = tid; i < kPN * kM1 / 4; i += kTh) {
      const int r = i / (kM1 / 4), c4 = i - r * (kM1 / 4), n = n0 + r;
      reinterpret_cast<float4*>(&v1s[r][0])[c4] = n < N
          ? reinterpret_cast<const float4*>(p.V1 + (trb + n) * kM1)[c4] : make_float4(0, 0, 0, 0);
    }
    for (int i = tid; i < kPN * kD2; i += kTh) {
      const int r = i / kD2, c = i - r * kD2, n = n0 + r;
      v2s[r][c] = n < N ? p.V2[(trb + n) * kM2 + c] : 0.f;
    }
    for (int d = tid; d < kD1; d += kTh) {
      vv[d] = p.v1[d];
#pragma unroll
      for (int f = 0; f < kF; ++f) locw[f][d] = p.locW[f * kD1 + d];
    }
    if (tid < kD2) vv2[tid] = p.v2[tid];
    if (tid < kJF) cw[tid] = p.convW[tid];
    if (tid < kF) cb[tid] = p.convb[tid];
  }

  // ---------------- prefetch of the forward histories (plain loads, one step ahead)
  struct YPre { float cv, dv, st, s2, ap, loc, sa; float4 z1[4]; float2 z2; };
  struct ZPre { float4 g4; float cp, dy, mc, mh; };
  auto prefetch_y = [&](int t, YPre& y) {
    const int64_t tb1 = (int64_t)(t + 1) * B + tb, tb0 = (int64_t)t * B + tb;
    y.cv = tid < kC ? p.REC0[tb1 * kK0 + tid] : 0.f;
    y.dv = tid < kC ? p.RD[tb0 * kK0 + tid] : 0.f;
    y.st = tid < nt ? p.S1[tb1 * N + n0 + tid] : 0.f;
    y.s2 = tid < nt ? p.S2[tb0 * N + n0 + tid] : 0.f;
    const int na = n0 - 1 + tid;
    y.ap = (tid <= nt && na >= 0 && na < N) ? p.AL1[tb0 * N + na] : 0.f;
    y.loc = tid < nt * kF ? p.LOC[(tb0 * N + n0) * kF + tid] : 0.f;
    y.sa = p.ST[tb0 * 4 + 2];
    // this lane's energy tanh values: source 1 float4 chunks part + 16k, source 2 dims 2 part..
    const float* zr = p.ZH + (tb0 * N + n0 + pl) * kQ;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int c = part + 16 * k;
      y.z1[k] = (pl < nt && c < kD1 / 4) ? reinterpret_cast<const float4*>(zr)[c]
                                          : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    y.z2 = pl < nt ? reinterpret_cast<const float2*>(zr + kD1)[part] : make_float2(0.f, 0.f);
  };
  auto prefetch_z = [&](int t, ZPre& z) {
    z.g4 = make_float4(0.f, 0.f, 0.f, 0.f);
    z.cp = 0.f; z.dy = 0.f; z.mc = 1.f - p.zc; z.mh = 1.f - p.zh;
    if (zlead) {
      const int64_t r = ((int64_t)t * B + zb) * kU + zunit;
      z.g4 = reinterpret_cast<const float4*>(p.G0 + ((int64_t)t * B + zb) * 4 * kU)[zunit];
      z.cp = p.C0[r];
      z.dy = p.DH0[r];
      if (p.mask_c) { z.mc = p.mask_c[r]; z.mh = p.mask_h[r]; }
    }
  };
  // 4 rows x 8 columns per lane, quad reduction, one 16-byte store per quad (lane cg == ub)
  auto rowdot_quads = [&](int ub, int base) {
    const float4 x0 = *reinterpret_cast<const float4*>(&dgs[ub][8 * cg]);
    const float4 x1 = *reinterpret_cast<const float4*>(&dgs[ub][8 * cg + 4]);
    float acc[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float* w = &wr[r * 8];
      float a0 = x0.x * w[0], a1 = x0.y * w[1];
      a0 = fmaf(x0.z, w[2], a0); a1 = fmaf(x0.w, w[3], a1);
      a0 = fmaf(x1.x, w[4], a0); a1 = fmaf(x1.y, w[5], a1);
      a0 = fmaf(x1.z, w[6], a0); a1 = fmaf(x1.w, w[7], a1);
      acc[r] = a0 + a1;
      acc[r] += dpp<0xB1>(acc[r]);
      acc[r] += dpp<0x4E>(acc[r]);
    }
    if (cg == (ub & 3)) stc4x(xl, rRDP, (base + wrow) / 4, make_float4(acc[0], acc[1], acc[2], acc[3]));
  };
  // part B: the recurrent-product rows (k >= 288) of DG0[t+1] (still in dgs) for step t
  auto rowdot_b = [&](int t) {
    if (t == T - 1 || wave >= 4) return;
#pragma unroll
    for (int ub = 0; ub < kUBmax; ++ub) {
      if (ub >= UB) break;
      rowdot_quads(ub, (((t & 1) * B + g + kG * ub) * kGW + j) * kK0);
    }
  };
  YPre ypre;
  ZPre zpre;
  if (tile_wg) prefetch_y(T - 1, ypre);
  prefetch_z(T - 1, zpre);
  float dh_c = 0.f, dc_c = 0.f;               // carries of the lead lanes
  __syncthreads();
  long long tp[16] = {};
  long long t0 = wall_clock64();
  auto tick = [&](int seg) {
    if (p.prof) {
      const long long t1 = wall_clock64();
      tp[seg] += t1 - t0;
      t0 = t1;
    }
  };

  for (int t = T - 1; t >= 0; --t) {
    const bool last = t == T - 1;
    const int slot = t & 1, nslot = (t + 1) & 1;
    // ===================== phase Y: attention backward of the tile
    if (tile_wg) {
      // ---- sc1 loads: the 32 row-dot partials of dL/dctx_t (wave w: rows 4w..4w+3), Y_{t+1}
      //      and dL/df_{t+1} over the tile plus halo, the tile sums of step t+1
      float4 pr[2][4];
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int c4 = min(lane + 64 * h, kC / 4 - 1);
          pr[h][r] = last ? make_float4(0.f, 0.f, 0.f, 0.f)
                          : ldc4(rRDP, (((slot * B + tb) * kGW + 4 * wave + r) * kK0) / 4 + c4);
        }
      float yh = 0.f, dfh = 0.f, pp = 0.f;
      if (!last) {
        if (tid <= nt && n0 + tid < N) yh = ldc(rYA, (nslot * B + tb) * N + n0 + tid);
        const int m = n0 - kHL + tid / kF;
        if (tid < kHalo * kF && m >= 0 && m < N)
          dfh = ldc(rDF, (((t + 1) * B + tb) * N + n0 - kHL) * kF + tid);
        if (tid < 2 * ntiles) pp = ldc(rPS, ((nslot * B + tb) * 8) * 2 + tid);
      }
      rowdot_b(t);
      // ---- stage in LDS
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
      if (tid <= kPN) ysh[tid] = yh;
      if (tid < kHalo * kF) dfsh[tid] = dfh;
      if (tid < 16) pps[tid] = pp;
      if (tid < kPN) { stv[tid] = ypre.st; s2v[tid] = ypre.s2; }
      if (tid <= kPN) apv[tid] = ypre.ap;
      if (tid < kPN * kF) fs[tid / kF][tid % kF] = ypre.loc;
      const float cv = ypre.cv, dv = ypre.dv, Sa = ypre.sa;
      float4 z1[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) z1[k] = ypre.z1[k];
      const float2 z2 = ypre.z2;
      tick(0);
      __syncthreads();
      // ---- full dL/dctx_t, the forward-context dots dc1.c1, dc2.c2
      float prod = 0.f;
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
        if (tile == 0) p.RD[((int64_t)t * B + tb) * kK0 + tid] = full;
        prod = full * cv;
      }
      {
        const float s = wave_sum_dpp(prod);          // waves 0-3: c1 (256), wave 4: c2 (32)
        if (lane == 0) red[wave] = s;
      }
      // next step's forward histories (consumed after the barrier of this step's Z)
      if (t > 0) prefetch_y(t - 1, ypre);
      tick(1);
      __syncthreads();
      // utterance-wide scalars: s1 = dc1.c1 + sum_n dalpha_next alpha_t, s3 = dc2.c2,
      // s2 = sum_n s_t DSN -- the two sums over n arrive as per-tile partials of step t+1
      float s1 = (red[0] + red[1]) + (red[2] + red[3]), s2 = 0.f;
      const float s3 = red[4];
      for (int tl = 0; tl < ntiles; ++tl) { s1 += pps[2 * tl]; s2 += pps[2 * tl + 1]; }
      const float rSa = 1.f / Sa;
      // ---- 16 lanes per position: DA = dc1.V1[n] (+ dalpha_next), DS2 = dc2.V2[n], DSN
      float a = 0.f, c2 = 0.f, dsn = 0.f;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int d = 4 * (part + 16 * k);
        const float4 dv4 = *reinterpret_cast<const float4*>(&dc[d]);
        const float4 v4 = *reinterpret_cast<const float4*>(&v1s[pl][d]);
        a = fmaf(dv4.x, v4.x, a); a = fmaf(dv4.y, v4.y, a);
        a = fmaf(dv4.z, v4.z, a); a = fmaf(dv4.w, v4.w, a);
      }
      c2 = fmaf(dc[kM1 + 2 * part], v2s[pl][2 * part], c2);
      c2 = fmaf(dc[kM1 + 2 * part + 1], v2s[pl][2 * part + 1], c2);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int jf = part + 16 * k;
        if (jf < kJF) {
          const int jj = jf / kF, f = jf - jj * kF;
          // DSN[n] = sum_{j,f} df_{t+1}[n - j + padl][f] convW[j][f]; halo index n - n0 + kHL
          dsn = fmaf(dfsh[(pl - jj + kPadL + kHL) * kF + f], cw[jf], dsn);
        }
      }
      a = group16_sum(a);
      c2 = group16_sum(c2);
      dsn = group16_sum(dsn);
      const bool valid = pl < nt;
      const float dan = (1.f - u) * ysh[pl] + u * ysh[pl + 1];
      const float DA = a + dan;
      const float st = stv[pl];
      const float da = (DA - s1) * rSa;
      const float prior = (1.f - u) * apv[pl + 1] + u * apv[pl];
      const float ds = dsn + da * (prior + 1e-7f);
      const float yv = st * da;
      const float e1v = st * (ds - s2), e2v = s2v[pl] * (c2 - s3);
      if (valid) {
        const int64_t o = ((int64_t)t * B + tb) * N + n0 + pl;
        if (part == 0) stcx(xl, rYA, (slot * B + tb) * N + n0 + pl, yv);
        else if (part == 1) p.DE1[o] = e1v;
        else if (part == 2) p.DE2[o] = e2v;
      }
      tick(2);
      // ---- back-propagate through the energies' tanh (kept by the forward): dp = de v (1 - z^2)
      float fl[kF], dfp[kF];
#pragma unroll
      for (int f = 0; f < kF; ++f) { fl[f] = fs[pl][f]; dfp[f] = 0.f; }
      float4 dq4[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        dq4[k] = make_float4(0.f, 0.f, 0.f, 0.f);
        const int c = part + 16 * k;
        if (c < kD1 / 4) {
          const int d = 4 * c;
          const float4 vw = *reinterpret_cast<const float4*>(&vv[d]);
          const float4 z = z1[k];
          float4 dp;
          dp.x = e1v * vw.x * fmaf(-z.x, z.x, 1.f); dp.y = e1v * vw.y * fmaf(-z.y, z.y, 1.f);
          dp.z = e1v * vw.z * fmaf(-z.z, z.z, 1.f); dp.w = e1v * vw.w * fmaf(-z.w, z.w, 1.f);
          dq4[k] = dp;
#pragma unroll
          for (int f = 0; f < kF; ++f) {
            const float4 lw = *reinterpret_cast<const float4*>(&locw[f][d]);
            dfp[f] = fmaf(dp.x, lw.x, dfp[f]); dfp[f] = fmaf(dp.y, lw.y, dfp[f]);
            dfp[f] = fmaf(dp.z, lw.z, dfp[f]); dfp[f] = fmaf(dp.w, lw.w, dfp[f]);
          }
        }
      }
      float dq2[2];
      dq2[0] = e2v * vv2[2 * part] * fmaf(-z2.x, z2.x, 1.f);
      dq2[1] = e2v * vv2[2 * part + 1] * fmaf(-z2.y, z2.y, 1.f);
      // dL/df_t of the position (-> DSN of step t-1) and its tile sums for step t-1:
      // P1 = sum_n Y_t[n] (prior_t[n] - 1e-7) (= sum_n dalpha_{t-1}[n] alpha_{t-1}[n]),
      // P2 = sum_n sum_f dL/df_t[n][f] (f_t[n][f] - convb[f]) (= sum_n s_{t-1}[n] DSN_{t-1}[n])
      float p2 = 0.f;
#pragma unroll
      for (int f = 0; f < kF; ++f) {
        const float v = group16_sum(dfp[f]);
        if (valid && part == f) stcx(xl, rDF, (((t * B + tb) * N) + n0 + pl) * kF + f, v);
        p2 = fmaf(v, fl[f] - cb[f], p2);
      }
      float p1 = valid ? yv * prior : 0.f;
      p2 = valid ? p2 : 0.f;
      p1 = rows4_sum(p1);
      p2 = rows4_sum(p2);
      if (lane == 0) { red2[wave][0] = p1; red2[wave][1] = p2; }
      // dq: sum over the 4 positions of the wave, then over the 8 waves in LDS
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        dq4[k].x = rows4_sum(dq4[k].x); dq4[k].y = rows4_sum(dq4[k].y);
        dq4[k].z = rows4_sum(dq4[k].z); dq4[k].w = rows4_sum(dq4[k].w);
      }
      dq2[0] = rows4_sum(dq2[0]);
      dq2[1] = rows4_sum(dq2[1]);
      if (lane < 16) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int c = part + 16 * k;
          if (c < kD1 / 4) *reinterpret_cast<float4*>(&dqred[wave][4 * c]) = dq4[k];
        }
        dqred[wave][kD1 + 2 * part] = dq2[0];
        dqred[wave][kD1 + 2 * part + 1] = dq2[1];
      }
      __syncthreads();
      if (tid < kQ / 4) {
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int w = 0; w < kWv; ++w) {
          const float4 v = *reinterpret_cast<const float4*>(&dqred[w][4 * tid]);
          acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
        }
        stc4x(xl, rDQ, ((t * B + tb) * ntiles + tile) * (kQ / 4) + tid, acc);
      } else if (tid >= kQ && tid < kQ + 2) {
        const int i = tid - kQ;
        float acc = 0.f;
#pragma unroll
        for (int w = 0; w < kWv; ++w) acc += red2[w][i];
        stcx(xl, rPS, ((slot * B + tb) * 8 + tile) * 2 + i, acc);
      }
      tick(3);
    } else {
      rowdot_b(t);
    }
    group_barrier(ctr, (++phase) * kGW, p.err);
    tick(4);

    // ===================== phase Z: the attention RNN's reverse step t for the 8 units
    {
      // ---- sc1 loads: recurrent-product partials (rows 2 part, 2 part + 1 of unit zunit),
      //      dq_t tile partials (utterance tid >> 6, float4 column tid & 63)
      float r0 = 0.f, r1 = 0.f;
      if (!last && zown) {
        const int base = ((slot * B + zb) * kGW + 2 * part) * kK0 + kC + zunit;
        r0 = ldc(rRDP, base);
        r1 = ldc(rRDP, base + kK0);
      }
      float4 dqv[8];
      const int qub = tid >> 6, qc4 = tid & 63;
#pragma unroll
      for (int tl = 0; tl < 8; ++tl) {
        dqv[tl] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (qub < UB && tl < ntiles)
          dqv[tl] = ldc4(rDQ, ((t * B + g + kG * qub) * ntiles + tl) * (kQ / 4) + qc4);
      }
      const ZPre z = zpre;
      if (t > 0) prefetch_z(t - 1, zpre);
      if (qub < UB) {
        float4 a = dqv[0];
#pragma unroll
        for (int tl = 1; tl < 8; ++tl) {
          a.x += dqv[tl].x; a.y += dqv[tl].y; a.z += dqv[tl].z; a.w += dqv[tl].w;
        }
        reinterpret_cast<float4*>(&dqs[qub][0])[qc4] = a;
      }
      tick(5);
      __syncthreads();
      // ---- recurrent product and query term of (zu, zunit): 16 lanes, then the lead lane's
      //      pointwise reverse step (lstm.hip lstm_bwd_block)
      float qt = 0.f;
      if (zown) {
        const float* dq = &dqs[zu][16 * part];
#pragma unroll
        for (int i = 0; i < 16; i += 4) {
          const float4 v = *reinterpret_cast<const float4*>(dq + i);
          qt = fmaf(v.x, wq[i], qt); qt = fmaf(v.y, wq[i + 1], qt);
          qt = fmaf(v.z, wq[i + 2], qt); qt = fmaf(v.w, wq[i + 3], qt);
        }
      }
      qt = group16_sum(qt);
      const float rec = group16_sum(r0 + r1);
      tick(8);
      if (zlead) {
        const float dh_t = rec + dh_c;
        const float dc_t = dc_c;
        const float gi = z.g4.x, gj = z.g4.y, gf = z.g4.z, go = z.g4.w;
        const float cn = gf * z.cp + gi * gj;
        const float tc = tanh_lstm(cn);
        const float dhn = z.dy + qt + z.mh * dh_t;
        const float dcn = z.mc * dc_t + dhn * go * (1.f - tc * tc);
        const float d_o = dhn * tc * go * (1.f - go);
        const float d_f = dcn * z.cp * gf * (1.f - gf);
        const float d_i = dcn * gj * gi * (1.f - gi);
        const float d_j = dcn * gi * (1.f - gj * gj);
        const float4 dg = make_float4(d_i, d_j, d_f, d_o);
        reinterpret_cast<float4*>(p.DG0 + ((int64_t)t * B + zb) * 4 * kU)[zunit] = dg;
        *reinterpret_cast<float4*>(&dgs[zu][4 * zuu]) = dg;
        dc_c = dcn * gf + (1.f - z.mc) * dc_t;
        dh_c = (1.f - z.mh) * dh_t;
      }
      tick(9);
      __syncthreads();
      tick(10);
      // ---- part A of this workgroup's share of step t-1's input gradients (k < 288)
      if (t > 0) {
        const int oslot = (t - 1) & 1;
#pragma unroll
        for (int ub = 0; ub < kUBmax; ++ub) {
          if (ub >= UB) break;
          const int base = ((oslot * B + g + kG * ub) * kGW + j) * kK0;
          if (wave >= 4) rowdot_quads(ub, base);
          else {
            const float4 x = *reinterpret_cast<const float4*>(&dgs[ub][4 * c8]);
            float a = x.x * wt[0];
            a = fmaf(x.y, wt[1], a); a = fmaf(x.z, wt[2], a); a = fmaf(x.w, wt[3], a);
            a = group8_sum(a);
            if (c8 == 0) stcx(xl, rRDP, base + 256 + tr, a);
          }
        }
      }
      tick(6);
    }
    group_barrier(ctr, (++phase) * kGW, p.err);
    tick(7);
  }
  if (p.prof && tid == 0)
    for (int i = 0; i < 16; ++i) p.prof[blockIdx.x * 16 + i] = tp[i];
}

}  // namespace
}  // namespace sat

using namespace sat;

extern "C" int sat_decoder_attention_bwd(const SatDecAttnBwd* a, void* stream) {
  SAT_CHECK_ARG(a && a->B > 0 && a->N > 0 && a->T > 0, "sat_decoder_attention_bwd: bad sizes");
  if (dec_attn_bwd8_eligible(a)) {               // one utterance per 8 workgroups (N <= 256)
    SAT_CHECK_ARG(a->REC0 && a->C0 && a->G0 && a->S1 && a->AL1 && a->S2 && a->ST && a->LOC &&
                  a->V1 && a->V2 && a->v1 && a->convW && a->convb && a->locW && a->v2 &&
                  a->W0r && a->Wq1 && a->Wq2 && a->DH0 && a->ZH && a->RD && a->DG0 && a->DE1 &&
                  a->DE2 && a->DFH && a->DQP && a->RDP && a->err,
                  "sat_decoder_attention_bwd: null pointer");
    SAT_CHECK_ARG((a->mask_c == nullptr) == (a->mask_h == nullptr), "sat_decoder_attention_bwd: masks come in pairs");
    SAT_CHECK_ARG(aligned16(a->W0r) && aligned16(a->G0) && aligned16(a->DG0) && aligned16(a->ZH) &&
                  aligned16(a->DQP) && aligned16(a->RDP) && aligned16(a->REC0),
                  "sat_decoder_attention_bwd: 16-byte aligned operands");
    return dec_attn_bwd8_launch(a, as_stream(stream));
  }
  SAT_CHECK_ARG(a->U == kU && a->M1 == kM1 && a->M2 == kM2 && a->D1 == kD1 && a->D2 == kD2 &&
                a->F == kF && a->KW == kKW,
                "sat_decoder_attention_bwd: compiled for the self-attention-tacotron shapes");
  SAT_CHECK_ARG(a->B <= kG * kUBmax, "sat_decoder_attention_bwd: B <= 32");
  const int ntiles = ceil_div(a->N, kPN);
  SAT_CHECK_ARG(ceil_div(a->B, kG) * ntiles <= kGW && ntiles <= 8,
                "sat_decoder_attention_bwd: ceil(B/8) * ceil(N/32) must be <= 32");
  SAT_CHECK_ARG(a->REC0 && a->C0 && a->G0 && a->S1 && a->AL1 && a->S2 && a->ST &&
                a->LOC && a->V1 && a->V2 && a->v1 && a->convW && a->convb &&
                a->locW && a->v2 && a->W0r && a->Wq1 && a->Wq2 && a->DH0 && a->ZH && a->RD && a->DG0 &&
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
  p.B = a->B; p.N = a->N; p.T = a->T; p.ntiles = ntiles; p.UB = ceil_div(a->B, kG);
  p.u = a->u; p.zc = a->zc; p.zh = a->zh;
  p.REC0 = a->REC0; p.C0 = a->C0; p.G0 = a->G0; p.S1 = a->S1; p.AL1 = a->AL1;
  p.S2 = a->S2; p.ST = a->ST; p.LOC = a->LOC;
  p.V1 = a->V1; p.V2 = a->V2;
  p.v1 = a->v1; p.convW = a->convW; p.convb = a->convb; p.locW = a->locW;
  p.v2 = a->v2;
  p.W0r = a->W0r; p.Wq1 = a->Wq1; p.Wq2 = a->Wq2; p.mask_c = a->mask_c; p.mask_h = a->mask_h;
  p.DH0 = a->DH0; p.ZH = a->ZH; p.RD = a->RD; p.DG0 = a->DG0; p.DE1 = a->DE1; p.DE2 = a->DE2;
  p.DFH = a->DFH; p.DQP = a->DQP; p.RDP = a->RDP; p.YA = a->YA; p.ctr = a->ctr; p.err = a->err; p.flags = xcd_local_env();
  p.prof = reinterpret_cast<long long*>(a->prof);
  hipStream_t s = as_stream(stream);
  if (zero_ranges(s, a->ctr, (kG * 64 + kG * kGW), a->err, 2) != hipSuccess) {
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
  if (ya_floats) *ya_floats = (int64_t)2 * B * N + (int64_t)2 * B * 8 * 2;
  return kG * 64 + kG * kGW;   // group counters + XID
}
