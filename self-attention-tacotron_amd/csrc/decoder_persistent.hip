// Persistent attention chain of the decoder forward: ALL T' steps of
//   attention RNN (ZoneoutLSTM 256)  ->  query layers  ->  dual-source attention (+ combine)
// in ONE launch (DualSourceAttentionRNN, modules/module.py:1017-1048, with ForwardAttention
// modules/forward_attention.py:88-122 and TF BahdanauAttention as attention2; zoneout LSTM as in
// lstm.hip; the arithmetic is the per-step kernels' -- attention.hip / lstm.hip -- restated).
//
// Why: per step the launch-based chain is 4 dependent launches (LSTM step, query row-dot, tile
// kernel, combine), each paying a ~1.5 us boundary plus a cold reload of its operands (the L2
// does not survive a boundary): K1/V1 (14 MB) and the LSTM weights (2.2 MB) stream from
// MALL/HBM 500 times.  Here each (utterance, 32-position tile) K1/V1/K2/V2 slice (68 KB) lives
// in one workgroup's LDS and each workgroup's 32 LSTM gate columns (68 floats per lane) and
// query rows live in registers for the whole decode; a step costs two in-kernel group barriers
// (~1.3-1.8 us each, measured by tools/probes/handoff_probe) plus on-chip arithmetic.
//
// Layout: 8 groups x 32 workgroups (256, one per CU).  Group g = blockIdx % 8 owns utterances
// b = g + 8*ub (ub < B/8 <= 4) -- workgroups b, b+8, ... share an XCD under the observed
// round-robin placement, so a group's hand-offs stay in one L2 (speed only; correctness never
// depends on placement).  Workgroup j = blockIdx / 8 of the group owns LSTM units [8j, 8j+8)
// and, if j < UB*ntiles, tile (ub = j / ntiles, tile = j % ntiles).  Per step t:
//   A: combine step t-1's tile partials (every workgroup, redundantly: the context is the LSTM
//      input); tile workgroups normalise step t-1 on their window (s_{t-1}, alpha_{t-1} from the
//      raw energies and the combine statistics); LSTM0 step t for the 8 units x UB utterances;
//      the units' query contribution q_part[j] = h0'_t[8 units] [Wq1 | Wq2][8 units, :]
//   C: tile workgroups sum the 32 query partials of their utterance, location features,
//      energies from LDS K1/K2, tile statistics and unnormalised partial contexts
// Every cross-workgroup operand of a phase is loaded in one batch at the phase start.
// Hand-offs (guide: MI355X_MICROARCH.md inter-workgroup visibility, "sc1 loads in place of the
// acquire" table row 1): producers store with sc1 and drain (s_waitcnt vmcnt(0)) before the
// workgroup barrier; one lane arrives on the group counter (agent-scope atomic) and polls it
// with sc1 loads; every load of another workgroup's bytes is an sc1 load.  Every spin is
// bounded: a timeout raises err[0] and all later barriers fall through, so the grid always
// drains.  All histories the backward needs are written exactly as the launch-based path.
#include "sat_common.h"
#include "persistent.h"

namespace sat {
namespace {

constexpr int kG = 8;          // groups
constexpr int kGW = 32;        // workgroups per group
constexpr int kPN = 32;        // tile positions
constexpr int kUBmax = 4;      // utterances per group
constexpr int kU = 256, kM1 = 256, kM2 = 32, kD1 = 224, kD2 = 32, kF = 5, kKW = 10;
constexpr int kK0 = kM1 + kM2 + kU;            // attention-RNN recurrent input [c1 | c2 | h0]
constexpr int kPST = 8 + kM1 + kM2;            // partial record stride (floats, 16-B multiple)
constexpr int kW0 = kK0 / 8;                   // recurrent weights per lane (k-slice of 8)
constexpr int kQ = kD1 + kD2;                  // query width (= U here)
constexpr int kUW = kU / kGW;                  // units per workgroup (8)
static_assert(kK0 % 8 == 0 && kU % kGW == 0 && kQ == 256 && kPST % 4 == 0, "layout");

struct DecAttnP {
  int B, N, T, ntiles, UB;
  float u, zc, zh;
  const float* X0;                                   // [T][B][4U] prenet part + bias
  const float* W0r;                                  // [K0][U][4]
  const float* Wq1; const float* Wq2;                // [U][D1], [U][D2]
  const float* K1; const float* V1; const float* K2; const float* V2;
  const int64_t* lengths;
  const float* v1; const float* b1; const float* convW; const float* convb; const float* locW;
  const float* v2;
  const float* mask_c; const float* mask_h;          // [T][B][U] or null (eval blend)
  float* REC0; float* C0; float* H0RAW; float* G0; float* Q;
  float* S1; float* AL1; float* S2; float* ST; float* LOC;
  float* ZH;                                         // [T][B][N][D1+D2] energy tanh (nullable)
  float* E;                                          // [2][B][2][N] raw energies
  float* PART;                                       // [2][B][ntiles][kPST]
  float* QP;                                         // [2][B][kGW][kQ] query partials
  unsigned* ctr;                                     // [kG * 64], zero at launch
  int* err;                                          // [2]
  long long* prof;                                   // [256][8] segment clocks (nullable)
};

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + __expf(-x)); }

// Per step t, two phases separated by group barriers:
//   A: every workgroup combines step t-1's tile partials (the context is the LSTM input), tile
//      workgroups normalise step t-1 on their window, then the LSTM0 step for the workgroup's
//      8 units and their query contribution q_part[j] = h0'[8 units] Wq[8 units, :];
//   C: tile workgroups sum the 32 query partials of their utterance and run the tile.
// Every cross-workgroup operand of a phase is loaded in one batch at the phase start.
__global__ void __launch_bounds__(256) dec_attn_fwd_kernel(DecAttnP p) {
  __shared__ __attribute__((aligned(16))) float k1s[kPN][kD1];
  __shared__ __attribute__((aligned(16))) float v1s[kPN][kM1];
  __shared__ __attribute__((aligned(16))) float k2s[kPN][kD2];
  __shared__ __attribute__((aligned(16))) float v2s[kPN][kM2];
  __shared__ __attribute__((aligned(16))) float rin[kUBmax][kK0];
  __shared__ float gsh[kUBmax][32];
  __shared__ float hown[kUBmax][kUW];
  __shared__ float stat[kUBmax][8];
  __shared__ __attribute__((aligned(16))) float4 qred[4][64];
  // tile phase
  __shared__ __attribute__((aligned(16))) float qb[kD1];
  __shared__ __attribute__((aligned(16))) float vv[kD1];
  __shared__ __attribute__((aligned(16))) float locw[kF][kD1];
  __shared__ __attribute__((aligned(16))) float q2s[kD2];
  __shared__ __attribute__((aligned(16))) float vv2[kD2];
  __shared__ float cw[kKW * kF + kF];
  __shared__ float fs[kPN][kF];
  __shared__ float sp[kPN + kKW], ap[kPN + 1];
  __shared__ float ew[kPN + kKW], e2w[kPN], aw[kPN + 2];
  __shared__ float e1s[kPN], e2s[kPN], w1s[kPN], w2s[kPN];
  __shared__ __attribute__((aligned(16))) float4 cred[4][64];
  __shared__ __attribute__((aligned(16))) float4 c2red[kPN][8];
  __shared__ float red[8];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = blockIdx.x % kG, j = blockIdx.x / kG;
  const int B = p.B, N = p.N, T = p.T, UB = p.UB, ntiles = p.ntiles;
  unsigned* ctr = p.ctr + 64 * g;
  unsigned phase = 0;
  const bool tile_wg = j < UB * ntiles;
  const int tub = tile_wg ? j / ntiles : 0, tile = tile_wg ? j % ntiles : 0;
  const int tb = g + kG * tub;                      // utterance of this workgroup's tile
  const int n0 = tile * kPN, nt = tile_wg ? min(kPN, N - n0) : 0;
  const int64_t trb = (int64_t)tb * N;
  const int padl = (kKW - 1) / 2;
  const int span = nt + kKW - 1;
  const float u = p.u;
  const auto rREC = rsrc(p.REC0), rAL = rsrc(p.AL1), rE = rsrc(p.E), rPT = rsrc(p.PART);
  const auto rQP = rsrc(p.QP);

  // ---------------- prologue: resident operands
  // LSTM: lane (column c = tid >> 3, k-block ks = tid & 7) holds W0r[68 ks + kk][32j + c], so
  // its recurrent inputs are 17 contiguous float4 of rin (conflict-free: 68 % 32 = 4 banks apart)
  const int cc = tid >> 3, ks = tid & 7;
  float w0[kW0];
#pragma unroll
  for (int kk = 0; kk < kW0; ++kk) w0[kk] = p.W0r[(int64_t)(kW0 * ks + kk) * (4 * kU) + 32 * j + cc];
  // query partial: lane = output column, holds Wq[8j + uu][col] for its 8 units
  float wq[kUW];
#pragma unroll
  for (int uu = 0; uu < kUW; ++uu) {
    const int k = kUW * j + uu;
    wq[uu] = tid < kD1 ? p.Wq1[k * kD1 + tid] : p.Wq2[k * kD2 + (tid - kD1)];
  }
  if (tile_wg) {
    for (int i = tid; i < kPN * kD1 / 4; i += 256) {
      const int r = i / (kD1 / 4), c4 = i - r * (kD1 / 4);
      const int n = n0 + r;
      reinterpret_cast<float4*>(&k1s[r][0])[c4] = n < N
          ? reinterpret_cast<const float4*>(p.K1 + (trb + n) * kD1)[c4] : make_float4(0, 0, 0, 0);
    }
    for (int i = tid; i < kPN * kM1 / 4; i += 256) {
      const int r = i / (kM1 / 4), c4 = i - r * (kM1 / 4);
      const int n = n0 + r;
      reinterpret_cast<float4*>(&v1s[r][0])[c4] = n < N
          ? reinterpret_cast<const float4*>(p.V1 + (trb + n) * kM1)[c4] : make_float4(0, 0, 0, 0);
    }
    for (int i = tid; i < kPN * kD2; i += 256) {
      const int r = i / kD2, c = i - r * kD2, n = n0 + r;
      k2s[r][c] = n < N ? p.K2[(trb + n) * kD2 + c] : 0.f;
      v2s[r][c] = n < N ? p.V2[(trb + n) * kM2 + c] : 0.f;
    }
    for (int d = tid; d < kD1; d += 256) {
      vv[d] = p.v1[d];
#pragma unroll
      for (int f = 0; f < kF; ++f) locw[f][d] = p.locW[f * kD1 + d];
    }
    if (tid < kD2) vv2[tid] = p.v2[tid];
    if (tid < kKW * kF) cw[tid] = p.convW[tid];
    if (tid < kF) cw[kKW * kF + tid] = p.convb[tid];
  }
  float c_own = 0.f, h_own = 0.f;   // lane tid < UB*8: (ub = tid >> 3, unit 8j + (tid & 7))
  const int len = tile_wg ? (int)p.lengths[tb] : 0;
  __syncthreads();

  // ---- phase A of step t (combining step s = t - 1); t == T is the epilogue (no LSTM)
  long long tp[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  long long t0 = wall_clock64();
  auto tick = [&](int seg) {
    if (p.prof) {
      const long long t1 = wall_clock64();
      tp[seg] += t1 - t0;
      t0 = t1;
    }
  };
  auto phase_a = [&](int t) {
    const int s = t - 1;
    // ======== batch of loads: partials of step s (wave ub), h0_{t-1}, tile windows, X0/masks
    float4 ph[2][8];
    float hd[5];
    const int pbase = ((s & 1) * B + g + kG * wave) * ntiles * kPST;   // floats
    if (t > 0 && wave < UB) {
#pragma unroll
      for (int jt = 0; jt < 8; ++jt) {
        const int jc = min(jt, ntiles - 1);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int c4 = min(lane + 64 * h, (kM1 + kM2) / 4 - 1);
          ph[h][jt] = ldc4(rPT, (pbase + jc * kPST + 8) / 4 + c4);
        }
      }
      const int jl = min(lane, ntiles - 1);
#pragma unroll
      for (int q = 0; q < 5; ++q) hd[q] = ldc(rPT, pbase + jl * kPST + q);
    }
    float4 h4 = make_float4(0.f, 0.f, 0.f, 0.f);
    const int hub = tid >> 6, hk = 4 * (tid & 63);
    if (t > 0 && t < p.T + 1 && hub < UB)
      h4 = ldc4(rREC, ((t * B + g + kG * hub) * kK0 + kM1 + kM2 + hk) / 4);
    float ewv = 0.f, e2v = 0.f, awv = 0.f;
    if (tile_wg && t > 0) {
      const int eb = (((s & 1) * B + tb) * 2) * N;
      if (tid < span) {
        const int n = n0 - padl + tid;
        ewv = (n >= 0 && n < N) ? ldc(rE, eb + n) : -INFINITY;
      } else if (tid >= 64 && tid < 64 + nt) {
        e2v = ldc(rE, eb + N + n0 + tid - 64);
      } else if (tid >= 128 && tid < 128 + nt + 2) {
        const int n = n0 - 2 + tid - 128;                       // alpha_{t-2} window
        awv = n >= 0 ? ldc(rAL, ((t - 1) * B + tb) * N + n) : 0.f;
      }
    }
    float4 xp = make_float4(0.f, 0.f, 0.f, 0.f);
    float mcv = 1.f - p.zc, mhv = 1.f - p.zh;
    const int pub = tid >> 3, puu = tid & 7, punit = kUW * j + puu, pb = g + kG * pub;
    const bool pw = t < T && tid < UB * 8;
    if (pw) {
      xp = reinterpret_cast<const float4*>(p.X0 + ((int64_t)t * B + pb) * 4 * kU)[punit];
      if (p.mask_c) {
        mcv = p.mask_c[((int64_t)t * B + pb) * kU + punit];
        mhv = p.mask_h[((int64_t)t * B + pb) * kU + punit];
      }
    }
    // ======== combine step s (one wave per utterance)
    if (t > 0 && wave < UB) {
      const int ub = wave, b = g + kG * ub;
      const bool on = lane < ntiles;
      const float hm1 = on ? hd[0] : -INFINITY, hz1 = on ? hd[1] : 0.f, ha1 = on ? hd[2] : 0.f;
      const float hm2 = on ? hd[3] : -INFINITY, hz2 = on ? hd[4] : 0.f;
      const float M1 = wave_max(hm1), M2 = wave_max(hm2);
      const float s1 = (hm1 == -INFINITY) ? 0.f : __expf(hm1 - M1);
      const float s2 = (hm2 == -INFINITY) ? 0.f : __expf(hm2 - M2);
      const float Z1 = wave_sum(hz1 * s1), A1 = wave_sum(ha1 * s1), Z2 = wave_sum(hz2 * s2);
      const float inv1 = 1.f / A1, inv2 = 1.f / Z2;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int c4 = lane + 64 * h;
        if (c4 >= (kM1 + kM2) / 4) break;
        const bool first = c4 < kM1 / 4;
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int jt = 0; jt < 8; ++jt) {          // lane jt's scale, broadcast by readlane
          const float w1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(s1), jt));
          const float w2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(s2), jt));
          const float w = jt < ntiles ? (first ? w1 : w2) : 0.f;
          acc.x = fmaf(ph[h][jt].x, w, acc.x); acc.y = fmaf(ph[h][jt].y, w, acc.y);
          acc.z = fmaf(ph[h][jt].z, w, acc.z); acc.w = fmaf(ph[h][jt].w, w, acc.w);
        }
        const float inv = first ? inv1 : inv2;
        acc.x *= inv; acc.y *= inv; acc.z *= inv; acc.w *= inv;
        reinterpret_cast<float4*>(&rin[ub][0])[c4] = acc;
        if (j == 0) reinterpret_cast<float4*>(p.REC0 + ((int64_t)t * B + b) * kK0)[c4] = acc;
      }
      if (lane == 0) {
        stat[ub][0] = M1; stat[ub][1] = Z1; stat[ub][2] = A1; stat[ub][3] = M2; stat[ub][4] = Z2;
        if (j == 0) {
          float* st = p.ST + ((int64_t)s * B + b) * 4;
          st[0] = M1; st[1] = Z1; st[2] = A1 / Z1; st[3] = Z2;
        }
      }
    } else if (t == 0 && wave < UB) {
      for (int d = lane; d < kM1 + kM2; d += 64) rin[wave][d] = 0.f;
    }
    if (hub < UB) *reinterpret_cast<float4*>(&rin[hub][kM1 + kM2 + hk]) = h4;
    tick(4);
    if (tile_wg) {
      if (tid < span) ew[tid] = ewv;
      else if (tid >= 64 && tid < 64 + nt) e2w[tid - 64] = e2v;
      else if (tid >= 128 && tid < 128 + nt + 2) aw[tid - 128] = awv;
    }
    __syncthreads();
    // ======== tile workgroups: s_{t-1} on the conv window, alpha_{t-1} on [n0-1, n0+nt)
    if (tile_wg) {
      if (t == 0) {
        if (tid < span) {
          const int n = n0 - padl + tid;
          sp[tid] = (n >= 0 && n < N) ? p.S1[trb + n] : 0.f;          // host rows
        }
        if (tid <= nt) ap[tid] = (n0 - 1 + tid >= 0) ? p.AL1[trb + n0 - 1 + tid] : 0.f;
      } else {
        const float M1 = stat[tub][0], Z1 = stat[tub][1], A1 = stat[tub][2];
        const float M2 = stat[tub][3], Z2 = stat[tub][4];
        if (tid < span) {
          const float e = ew[tid];
          sp[tid] = e == -INFINITY ? 0.f : __expf(e - M1) / Z1;
        }
        if (tid <= nt) {
          const int n = n0 - 1 + tid;
          float av = 0.f;
          if (n >= 0) {
            const float e = ew[tid + padl - 1];
            const float pe = e == -INFINITY ? 0.f : __expf(e - M1);
            av = ((1.f - u) * aw[tid + 1] + u * aw[tid] + 1e-7f) * pe / A1;
          }
          ap[tid] = av;
        }
        __syncthreads();
        if (tid < nt) {   // own positions of the history rows s_{t-1}, alpha_{t-1}, s2_{t-1}
          const int n = n0 + tid;
          p.S1[((int64_t)t * B + tb) * N + n] = sp[tid + padl];
          stc(rAL, (t * B + tb) * N + n, ap[tid + 1]);
          const float e = e2w[tid];
          p.S2[((int64_t)s * B + tb) * N + n] = e == -INFINITY ? 0.f : __expf(e - M2) / Z2;
        }
      }
    }
    if (t == T) return;
    __syncthreads();
    tick(5);
    // ======== LSTM0 step t: gates for 32 columns x UB utterances
    {
      float acc[kUBmax] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
      for (int ub = 0; ub < kUBmax; ++ub) {        // not unrolled: 17 float4 of rin in flight
        if (ub >= UB) break;
        const float4* r4 = reinterpret_cast<const float4*>(&rin[ub][kW0 * ks]);
        float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;   // four independent FMA chains
#pragma unroll
        for (int k4 = 0; k4 < kW0 / 4; ++k4) {      // fully unrolled: w0 stays in registers
          const float4 x = r4[k4];
          a0 = fmaf(x.x, w0[4 * k4], a0);
          a1 = fmaf(x.y, w0[4 * k4 + 1], a1);
          a2 = fmaf(x.z, w0[4 * k4 + 2], a2);
          a3 = fmaf(x.w, w0[4 * k4 + 3], a3);
        }
        acc[ub] = (a0 + a1) + (a2 + a3);
      }
#pragma unroll
      for (int ub = 0; ub < kUBmax; ++ub) {
        float a = acc[ub];
        a += __shfl_xor(a, 1, 64);
        a += __shfl_xor(a, 2, 64);
        a += __shfl_xor(a, 4, 64);
        if (ks == 0 && ub < UB) gsh[ub][cc] = a;
      }
    }
    __syncthreads();
    tick(6);
    if (pw) {
      const int64_t tbu = ((int64_t)t * B + pb) * kU + punit;
      const float gi = sigm(gsh[pub][4 * puu] + xp.x);
      const float gj = tanhf(gsh[pub][4 * puu + 1] + xp.y);
      const float gf = sigm(gsh[pub][4 * puu + 2] + xp.z + 1.0f);   // forget_bias = 1.0
      const float go = sigm(gsh[pub][4 * puu + 3] + xp.w);
      const float cn = gf * c_own + gi * gj;
      const float hn = go * tanhf(cn);
      const float c2 = mcv * cn + (1.f - mcv) * c_own;
      const float h2 = mhv * hn + (1.f - mhv) * h_own;
      c_own = c2; h_own = h2;
      hown[pub][puu] = hn;
      p.C0[((int64_t)(t + 1) * B + pb) * kU + punit] = c2;
      stc(rREC, ((t + 1) * B + pb) * kK0 + kM1 + kM2 + punit, h2);
      p.H0RAW[tbu] = hn;
      reinterpret_cast<float4*>(p.G0 + ((int64_t)t * B + pb) * 4 * kU)[punit] = make_float4(gi, gj, gf, go);
    }
    __syncthreads();
    tick(7);
    // ======== query contribution of the workgroup's units: lane = output column
#pragma unroll
    for (int ub = 0; ub < kUBmax; ++ub) {
      if (ub >= UB) break;
      float a = 0.f;
#pragma unroll
      for (int uu = 0; uu < kUW; ++uu) a = fmaf(hown[ub][uu], wq[uu], a);
      stc(rQP, (((t & 1) * B + g + kG * ub) * kGW + j) * kQ + tid, a);
    }
  };

  for (int t = 0; t < T; ++t) {
    phase_a(t);
    tick(0);
    group_barrier(ctr, (++phase) * kGW, p.err);
    tick(1);

    // ===================== phase C: attention tile (energies from LDS-resident K1/K2)
    if (tile_wg) {
      {   // q_t = sum of the 32 query partials of this utterance: 8 float4 loads per lane
        const int base4 = (((t & 1) * B + tb) * kGW) * (kQ / 4);
        float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
        float4 v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = ldc4(rQP, base4 + (wave * 8 + i) * (kQ / 4) + lane);
#pragma unroll
        for (int i = 0; i < 8; ++i) { a.x += v[i].x; a.y += v[i].y; a.z += v[i].z; a.w += v[i].w; }
        qred[wave][lane] = a;
      }
      __syncthreads();
      if (tid < kQ / 4) {
        const float4 a0 = qred[0][tid], a1 = qred[1][tid], a2 = qred[2][tid], a3 = qred[3][tid];
        const float4 qv = make_float4((a0.x + a1.x) + (a2.x + a3.x), (a0.y + a1.y) + (a2.y + a3.y),
                                      (a0.z + a1.z) + (a2.z + a3.z), (a0.w + a1.w) + (a2.w + a3.w));
        if (tile == 0) reinterpret_cast<float4*>(p.Q + ((int64_t)t * B + tb) * kQ)[tid] = qv;
        const int d = 4 * tid;
        if (d < kD1) {
          qb[d] = qv.x + p.b1[d]; qb[d + 1] = qv.y + p.b1[d + 1];
          qb[d + 2] = qv.z + p.b1[d + 2]; qb[d + 3] = qv.w + p.b1[d + 3];
        } else {
          q2s[d - kD1] = qv.x; q2s[d - kD1 + 1] = qv.y; q2s[d - kD1 + 2] = qv.z; q2s[d - kD1 + 3] = qv.w;
        }
      }
      if (tid < kPN * kF) {       // location features f = Conv1D_SAME(s_{t-1}) + bias
        const int i = tid / kF, f = tid - i * kF;
        float acc = cw[kKW * kF + f];
#pragma unroll
        for (int jj = 0; jj < kKW; ++jj) acc = fmaf(sp[i + jj], cw[jj * kF + f], acc);
        fs[i][f] = acc;
        if (p.LOC && i < nt) p.LOC[(((int64_t)t * B + tb) * N + n0 + i) * kF + f] = acc;
      }
      __syncthreads();
      // energies: 8 lanes per position, 28 dims (7 float4) of K1 per lane, 4 dims of K2
      const int nl = tid >> 3, part = tid & 7;
      // the tanh values are kept for the BPTT (decoder_persistent_bwd.hip recomputes nothing)
      float* zrow = (p.ZH && nl < nt) ? p.ZH + ((((int64_t)t * B + tb) * N) + n0 + nl) * kQ : nullptr;
      float acc = 0.f;
      {
        float fl[kF];
#pragma unroll
        for (int f = 0; f < kF; ++f) fl[f] = fs[nl][f];
#pragma unroll
        for (int jj = 0; jj < kD1 / 32; ++jj) {
          const int d = part * (kD1 / 8) + 4 * jj;
          const float4 kv = *reinterpret_cast<const float4*>(&k1s[nl][d]);
          const float4 qv = *reinterpret_cast<const float4*>(&qb[d]);
          const float4 vw = *reinterpret_cast<const float4*>(&vv[d]);
          float4 pre = make_float4(kv.x + qv.x, kv.y + qv.y, kv.z + qv.z, kv.w + qv.w);
#pragma unroll
          for (int f = 0; f < kF; ++f) {
            const float4 lw = *reinterpret_cast<const float4*>(&locw[f][d]);
            pre.x = fmaf(fl[f], lw.x, pre.x); pre.y = fmaf(fl[f], lw.y, pre.y);
            pre.z = fmaf(fl[f], lw.z, pre.z); pre.w = fmaf(fl[f], lw.w, pre.w);
          }
          const float4 z = make_float4(tanh_fast(pre.x), tanh_fast(pre.y), tanh_fast(pre.z),
                                       tanh_fast(pre.w));
          if (zrow) *reinterpret_cast<float4*>(zrow + d) = z;
          acc = fmaf(vw.x, z.x, acc);
          acc = fmaf(vw.y, z.y, acc);
          acc = fmaf(vw.z, z.z, acc);
          acc = fmaf(vw.w, z.w, acc);
        }
      }
      float acc2;
      {
        const int d = 4 * part;
        const float4 kv = *reinterpret_cast<const float4*>(&k2s[nl][d]);
        const float4 qv = *reinterpret_cast<const float4*>(&q2s[d]);
        const float4 vw = *reinterpret_cast<const float4*>(&vv2[d]);
        const float4 z = make_float4(tanh_fast(kv.x + qv.x), tanh_fast(kv.y + qv.y),
                                     tanh_fast(kv.z + qv.z), tanh_fast(kv.w + qv.w));
        if (zrow) *reinterpret_cast<float4*>(zrow + kD1 + d) = z;
        acc2 = vw.x * z.x;
        acc2 = fmaf(vw.y, z.y, acc2);
        acc2 = fmaf(vw.z, z.z, acc2);
        acc2 = fmaf(vw.w, z.w, acc2);
      }
      acc = group8_sum(acc);
      acc2 = group8_sum(acc2);
      const int eb = (((t & 1) * B + tb) * 2) * N;
      if (part == 0 && nl < nt) {
        const bool valid = n0 + nl < len;
        const float ev1 = valid ? acc : -INFINITY, ev2 = valid ? acc2 : -INFINITY;
        e1s[nl] = ev1;
        e2s[nl] = ev2;
        stc(rE, eb + n0 + nl, ev1);
        stc(rE, eb + N + n0 + nl, ev2);
      }
      __syncthreads();
      if (wave == 0) {            // tile statistics
        const float e1v = lane < nt ? e1s[lane] : -INFINITY;
        const float e2v = lane < nt ? e2s[lane] : -INFINITY;
        const float m1 = wave_max(e1v), m2 = wave_max(e2v);
        const float pe = (e1v == -INFINITY) ? 0.f : __expf(e1v - m1);
        const float pe2 = (e2v == -INFINITY) ? 0.f : __expf(e2v - m2);
        const float w = lane < nt ? ((1.f - u) * ap[lane + 1] + u * ap[lane] + 1e-7f) * pe : 0.f;
        if (lane < kPN) { w1s[lane] = w; w2s[lane] = lane < nt ? pe2 : 0.f; }
        const float z1 = wave_sum_dpp(pe), a1 = wave_sum_dpp(w), z2 = wave_sum_dpp(pe2);
        if (lane == 0) { red[0] = m1; red[1] = z1; red[2] = a1; red[3] = m2; red[4] = z2; }
      }
      __syncthreads();
      const int pout = (((t & 1) * B + tb) * ntiles + tile) * kPST;
      if (tid < 5) stc(rPT, pout + tid, red[tid]);
      {   // unnormalised partial contexts: wave owns 8 positions, lane a float4 column
        float4 c = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int i = 0; i < kPN / 4; ++i) {
          const int r = wave * (kPN / 4) + i;
          const float w = w1s[r];
          const float4 v = *reinterpret_cast<const float4*>(&v1s[r][4 * lane]);
          c.x = fmaf(w, v.x, c.x); c.y = fmaf(w, v.y, c.y);
          c.z = fmaf(w, v.z, c.z); c.w = fmaf(w, v.w, c.w);
        }
        cred[wave][lane] = c;
        if (part < kD2 / 4) {
          const float w = w2s[nl];
          const float4 v = *reinterpret_cast<const float4*>(&v2s[nl][4 * part]);
          c2red[nl][part] = make_float4(w * v.x, w * v.y, w * v.z, w * v.w);
        }
      }
      __syncthreads();
      if (tid < kM1 / 4) {
        const float4 a0 = cred[0][tid], a1 = cred[1][tid], a2 = cred[2][tid], a3 = cred[3][tid];
        stc4(rPT, (pout + 8) / 4 + tid,
             make_float4((a0.x + a1.x) + (a2.x + a3.x), (a0.y + a1.y) + (a2.y + a3.y),
                         (a0.z + a1.z) + (a2.z + a3.z), (a0.w + a1.w) + (a2.w + a3.w)));
      } else if (tid >= 64 && tid < 64 + kM2 / 4) {
        const int jj = tid - 64;
        float4 sm = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 8
        for (int i = 0; i < kPN; ++i) {
          const float4 v = c2red[i][jj];
          sm.x += v.x; sm.y += v.y; sm.z += v.z; sm.w += v.w;
        }
        stc4(rPT, (pout + 8 + kM1) / 4 + jj, sm);
      }
    }
    tick(2);
    group_barrier(ctr, (++phase) * kGW, p.err);
    tick(3);
  }
  if (p.prof && tid == 0)
    for (int i = 0; i < 8; ++i) p.prof[blockIdx.x * 8 + i] = tp[i];
  // ===================== epilogue: step T-1's context, statistics and normalised rows
  phase_a(T);
}

}  // namespace
}  // namespace sat

using namespace sat;

extern "C" int sat_decoder_attention_fwd(const SatDecAttnFwd* a, void* stream) {
  SAT_CHECK_ARG(a && a->B > 0 && a->N > 0 && a->T > 0, "sat_decoder_attention_fwd: bad sizes");
  SAT_CHECK_ARG(a->U == kU && a->M1 == kM1 && a->M2 == kM2 && a->D1 == kD1 && a->D2 == kD2 &&
                a->F == kF && a->KW == kKW,
                "sat_decoder_attention_fwd: compiled for U=256, M1=256, M2=32, D1=224, D2=32, "
                "F=5, KW=10 (the self-attention-tacotron configs)");
  SAT_CHECK_ARG(a->B % kG == 0 && a->B / kG <= kUBmax, "sat_decoder_attention_fwd: B in {8,16,24,32}");
  const int ntiles = ceil_div(a->N, kPN);
  SAT_CHECK_ARG((a->B / kG) * ntiles <= kGW && ntiles <= 8,
                "sat_decoder_attention_fwd: (B/8) * ceil(N/32) must be <= 32");
  SAT_CHECK_ARG(a->X0 && a->W0r && a->Wq1 && a->Wq2 && a->K1 && a->V1 && a->K2 && a->V2 &&
                a->lengths && a->v1 && a->b1 && a->convW && a->convb && a->locW && a->v2 &&
                a->REC0 && a->C0 && a->H0RAW && a->G0 && a->Q && a->S1 && a->AL1 && a->S2 &&
                a->ST && a->E && a->PART && a->QP && a->ctr && a->err,
                "sat_decoder_attention_fwd: null pointer");
  SAT_CHECK_ARG((a->mask_c == nullptr) == (a->mask_h == nullptr), "sat_decoder_attention_fwd: masks come in pairs");
  SAT_CHECK_ARG(aligned16(a->X0) && aligned16(a->G0) && aligned16(a->K1) && aligned16(a->V1),
                "sat_decoder_attention_fwd: 16-byte aligned operands");
  // the grid must be co-resident (one workgroup per CU): refuse rather than hang
  int dev = 0, cus = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, dec_attn_fwd_kernel, 256, 0) != hipSuccess) {
    set_error("sat_decoder_attention_fwd: device query failed");
    return SAT_ERR_HIP;
  }
  SAT_CHECK_ARG((int64_t)cus * per_cu >= kG * kGW,
                "sat_decoder_attention_fwd: fewer than 256 co-resident workgroups on this device");
  DecAttnP p;
  p.B = a->B; p.N = a->N; p.T = a->T; p.ntiles = ntiles; p.UB = a->B / kG;
  p.u = a->u; p.zc = a->zc; p.zh = a->zh;
  p.X0 = a->X0; p.W0r = a->W0r; p.Wq1 = a->Wq1; p.Wq2 = a->Wq2;
  p.K1 = a->K1; p.V1 = a->V1; p.K2 = a->K2; p.V2 = a->V2; p.lengths = a->lengths;
  p.v1 = a->v1; p.b1 = a->b1; p.convW = a->convW; p.convb = a->convb; p.locW = a->locW;
  p.v2 = a->v2; p.mask_c = a->mask_c; p.mask_h = a->mask_h;
  p.REC0 = a->REC0; p.C0 = a->C0; p.H0RAW = a->H0RAW; p.G0 = a->G0; p.Q = a->Q;
  p.S1 = a->S1; p.AL1 = a->AL1; p.S2 = a->S2; p.ST = a->ST; p.LOC = a->LOC;
  p.E = a->E; p.PART = a->PART; p.QP = a->QP; p.ctr = a->ctr; p.err = a->err;
  p.prof = reinterpret_cast<long long*>(a->prof);
  p.ZH = a->ZH;
  hipStream_t s = as_stream(stream);
  if (hipMemsetAsync(a->ctr, 0, kG * 64 * sizeof(unsigned), s) != hipSuccess ||
      hipMemsetAsync(a->err, 0, 2 * sizeof(int), s) != hipSuccess) {
    set_error("sat_decoder_attention_fwd: memset failed");
    return SAT_ERR_HIP;
  }
  hipLaunchKernelGGL(dec_attn_fwd_kernel, dim3(kG * kGW), dim3(256), 0, s, p);
  SAT_LAUNCH_CHECK("sat_decoder_attention_fwd");
  return SAT_OK;
}

extern "C" int64_t sat_decoder_attention_scratch(int32_t B, int32_t N, int64_t* e_floats,
                                                 int64_t* part_floats, int64_t* qp_floats) {
  const int ntiles = ceil_div(N, kPN);
  if (e_floats) *e_floats = (int64_t)2 * B * 2 * N;
  if (part_floats) *part_floats = (int64_t)2 * B * ntiles * kPST;
  if (qp_floats) *qp_floats = (int64_t)2 * B * kGW * kQ;
  return kG * 64;   // counter words
}
