// Persistent BPTT of the decoder's attention chain, one utterance per group of 8 workgroups:
// ALL T' reverse steps of
//   dual-source attention backward  ->  attention-RNN (ZoneoutLSTM 256) reverse step
// in ONE launch -- the mirror of decoder_persistent8.hip and the same arithmetic as
// decoder_persistent_bwd.hip (attention.hip attn_bwd_kernel, lstm.hip lstm_bwd_block), which
// it replaces for N <= 256.
//
// Layout: group g = utterance g owns workgroups blockIdx = g + 32 j (one XCD under the
// observed round-robin placement); workgroup j holds LSTM units [32j, 32j+32) (their 128 gate
// columns x 512 rows of W0r in registers, the 32 c2 rows and the 32 query rows in LDS) and
// memory positions [jP, jP+P) (V1/V2 rows in LDS).  Per reverse step t two 8-producer
// hand-offs, data-tagged like the forward (persistent.h lsb_tag; sequence q = T-1-t):
//   record Q_t (phase Y -> Z): the tile's query-gradient partial sum_n dp_t[n] (256), its
//     sums P1 = sum_n Y_t (prior_t - 1e-7), P2 = sum_n dL/df_t . (f_t - convb), Y_t at the
//     first own position and dL/df_t at the first 4 / last 5 own positions (the halos of the
//     neighbours' alignment recursion and transposed location convolution);
//   record R_t (phase Z -> Y of step t-1): the row-dot partial DG0_t[own 128 columns] .
//     W0r[k, own columns] for all 544 inputs k (c part: dL/dctx_{t-1}; h part: the recurrent
//     product of step t-1).
// Phase Y(t): dL/dctx_t = RD[t] (LSTM1's part) + sum of the 8 R_{t+1} c parts; the tile's
// attention backward (Y_t, DE1/DE2, back through the kept energy tanh: dq partial, dL/df_t);
// publish Q_t.  Phase Z(t): dq_t = sum of the 8 Q_t partials; the own units' reverse LSTM
// step (recurrent product from the R_{t+1} h parts, dy += dq_t . Wq[unit]); DG0[t]; the
// row-dot partial R_t; publish.  Every value that crosses a workgroup boundary is tagged when
// it is made and its maker uses the tagged value too.  Outputs: DG0, DE1/DE2, DFH, the full
// dL/dctx_t in RD[:, :, :288], and dq_t fully reduced in DQP[t][b][0][:] (one part per step:
// sat_decoder_attention_bwd_dq_parts).  Bounded spins as everywhere (persistent.h).
#include "sat_common.h"
#include "persistent.h"

#ifndef SAT_BWD8_ZSUM
// every wave forms dq_t itself from the 8 staged Q partials (no wave-0 sum + second barrier),
// bitwise the same dq: 5.80-5.82 -> 5.74-5.77 us/step (two A/B rounds on one box, round 6)
#define SAT_BWD8_ZSUM 1
#endif
// trace builds only: the wave whose lane 0 keeps the segment clocks, and a split of segment 2
// at the history prefetch (slot 15)
#ifndef SAT_BWD8_TICKW
#define SAT_BWD8_TICKW 0
#endif
#ifndef SAT_BWD8_TICK15
#define SAT_BWD8_TICK15 0
#endif
#ifndef SAT_BWD8_MERGE3
// A/B: the per-position scalar chain (3b) on the lanes of the wave that owns the position,
// right after its DA / DS2 reduction (3a), instead of on wave 0 alone between two extra
// barriers -- correct (tests green) but 5.77-5.79 vs 5.74-5.77 us/step with ZSUM: not kept
#define SAT_BWD8_MERGE3 0
#endif

namespace sat {
namespace {

constexpr int kW = 8;                  // workgroups per utterance
constexpr int kGmax = 32;              // utterances (groups); grid = 256
constexpr int kTh = 512;               // 8 waves, 2 per SIMD
constexpr int kU = 256, kM1 = 256, kM2 = 32, kD1 = 224, kD2 = 32, kF = 5, kKW = 10;
constexpr int kC = kM1 + kM2;          // 288
constexpr int kK0 = kC + kU;           // 544
constexpr int kQ = kD1 + kD2;          // 256
constexpr int kUW = kU / kW;           // 32 units per workgroup
constexpr int kPmax = 32;
constexpr int kPadL = (kKW - 1) / 2;   // 4
constexpr int kHL = kKW - 1 - kPadL;   // 5: left halo of the transposed convolution
constexpr int kHR = kPadL;             // 4: right halo
constexpr int kJF = kKW * kF;          // 50 taps
constexpr int kRQ = 320;               // record Q floats
constexpr int kQP = kQ, kQY = kQ + 2, kQDH = kQ + 4, kQDT = kQDH + kHR * kF;   // 256, 258, 260, 280
constexpr int kRR = kK0;               // record R floats (544)
static_assert(kQDT + kHL * kF <= kRQ && kRR % 4 == 0, "layout");

struct Bwd8P {
  int B, N, T, P, flags;
  float u, zc, zh;
  const float* REC0; const float* C0; const float* G0;
  const float* S1; const float* AL1; const float* S2; const float* ST; const float* LOC;
  const float* V1; const float* V2;
  const float* v1; const float* convW; const float* convb; const float* locW; const float* v2;
  const float* W0r; const float* Wq1; const float* Wq2;
  const float* mask_c; const float* mask_h;
  const float* DH0; const float* ZH;
  float* RD; float* DG0; float* DE1; float* DE2; float* DFH; float* DQP;
  float* RQ;        // [2][B][8][kRQ] tagged
  float* RR;        // [2][B][8][kRR] tagged
  unsigned* XID; int* err;
  long long* prof;  // [256][16] segment clocks (nullable)
};

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ bool any_lane(bool v) { return __builtin_amdgcn_ballot_w64(v) != 0; }
__device__ __forceinline__ float rdl(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ float4 add4(float4 a, float4 b) {
  return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}
// x[l] + x[l ^ 32] in lanes l < 32 (gfx950 v_permlane32_swap)
__device__ __forceinline__ float fold32(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float from_upper32(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[1]);
}
// 4 outputs: row r (lanes 16r .. 16r+15) holds output r
__device__ __forceinline__ void transpose_reduce4(float* v) {
  v[0] = fsum_swap32(v[0], v[2]);
  v[1] = fsum_swap32(v[1], v[3]);
  v[0] = fsum_swap16(v[0], v[1]);
  v[0] = group16_sum(v[0]);
}

__global__ void __launch_bounds__(kTh) dec_attn_bwd8_kernel(Bwd8P p) {
  __shared__ __attribute__((aligned(16))) float v1s[kPmax][kM1];
  __shared__ __attribute__((aligned(16))) float v2s[kPmax][kM2];
  __shared__ __attribute__((aligned(16))) float wqs[kUW][kQ];
  __shared__ __attribute__((aligned(16))) float wc2[kM2][4 * kUW + 4];
  __shared__ __attribute__((aligned(16))) float locw[kF][kQ];        // columns >= D1 zero
  __shared__ __attribute__((aligned(16))) float vcat[kQ];            // [v1 | v2]
  __shared__ float cw[kJF + kF];
  // per step
  __shared__ __attribute__((aligned(16))) float rst[kW][kC + kUW];   // staged R: c part + own h rows
  __shared__ __attribute__((aligned(16))) float4 qst[kW][64];        // staged dq partials / dq reduce
  __shared__ __attribute__((aligned(16))) float dcb[kC];             // dL/dctx_t
#if !SAT_BWD8_ZSUM
  __shared__ __attribute__((aligned(16))) float qb[kQ];              // dq_t
#endif
  __shared__ __attribute__((aligned(16))) float wred[kW][kK0];       // row-dot partials per wave
  __shared__ float ysh[2][kPmax + 1];       // Y_{t+1} at n0..n0+nt (last = right neighbour's)
  __shared__ float dfh[2][(kPmax + kHL + kHR) * kF];   // dL/df_{t+1} on n0-5 .. n0+nt+3
  __shared__ float pst[kW][2];              // P1, P2 of step t+1 per tile
  __shared__ float dsn[kPmax];
  __shared__ float daS[kPmax], ds2S[kPmax], e1S[kPmax], e2S[kPmax];
  __shared__ float lfS[kPmax][kF];          // f_t - convb of the own positions
  __shared__ __attribute__((aligned(16))) float4 qz[kW][64];        // staged Q_t dq partials
  __shared__ float red[8];
  __shared__ float pw[kW][2];               // per-wave P1 / P2 partials
  __shared__ long long tp[16];

  const int tid0 = threadIdx.x;
  const int g = blockIdx.x % kGmax, j = blockIdx.x / kGmax;
  const int B = p.B, N = p.N, T = p.T, P = p.P;
  if (g >= B) return;
  const int b = g;
  const int n0 = j * P, nt = max(0, min(P, N - n0));
  const bool has_left = j > 0, has_right = j + 1 < kW && n0 + P < N;
  const int64_t bN = (int64_t)b * N;
  const float u = p.u;
  const auto rRQ = rsrc(p.RQ), rRR = rsrc(p.RR);

  // ---------------- prologue (weights exactly as the forward: wave w = columns 16w..16w+15)
  f2 w0[8][8];
  {
    const int lane = tid0 & 63, wave = tid0 >> 6;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int r = i < 4 ? kC + 64 * i + lane : 64 * (i - 4) + lane;
      const float4* src = reinterpret_cast<const float4*>(p.W0r + (int64_t)r * (4 * kU) +
                                                          128 * j + 16 * wave);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 a = src[q];
        w0[i][2 * q] = f2{a.x, a.y};
        w0[i][2 * q + 1] = f2{a.z, a.w};
      }
    }
  }
  for (int i = tid0; i < kM2 * 32; i += kTh) {
    const int r = i >> 5, c4 = i & 31;
    *reinterpret_cast<float4*>(&wc2[r][4 * c4]) =
        reinterpret_cast<const float4*>(p.W0r + (int64_t)(kM1 + r) * (4 * kU) + 128 * j)[c4];
  }
  for (int i = tid0; i < kUW * kQ; i += kTh) {
    const int uu = i / kQ, c = i - uu * kQ, k = kUW * j + uu;
    wqs[uu][c] = c < kD1 ? p.Wq1[k * kD1 + c] : p.Wq2[k * kD2 + (c - kD1)];
  }
  for (int i = tid0; i < kPmax * kM1 / 4; i += kTh) {
    const int r = i / (kM1 / 4), c4 = i - r * (kM1 / 4);
    reinterpret_cast<float4*>(&v1s[r][0])[c4] = r < nt
        ? reinterpret_cast<const float4*>(p.V1 + (bN + n0 + r) * kM1)[c4] : make_float4(0, 0, 0, 0);
  }
  for (int i = tid0; i < kPmax * kM2; i += kTh) {
    const int r = i / kM2, c = i - r * kM2;
    v2s[r][c] = r < nt ? p.V2[(bN + n0 + r) * kM2 + c] : 0.f;
  }
  for (int d = tid0; d < kQ; d += kTh) {
    vcat[d] = d < kD1 ? p.v1[d] : p.v2[d - kD1];
#pragma unroll
    for (int f = 0; f < kF; ++f) locw[f][d] = d < kD1 ? p.locW[f * kD1 + d] : 0.f;
  }
  if (tid0 < kJF) cw[tid0] = p.convW[tid0];
  if (tid0 < kF) cw[kJF + tid0] = p.convb[tid0];
  if (tid0 < 16) tp[tid0] = 0;
  // nothing flows in from step T: Y_T = 0, dL/df_T = 0, P_T = 0
  for (int i = tid0; i < 2 * (kPmax + 1); i += kTh) (&ysh[0][0])[i] = 0.f;
  for (int i = tid0; i < 2 * (kPmax + kHL + kHR) * kF; i += kTh) (&dfh[0][0])[i] = 0.f;
  if (tid0 < 2 * kW) (&pst[0][0])[tid0] = 0.f;

  // ---- prefetch of the forward histories (plain loads, one step ahead)
  //   Y inputs: thread d < 288: c_t[d] (REC0 row t+1), RD[t][d]; thread r < nt (position
  //   n0 + r): s_t, s2_t, alpha_{t-1} at n and n-1, f_t; every lane: Sa; lane-chunk c of wave
  //   w: the energy tanh of positions 4w..4w+3.  Z inputs (cell lanes 16q of wave w, unit
  //   32j + 4w + q): G0, C0, DH0, masks.
  struct YPre { float cv, dv, st, s2, apn, apm, sa; float lf[kF]; float4 z[4]; };
  struct ZPre { float4 g4; float cp, dy, mc, mh; };
  auto prefetch_y = [&](int t, int tid, int lane, int wave, YPre& y) {
    const int64_t tb1 = (int64_t)(t + 1) * B + b, tb0 = (int64_t)t * B + b;
    y.cv = tid < kC ? p.REC0[tb1 * kK0 + tid] : 0.f;
    y.dv = tid < kC ? p.RD[tb0 * kK0 + tid] : 0.f;
#if SAT_BWD8_MERGE3
    const int pr = 4 * wave + (lane >> 3);
    const bool pos = (lane & 7) == 0 && lane < 32 && pr < nt;
    const int n = n0 + pr;
#else
    const bool pos = tid < nt;
    const int n = n0 + tid;
#endif
    y.st = pos ? p.S1[tb1 * N + n] : 0.f;
    y.s2 = pos ? p.S2[tb0 * N + n] : 0.f;
    y.apn = pos ? p.AL1[tb0 * N + n] : 0.f;
    y.apm = (pos && n >= 1) ? p.AL1[tb0 * N + n - 1] : 0.f;
#pragma unroll
    for (int f = 0; f < kF; ++f) y.lf[f] = pos ? p.LOC[(tb0 * N + n) * kF + f] : 0.f;
    y.sa = p.ST[tb0 * 4 + 2];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = 4 * wave + i;
      y.z[i] = r < nt ? reinterpret_cast<const float4*>(p.ZH + (tb0 * N + n0 + r) * kQ)[lane]
                      : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  const bool masked = p.mask_c != nullptr;
  auto prefetch_z = [&](int t, int lane, int wave, ZPre& z) {
    const bool cl = (lane & 15) == 0;
    const int64_t r = ((int64_t)t * B + b) * kU + kUW * j + 4 * wave + (lane >> 4);
    z.g4 = cl ? reinterpret_cast<const float4*>(p.G0)[r] : make_float4(0.f, 0.f, 0.f, 0.f);
    z.cp = cl ? p.C0[r] : 0.f;
    z.dy = cl ? p.DH0[r] : 0.f;
    z.mc = (cl && masked) ? p.mask_c[r] : 1.f - p.zc;
    z.mh = (cl && masked) ? p.mask_h[r] : 1.f - p.zh;
  };
  YPre ypre;
  ZPre zpre;
  prefetch_y(T - 1, tid0, tid0 & 63, tid0 >> 6, ypre);
  prefetch_z(T - 1, tid0 & 63, tid0 >> 6, zpre);
  float dh_c = 0.f, dc_c = 0.f;              // carries of the cell lanes
  __syncthreads();

  const bool xl = (p.flags & 1) ? xcd_local_group(p.XID, g, kGmax, kW, p.err) : false;
  long long t0 = p.prof ? wall_clock64() : 0;
  auto tick = [&](int seg) {
    if (p.prof && tid0 == 64 * SAT_BWD8_TICKW) {
      const long long t1 = wall_clock64();
      tp[seg] += t1 - t0;
      t0 = t1;
    }
  };
  bool gave_up = false;

  for (int t = T - 1; t >= 0; --t) {
    int tid = tid0;
    asm volatile("" : "+v"(tid));
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int q = T - 1 - t;                   // hand-off sequence number of step t
    const bool last = t == T - 1;
    const int yb = q & 1;                      // ysh / dfh buffer holding step t+1's values
    const unsigned bit = lsb_tag(q);
    // ===================== phase Y(t)
    // ---- 1. records R_{t+1} (wave jj stages record jj: c part + the own units' h rows) and
    //         the sum / halo words of records Q_{t+1} (wave 0 lanes 16..52, wave 1 lanes < 25)
    if (!last) {
      const int qp = q - 1;                    // sequence number of step t+1
      const unsigned want = lsb_tag(qp);
      const int rr = (((qp & 1) * B + b) * kW + wave) * kRR;
      const bool two = lane < kM2 / 4 + kUW / 4;      // c2 chunk (lanes < 8) or own h (8..15)
      const int i2 = lane < kM2 / 4 ? (rr + kM1) / 4 + lane : (rr + kC + kUW * j) / 4 + (lane - kM2 / 4);
      const int rq0 = ((qp & 1) * B + b) * kW;
      const int hq = lane - 16;
      int hw = -1;
      if (wave == 0 && hq >= 0) {
        if (hq < 2 * kW) hw = (rq0 + (hq >> 1)) * kRQ + kQP + (hq & 1);
        else if (hq == 2 * kW) hw = has_right ? (rq0 + j + 1) * kRQ + kQY : -2;
        else if (hq < 2 * kW + 1 + kHR * kF) hw = has_right ? (rq0 + j + 1) * kRQ + kQDH + (hq - 2 * kW - 1) : -2;
      }
      if (wave == 1 && lane < kHL * kF) hw = has_left ? (rq0 + j - 1) * kRQ + kQDT + lane : -2;
      float4 x1 = make_float4(0.f, 0.f, 0.f, 0.f), x2 = x1;
      float hv = 0.f;
      bool ok1 = false, ok2 = !two, ok3 = hw < 0;
      for (unsigned spins = 0;; ++spins) {
        if (!ok1) x1 = ldc4(rRR, rr / 4 + lane);
        if (!ok2) x2 = ldc4(rRR, i2);
        if (!ok3) hv = ldc(rRQ, hw);
        ok1 = tag_ok4(x1, want);
        ok2 = ok2 || tag_ok4(x2, want);
        ok3 = ok3 || tag_ok(hv, want);
        if (!any_lane(!(ok1 && ok2 && ok3)) || gave_up) break;
        if (poll_give_up(spins, p.err)) { gave_up = true; break; }
        __builtin_amdgcn_s_sleep(1);
      }
      reinterpret_cast<float4*>(&rst[wave][0])[lane] = x1;
      if (lane < kM2 / 4) reinterpret_cast<float4*>(&rst[wave][kM1])[lane] = x2;
      else if (two) reinterpret_cast<float4*>(&rst[wave][kC])[lane - kM2 / 4] = x2;
      if (wave == 0 && hq >= 0) {
        if (hq < 2 * kW) pst[hq >> 1][hq & 1] = hv;
        else if (hq == 2 * kW) ysh[yb][nt] = hv;                        // Y_{t+1}(n0 + nt)
        else if (hq < 2 * kW + 1 + kHR * kF)
          dfh[yb][(kHL + nt) * kF + (hq - 2 * kW - 1)] = hv;            // n0+nt .. n0+nt+3
      }
      if (wave == 1 && lane < kHL * kF) dfh[yb][lane] = hv;             // n0-5 .. n0-1
    }
    tick(0);
    lds_barrier();
    tick(1);
    // ---- 2. dL/dctx_t (thread d < 288, record order) and the forward-context dots; the
    //         transposed location convolution DSN (16 lanes per position, one tap each)
    const YPre y = ypre;
    if (wave < (kC + 63) / 64) {
      float a = y.dv;
      if (!last && tid < kC) {
#pragma unroll
        for (int k = 0; k < kW; ++k) a += rst[k][tid];
      }
      if (tid < kC) {
        dcb[tid] = a;
        if (j == 0) p.RD[((int64_t)t * B + b) * kK0 + tid] = a;
      }
      const float s = wave_sum_dpp(tid < kC ? a * y.cv : 0.f);   // waves 0-3: dc1.c1, 4: dc2.c2
      if (lane == 0) red[wave] = s;
    }
    {
      const int pos = tid >> 4, tap = tid & 15;
      float a = 0.f;
      if (tap < kKW && pos < nt) {
        // DSN[n] = sum_{k,f} dfh_{t+1}[n - k + padl][f] convW[k][f]; dfh index (n - n0) + kHL
        const float* dr = &dfh[yb][(pos - tap + kPadL + kHL) * kF];
#pragma unroll
        for (int f = 0; f < kF; ++f) a = fmaf(dr[f], cw[tap * kF + f], a);
      }
      a = group16_sum(a);
      if (tap == 0) dsn[pos] = a;
    }
#if SAT_BWD8_TICK15
    tick(15);
#endif
    if (t > 0) prefetch_y(t - 1, tid, lane, wave, ypre);
    tick(2);
    lds_barrier();
    tick(3);
    // ---- 3a. DA = dc1 . V1[n], DS2 = dc2 . V2[n] (lane = column chunk, wave = positions
    //          4w..4w+3; the 8 c2 chunks on lanes 0..7)
    if (4 * wave < nt) {
      const float4 dc4 = *reinterpret_cast<const float4*>(&dcb[4 * lane]);
      const float4 dc2 = lane < kM2 / 4 ? *reinterpret_cast<const float4*>(&dcb[kM1 + 4 * lane])
                                        : make_float4(0.f, 0.f, 0.f, 0.f);
      float e[8];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = 4 * wave + i;
        const float4 v = *reinterpret_cast<const float4*>(&v1s[r][4 * lane]);
        float a = dc4.x * v.x;
        a = fmaf(dc4.y, v.y, a); a = fmaf(dc4.z, v.z, a); a = fmaf(dc4.w, v.w, a);
        e[i] = a;
        float c = 0.f;
        if (lane < kM2 / 4) {
          const float4 w = *reinterpret_cast<const float4*>(&v2s[r][4 * lane]);
          c = dc2.x * w.x;
          c = fmaf(dc2.y, w.y, c); c = fmaf(dc2.z, w.z, c); c = fmaf(dc2.w, w.w, c);
        }
        e[4 + i] = c;
      }
      transpose_reduce8(e, lane);              // lanes 8m: m < 4 DA(4w+m), m >= 4 DS2(4w+m-4)
#if SAT_BWD8_MERGE3
      // ---- 3b on the owning wave: lane 8m (m < 4) runs position r = 4w + m's scalar chain
      //      with DS2 brought over from lane 8m + 32 (v_permlane32_swap) and the position's
      //      history operands prefetched into that lane (prefetch_y)
      {
        const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(e[0]), __float_as_uint(e[0]),
                                                         false, false);
        const float ds2v = __uint_as_float(sw[1]);       // lane l < 32: lane l + 32's value
        const float s1 = (red[0] + red[1]) + (red[2] + red[3]), s3 = red[4];
        float P1n = 0.f, P2n = 0.f;
#pragma unroll
        for (int k = 0; k < kW; ++k) { P1n += pst[k][0]; P2n += pst[k][1]; }
        const int r = 4 * wave + (lane >> 3);
        float p1 = 0.f;
        if ((lane & 7) == 0 && lane < 32 && r < nt) {
          const float* yn = ysh[yb];
          const float dan = (1.f - u) * yn[r] + u * yn[r + 1];
          const float da = (e[0] + dan - (s1 + P1n)) * __builtin_amdgcn_rcpf(y.sa);
          const float prior = (1.f - u) * y.apn + u * y.apm;
          const float ds = dsn[r] + da * (prior + 1e-7f);
          const float yv = tagf(y.st * da, bit);
          const float e1v = y.st * (ds - P2n);
          const float e2v = y.s2 * (ds2v - s3);
          const int64_t o = ((int64_t)t * B + b) * N + n0 + r;
          p.DE1[o] = e1v;
          p.DE2[o] = e2v;
          ysh[1 - yb][r] = yv;
          e1S[r] = e1v;
          e2S[r] = e2v;
          p1 = yv * prior;
#pragma unroll
          for (int f = 0; f < kF; ++f) lfS[r][f] = y.lf[f] - cw[kJF + f];
        }
        p1 = wave_sum_dpp(p1);
        if (lane == 0) pw[wave][0] = p1;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // own e1S / e2S / lfS for phase 4
    } else if (lane == 0) {
      pw[wave][0] = 0.f;                       // no own positions: no P1 partial
    }
    tick(4);
#else
      if ((lane & 7) == 0) {
        const int m = lane >> 3;
        if (m < 4) daS[4 * wave + m] = e[0]; else ds2S[4 * wave + m - 4] = e[0];
      }
    }
    tick(4);
    lds_barrier();
    // ---- 3b. the scalar chain of position r (thread r < nt holds its history operands):
    //          da = (DA + dalpha_next - s1) / Sa, ds = DSN + da (prior + 1e-7), Y_t = s da,
    //          DE1 = s (ds - s2), DE2 = s2 (DS2 - s3); P1 partial = Y_t prior
    if (wave == 0) {
      const float s1 = (red[0] + red[1]) + (red[2] + red[3]), s3 = red[4];
      float P1n = 0.f, P2n = 0.f;
#pragma unroll
      for (int k = 0; k < kW; ++k) { P1n += pst[k][0]; P2n += pst[k][1]; }
      const int r = lane;
      float p1 = 0.f;
      if (r < nt) {
        const float* yn = ysh[yb];
        const float dan = (1.f - u) * yn[r] + u * yn[r + 1];
        const float da = (daS[r] + dan - (s1 + P1n)) * __builtin_amdgcn_rcpf(y.sa);
        const float prior = (1.f - u) * y.apn + u * y.apm;
        const float ds = dsn[r] + da * (prior + 1e-7f);
        const float yv = tagf(y.st * da, bit);
        const float e1v = y.st * (ds - P2n);
        const float e2v = y.s2 * (ds2S[r] - s3);
        const int64_t o = ((int64_t)t * B + b) * N + n0 + r;
        p.DE1[o] = e1v;
        p.DE2[o] = e2v;
        ysh[1 - yb][r] = yv;
        e1S[r] = e1v;
        e2S[r] = e2v;
        p1 = yv * prior;
#pragma unroll
        for (int f = 0; f < kF; ++f) lfS[r][f] = y.lf[f] - cw[kJF + f];
      }
      p1 = wave_sum_dpp(p1);
      if (lane == 0) pw[0][0] = p1;
    }
    tick(5);
    lds_barrier();
    tick(6);
#endif
    // ---- 4. back through the kept energy tanh: dp = DE v (1 - z^2) (lane = chunk, wave =
    //         positions 4w..4w+3); the dq partial (sum over positions) and dL/df_t
    {
      const int c = lane;
      const float4 v4 = *reinterpret_cast<const float4*>(&vcat[4 * c]);
      const bool d1 = c < kD1 / 4;
      float4 dqa = make_float4(0.f, 0.f, 0.f, 0.f);
      // dL/df of the wave's 4 positions: taps f < 4 as 16 outputs, tap 4 as 4 (a 32-output
      // reduction of the 20 values paid 12 exchanges of constant zeros)
      float dfa[16], dfb[4];
#pragma unroll
      for (int k = 0; k < 16; ++k) dfa[k] = 0.f;
#pragma unroll
      for (int k = 0; k < 4; ++k) dfb[k] = 0.f;
      float4 lw[kF];
#pragma unroll
      for (int f = 0; f < kF; ++f) lw[f] = *reinterpret_cast<const float4*>(&locw[f][4 * c]);
      if (4 * wave < nt) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = 4 * wave + i;
          const float ev = r < nt ? (d1 ? e1S[r] : e2S[r]) : 0.f;
          const float4 z = y.z[i];
          const float4 dp = make_float4(ev * v4.x * fmaf(-z.x, z.x, 1.f), ev * v4.y * fmaf(-z.y, z.y, 1.f),
                                        ev * v4.z * fmaf(-z.z, z.z, 1.f), ev * v4.w * fmaf(-z.w, z.w, 1.f));
          dqa = add4(dqa, dp);
#pragma unroll
          for (int f = 0; f < kF; ++f) {        // locw is zero on the D2 chunks
            float a = dp.x * lw[f].x;
            a = fmaf(dp.y, lw[f].y, a); a = fmaf(dp.z, lw[f].z, a); a = fmaf(dp.w, lw[f].w, a);
            if (f < 4) dfa[4 * i + f] = a; else dfb[i] = a;
          }
        }
      }
      qst[wave][c] = dqa;
      transpose_reduce16(dfa, lane);           // lanes 4m..4m+3: position 4w + m / 4, tap m % 4
      transpose_reduce4(dfb);                  // lanes 16i..16i+15: position 4w + i, tap 4
      float p2 = 0.f;
      {
        const int r = 4 * wave + (lane >> 4);
        const int64_t o = (((int64_t)t * B + b) * N + n0 + r) * kF;
        if ((lane & 3) == 0 && r < nt) {
          const int f = (lane >> 2) & 3;
          const float v = tagf(dfa[0], bit);
          p.DFH[o + f] = v;
          dfh[1 - yb][(kHL + r) * kF + f] = v;
          p2 = v * lfS[r][f];
        }
        if ((lane & 15) == 0 && r < nt) {
          const float v = tagf(dfb[0], bit);
          p.DFH[o + 4] = v;
          dfh[1 - yb][(kHL + r) * kF + 4] = v;
          p2 += v * lfS[r][4];
        }
      }
      p2 = wave_sum_dpp(p2);
      if (lane == 0) pw[wave][1] = p2;
    }
    tick(7);
    lds_barrier();
    tick(8);
    // ---- 5. publish record Q_t: wave 0 the dq partial; wave 1 the sums word (lane 0) and the
    //         dL/df_t head / tail words (lanes 1..45), addresses and values chosen branch-free
    //         (one store per lane; the per-lane-range branches serialised the segment)
    if (wave == 0) {
      const int rq = (((q & 1) * B + b) * kW + j) * kRQ;
      float4 a = qst[0][lane];
#pragma unroll
      for (int w = 1; w < kW; ++w) a = add4(a, qst[w][lane]);
      stc4x(xl, rRQ, rq / 4 + lane, tagf4(a, bit));
    } else if (wave == 1) {
      const int rq = (((q & 1) * B + b) * kW + j) * kRQ;
      float P2 = 0.f;
#pragma unroll
      for (int w = 0; w < kW; ++w) P2 += pw[w][1];
#if SAT_BWD8_MERGE3
      float P1 = 0.f;                          // per-wave partials of the position owners
#pragma unroll
      for (int w = 0; w < kW; ++w) P1 += pw[w][0];
#else
      const float P1 = pw[0][0];
#endif
      const float4 pword = tagf4(make_float4(P1, P2, ysh[1 - yb][0], 0.f), bit);
      const bool head = lane >= 1 && lane <= kHR * kF;                   // n0 .. n0+3
      const bool tail = lane > kHR * kF && lane <= kHR * kF + kHL * kF;  // n0+nt-5 .. n0+nt-1
      const int kh = lane - 1, kt = lane - 1 - kHR * kF;
      const int it = nt - kHL + kt / kF;
      const int src = head ? kHL * kF + kh : (kHL + max(it, 0)) * kF + (kt % kF);
      const float dv = dfh[1 - yb][min(max(src, 0), (kPmax + kHL + kHR) * kF - 1)];
      const bool valid = head ? (kh / kF) < nt : it >= 0;
      const float v = valid ? dv : tagf(0.f, bit);
      const int idx = head ? rq + kQDH + kh : rq + kQDT + kt;
      if (lane == 0) stc4x(xl, rRQ, (rq + kQP) / 4, pword);
      else if (head || tail) stcx(xl, rRQ, idx, v);
    }
    tick(9);

    // ===================== phase Z(t)
    // ---- 1. records Q_t (wave jj stages record jj's dq partial)
    {
      const int rq = (((q & 1) * B + b) * kW + wave) * kRQ;
      float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
      for (unsigned spins = 0;; ++spins) {
        x = ldc4(rRQ, rq / 4 + lane);
        if (!any_lane(!tag_ok4(x, bit)) || gave_up) break;
        if (poll_give_up(spins, p.err)) { gave_up = true; break; }
        __builtin_amdgcn_s_sleep(1);
      }
      qz[wave][lane] = x;
    }
    tick(10);
    lds_barrier();
#if SAT_BWD8_ZSUM
    // every wave sums the 8 staged partials of its lane's chunk itself (record order: the same
    // bits wave 0 formed into qb) -- no wave-0-only phase and no second barrier
    float4 dqz = qz[0][lane];
#pragma unroll
    for (int w = 1; w < kW; ++w) dqz = add4(dqz, qz[w][lane]);
    if (wave == 0 && j == 0) reinterpret_cast<float4*>(p.DQP + ((int64_t)t * B + b) * kQ)[lane] = dqz;
#else
    if (wave == 0) {
      float4 a = qz[0][lane];
#pragma unroll
      for (int w = 1; w < kW; ++w) a = add4(a, qz[w][lane]);
      reinterpret_cast<float4*>(qb)[lane] = a;
      if (j == 0) reinterpret_cast<float4*>(p.DQP + ((int64_t)t * B + b) * kQ)[lane] = a;
    }
    lds_barrier();
#endif
    tick(11);
    // ---- 2. the own units' reverse step: query term dq_t . Wq[unit] (wave w, units 4w..4w+3:
    //         row q of the wave holds unit q's sum), recurrent product from the R_{t+1} h rows,
    //         then the cell lane's pointwise reverse step (lstm.hip lstm_bwd_block)
    f2 dgp[8];
    {
#if SAT_BWD8_ZSUM
      const float4 dq4 = dqz;
#else
      const float4 dq4 = *reinterpret_cast<const float4*>(&qb[4 * lane]);
#endif
      float v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float4 w4 = *reinterpret_cast<const float4*>(&wqs[4 * wave + k][4 * lane]);
        float a = dq4.x * w4.x;
        a = fmaf(dq4.y, w4.y, a); a = fmaf(dq4.z, w4.z, a); a = fmaf(dq4.w, w4.w, a);
        v[k] = a;
      }
      transpose_reduce4(v);                    // row cq = lane >> 4 holds unit 4w + cq's term
      const int cq = lane >> 4, ul = 4 * wave + cq;
      const ZPre z = zpre;
      float4 dg = make_float4(0.f, 0.f, 0.f, 0.f);
      if ((lane & 15) == 0) {
        float rec = 0.f;
        if (!last) {
#pragma unroll
          for (int k = 0; k < kW; ++k) rec += rst[k][kC + ul];
        }
        const float dh_t = rec + dh_c;
        const float dc_t = dc_c;
        const float gi = z.g4.x, gj = z.g4.y, gf = z.g4.z, go = z.g4.w;
        const float cn = gf * z.cp + gi * gj;
        // tanh(c) exactly as the forward formed it (decoder_persistent8.hip: 2 sigm(2c) - 1
        // with one v_exp and one v_rcp), so the derivative is taken at the forward's value
        const float tc = fmaf(2.f, __builtin_amdgcn_rcpf(1.f + __expf(-2.f * cn)), -1.f);
        const float dhn = z.dy + v[0] + z.mh * dh_t;
        const float dcn = z.mc * dc_t + dhn * go * (1.f - tc * tc);
        const float d_o = dhn * tc * go * (1.f - go);
        const float d_f = dcn * z.cp * gf * (1.f - gf);
        const float d_i = dcn * gj * gi * (1.f - gi);
        const float d_j = dcn * gi * (1.f - gj * gj);
        dg = make_float4(d_i, d_j, d_f, d_o);
        reinterpret_cast<float4*>(p.DG0 + ((int64_t)t * B + b) * 4 * kU)[kUW * j + ul] = dg;
        dc_c = dcn * gf + (1.f - z.mc) * dc_t;
        dh_c = (1.f - z.mh) * dh_t;
      }
      // the wave's 16 gate gradients to every lane (column order 4 unit + gate)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        dgp[2 * k] = f2{rdl(dg.x, 16 * k), rdl(dg.y, 16 * k)};
        dgp[2 * k + 1] = f2{rdl(dg.z, 16 * k), rdl(dg.w, 16 * k)};
      }
      if (t > 0) prefetch_z(t - 1, lane, wave, zpre);
    }
    tick(12);
    // ---- 3. row-dot partial R_t[k] = sum over the own 128 columns of DG0_t[col] W0r[k][col]:
    //         per wave over its 16 columns (lane rows as in the forward), summed over waves
    if (t > 0) {
      // two rows at a time, each as two 4-deep chains: the compiler otherwise serialises all
      // 8 rows into one 8-deep dependent pk_fma chain (register pressure at the 256 cap)
#pragma unroll
      for (int i = 0; i < 8; i += 2) {
        f2 a0 = w0[i][0] * dgp[0], a1 = w0[i][4] * dgp[4];
        f2 b0 = w0[i + 1][0] * dgp[0], b1 = w0[i + 1][4] * dgp[4];
#pragma unroll
        for (int k = 1; k < 4; ++k) {
          a0 = __builtin_elementwise_fma(w0[i][k], dgp[k], a0);
          a1 = __builtin_elementwise_fma(w0[i][k + 4], dgp[k + 4], a1);
          b0 = __builtin_elementwise_fma(w0[i + 1][k], dgp[k], b0);
          b1 = __builtin_elementwise_fma(w0[i + 1][k + 4], dgp[k + 4], b1);
        }
        const f2 a = a0 + a1, b2 = b0 + b1;
        const int row = i < 4 ? kC + 64 * i + lane : 64 * (i - 4) + lane;
        const int row1 = i + 1 < 4 ? kC + 64 * (i + 1) + lane : 64 * (i + 1 - 4) + lane;
        wred[wave][row] = a.x + a.y;
        wred[wave][row1] = b2.x + b2.y;
      }
      {
        const int r2 = lane & 31, hsel = lane >> 5;
        const float4 wa = *reinterpret_cast<const float4*>(&wc2[r2][16 * wave + 8 * hsel]);
        const float4 wb = *reinterpret_cast<const float4*>(&wc2[r2][16 * wave + 8 * hsel + 4]);
        // (hsel is per lane: select the 4 gate-gradient pairs explicitly -- indexing the
        // register array with it compiled to a 16-way v_cmp/v_cndmask chain per operand)
        const bool hi = hsel != 0;
        const f2 g0 = hi ? dgp[4] : dgp[0], g1 = hi ? dgp[5] : dgp[1];
        const f2 g2 = hi ? dgp[6] : dgp[2], g3 = hi ? dgp[7] : dgp[3];
        f2 a = f2{wa.x, wa.y} * g0;
        a = __builtin_elementwise_fma(f2{wa.z, wa.w}, g1, a);
        a = __builtin_elementwise_fma(f2{wb.x, wb.y}, g2, a);
        a = __builtin_elementwise_fma(f2{wb.z, wb.w}, g3, a);
        const float s = fold32(a.x + a.y);
        if (lane < kM2) wred[wave][kM1 + lane] = s;
      }
      tick(13);
      lds_barrier();
      // sum over the 8 waves (136 float4) and publish R_t
      if (tid < kK0 / 4) {
        float4 a = reinterpret_cast<const float4*>(&wred[0][0])[tid];
#pragma unroll
        for (int w = 1; w < kW; ++w) a = add4(a, reinterpret_cast<const float4*>(&wred[w][0])[tid]);
        const int rr = (((q & 1) * B + b) * kW + j) * kRR;
        stc4x(xl, rRR, rr / 4 + tid, tagf4(a, bit));
      }
    }
    tick(14);
  }
  if (p.prof && tid0 == 0)
    for (int i = 0; i < 16; ++i) p.prof[blockIdx.x * 16 + i] = tp[i];
}

}  // namespace

bool dec_attn_bwd8_eligible(const SatDecAttnBwd* a) {
  const char* e = getenv("SAT_ATTN_BWD8");
  if (e && e[0] == '0') return false;
  return a->U == kU && a->M1 == kM1 && a->M2 == kM2 && a->D1 == kD1 && a->D2 == kD2 &&
         a->F == kF && a->KW == kKW && a->B >= 1 && a->B <= kGmax && a->N >= 1 &&
         a->N <= kW * kPmax;
}

// Scratch: records Q / R and the placement words live in the RDP buffer of
// sat_decoder_attention_bwd_scratch (2 B 32 544 floats >= 2 B 8 (320 + 544) + 256).
int dec_attn_bwd8_launch(const SatDecAttnBwd* a, hipStream_t s) {
  int dev = 0, cus = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, dec_attn_bwd8_kernel, kTh, 0) != hipSuccess) {
    set_error("sat_decoder_attention_bwd: device query failed");
    return SAT_ERR_HIP;
  }
  SAT_CHECK_ARG((int64_t)cus * per_cu >= kGmax * kW,
                "sat_decoder_attention_bwd: fewer than 256 co-resident workgroups on this device");
  Bwd8P p;
  p.B = a->B; p.N = a->N; p.T = a->T;
  p.P = std::max(kHL, ceil_div(a->N, kW));
  p.u = a->u; p.zc = a->zc; p.zh = a->zh;
  p.REC0 = a->REC0; p.C0 = a->C0; p.G0 = a->G0; p.S1 = a->S1; p.AL1 = a->AL1;
  p.S2 = a->S2; p.ST = a->ST; p.LOC = a->LOC; p.V1 = a->V1; p.V2 = a->V2;
  p.v1 = a->v1; p.convW = a->convW; p.convb = a->convb; p.locW = a->locW; p.v2 = a->v2;
  p.W0r = a->W0r; p.Wq1 = a->Wq1; p.Wq2 = a->Wq2; p.mask_c = a->mask_c; p.mask_h = a->mask_h;
  p.DH0 = a->DH0; p.ZH = a->ZH; p.RD = a->RD; p.DG0 = a->DG0; p.DE1 = a->DE1; p.DE2 = a->DE2;
  p.DFH = a->DFH; p.DQP = a->DQP;
  const int64_t rq = (int64_t)2 * a->B * kW * kRQ, rr = (int64_t)2 * a->B * kW * kRR;
  p.RQ = a->RDP;
  p.RR = a->RDP + rq;
  p.XID = reinterpret_cast<unsigned*>(a->RDP + rq + rr);
  p.err = a->err;
  p.flags = xcd_local_env();
  p.prof = reinterpret_cast<long long*>(a->prof);
  if (zero_ranges(s, a->RDP, rq + rr + kGmax * kW, a->err, 2) != hipSuccess) {
    set_error("sat_decoder_attention_bwd: scratch clear failed");
    return SAT_ERR_HIP;
  }
  hipLaunchKernelGGL(dec_attn_bwd8_kernel, dim3(kGmax * kW), dim3(kTh), 0, s, p);
  SAT_LAUNCH_CHECK("sat_decoder_attention_bwd");
  return SAT_OK;
}

}  // namespace sat

// query-gradient parts per step the BPTT writes into DQP [T][B][parts][D1+D2]: 1 when the
// one-utterance-per-8-workgroups kernel applies (dq_t fully reduced), else ceil(N / 32)
extern "C" int32_t sat_decoder_attention_bwd_dq_parts(int32_t B, int32_t N) {
  SatDecAttnBwd a{};
  a.B = B; a.N = N; a.U = sat::kU; a.M1 = sat::kM1; a.M2 = sat::kM2; a.D1 = sat::kD1;
  a.D2 = sat::kD2; a.F = sat::kF; a.KW = sat::kKW;
  return sat::dec_attn_bwd8_eligible(&a) ? 1 : (N + 31) / 32;
}
