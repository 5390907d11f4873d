// Persistent attention chain of the decoder forward, one utterance per group of 8 workgroups:
// ALL T' steps of
//   attention RNN (ZoneoutLSTM 256)  ->  query layers  ->  dual-source attention (+ contexts)
// in ONE launch (DualSourceAttentionRNN, modules/module.py:1017-1048, with ForwardAttention
// modules/forward_attention.py:88-122 and TF BahdanauAttention as attention2; zoneout LSTM as in
// lstm.hip).  Same histories as decoder_persistent.hip (which it replaces for N <= 256).
//
// Why a second layout: the 8 x 32 layout (4 utterances per 32-workgroup group) pays two
// 32-producer all-gathers per decoder step -- every workgroup re-reads ~33 KB of tile records,
// every tile workgroup 32 KB of query partials -- and those hand-offs were 60 % of its 11 us
// per step.  Here group g = utterance g owns 8 workgroups (blockIdx = g + 32 j, one XCD under
// the observed round-robin placement); workgroup j holds
//   * LSTM units [32j, 32j+32): their 128 gate columns x 512 inputs in registers (128 per lane
//     at 512 threads; the 32 c2 rows in LDS), and their 32 query rows (32 KB) in LDS;
//   * memory positions [jP, jP+P), P = max(5, ceil(N/8)) <= 32: K1/V1/K2/V2 rows in LDS.
// Per decoder step two 8-producer hand-offs of ~1.2 KB records, both data-tagged (every word
// carries the step parity in its mantissa LSB, persistent.h lsb_tag):
//   record A_t = {query partial of the own units (256), h_t state of the own units (32)};
//   record B_t = {tile statistics (m1, z1, a1, m2, z2), unnormalised partial contexts (288),
//                 the tile's first 5 / last 4 energies and last 2 alignments (the halos the
//                 neighbours' location convolution and alignment recursion need)}.
// Iteration t:  [B_{t-1}: combine c_{t-1}] -> LSTM step t (h part of the dot done at the end of
// iteration t-1) -> publish A_t -> [normalise s_{t-1}, alpha_{t-1} on the own positions,
// location features, query-independent part of the energies -- all in the shadow of A_t's
// latency] -> [A_t: q_t, h_t] -> energies, tile statistics, partial contexts -> publish B_t ->
// h part of step t+1's gate sums.
// Consistency rule: every value that crosses a workgroup boundary is tagged when it is made and
// its maker uses the tagged value too, so all readers (and the histories) see identical bits.
// Every spin is bounded (persistent.h poll_give_up): a timeout raises err[0], later polls give
// up and the grid drains.
#include "sat_common.h"
#include "persistent.h"

#ifndef SAT_FWD8_TRACE
#define SAT_FWD8_TRACE 0
#endif
#ifndef SAT_FWD8_NORM3
#define SAT_FWD8_NORM3 1     // the normalise window's history stores on wave 7 (A/B switch)
#endif
#ifndef SAT_FWD8_HSTORE7
#define SAT_FWD8_HSTORE7 1   // the cell's C0 / REC0 / H0RAW / G0 stores on wave 7 (A/B switch)
#endif
#ifndef SAT_FWD8_ESCALE
// the energies' tanh argument pre-scaled: K + b1 + convb W_loc and the folded location weights
// held x 2 log2(e) in LDS, so tanh(a + q) = 1 - 2 / (1 + exp2(fma(q, 2 log2 e, a'))) takes one
// fma where the plain form took an add and a multiply (16 per lane per step): 5.65 -> 5.58 us
// per step over three interleaved rounds on one box (profiles/r05_fwd8_ab.txt)
#define SAT_FWD8_ESCALE 1
#endif
#ifndef SAT_FWD8_POLL1
// the hand-off polls' first attempt branch-free: every lane issues its loads (clamped in-record
// addresses for lanes without one), the tags are checked, and only a miss enters the retry
// loop -- the first attempt succeeds on the critical path (trace: 0 spins), where the loop's
// per-load exec-mask branches were ~30 branches + 150 scalar instructions of the staging phase
#define SAT_FWD8_POLL1 1
#endif
#ifndef SAT_FWD8_HMERGE
// the h part of the gate sums inside the cell phase's dot (one dot, one transpose-reduce) rather
// than a separate h-dot after publishing record B: 5.84 -> 5.78 us/step (three interleaved
// rounds on one box).  The separate h-dot was meant to hide in B's latency, but the group's
// last publisher (whichever workgroup it is) never waits -- every other record is already
// there when it polls -- so its h-dot sat on the group's period (0: the old placement, A/B)
#define SAT_FWD8_HMERGE 1
#endif

#ifndef SAT_FWD8_R1
// the S1 / S2 / ST history stores of step t-1 on wave 7 in the location-term window (where it
// holds no positions and idles until record A_t arrives) instead of the combine window, where
// the trace showed wave 7 finishing last (1.51 vs <= 1.39 us into the step): with R2,
// 5.16 -> 5.10 us/step (two A/B rounds on one box, profiles/r06i_fwd8_rebalance_ab.txt)
#define SAT_FWD8_R1 1
#endif
#ifndef SAT_FWD8_R2
// record B's halo words published by wave 7 at the start of the statistics phase (the energies
// and alpha_{t-1} are final there) instead of by wave 1 after its contexts: wave 1, which also
// publishes the statistics, was the group's last B publisher in the trace: with R1,
// 5.21 -> 5.10 us/step
#define SAT_FWD8_R2 1
#endif
#ifndef SAT_FWD8_STW
#define SAT_FWD8_STW 1   // the wave that sums and publishes record B's statistics words
#endif
#ifndef SAT_FWD8_R4
#define SAT_FWD8_R4 0    // A/B: the AL1 history store on wave 7 in the location window
#endif
#ifndef SAT_FWD8_C2W
// the wave that forms the 32 c2 partial contexts besides its own c1 columns (A/B: wave 3, the
// trace's earliest B publisher, measured 5.10 -> 5.14 us/step against wave 0)
#define SAT_FWD8_C2W 0
#endif

namespace sat {
namespace {

constexpr int kW = 8;                  // workgroups per utterance
constexpr int kGmax = 32;              // utterances (groups); grid = 256
constexpr int kTh = 512;               // threads: 8 waves, 2 per SIMD (256 registers each)
constexpr int kU = 256, kM1 = 256, kM2 = 32, kD1 = 224, kD2 = 32, kF = 5, kKW = 10;
constexpr int kC = kM1 + kM2;          // 288 context dims
constexpr int kK0 = kC + kU;           // 544 inputs of the attention RNN's recurrent product
constexpr int kQ = kD1 + kD2;          // 256 query dims
constexpr int kUW = kU / kW;           // 32 units per workgroup
constexpr int kPmax = 32;              // memory positions per workgroup
constexpr int kPadL = (kKW - 1) / 2;   // 4: SAME padding of the location convolution
constexpr int kPadR = kKW - 1 - kPadL; // 5
constexpr int kRA = kQ + kUW;          // record A floats
constexpr int kRB = 320;               // record B floats (307 used)
constexpr int kRBctx = 8, kRBeh = kRBctx + kC, kRBet = kRBeh + kPadR, kRBal = kRBet + kPadL;
constexpr int kR4 = 2 + kC / 4;        // staged record B: 2 statistics float4 + 72 context float4
constexpr float kTwoLog2e = 2.8853900817779268f;   // 2 log2(e)
static_assert(kRBal + 2 <= kRB && kK0 == 544 && kQ == 256 && kD1 % 16 == 0, "layout");

struct Fwd8P {
  int B, N, T, P, flags;
  float u, zc, zh;
  const float* X0; const float* W0r; const float* Wq1; const float* Wq2;
  const float* K1; const float* V1; const float* K2; const float* V2;
  const int64_t* lengths;
  const float* v1; const float* b1; const float* convW; const float* convb; const float* locW;
  const float* v2;
  const float* mask_c; const float* mask_h;
  float* REC0; float* C0; float* H0RAW; float* G0; float* Q;
  float* S1; float* AL1; float* S2; float* ST; float* LOC; float* ZH;
  float* RA;        // [2][B][8][kRA] tagged
  float* RB;        // [2][B][8][kRB] tagged
  unsigned* XID;    // [256] XCC_ID + 1 per workgroup (zeroed)
  int* err;
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
// logistic with one v_exp and one v_rcp (1-ulp reciprocal; no IEEE division sequence)
__device__ __forceinline__ float sigm_fast(float x) {
  return __builtin_amdgcn_rcpf(1.f + __expf(-x));
}
// x[l] + x[l ^ 32] in lanes l < 32 (gfx950 v_permlane32_swap)
__device__ __forceinline__ float fold32(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// lanes 4k (k < 8) gather the values of lanes 4k .. 4k+3 (row shifts inside 16-lane rows)
__device__ __forceinline__ float4 quad_gather(float x) {
  return make_float4(x, dpp_mov<0x101>(x), dpp_mov<0x102>(x), dpp_mov<0x103>(x));
}

__global__ void __launch_bounds__(kTh) dec_attn_fwd8_kernel(Fwd8P p) {
  // resident operands
  __shared__ __attribute__((aligned(16))) float kc[kPmax][kQ];       // [K1 + b1 | K2] rows
  __shared__ __attribute__((aligned(16))) float v1s[kPmax][kM1];
  __shared__ __attribute__((aligned(16))) float v2s[kPmax][kM2];
  __shared__ __attribute__((aligned(16))) float wqs[kUW][kQ];
  __shared__ __attribute__((aligned(16))) float wc2[kM2][4 * kUW + 4];   // padded rows (banks)
  // the location term folded: l[n] = f[n] W_loc = convb W_loc + sum_k s[n-4+k] (W_conv[k] W_loc)
  __shared__ __attribute__((aligned(16))) float cwl[kKW][kQ];        // W_conv W_loc, cols >= D1 zero
  __shared__ __attribute__((aligned(16))) float vcat[kQ];            // [v1 | v2]
  __shared__ float cw[kKW * kF + kF];
  // per step
  __shared__ __attribute__((aligned(16))) float hbuf[kU];        // h_t states (next LSTM input)
  __shared__ __attribute__((aligned(16))) float cbuf[kC];        // c_{t-1}
  __shared__ __attribute__((aligned(16))) float4 qst[kW][64];    // staged query partials
  __shared__ __attribute__((aligned(16))) float4 recs[kW][kR4];  // staged records B_{t-1}
  __shared__ __attribute__((aligned(16))) float hst[kUW];        // own units' h_t (tagged)
  __shared__ __attribute__((aligned(16))) float hraw[kUW];       // own units' raw outputs
  __shared__ float cown[kUW];                                    // own units' c_t
  __shared__ __attribute__((aligned(16))) float4 gown[kUW];      // own units' gates (i, j, f, o)
  __shared__ float gsum[8][64];             // h part of the gate sums (transpose-reduced)
  __shared__ float halo[12];                // e_{t-1} left 4 | right 5 ; alpha_{t-2} at n0-2, n0-1
  __shared__ float eown[kPmax], e2own[kPmax];
  __shared__ float alf[2][kPmax + 1];       // alf[t & 1][k] = alpha_{t-1} at n0 - 1 + k
  __shared__ float sp[kPmax + kKW];         // s_{t-1} on n0-4 .. n0+nt+4
  __shared__ __attribute__((aligned(16))) float wsc[8][2][kPmax];     // per-wave alignment weights
  __shared__ long long tp[16];              // optional segment clocks of thread 0

  const int tid0 = threadIdx.x;
  const int g = blockIdx.x % kGmax, j = blockIdx.x / kGmax;
  const int B = p.B, N = p.N, T = p.T, P = p.P;
  if (g >= B) return;                       // no utterance: no partner outside this group
  const int b = g;
  const int n0 = j * P, nt = max(0, min(P, N - n0));
  const bool has_left = j > 0, has_right = j + 1 < kW && n0 + P < N;
  // wave 7 holds no energy positions when nt <= 28: it then stores the cell's histories in the
  // location-term phase (from LDS) instead of the cell lanes of every wave
  const bool w7_stores = SAT_FWD8_HSTORE7 && 4 * 7 >= nt;
  const int64_t bN = (int64_t)b * N;
  const int len = (int)p.lengths[b];
  const float u = p.u;
  const auto rRA = rsrc(p.RA), rRB = rsrc(p.RB);

  // ---------------- prologue
  // LSTM: wave w owns gate columns 128j + 16w + m (m < 16: unit 32j + 4w + m/4, gate m%4);
  // lane owns input rows: chunk i < 4 -> h row 64i + lane, 4 <= i < 8 -> c1 row 64(i-4) +
  // lane; the 32 c2 rows sit in LDS (wc2).  W0r rows are [c1 | c2 | h].
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
  for (int i = tid0; i < kPmax * kQ; i += kTh) {
    const int r = i / kQ, c = i - r * kQ;
    float lb = 0.f;                              // convb W_loc (the location term's constant)
    if (c < kD1) {
#pragma unroll
      for (int f = 0; f < kF; ++f) lb = fmaf(p.convb[f], p.locW[f * kD1 + c], lb);
    }
    const float kv = r >= nt ? 0.f : c < kD1 ? p.K1[(bN + n0 + r) * kD1 + c] + p.b1[c] + lb
                                            : p.K2[(bN + n0 + r) * kD2 + (c - kD1)];
    kc[r][c] = SAT_FWD8_ESCALE ? kv * kTwoLog2e : kv;
  }
  for (int i = tid0; i < kKW * kQ; i += kTh) {
    const int k = i / kQ, c = i - k * kQ;
    float a = 0.f;
    if (c < kD1) {
#pragma unroll
      for (int f = 0; f < kF; ++f) a = fmaf(p.convW[k * kF + f], p.locW[f * kD1 + c], a);
    }
    cwl[k][c] = SAT_FWD8_ESCALE ? a * kTwoLog2e : a;
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
  for (int d = tid0; d < kQ; d += kTh) vcat[d] = d < kD1 ? p.v1[d] : p.v2[d - kD1];
  if (tid0 < kKW * kF) cw[tid0] = p.convW[tid0];
  if (tid0 < kF) cw[kKW * kF + tid0] = p.convb[tid0];
  if (tid0 < kU) hbuf[tid0] = 0.f;                                  // h_{-1}
  if (tid0 < 16) tp[tid0] = 0;
  gsum[tid0 >> 6][tid0 & 63] = 0.f;          // h_{-1} = 0: no h part at step 0
  // initial state rows (host): s_{-1} on the conv window, alpha_{-1} on n0-1 .. n0+nt-1
  // (tagged with step 0's bit: they travel in record B_0)
  if (tid0 < nt + kKW - 1) {
    const int n = n0 - kPadL + tid0;
    sp[tid0] = (n >= 0 && n < N) ? p.S1[bN + n] : 0.f;
  }
  if (tid0 >= 64 && tid0 - 64 <= nt) {
    const int n = n0 - 1 + (tid0 - 64);
    alf[0][tid0 - 64] = tagf(n >= 0 ? p.AL1[bN + n] : 0.f, lsb_tag(0));
  }
  // after the transpose-reduce lane l holds gate column m = l >> 2 of its wave: unit
  // 32j + 4 wave + (m >> 2), gate m & 3; it prefetches that gate's X0 term, cell lanes (16q)
  // also the zoneout masks
  float c_own = 0.f, h_own = 0.f;
  const bool masked = p.mask_c != nullptr;
  auto load_ops = [&](int tt, int lane_, int wave_, float& xg_, float& mc_, float& mh_) {
    const int m = lane_ >> 2;
    const int64_t bu = ((int64_t)(tt < T ? tt : 0) * B + b) * kU + kUW * j + 4 * wave_ + (m >> 2);
    xg_ = p.X0[4 * bu + (m & 3)];
    const bool cl = (lane_ & 15) == 0 && masked;
    mc_ = cl ? p.mask_c[bu] : 1.f - p.zc;
    mh_ = cl ? p.mask_h[bu] : 1.f - p.zh;
  };
  float xgn, mcn, mhn;
  load_ops(0, tid0 & 63, tid0 >> 6, xgn, mcn, mhn);
  __syncthreads();

  const bool xl = (p.flags & 1) ? xcd_local_group(p.XID, g, kGmax, kW, p.err) : false;

#if SAT_FWD8_TRACE || SAT_SEGMENT_CLOCKS
  long long t0 = p.prof ? wall_clock64() : 0;
  auto tick = [&](int seg) {
    if (p.prof && tid0 == 0) {
      const long long t1 = wall_clock64();
      tp[seg] += t1 - t0;
      t0 = t1;
    }
  };
#else
  auto tick = [](int) {};   // production build: no clock reads and no per-phase flag tests
#endif
  bool gave_up = false;
  // location features f_t of the own positions from s_{t-1} in sp (the BPTT's LOC history;
  // the forward itself uses the folded form, section 4)
  auto store_loc = [&](int tt, int lane_) {
    if (!p.LOC) return;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int o = lane_ + 64 * h;
      if (o < nt * kF) {
        const int i = o / kF, f = o - i * kF;
        float a = cw[kKW * kF + f];
#pragma unroll
        for (int k = 0; k < kKW; ++k) a = fmaf(sp[i + k], cw[k * kF + f], a);
        p.LOC[(((int64_t)tt * B + b) * N + n0) * kF + o] = a;
      }
    }
  };
  if ((tid0 >> 6) == 5) store_loc(0, tid0 & 63);   // f_0 from the initial state s_{-1}
#if SAT_FWD8_TRACE
  // per-wave event clocks of workgroup 1 over steps 100..107: prof[4096 + ...] (build with
  // -DSAT_FWD8_TRACE=1; tools/probes/fwd8_profile.py prints them)
  // (workgroup 1 = group 1's first: the per-wave stores must not perturb group 0, whose
  // hand-off skew gevt measures)
  long long* evt = (p.prof && blockIdx.x == 1) ? p.prof + 256 * 16 : nullptr;
  // group 0's eight workgroups, wave 0: {A published, A staged, B published, B staged} of steps
  // 100..107 at prof[256 * 16 + 8 * 8 * 20 + ((t - 100) * 8 + j) * 4 + k] (hand-off skew)
  long long* gevt = (p.prof && g == 0) ? p.prof + 256 * 16 + 8 * 8 * 20 + j * 4 : nullptr;
#endif

  // e_{t-1}(n) on the window around the own positions, -inf where masked (the own energies of
  // step t-1 in eown until the energies phase of step t rewrites them; the neighbours' in halo)
  auto e_at = [&](int n) -> float {
    if (n < 0 || n >= len) return -INFINITY;
    if (n < n0) return halo[n - n0 + kPadL];
    if (n < n0 + nt) return eown[n - n0];
    return halo[kPadL + (n - n0 - nt)];
  };
  // step t-1's histories S1 / S2 / ST (normalised alignments of both sources, statistics)
  auto store_hist = [&](int tt, int lane_, float M1, float Z1, float A1, float M2, float Z2) {
    const int ss = tt - 1;
    if (lane_ >= kPadL && lane_ < nt + kPadL) {
      const float e = e_at(n0 - kPadL + lane_);
      p.S1[((int64_t)tt * B + b) * N + n0 + lane_ - kPadL] =
          e == -INFINITY ? 0.f : __expf(e - M1) * __builtin_amdgcn_rcpf(Z1);
    }
    if (lane_ < nt) {
      const float e2 = e2own[lane_];
      p.S2[((int64_t)ss * B + b) * N + n0 + lane_] =
          e2 == -INFINITY ? 0.f : __expf(e2 - M2) * __builtin_amdgcn_rcpf(Z2);
    }
    if (j == 0 && lane_ == 0) {
      float* stp = p.ST + ((int64_t)ss * B + b) * 4;
      stp[0] = M1; stp[1] = Z1; stp[2] = A1 / Z1; stp[3] = Z2;
    }
  };

  for (int t = 0; t <= T; ++t) {
    const int s = t - 1;
    float M1 = 0.f, Z1 = 1.f, A1 = 1.f, M2 = 0.f, Z2 = 1.f;   // statistics of step t-1
    // lane-dependent indices re-derived from an opaque copy of the thread id every step: the
    // compiler cannot hoist per-lane addresses out of the loop (which kept ~150 of them live
    // and spilled the register-resident weights)
    int tid = tid0;
    asm volatile("" : "+v"(tid));
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform (scalar)
    auto ev = [&](int k) {
#if SAT_FWD8_TRACE
      if (evt && t >= 100 && t < 108 && lane == 0) evt[((t - 100) * 8 + wave) * 16 + k] = wall_clock64();
      if (gevt && t >= 100 && t < 108 && tid == 0 && (k == 7 || k == 10 || k == 15 || k == 2)) {
        const int slot = k == 7 ? 0 : k == 10 ? 1 : k == 15 ? 2 : 3;
        // B staged (k == 2) belongs to step t - 1's records
        const int ts = k == 2 ? t - 1 : t;
        if (ts >= 100) gevt[(ts - 100) * 32 + slot] = wall_clock64();
      }
#else
      (void)k;
#endif
    };
    ev(0);
    // ============ 1. records B_{t-1}: wave jj stages record jj (wave 0 lanes 16..26 the halos)
    if (t > 0) {
      const int rb0 = ((s & 1) * B + b) * kW;
      const unsigned want = lsb_tag(s);
      const int rec = (rb0 + wave) * kRB;
      // load 1: c1 chunk `lane`; load 2: lanes 0..7 the c2 chunk, 8..9 the statistics
      const bool two = lane < kM2 / 4 + 2;
      const int i2 = lane < kM2 / 4 ? (rec + kRBctx + kM1) / 4 + lane : rec / 4 + (lane - kM2 / 4);
      // halo words (wave 0 lanes 16..26): 0..3 e_{t-1} at n0-4..n0-1 (left tail), 4..8 at
      // n0+P.. (right head), 9, 10 alpha_{t-2} at n0-2, n0-1 (left)
      const int hq = lane - 16;
      const bool hl = wave == 0 && hq >= 0 && hq < 11;
      const bool hleft = hq < kPadL || hq >= kPadL + kPadR;
      const bool hsrc = hl && (hleft ? has_left : has_right);
      const int hw = (rb0 + (hleft ? j - 1 : j + 1)) * kRB +
                     (hq < kPadL ? kRBet + hq : hq < kPadL + kPadR ? kRBeh + hq - kPadL
                                                                   : kRBal + hq - kPadL - kPadR);
      float4 x1 = make_float4(0.f, 0.f, 0.f, 0.f), x2 = x1;
      float hv = 0.f;
      bool ok1 = false, ok2 = !two, ok3 = !hsrc;
#if SAT_FWD8_TRACE
      // trace build: drain the wave's own earlier stores first, then time the poll alone
      const long long tq0 = wall_clock64();
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const long long tq1 = wall_clock64();
#endif
      bool retry = true;
      if (SAT_FWD8_POLL1) {
        x1 = ldc4(rRB, (rec + kRBctx) / 4 + lane);
        x2 = ldc4(rRB, i2);                    // (lanes >= 10: in-record words, unused)
        const float h0 = ldc(rRB, hsrc ? hw : 0);
        hv = hsrc ? h0 : 0.f;                  // an absent neighbour's halo words stay 0
        ok1 = tag_ok4(x1, want);
        ok2 = ok2 || tag_ok4(x2, want);
        ok3 = ok3 || tag_ok(hv, want);
        retry = any_lane(!(ok1 && ok2 && ok3)) && !gave_up;
      }
      if (retry) {
        for (unsigned spins = 0;; ++spins) {
          if (!ok1) x1 = ldc4(rRB, (rec + kRBctx) / 4 + lane);
          if (!ok2) x2 = ldc4(rRB, i2);
          if (!ok3) hv = ldc(rRB, hsrc ? hw : 0);
          ok1 = tag_ok4(x1, want);
          ok2 = ok2 || tag_ok4(x2, want);
          ok3 = ok3 || tag_ok(hv, want);
          if (!any_lane(!(ok1 && ok2 && ok3)) || gave_up) break;
          if (poll_give_up(spins, p.err)) { gave_up = true; break; }
          __builtin_amdgcn_s_sleep(1);
        }
      }
#if SAT_FWD8_TRACE
      {
        const long long tq2 = wall_clock64();
        if (evt && t >= 100 && t < 108 && lane == 0) {
          evt[8 * 8 * 16 + ((t - 100) * 8 + wave) * 4 + 0] = tq1 - tq0;
          evt[8 * 8 * 16 + ((t - 100) * 8 + wave) * 4 + 1] = tq2 - tq1;
        }
      }
#endif
      recs[wave][2 + lane] = x1;
      if (lane < kM2 / 4) recs[wave][2 + kM1 / 4 + lane] = x2;
      else if (two) recs[wave][lane - kM2 / 4] = x2;
      if (hl) halo[hq] = hv;
      tick(0);
    ev(1);
      lds_barrier();
      tick(1);
    ev(2);
      // combine: thread d < 288 one context dim; the record scales from lanes 0..7 of each
      // wave (DPP, identical arithmetic in every workgroup of the group), broadcast by readlane.
      // Waves 5 and 6 normalise step t-1 on the own positions meanwhile (the statistics
      // formed the same way): s_{t-1} on the convolution window (the next energies' location
      // term reads it) and alpha_{t-1} (tagged for record B_t) -- off the step's critical
      // path, which used to run them after publishing A_t.
      {
        const int jj = lane & 7;
        const float4 st = recs[jj][0];
        const float z2 = recs[jj][1].x;
        M1 = lanes8_max(st.x);
        M2 = lanes8_max(st.w);
        const float sc1 = __expf(st.x - M1), sc2 = __expf(st.w - M2);
        Z1 = lanes8_sum(st.y * sc1);
        A1 = lanes8_sum(st.z * sc1);
        Z2 = lanes8_sum(z2 * sc2);
        if (wave < (kC + 63) / 64) {
          if (tid < kC) {
            const bool first = wave < kM1 / 64;    // wave-uniform: c1 dims (waves 0..3) or c2
            const float sc = first ? sc1 : sc2;
            const float* rf = reinterpret_cast<const float*>(&recs[0][2]) + tid;
            float a = 0.f;
#pragma unroll
            for (int k = 0; k < kW; ++k) a = fmaf(rf[k * kR4 * 4], rdl(sc, k), a);
            a *= __builtin_amdgcn_rcpf(first ? A1 : Z2);
            cbuf[tid] = a;
            // the REC0 context row: every workgroup forms all 288 dims, each stores its own 36
            // (the whole row from workgroup 0 alone put it a step-long offset behind its group)
            if (tid / (kC / kW) == j) p.REC0[((int64_t)t * B + b) * kK0 + tid] = a;
          }
        } else {
          const unsigned bit = lsb_tag(t);
          if (wave == 5) {
            // s_{t-1} = softmax on n0-4 .. n0+nt+4, then (same wave, no barrier) the location
            // features f_t of the own positions for the LOC history of the BPTT
            if (lane < nt + kKW - 1) {
              const float e = e_at(n0 - kPadL + lane);
              const float sv = e == -INFINITY ? 0.f : __expf(e - M1) * __builtin_amdgcn_rcpf(Z1);
              sp[lane] = sv;
              if (!SAT_FWD8_NORM3 && lane >= kPadL && lane < nt + kPadL)
                p.S1[((int64_t)t * B + b) * N + n0 + lane - kPadL] = sv;
            }
            if (t < T && 4 * 7 < nt) {         // no idle energy wave (N > 224): here
              asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
              store_loc(t, lane);
            }
          } else if (wave == 6) {
            const float* ap = alf[(t - 1) & 1];      // alpha_{t-2} at n0-1+k
            if (lane <= nt) {
              const int k = lane, n = n0 - 1 + k;
              float av = 0.f;
              if (n >= 0) {
                // alpha_{t-2} at n and n-1: own from ap, n0-1 / n0-2 from the left halo
                const float a_n = k >= 1 ? ap[k] : halo[kPadL + kPadR + 1];
                const float a_m = k >= 2 ? ap[k - 1] : halo[kPadL + kPadR + k];
                const float e = e_at(n);
                const float pe = e == -INFINITY ? 0.f : __expf(e - M1);
                av = ((1.f - u) * a_n + u * a_m + 1e-7f) * pe * __builtin_amdgcn_rcpf(A1);
              }
              const float at = tagf(av, bit);
              alf[t & 1][k] = at;
              if (k >= 1 && !(SAT_FWD8_R4 && w7_stores && t < T))
                p.AL1[((int64_t)t * B + b) * N + n] = at;
            }
          }
          // wave 7 (idle in this window): the S1 / S2 / ST history stores (S1 recomputed with
          // wave 5's arithmetic: the same bits), off waves 5 and 6 whose LDS results the next
          // phases wait for
          // (deferred to wave 7's location-term window when it idles there, SAT_FWD8_R1; the
          // last step's here)
          const bool defer = SAT_FWD8_R1 && w7_stores && t < T;
          if (SAT_FWD8_NORM3 ? (wave == 7 && !defer) : wave == 6) {
            if (SAT_FWD8_NORM3) {
              store_hist(t, lane, M1, Z1, A1, M2, Z2);
            } else {
              if (lane < nt) {
                const float e2 = e2own[lane];
                p.S2[((int64_t)s * B + b) * N + n0 + lane] =
                    e2 == -INFINITY ? 0.f : __expf(e2 - M2) * __builtin_amdgcn_rcpf(Z2);
              }
              if (j == 0 && lane == 0) {
                float* stp = p.ST + ((int64_t)s * B + b) * 4;
                stp[0] = M1; stp[1] = Z1; stp[2] = A1 / Z1; stp[3] = Z2;
              }
            }
          }
        }
      }
    }
    tick(2);
    ev(3);
    lds_barrier();
    tick(3);
    ev(4);

    // ============ 2. LSTM step t: c part of the dot, gates (one activation per lane), cell;
    //                 publish record A_t
    if (t < T) {
      f2 acc[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] = f2{0.f, 0.f};
      if (t > 0) {
#if SAT_FWD8_HMERGE
        // h_{t-1} (staged with records A_{t-1}) and c_{t-1} in ONE dot and ONE transpose-reduce
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float xv = hbuf[64 * i + lane];
          const f2 xx = {xv, xv};
#pragma unroll
          for (int q = 0; q < 8; ++q) acc[q] = __builtin_elementwise_fma(xx, w0[i][q], acc[q]);
        }
#endif
#pragma unroll
        for (int i = 4; i < 8; ++i) {
          const float xv = cbuf[64 * (i - 4) + lane];
          const f2 xx = {xv, xv};
#pragma unroll
          for (int q = 0; q < 8; ++q) acc[q] = __builtin_elementwise_fma(xx, w0[i][q], acc[q]);
        }
        // c2 rows from LDS: lane l takes row l & 31 and columns 8 (l >> 5) .. + 7
        const int r2 = lane & 31, hsel = lane >> 5;
        const float xv = cbuf[kM1 + r2];
        const f2 xx = {xv, xv};
        const float4 wa = *reinterpret_cast<const float4*>(&wc2[r2][16 * wave + 8 * hsel]);
        const float4 wb = *reinterpret_cast<const float4*>(&wc2[r2][16 * wave + 8 * hsel + 4]);
        const f2 c0 = __builtin_elementwise_fma(xx, f2{wa.x, wa.y}, f2{0.f, 0.f});
        const f2 c1 = __builtin_elementwise_fma(xx, f2{wa.z, wa.w}, f2{0.f, 0.f});
        const f2 c2 = __builtin_elementwise_fma(xx, f2{wb.x, wb.y}, f2{0.f, 0.f});
        const f2 c3 = __builtin_elementwise_fma(xx, f2{wb.z, wb.w}, f2{0.f, 0.f});
        if (hsel == 0) { acc[0] += c0; acc[1] += c1; acc[2] += c2; acc[3] += c3; }
        else { acc[4] += c0; acc[5] += c1; acc[6] += c2; acc[7] += c3; }
      }
      float v[16];
#pragma unroll
      for (int q = 0; q < 8; ++q) { v[2 * q] = acc[q].x; v[2 * q + 1] = acc[q].y; }
      transpose_reduce16(v, lane);
      // lane holds column m = lane >> 2: activation of its gate (i, f, o sigmoid; j tanh via
      // 2 sigm(2x) - 1; forget_bias 1.0), then the cell lane (16q) gathers its unit's 4 gates
      const int gate = (lane >> 2) & 3;
#if SAT_FWD8_HMERGE
      const float pre = v[0] + xgn;
#else
      const float pre = v[0] + gsum[wave][lane] + xgn;
#endif
      const float sg = sigm_fast(gate == 1 ? 2.f * pre : pre + (gate == 2 ? 1.0f : 0.f));
      const float act = gate == 1 ? fmaf(2.f, sg, -1.f) : sg;
      const float gj = dpp_mov<0x104>(act);        // row_shl:4, 8, 12
      const float gf = dpp_mov<0x108>(act);
      const float go = dpp_mov<0x10C>(act);
      const bool cell = (lane & 15) == 0;
      const int cq = lane >> 4, cunit = kUW * j + 4 * wave + cq;
      const float mc = mcn, mh = mhn;
      const unsigned bit = lsb_tag(t);
      if (cell) {
        const float gi = act;
        const float cn = gf * c_own + gi * gj;
        const float hn = go * fmaf(2.f, sigm_fast(2.f * cn), -1.f);   // o * tanh(c)
        const float c2 = mc * cn + (1.f - mc) * c_own;
        const float h2 = tagf(mh * hn + (1.f - mh) * h_own, bit);   // what every reader sees
        c_own = c2; h_own = h2;
        hst[4 * wave + cq] = h2;
        hraw[4 * wave + cq] = hn;
        if (w7_stores) {
          cown[4 * wave + cq] = c2;
          gown[4 * wave + cq] = make_float4(gi, gj, gf, go);
        } else {
          const int64_t tbu = ((int64_t)t * B + b) * kU + cunit;
          p.C0[((int64_t)(t + 1) * B + b) * kU + cunit] = c2;
          p.REC0[((int64_t)(t + 1) * B + b) * kK0 + kC + cunit] = h2;
          p.H0RAW[tbu] = hn;
          reinterpret_cast<float4*>(p.G0)[tbu] = make_float4(gi, gj, gf, go);
        }
      }
      load_ops(t + 1, lane, wave, xgn, mcn, mhn);
      tick(4);
    ev(5);
      lds_barrier();
      tick(5);
    ev(6);
      // query partial over the own 32 units: wave w owns query columns 32w .. 32w+31; lane l
      // column 32w + (l & 31), units 16 (l >> 5) .. + 15; halves folded, quads gathered
      {
        const int col = 32 * wave + (lane & 31), u0 = 16 * (lane >> 5);
        float a = 0.f;
#pragma unroll
        for (int k4 = 0; k4 < 4; ++k4) {
          const float4 h4 = *reinterpret_cast<const float4*>(&hraw[u0 + 4 * k4]);
          a = fmaf(h4.x, wqs[u0 + 4 * k4][col], a);
          a = fmaf(h4.y, wqs[u0 + 4 * k4 + 1][col], a);
          a = fmaf(h4.z, wqs[u0 + 4 * k4 + 2][col], a);
          a = fmaf(h4.w, wqs[u0 + 4 * k4 + 3][col], a);
        }
        const float4 q4 = quad_gather(fold32(a));
        const int ra = (((t & 1) * B + b) * kW + j) * kRA;
        if (lane < 32 && (lane & 3) == 0) stc4x(xl, rRA, ra / 4 + 8 * wave + (lane >> 2), tagf4(q4, bit));
        if (wave == 1 && lane < kUW / 4)
          stc4x(xl, rRA, (ra + kQ) / 4 + lane, *reinterpret_cast<const float4*>(&hst[4 * lane]));
      }
      tick(6);
    ev(7);
    }

    if (t == T) break;
    tick(7);
    ev(8);

    // ============ 4. the query-independent energy part of step t (s_{t-1} came from wave 5
    //                 before the last barrier): a = K + b1 + convb W_loc + sum_k s_{t-1}[n-4+k]
    //                 (W_conv[k] W_loc) -- the location convolution and layer folded into one
    //                 10-tap product (modules/forward_attention.py:98-101)
    // energy role: lane = dim chunk c (4 dims of [D1 | D2]), wave = positions 4w .. 4w+3
    float4 Lr[4];
    if (SAT_FWD8_R1 && SAT_FWD8_NORM3 && w7_stores && wave == 7 && t > 0)
      store_hist(t, lane, M1, Z1, A1, M2, Z2);   // wave 7 holds no positions: idle here
    if (SAT_FWD8_R4 && w7_stores && wave == 7 && t > 0 && lane >= 1 && lane <= nt &&
        n0 - 1 + lane >= 0)
      p.AL1[((int64_t)t * B + b) * N + n0 - 1 + lane] = alf[t & 1][lane];   // alpha_{t-1}
    if (4 * wave < nt) {
      const int c = lane;
#pragma unroll
      for (int i = 0; i < 4; ++i) Lr[i] = *reinterpret_cast<const float4*>(&kc[4 * wave + i][4 * c]);
#pragma unroll
      for (int k = 0; k < kKW; ++k) {
        const float4 wk = *reinterpret_cast<const float4*>(&cwl[k][4 * c]);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float sv = sp[4 * wave + i + k];
          Lr[i].x = fmaf(sv, wk.x, Lr[i].x); Lr[i].y = fmaf(sv, wk.y, Lr[i].y);
          Lr[i].z = fmaf(sv, wk.z, Lr[i].z); Lr[i].w = fmaf(sv, wk.w, Lr[i].w);
        }
      }
    }
    tick(8);
    ev(9);

    // ============ 5. records A_t: wave jj stages record jj (query partial, h_t states)
    {
      const unsigned want = lsb_tag(t);
      const int ra = (((t & 1) * B + b) * kW + wave) * kRA;
      const bool two = lane < kUW / 4;
      float4 x1 = make_float4(0.f, 0.f, 0.f, 0.f), x2 = x1;
      bool ok1 = false, ok2 = !two;
#if SAT_FWD8_TRACE
      const long long tq0 = wall_clock64();
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const long long tq1 = wall_clock64();
#endif
      bool retry = true;
      if (SAT_FWD8_POLL1) {
        x1 = ldc4(rRA, ra / 4 + lane);
        x2 = ldc4(rRA, (ra + kQ) / 4 + (two ? lane : 0));
        ok1 = tag_ok4(x1, want);
        ok2 = ok2 || tag_ok4(x2, want);
        retry = any_lane(!(ok1 && ok2)) && !gave_up;
      }
      if (retry) {
        for (unsigned spins = 0;; ++spins) {
          if (!ok1) x1 = ldc4(rRA, ra / 4 + lane);
          if (!ok2) x2 = ldc4(rRA, (ra + kQ) / 4 + lane);
          ok1 = tag_ok4(x1, want);
          ok2 = ok2 || tag_ok4(x2, want);
          if (!any_lane(!(ok1 && ok2)) || gave_up) break;
          if (poll_give_up(spins, p.err)) { gave_up = true; break; }
          __builtin_amdgcn_s_sleep(1);
        }
      }
#if SAT_FWD8_TRACE
      {
        const long long tq2 = wall_clock64();
        if (evt && t >= 100 && t < 108 && lane == 0) {
          evt[8 * 8 * 16 + ((t - 100) * 8 + wave) * 4 + 2] = tq1 - tq0;
          evt[8 * 8 * 16 + ((t - 100) * 8 + wave) * 4 + 3] = tq2 - tq1;
        }
      }
#endif
      qst[wave][lane] = x1;
      if (two) reinterpret_cast<float4*>(hbuf)[(kUW / 4) * wave + lane] = x2;   // units 32 jj + 4 lane
    }
    tick(9);
    ev(10);
    lds_barrier();
    tick(10);
    ev(11);

    // ============ 6. energies: q chunk summed per lane (record order), tanh, dots with v
    if (4 * wave < nt) {
      const unsigned bit = lsb_tag(t);
      const int c = lane;
      float4 q = qst[0][c];
#pragma unroll
      for (int k = 1; k < kW; ++k) q = add4(q, qst[k][c]);
      // the Q row likewise: chunks 8j .. 8j+7 from workgroup j
      if (wave == 0 && (c >> 3) == j) reinterpret_cast<float4*>(p.Q + ((int64_t)t * B + b) * kQ)[c] = q;
      const float4 v4 = *reinterpret_cast<const float4*>(&vcat[4 * c]);
      const bool d1 = c < kD1 / 4;
      float e[8];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = 4 * wave + i;
#if SAT_FWD8_ESCALE
        auto tz = [](float a2, float qv) {        // tanh(a + q) from a' = 2 log2(e) a
          return fmaf(-2.f, __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(fmaf(qv, kTwoLog2e, a2))), 1.f);
        };
        const float4 z = make_float4(tz(Lr[i].x, q.x), tz(Lr[i].y, q.y), tz(Lr[i].z, q.z),
                                     tz(Lr[i].w, q.w));
#else
        const float4 z = make_float4(tanh_fast(Lr[i].x + q.x), tanh_fast(Lr[i].y + q.y),
                                     tanh_fast(Lr[i].z + q.z), tanh_fast(Lr[i].w + q.w));
#endif
        float a = v4.x * z.x;
        a = fmaf(v4.y, z.y, a); a = fmaf(v4.z, z.z, a); a = fmaf(v4.w, z.w, a);
        e[i] = d1 ? a : 0.f;
        e[4 + i] = d1 ? 0.f : a;
        if (p.ZH && r < nt)                    // energy tanh history for the BPTT (streamed out)
          __builtin_nontemporal_store(f4v{z.x, z.y, z.z, z.w},
                                      reinterpret_cast<f4v*>(p.ZH + (((int64_t)t * B + b) * N + n0 + r) * kQ + 4 * c));
      }
      transpose_reduce8(e, lane);              // lanes 8m..8m+7 hold sum m
      if ((lane & 7) == 0) {
        const int m = lane >> 3, r = 4 * wave + (m & 3);
        const bool valid = r < nt && n0 + r < len;
        const float ev = valid ? tagf(e[0], bit) : -INFINITY;
        if (m < 4) eown[r] = ev; else e2own[r] = ev;
      }
    } else {                                   // idle wave: its positions are padding
      const int r = 4 * wave + (lane & 3);
      if (lane < 4) eown[r] = -INFINITY; else if (lane < 8) e2own[r] = -INFINITY;
      if (wave == 0 && (lane >> 3) == j) {
        // no own positions (nt == 0, small N): the Q row's chunks 8j .. 8j+7 are still this
        // workgroup's to store, summed in the same record order as the energy waves'
        float4 q = qst[0][lane];
#pragma unroll
        for (int k = 1; k < kW; ++k) q = add4(q, qst[k][lane]);
        reinterpret_cast<float4*>(p.Q + ((int64_t)t * B + b) * kQ)[lane] = q;
      }
      if (wave == 7) {
        store_loc(t, lane);                    // the LOC history, off the critical path
        if (w7_stores && lane < kUW) {
          // the cell's histories of step t for the own 32 units (in LDS since the cell
          // barrier; rewritten only by step t+1's cell): one coalesced store each instead of
          // four scattered ones per cell lane of every wave
          const int cunit = kUW * j + lane;
          const int64_t tbu = ((int64_t)t * B + b) * kU + cunit;
          p.C0[((int64_t)(t + 1) * B + b) * kU + cunit] = cown[lane];
          p.REC0[((int64_t)(t + 1) * B + b) * kK0 + kC + cunit] = hst[lane];
          p.H0RAW[tbu] = hraw[lane];
          reinterpret_cast<float4*>(p.G0)[tbu] = gown[lane];
        }
      }
    }
    tick(11);
    ev(12);
    lds_barrier();
    tick(12);
    ev(13);
    // tile statistics (every wave redundantly, lane = position) and the wave's own copy of
    // the alignment weights; wave 1 publishes the statistics words
    {
      const unsigned bit = lsb_tag(t);
      const float* al = alf[t & 1];            // alpha_{t-1} at n0-1+k
      if (SAT_FWD8_R2 && wave == 7 && lane < kPadR + kPadL + 2) {
        // record B's halo words (first 5 / last 4 energies, last 2 alpha_{t-1}): final since the
        // energies barrier
        const int rb = (((t & 1) * B + b) * kW + j) * kRB;
        const int q = lane;
        float v;
        if (q < kPadR) v = q < nt ? eown[q] : -INFINITY;
        else if (q < kPadR + kPadL) { const int i = nt - kPadL + (q - kPadR); v = i >= 0 ? eown[i] : -INFINITY; }
        else { const int k = nt - 1 + (q - kPadR - kPadL); v = k >= 0 ? al[k] : 0.f; }
        stcx(xl, rRB, rb + kRBeh + q, tagf(v == -INFINITY ? 0.f : v, bit));
      }
      const float e1v = lane < kPmax ? eown[lane] : -INFINITY;
      const float e2v = lane < kPmax ? e2own[lane] : -INFINITY;
      const float m1 = tagf(fmaxf(wave_max_dpp(e1v), -3.402823466e38f), bit);
      const float m2 = tagf(fmaxf(wave_max_dpp(e2v), -3.402823466e38f), bit);
      const float pe = e1v == -INFINITY ? 0.f : __expf(e1v - m1);
      const float pe2 = e2v == -INFINITY ? 0.f : __expf(e2v - m2);
      const float w = lane < nt ? ((1.f - u) * al[lane + 1] + u * al[lane] + 1e-7f) * pe : 0.f;
      if (lane < kPmax) { wsc[wave][0][lane] = w; wsc[wave][1][lane] = lane < nt ? pe2 : 0.f; }
      if (wave == SAT_FWD8_STW) {
        const float z1 = tagf(wave_sum_dpp(pe), bit), a1 = tagf(wave_sum_dpp(w), bit);
        const float z2 = tagf(wave_sum_dpp(pe2), bit);
        if (lane == 0) {
          const int rb = (((t & 1) * B + b) * kW + j) * kRB;
          stc4x(xl, rRB, rb / 4, make_float4(m1, z1, a1, m2));
          stc4x(xl, rRB, rb / 4 + 1, tagf4(make_float4(z2, 0.f, 0.f, 0.f), bit));
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // own-wave LDS copy is ready
    }
    tick(13);
    ev(14);
    // partial contexts, published per wave: wave w owns c1 columns 32w .. 32w+31 (lane l:
    // column 32w + (l & 31), positions 16 (l >> 5) .. + 15); wave SAT_FWD8_C2W also the 32 c2
    // columns; wave 1 the halo words unless SAT_FWD8_R2 (then wave 7 in the statistics phase)
    {
      const unsigned bit = lsb_tag(t);
      const int rb = (((t & 1) * B + b) * kW + j) * kRB;
      const int col = lane & 31, r0 = 16 * (lane >> 5);
      const float* ws = &wsc[wave][0][r0];
      float c = 0.f;
#pragma unroll
      for (int k4 = 0; k4 < 4; ++k4) {
        const float4 w4 = *reinterpret_cast<const float4*>(ws + 4 * k4);
        c = fmaf(w4.x, v1s[r0 + 4 * k4][32 * wave + col], c);
        c = fmaf(w4.y, v1s[r0 + 4 * k4 + 1][32 * wave + col], c);
        c = fmaf(w4.z, v1s[r0 + 4 * k4 + 2][32 * wave + col], c);
        c = fmaf(w4.w, v1s[r0 + 4 * k4 + 3][32 * wave + col], c);
      }
      const float4 c4 = quad_gather(fold32(c));
      if (lane < 32 && (lane & 3) == 0)
        stc4x(xl, rRB, (rb + kRBctx) / 4 + 8 * wave + (lane >> 2), tagf4(c4, bit));
      if (wave == SAT_FWD8_C2W) {
        const float* ws2 = &wsc[SAT_FWD8_C2W][1][r0];
        float c2 = 0.f;
#pragma unroll
        for (int k = 0; k < 16; ++k) c2 = fmaf(ws2[k], v2s[r0 + k][col], c2);
        const float4 q4 = quad_gather(fold32(c2));
        if (lane < 32 && (lane & 3) == 0)
          stc4x(xl, rRB, (rb + kRBctx + kM1) / 4 + (lane >> 2), tagf4(q4, bit));
      } else if (!SAT_FWD8_R2 && wave == 1 && lane < kPadR + kPadL + 2) {
        const int q = lane;
        float v;
        if (q < kPadR) v = q < nt ? eown[q] : -INFINITY;
        else if (q < kPadR + kPadL) { const int i = nt - kPadL + (q - kPadR); v = i >= 0 ? eown[i] : -INFINITY; }
        else { const int k = nt - 1 + (q - kPadR - kPadL); v = k >= 0 ? alf[t & 1][k] : 0.f; }
        stcx(xl, rRB, rb + kRBeh + q, tagf(v == -INFINITY ? 0.f : v, bit));
      }
    }
    tick(14);
    ev(15);
    // ============ 7. h part of step t+1's gate sums (h_t arrived with records A_t)
    if (!SAT_FWD8_HMERGE && t + 1 < T) {
      f2 acc[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] = f2{0.f, 0.f};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float xv = hbuf[64 * i + lane];
        const f2 xx = {xv, xv};
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[q] = __builtin_elementwise_fma(xx, w0[i][q], acc[q]);
      }
      float v[16];
#pragma unroll
      for (int q = 0; q < 8; ++q) { v[2 * q] = acc[q].x; v[2 * q + 1] = acc[q].y; }
      transpose_reduce16(v, lane);
      gsum[wave][lane] = v[0];                    // own wave's slot: no barrier needed
    }
    tick(15);
  }
#if SAT_FWD8_TRACE || SAT_SEGMENT_CLOCKS
  if (p.prof && tid0 == 0)
    for (int i = 0; i < 16; ++i) p.prof[blockIdx.x * 16 + i] = tp[i];
#endif
}

}  // namespace

bool dec_attn_fwd8_eligible(const SatDecAttnFwd* a) {
  return a->U == kU && a->M1 == kM1 && a->M2 == kM2 && a->D1 == kD1 && a->D2 == kD2 &&
         a->F == kF && a->KW == kKW && a->B >= 1 && a->B <= kGmax && a->N >= 1 &&
         a->N <= kW * kPmax;
}

// Scratch: records A / B and the placement words live in the QP buffer of
// sat_decoder_attention_scratch (2 B 32 256 floats >= 2 B 8 (288 + 320) + 256).
int dec_attn_fwd8_launch(const SatDecAttnFwd* a, hipStream_t s) {
  int dev = 0, cus = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, dec_attn_fwd8_kernel, kTh, 0) != hipSuccess) {
    set_error("sat_decoder_attention_fwd: device query failed");
    return SAT_ERR_HIP;
  }
  SAT_CHECK_ARG((int64_t)cus * per_cu >= kGmax * kW,
                "sat_decoder_attention_fwd: fewer than 256 co-resident workgroups on this device");
  Fwd8P p;
  p.B = a->B; p.N = a->N; p.T = a->T;
  p.P = std::max(kPadR, ceil_div(a->N, kW));
  p.u = a->u; p.zc = a->zc; p.zh = a->zh;
  p.X0 = a->X0; p.W0r = a->W0r; p.Wq1 = a->Wq1; p.Wq2 = a->Wq2;
  p.K1 = a->K1; p.V1 = a->V1; p.K2 = a->K2; p.V2 = a->V2; p.lengths = a->lengths;
  p.v1 = a->v1; p.b1 = a->b1; p.convW = a->convW; p.convb = a->convb; p.locW = a->locW;
  p.v2 = a->v2; p.mask_c = a->mask_c; p.mask_h = a->mask_h;
  p.REC0 = a->REC0; p.C0 = a->C0; p.H0RAW = a->H0RAW; p.G0 = a->G0; p.Q = a->Q;
  p.S1 = a->S1; p.AL1 = a->AL1; p.S2 = a->S2; p.ST = a->ST; p.LOC = a->LOC; p.ZH = a->ZH;
  const int64_t ra = (int64_t)2 * a->B * kW * kRA, rb = (int64_t)2 * a->B * kW * kRB;
  p.RA = a->QP;
  p.RB = a->QP + ra;
  p.XID = reinterpret_cast<unsigned*>(a->QP + ra + rb);
  p.err = a->err;
  p.flags = xcd_local_env();
  p.prof = reinterpret_cast<long long*>(a->prof);
  if (zero_ranges(s, a->QP, ra + rb + kGmax * kW, a->err, 2) != hipSuccess) {
    set_error("sat_decoder_attention_fwd: scratch clear failed");
    return SAT_ERR_HIP;
  }
  hipLaunchKernelGGL(dec_attn_fwd8_kernel, dim3(kGmax * kW), dim3(kTh), 0, s, p);
  SAT_LAUNCH_CHECK("sat_decoder_attention_fwd");
  return SAT_OK;
}

}  // namespace sat
