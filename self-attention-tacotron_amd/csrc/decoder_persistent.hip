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
// in one workgroup's LDS and each workgroup's 32 LSTM gate columns (72 floats per lane) and
// query rows (32 floats per lane) live in registers for the whole decode.
//
// Layout: 8 groups x 32 workgroups (256, one per CU).  Group g = blockIdx % 8 owns utterances
// b = g + 8*ub < B (ub < 4) -- workgroups b, b+8, ... share an XCD under the observed
// round-robin placement (speed only; correctness never depends on placement).  Workgroup
// j = blockIdx / 8 of the group owns LSTM units [8j, 8j+8) and, if j < UB*ntiles, tile
// (ub = j / ntiles, tile = j % ntiles).  Per step t:
//   A (every workgroup): combine step t-1's tile partial records (redundantly: the context is
//      the LSTM input); LSTM0 step t for its 8 units x UB utterances; publish its units' h_t
//      and its query contribution q_part[j] = h0'_t[8 units] [Wq1 | Wq2][8 units, :];
//      tile workgroups then normalise step t-1 on their window (s_{t-1}, alpha_{t-1}).
//   C (tile workgroups): sum the 32 query partials of their utterance, location features,
//      energies from LDS K1/K2, tile statistics and the unnormalised partial context.
// Hand-offs (MI355X_MICROARCH.md price list "handoff-1to1": the data IS the flag): no group
// barrier, no drain, no counter.  Bulk payloads (partial records, query partials, h) carry the
// step parity in every float's mantissa LSB (persistent.h lsb_tag); energy and alignment halos
// travel as 8-byte {value, step+1} granules.  Producers store sc1, consumers load sc1 and
// re-load only the words whose tag is stale.  Slots alternate by step parity; a producer can
// reach step t+2 only after every consumer of its step-t slot has consumed it (each step needs
// every workgroup's query partial and every tile's record), so slots are never overwritten
// early.  Every spin is bounded: a timeout raises err[0] and all later polls give up, so the
// grid always drains.  All histories the backward needs are written exactly as the launch-based
// path writes them (the tagged values where a tagged value was consumed).
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
constexpr int kKP = 576;                       // kK0 padded to 9 x 64 (zero tail)
constexpr int kPST = 8 + kM1 + kM2;            // partial record: 8 statistics + 288 context
constexpr int kP4 = kPST / 4;                  // float4 per record (74)
constexpr int kQ = kD1 + kD2;                  // query width (= U here)
constexpr int kUW = kU / kGW;                  // units per workgroup (8)
constexpr int kPadL = (kKW - 1) / 2;           // 4: SAME padding of the location convolution
constexpr int kPadR = kKW - 1 - kPadL;         // 5
constexpr int kEH = 16;                        // energy-halo granules per tile record (9 used)
constexpr int kAH = 2;                         // alignment-halo granules per tile record
static_assert(kK0 <= kKP && kKP == 9 * 64 && kU % kGW == 0 && kQ == 256 && kPST % 4 == 0 &&
              kD1 % 4 == 0, "layout");

struct DecAttnP {
  int B, N, T, ntiles, UB, flags;
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
  float* HX;                                         // [2][B][U]            tagged h
  float* EH;                                         // [2][B][ntiles][kEH]  granules
  float* AH;                                         // [2][B][ntiles][kAH]  granules
  float* PART;                                       // [2][B][ntiles][kPST] tagged
  float* QP;                                         // [2][B][kGW][kQ]      tagged
  unsigned* XID;                                     // [256] XCC_ID + 1 per workgroup (zeroed)
  int* err;                                          // [2]
  long long* prof;                                   // [256][16] segment clocks + [T][256][4] trace (nullable)
};

typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float sigm(float x) { return sigmoid_fast(x); }   // as every LSTM kernel
__device__ __forceinline__ bool any_lane(bool v) { return __builtin_amdgcn_ballot_w64(v) != 0; }

__global__ void __launch_bounds__(256) dec_attn_fwd_kernel(DecAttnP p) {
  __shared__ __attribute__((aligned(16))) float k1s[kPN][kD1];
  __shared__ __attribute__((aligned(16))) float v1s[kPN][kM1];
  __shared__ __attribute__((aligned(16))) float k2s[kPN][kD2];
  __shared__ __attribute__((aligned(16))) float v2s[kPN][kM2];
  __shared__ __attribute__((aligned(16))) float rin[kUBmax][kKP];
  __shared__ __attribute__((aligned(16))) float hown[kUBmax][kUW];   // raw outputs (query input)
  __shared__ __attribute__((aligned(16))) float hst[kUBmax][kUW];    // zoneout states (tagged)
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
  __shared__ float ew[kPN + kKW], halo[kPadL + kPadR + kAH];
  __shared__ float aown[kPN];                        // alpha_{t-2} on the own positions
  __shared__ float e1s[kPN], e2s[kPN], w1s[kPN], w2s[kPN];
  __shared__ __attribute__((aligned(16))) float4 cred[4][64];
  __shared__ __attribute__((aligned(16))) float4 c2red[kPN][8];
  __shared__ float red[8];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = blockIdx.x % kG, j = blockIdx.x / kG;
  const int B = p.B, N = p.N, T = p.T, ntiles = p.ntiles;
  // utterances of this group (b = g + 8 ub < B); a group without any has no hand-off partner
  // outside itself, so it leaves at once
  const int UB = g < B ? (B - 1 - g) / kG + 1 : 0;
  if (UB == 0) return;
  const bool tile_wg = j < UB * ntiles;
  const int tub = tile_wg ? j / ntiles : 0, tile = tile_wg ? j % ntiles : 0;
  const int tb = g + kG * tub;                      // utterance of this workgroup's tile
  const int n0 = tile * kPN, nt = tile_wg ? min(kPN, N - n0) : 0;
  const int64_t trb = (int64_t)tb * N;
  const int span = nt + kKW - 1;
  const bool has_left = tile_wg && tile > 0, has_right = tile_wg && tile + 1 < ntiles;
  const float u = p.u;
  const auto rPT = rsrc(p.PART), rQP = rsrc(p.QP), rHX = rsrc(p.HX);
  const auto rEH = rsrc(p.EH), rAH = rsrc(p.AH);

  // ---------------- prologue: resident operands
  // LSTM (wave-transposed dot): wave w owns local gate columns 8w..8w+7 (units 8j+2w, +1, gates
  // i j f o), lane owns input rows k = lane + 64 i (i < 9; rows >= 544 are zero)
  f2 w0[9][4];
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int k = lane + 64 * i;
    if (k < kK0) {
      const float4* src = reinterpret_cast<const float4*>(p.W0r + (int64_t)k * (4 * kU) + 32 * j + 8 * wave);
      const float4 a = src[0], b = src[1];
      w0[i][0] = f2{a.x, a.y}; w0[i][1] = f2{a.z, a.w}; w0[i][2] = f2{b.x, b.y}; w0[i][3] = f2{b.z, b.w};
    } else {
#pragma unroll
      for (int c = 0; c < 4; ++c) w0[i][c] = f2{0.f, 0.f};
    }
  }
  // query partial: wave = utterance, lane = 4 output columns, 8 unit rows
  float4 wq[kUW];
  {
    const int c = 4 * lane;
#pragma unroll
    for (int uu = 0; uu < kUW; ++uu) {
      const int k = kUW * j + uu;
      wq[uu] = c < kD1 ? *reinterpret_cast<const float4*>(p.Wq1 + k * kD1 + c)
                       : *reinterpret_cast<const float4*>(p.Wq2 + k * kD2 + (c - kD1));
    }
  }
  for (int i = tid; i < kUBmax * kKP; i += 256) rin[i / kKP][i % kKP] = 0.f;   // pad, rows >= UB
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
  // cell role: after the transpose-reduce the 4 gate sums of (utterance cub, unit cu) sit in
  // lanes L, L+2, L+4, L+6 with L = 16 cub + 8 cu; lane L runs the cell, its state in registers
  const int cub = lane >> 4, cu = (lane >> 3) & 1;
  const int cunit = kUW * j + 2 * wave + cu, cb = g + kG * cub;
  const bool cell = (lane & 7) == 0 && cub < UB;
  float c_own = 0.f, h_own = 0.f;
  const bool masked = p.mask_c != nullptr;
  // prefetched cell operands: branch-free loads (clamped address, raw values, defaults applied
  // at the use), so the prefetch stays in flight across the barrier and hand-off waits
  auto load_ops = [&](int tt, float4& xp_, float& mc_, float& mh_) {
    const int64_t bu = (cell && tt < T) ? ((int64_t)tt * B + cb) * kU + cunit : 0;
    const float* Mc = masked ? p.mask_c : p.X0;
    const float* Mh = masked ? p.mask_h : p.X0;
    xp_ = reinterpret_cast<const float4*>(p.X0)[bu];
    mc_ = Mc[bu];
    mh_ = Mh[bu];
  };
  float4 xpn;
  float mcn, mhn;
  load_ops(0, xpn, mcn, mhn);
  const int len = tile_wg ? (int)p.lengths[tb] : 0;
  const float4 b1r = tile_wg && tid < kD1 / 4 ? reinterpret_cast<const float4*>(p.b1)[tid]
                                                : make_float4(0.f, 0.f, 0.f, 0.f);
  __syncthreads();

  // hand-off store policy: plain stores (lines kept in the XCD's L2) iff the whole group was
  // found on one XCD, else sc1 (persistent.h xcd_local_group; placement is observed, not promised)
  const bool xl = (p.flags & 1) ? xcd_local_group(p.XID, g, kG, kGW, p.err) : false;

  long long tp[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) tp[i] = 0;
  long long t0 = wall_clock64();
  // optional event trace behind the segment sums: [T][256][4] clocks of thread 0 (A-poll
  // done for utterance 0, query partial published, query partials received, record published)
  long long* trace = p.prof ? p.prof + 256 * 16 : nullptr;
  auto ev = [&](int t, int k) {
    if (trace && tid == 0 && t < T) trace[((int64_t)t * 256 + blockIdx.x) * 8 + k] = wall_clock64();
  };
  auto tick = [&](int seg) {
    if (p.prof) {
      const long long t1 = wall_clock64();
      tp[seg] += t1 - t0;
      t0 = t1;
    }
  };
  bool gave_up = false;   // a poll timed out (err raised): stop waiting, drain the grid

  for (int t = 0; t <= T; ++t) {
    const int s = t - 1;
    // ======== A1: step s's partial records (wave = utterance) and h_s; halo granules
    ev(t, 6);
    v2u hg = {0u, 0u};      // tile workgroups, wave 0 lanes < 11: energy / alignment halo
    if (t > 0 && tile_wg && wave == 0) {
      const int sl = s & 1;
      if (lane < kPadL && has_left)
        hg = ldg(rEH, ((sl * B + tb) * ntiles + tile - 1) * kEH + kPadR + lane);
      else if (lane >= kPadL && lane < kPadL + kPadR && has_right)
        hg = ldg(rEH, ((sl * B + tb) * ntiles + tile + 1) * kEH + lane - kPadL);
      else if (lane >= kPadL + kPadR && lane < kPadL + kPadR + kAH && has_left && t >= 2)
        hg = ldg(rAH, ((sl * B + tb) * ntiles + tile - 1) * kAH + lane - kPadL - kPadR);
    }
    if (t > 0 && wave < UB) {
      const unsigned want = lsb_tag(s);
      const int b = g + kG * wave;
      const int pb4 = ((s & 1) * B + b) * ntiles * kP4;
      const int hx4 = (((s & 1) * B + b) * kU) / 4 + lane;
      const bool need_h = t < T;
      float4 ph[2][8], hs[2], h4;
      // optimistic full load; while any tile's statistics are stale only those are re-polled
      // (the producer stores them after its context), then the stale payload words are reloaded
      unsigned bad = 0xFFFFFFFFu;
      bool light = false;
      for (unsigned spins = 0;; ++spins) {
        const unsigned ld = light ? (bad & (3u << 16)) : bad;
#pragma unroll
        for (int jt = 0; jt < 8; ++jt)
#pragma unroll
          for (int h = 0; h < 2; ++h)
            if (jt < ntiles && lane + 64 * h < (kM1 + kM2) / 4 && ((ld >> (h * 8 + jt)) & 1))
              ph[h][jt] = ldc4(rPT, pb4 + jt * kP4 + 2 + lane + 64 * h);
        if (lane < ntiles) {
          if ((ld >> 16) & 1) hs[0] = ldc4(rPT, pb4 + lane * kP4);
          if ((ld >> 17) & 1) hs[1] = ldc4(rPT, pb4 + lane * kP4 + 1);
        }
        if (need_h && ((ld >> 18) & 1)) h4 = ldc4(rHX, hx4);
        bad = 0;
#pragma unroll
        for (int jt = 0; jt < 8; ++jt)
#pragma unroll
          for (int h = 0; h < 2; ++h)
            if (jt < ntiles && lane + 64 * h < (kM1 + kM2) / 4 && !tag_ok4(ph[h][jt], want))
              bad |= 1u << (h * 8 + jt);
        if (lane < ntiles) {
          if (!tag_ok4(hs[0], want)) bad |= 1u << 16;
          if (!tag_ok4(hs[1], want)) bad |= 1u << 17;
        }
        if (need_h && !tag_ok4(h4, want)) bad |= 1u << 18;
        if (!any_lane(bad != 0) || gave_up) break;
        const bool was_light = light;
        light = any_lane((bad & (3u << 16)) != 0);
        if (was_light && !light) ev(t, 4);
        if (poll_give_up(spins, p.err)) { gave_up = true; break; }
        __builtin_amdgcn_s_sleep(1);
      }
      tick(0);
      ev(t, 0);
      // ---- combine step s (wave = utterance)
      const bool on = lane < ntiles;
      const float hm1 = on ? hs[0].x : -INFINITY, hz1 = on ? hs[0].y : 0.f, ha1 = on ? hs[0].z : 0.f;
      const float hm2 = on ? hs[0].w : -INFINITY, hz2 = on ? hs[1].x : 0.f;
      // ntiles <= 8: the tile statistics sit in lanes 0..7 (DPP reductions, no LDS crossbar)
      const float M1 = lanes8_max(hm1), M2 = lanes8_max(hm2);
      const float s1 = on ? __expf(hm1 - M1) : 0.f;   // an empty tile's max is -FLT_MAX: 0
      const float s2 = on ? __expf(hm2 - M2) : 0.f;
      const float Z1 = lanes8_sum(hz1 * s1), A1 = lanes8_sum(ha1 * s1), Z2 = lanes8_sum(hz2 * s2);
      const float inv1 = 1.f / A1, inv2 = 1.f / Z2;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int c4 = lane + 64 * h;
        if (c4 >= (kM1 + kM2) / 4) break;
        const bool first = c4 < kM1 / 4;
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int jt = 0; jt < 8; ++jt) {          // lane jt's scale, broadcast by readlane
          if (jt >= ntiles) break;
          const float w1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(s1), jt));
          const float w2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(s2), jt));
          const float w = first ? w1 : w2;
          acc.x = fmaf(ph[h][jt].x, w, acc.x); acc.y = fmaf(ph[h][jt].y, w, acc.y);
          acc.z = fmaf(ph[h][jt].z, w, acc.z); acc.w = fmaf(ph[h][jt].w, w, acc.w);
        }
        const float inv = first ? inv1 : inv2;
        acc.x *= inv; acc.y *= inv; acc.z *= inv; acc.w *= inv;
        reinterpret_cast<float4*>(&rin[wave][0])[c4] = acc;
        if (j == 0) reinterpret_cast<float4*>(p.REC0 + ((int64_t)t * B + b) * kK0)[c4] = acc;
      }
      if (need_h) reinterpret_cast<float4*>(&rin[wave][kM1 + kM2])[lane] = h4;
      if (lane == 0) {
        stat[wave][0] = M1; stat[wave][1] = Z1; stat[wave][2] = A1; stat[wave][3] = M2;
        stat[wave][4] = Z2;
        if (j == 0) {
          float* st = p.ST + ((int64_t)s * B + b) * 4;
          st[0] = M1; st[1] = Z1; st[2] = A1 / Z1; st[3] = Z2;
        }
      }
    } else if (t == 0 && wave < UB) {
      for (int d = lane; d < kK0; d += 64) rin[wave][d] = 0.f;   // zero initial state
    } else {
      tick(0);
    }
    __syncthreads();
    tick(1);

    if (t < T) {
      // ======== A2: LSTM0 step t, 8 gate columns x UB utterances per wave
      f2 v2[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) v2[q] = f2{0.f, 0.f};
#pragma unroll
      for (int i = 0; i < 9; ++i) {
        float x[kUBmax];
#pragma unroll
        for (int ub = 0; ub < kUBmax; ++ub) x[ub] = rin[ub][lane + 64 * i];
#pragma unroll
        for (int ub = 0; ub < kUBmax; ++ub) {
          const f2 xx = {x[ub], x[ub]};
#pragma unroll
          for (int cp = 0; cp < 4; ++cp)
            v2[ub * 4 + cp] = __builtin_elementwise_fma(xx, w0[i][cp], v2[ub * 4 + cp]);
        }
      }
      float v[32];
#pragma unroll
      for (int q = 0; q < 16; ++q) { v[2 * q] = v2[q].x; v[2 * q + 1] = v2[q].y; }
      transpose_reduce32(v, lane);
      const float gj_ = dpp_mov<0x102>(v[0]);
      const float gf_ = dpp_mov<0x104>(v[0]);
      const float go_ = dpp_mov<0x106>(v[0]);
      tick(2);
      const float4 xp = xpn;                       // used by cell lanes only (t < T here)
      const float mc = masked ? mcn : 1.f - p.zc, mh = masked ? mhn : 1.f - p.zh;
      const unsigned bit = lsb_tag(t);
      if (cell) {
        const float gi = sigm(v[0] + xp.x);
        const float gj = tanh_lstm(gj_ + xp.y);
        const float gf = sigm(gf_ + xp.z + 1.0f);   // forget_bias = 1.0
        const float go = sigm(go_ + xp.w);
        const float cn = gf * c_own + gi * gj;
        const float hn = go * tanh_lstm(cn);
        const float c2 = mc * cn + (1.f - mc) * c_own;
        const float h2 = tagf(mh * hn + (1.f - mh) * h_own, bit);   // the value every reader sees
        c_own = c2; h_own = h2;
        hown[cub][2 * wave + cu] = hn;
        hst[cub][2 * wave + cu] = h2;
        const int64_t tbu = ((int64_t)t * B + cb) * kU + cunit;
        p.C0[((int64_t)(t + 1) * B + cb) * kU + cunit] = c2;
        p.REC0[((int64_t)(t + 1) * B + cb) * kK0 + kM1 + kM2 + cunit] = h2;
        p.H0RAW[tbu] = hn;
        reinterpret_cast<float4*>(p.G0)[tbu] = make_float4(gi, gj, gf, go);
      }
      load_ops(t + 1, xpn, mcn, mhn);
      tick(12);
      __syncthreads();
      tick(13);
      // ======== publish h_t (own units' zoneout states) and the query contribution of the own
      //          units' raw outputs
      if (tid < 2 * UB) {
        const int ub = tid >> 1, hf = tid & 1;
        stc4x(xl, rHX, (((t & 1) * B + g + kG * ub) * kU + kUW * j) / 4 + hf,
             *reinterpret_cast<const float4*>(&hst[ub][4 * hf]));
      }
      if (wave < UB) {
        float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int uu = 0; uu < kUW; ++uu) {
          const float h = hown[wave][uu];
          a.x = fmaf(h, wq[uu].x, a.x); a.y = fmaf(h, wq[uu].y, a.y);
          a.z = fmaf(h, wq[uu].z, a.z); a.w = fmaf(h, wq[uu].w, a.w);
        }
        stc4x(xl, rQP, ((((t & 1) * B + g + kG * wave) * kGW + j) * kQ) / 4 + lane, tagf4(a, bit));
      }
      tick(3);
      ev(t, 1);
    }

    // ======== A3 (tile workgroups): s_{t-1} on the conv window, alpha_{t-1} on [n0-1, n0+nt)
    if (tile_wg) {
      if (t == 0) {
        if (tid < span) {
          const int n = n0 - kPadL + tid;
          sp[tid] = (n >= 0 && n < N) ? p.S1[trb + n] : 0.f;          // host rows
        }
        if (tid <= nt) ap[tid] = (n0 - 1 + tid >= 0) ? p.AL1[trb + n0 - 1 + tid] : 0.f;
        if (tid < nt) aown[tid] = p.AL1[trb + n0 + tid];
        if (tid < kAH) halo[kPadL + kPadR + tid] = n0 - kAH + tid >= 0 ? p.AL1[trb + n0 - kAH + tid] : 0.f;
      } else {
        if (wave == 0 && lane < kPadL + kPadR + kAH) {   // halo granules: check, re-poll stale
          const int sl = s & 1;
          const bool is_el = lane < kPadL, is_er = lane >= kPadL && lane < kPadL + kPadR;
          const bool src = is_el ? has_left : is_er ? has_right : (has_left && t >= 2);
          const unsigned want = (unsigned)t;   // step t-1's granules carry tag t
          bool ok = !src || hg[1] == want;
          for (unsigned spins = 0; !ok && !gave_up; ++spins) {
            if (poll_give_up(spins, p.err)) { gave_up = true; break; }
            __builtin_amdgcn_s_sleep(1);
            if (is_el) hg = ldg(rEH, ((sl * B + tb) * ntiles + tile - 1) * kEH + kPadR + lane);
            else if (is_er) hg = ldg(rEH, ((sl * B + tb) * ntiles + tile + 1) * kEH + lane - kPadL);
            else hg = ldg(rAH, ((sl * B + tb) * ntiles + tile - 1) * kAH + lane - kPadL - kPadR);
            ok = hg[1] == want;
          }
          if (src) halo[lane] = __uint_as_float(hg[0]);
          else if (is_el || is_er) halo[lane] = -INFINITY;
          else if (t >= 2) halo[lane] = 0.f;   // alpha left of position 0 (t == 1: host rows)
        }
        __syncthreads();
        const float M1 = stat[tub][0], Z1 = stat[tub][1], A1 = stat[tub][2];
        const float M2 = stat[tub][3], Z2 = stat[tub][4];
        if (tid < span) {   // e_{t-1} on [n0-4, n0+nt+5): halos and the own energies
          const float e = tid < kPadL ? halo[tid] : tid < kPadL + nt ? e1s[tid - kPadL]
                                                                     : halo[tid - nt];
          ew[tid] = e;
          sp[tid] = e == -INFINITY ? 0.f : __expf(e - M1) / Z1;
        }
        __syncthreads();
        if (tid <= nt) {
          const int n = n0 - 1 + tid;
          float av = 0.f;
          if (n >= 0) {
            // alpha_{t-2} at n (and n-1): own positions from aown, the left two from the halo
            const float a_n = tid >= 1 ? aown[tid - 1] : halo[kPadL + kPadR + 1];
            const float a_m = tid >= 2 ? aown[tid - 2] : halo[kPadL + kPadR + tid];
            const float e = ew[tid + kPadL - 1];
            const float pe = e == -INFINITY ? 0.f : __expf(e - M1);
            av = ((1.f - u) * a_n + u * a_m + 1e-7f) * pe / A1;
          }
          ap[tid] = av;
        }
        __syncthreads();
        if (tid < nt) {   // own positions of the history rows s_{t-1}, alpha_{t-1}, s2_{t-1}
          const int n = n0 + tid;
          p.S1[((int64_t)t * B + tb) * N + n] = sp[tid + kPadL];
          p.AL1[((int64_t)t * B + tb) * N + n] = ap[tid + 1];
          aown[tid] = ap[tid + 1];
          const float e = e2s[tid];
          p.S2[((int64_t)s * B + tb) * N + n] = e == -INFINITY ? 0.f : __expf(e - M2) / Z2;
        }
        if (tid < kAH && t < T)   // alpha_{t-1} at the last two own positions, for the right tile
          stgx(xl, rAH, ((t & 1) * B + tb) * ntiles * kAH + tile * kAH + tid, ap[nt - 1 + tid],
              (unsigned)(t + 1));
      }
    }
    if (t == T) break;
    __syncthreads();
    tick(4);

    // ===================== phase C: attention tile (energies from LDS-resident K1/K2)
    if (tile_wg) {
      const unsigned want = lsb_tag(t);
      const int base4 = (((t & 1) * B + tb) * kGW + wave * 8) * (kQ / 4) + lane;
      ev(t, 7);
      float4 qv8[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) qv8[i] = ldc4(rQP, base4 + i * (kQ / 4));
      // location features f = Conv1D_SAME(s_{t-1}) + bias (no dependence on the query)
      float locv = 0.f;
      if (tid < kPN * kF) {
        const int i = tid / kF, f = tid - i * kF;
        float acc = cw[kKW * kF + f];
#pragma unroll
        for (int jj = 0; jj < kKW; ++jj) acc = fmaf(sp[i + jj], cw[jj * kF + f], acc);
        fs[i][f] = acc;
        locv = acc;
      }
      // optimistic full load; while any of the wave's 8 rows is stale, lane i < 8 re-polls one
      // word of row i only, then the stale words are reloaded
      unsigned bad = 0;
#pragma unroll
      for (int i = 0; i < 8; ++i) bad |= tag_ok4(qv8[i], want) ? 0u : 1u << i;
      for (unsigned spins = 0; any_lane(bad != 0) && !gave_up; ++spins) {
        if (poll_give_up(spins, p.err)) { gave_up = true; break; }
        __builtin_amdgcn_s_sleep(1);
        const bool light = any_lane(lane < 8 && ((bad >> lane) & 1));
        if (!light) ev(t, 5);
#pragma unroll
        for (int i = 0; i < 8; ++i)
          if (((bad >> i) & 1) && (!light || lane == i)) qv8[i] = ldc4(rQP, base4 + i * (kQ / 4));
        bad = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) bad |= tag_ok4(qv8[i], want) ? 0u : 1u << i;
      }
      tick(5);
      ev(t, 2);
      {
        float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int i = 0; i < 8; ++i) { a.x += qv8[i].x; a.y += qv8[i].y; a.z += qv8[i].z; a.w += qv8[i].w; }
        qred[wave][lane] = a;
      }
      __syncthreads();
      tick(14);
      if (tid < kQ / 4) {
        const float4 a0 = qred[0][tid], a1 = qred[1][tid], a2 = qred[2][tid], a3 = qred[3][tid];
        const float4 qv = make_float4((a0.x + a1.x) + (a2.x + a3.x), (a0.y + a1.y) + (a2.y + a3.y),
                                      (a0.z + a1.z) + (a2.z + a3.z), (a0.w + a1.w) + (a2.w + a3.w));
        if (tile == 0) reinterpret_cast<float4*>(p.Q + ((int64_t)t * B + tb) * kQ)[tid] = qv;
        const int d = 4 * tid;
        if (d < kD1) {
          qb[d] = qv.x + b1r.x; qb[d + 1] = qv.y + b1r.y;
          qb[d + 2] = qv.z + b1r.z; qb[d + 3] = qv.w + b1r.w;
        } else {
          q2s[d - kD1] = qv.x; q2s[d - kD1 + 1] = qv.y; q2s[d - kD1 + 2] = qv.z; q2s[d - kD1 + 3] = qv.w;
        }
      }
      __syncthreads();
      // energies: 8 lanes per position, 28 dims (7 float4) of K1 per lane, 4 dims of K2; the
      // tanh values are kept for the BPTT (stored after the hand-off is published)
      const int nl = tid >> 3, part = tid & 7;
      float4 zk[kD1 / 32 + 1];
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
          zk[jj] = z;
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
        zk[kD1 / 32] = z;
        acc2 = vw.x * z.x;
        acc2 = fmaf(vw.y, z.y, acc2);
        acc2 = fmaf(vw.z, z.z, acc2);
        acc2 = fmaf(vw.w, z.w, acc2);
      }
      acc = group8_sum(acc);
      acc2 = group8_sum(acc2);
      tick(6);
      if (part == 0) {
        const bool valid = nl < nt && n0 + nl < len;
        e1s[nl] = valid ? acc : -INFINITY;
        e2s[nl] = valid ? acc2 : -INFINITY;
      }
      __syncthreads();
      if (wave == 0) {            // tile statistics
        const float e1v = lane < kPN ? e1s[lane] : -INFINITY;
        const float e2v = lane < kPN ? e2s[lane] : -INFINITY;
        const float m1 = wave_max_dpp(e1v), m2 = wave_max_dpp(e2v);
        const float pe = (e1v == -INFINITY) ? 0.f : __expf(e1v - m1);
        const float pe2 = (e2v == -INFINITY) ? 0.f : __expf(e2v - m2);
        const float w = lane < nt ? ((1.f - u) * ap[lane + 1] + u * ap[lane] + 1e-7f) * pe : 0.f;
        if (lane < kPN) { w1s[lane] = w; w2s[lane] = lane < nt ? pe2 : 0.f; }
        const float z1 = wave_sum_dpp(pe), a1 = wave_sum_dpp(w), z2 = wave_sum_dpp(pe2);
        if (lane == 0) {   // an empty tile's maxima are -inf: published as -FLT_MAX (finite)
          red[0] = fmaxf(m1, -3.402823466e38f); red[1] = z1; red[2] = a1;
          red[3] = fmaxf(m2, -3.402823466e38f); red[4] = z2;
          red[5] = 0.f; red[6] = 0.f; red[7] = 0.f;
        }
      }
      __syncthreads();
      tick(8);
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
      tick(9);
      // ---- publish the tile record (tagged) and the energy halo granules
      const int pout4 = (((t & 1) * B + tb) * ntiles + tile) * kP4;
      if (tid < kM1 / 4) {
        const float4 a0 = cred[0][tid], a1 = cred[1][tid], a2 = cred[2][tid], a3 = cred[3][tid];
        stc4x(xl, rPT, pout4 + 2 + tid,
             tagf4(make_float4((a0.x + a1.x) + (a2.x + a3.x), (a0.y + a1.y) + (a2.y + a3.y),
                               (a0.z + a1.z) + (a2.z + a3.z), (a0.w + a1.w) + (a2.w + a3.w)), want));
        if (tid < 2)   // statistics last: consumers poll them before the context words
          stc4x(xl, rPT, pout4 + tid, tagf4(make_float4(red[4 * tid], red[4 * tid + 1], red[4 * tid + 2],
                                                   red[4 * tid + 3]), want));
      } else if (tid >= 64 && tid < 64 + kM2 / 4) {
        const int jj = tid - 64;
        float4 sm = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 8
        for (int i = 0; i < kPN; ++i) {
          const float4 v = c2red[i][jj];
          sm.x += v.x; sm.y += v.y; sm.z += v.z; sm.w += v.w;
        }
        stc4x(xl, rPT, pout4 + 2 + kM1 / 4 + jj, tagf4(sm, want));
      } else if (tid >= 192 && tid < 192 + kPadR + kPadL) {   // first 5, last 4 energies
        const int q = tid - 192;
        stgx(xl, rEH, ((t & 1) * B + tb) * ntiles * kEH + tile * kEH + q,
            e1s[q < kPadR ? q : kPN - kPadL + (q - kPadR)], (unsigned)(t + 1));
      }
      tick(10);
      ev(t, 3);
      // ---- histories nobody waits for: energy tanh (for the BPTT), location features
      if (p.ZH && nl < nt) {
        float* zrow = p.ZH + ((((int64_t)t * B + tb) * N) + n0 + nl) * kQ;
#pragma unroll
        for (int jj = 0; jj < kD1 / 32; ++jj)
          *reinterpret_cast<float4*>(zrow + part * (kD1 / 8) + 4 * jj) = zk[jj];
        *reinterpret_cast<float4*>(zrow + kD1 + 4 * part) = zk[kD1 / 32];
      }
      if (p.LOC && tid < kPN * kF && tid / kF < nt)
        p.LOC[(((int64_t)t * B + tb) * N + n0) * kF + tid] = locv;
      tick(11);
    }
  }
  if (p.prof && tid == 0)
    for (int i = 0; i < 16; ++i) p.prof[blockIdx.x * 16 + i] = tp[i];
}

}  // namespace
}  // namespace sat

using namespace sat;

static int64_t hx_floats(int B) { return (int64_t)2 * B * kU; }
static int64_t eh_floats(int B, int ntiles) { return (int64_t)2 * B * ntiles * kEH * 2; }
static int64_t ah_floats(int B, int ntiles) { return (int64_t)2 * B * ntiles * kAH * 2; }
static constexpr int64_t kXidWords = kG * kGW;

// SAT_ATTN_FWD8=0 selects the 8-groups x 32-workgroups layout below even where the
// one-utterance-per-8-workgroups layout (decoder_persistent8.hip, N <= 256) applies (A/B switch)
static bool fwd8_enabled() {
  const char* e = getenv("SAT_ATTN_FWD8");
  return !(e && e[0] == '0');
}

extern "C" int sat_decoder_attention_fwd(const SatDecAttnFwd* a, void* stream) {
  SAT_CHECK_ARG(a && a->B > 0 && a->N > 0 && a->T > 0, "sat_decoder_attention_fwd: bad sizes");
  if (fwd8_enabled() && dec_attn_fwd8_eligible(a)) {
    SAT_CHECK_ARG(a->X0 && a->W0r && a->Wq1 && a->Wq2 && a->K1 && a->V1 && a->K2 && a->V2 &&
                  a->lengths && a->v1 && a->b1 && a->convW && a->convb && a->locW && a->v2 &&
                  a->REC0 && a->C0 && a->H0RAW && a->G0 && a->Q && a->S1 && a->AL1 && a->S2 &&
                  a->ST && a->QP && a->err,
                  "sat_decoder_attention_fwd: null pointer");
    SAT_CHECK_ARG((a->mask_c == nullptr) == (a->mask_h == nullptr), "sat_decoder_attention_fwd: masks come in pairs");
    SAT_CHECK_ARG(aligned16(a->X0) && aligned16(a->G0) && aligned16(a->K1) && aligned16(a->V1) &&
                  aligned16(a->W0r) && aligned16(a->REC0) && aligned16(a->Q) && aligned16(a->QP) &&
                  (a->ZH == nullptr || ((uintptr_t)a->ZH & 7) == 0),
                  "sat_decoder_attention_fwd: 16-byte aligned operands");
    return dec_attn_fwd8_launch(a, as_stream(stream));
  }
  SAT_CHECK_ARG(a->U == kU && a->M1 == kM1 && a->M2 == kM2 && a->D1 == kD1 && a->D2 == kD2 &&
                a->F == kF && a->KW == kKW,
                "sat_decoder_attention_fwd: compiled for U=256, M1=256, M2=32, D1=224, D2=32, "
                "F=5, KW=10 (the self-attention-tacotron configs)");
  SAT_CHECK_ARG(a->B <= kG * kUBmax, "sat_decoder_attention_fwd: B <= 32");
  const int ntiles = ceil_div(a->N, kPN);
  SAT_CHECK_ARG(ceil_div(a->B, kG) * ntiles <= kGW && ntiles <= 8,
                "sat_decoder_attention_fwd: ceil(B/8) * ceil(N/32) must be <= 32");
  SAT_CHECK_ARG(a->X0 && a->W0r && a->Wq1 && a->Wq2 && a->K1 && a->V1 && a->K2 && a->V2 &&
                a->lengths && a->v1 && a->b1 && a->convW && a->convb && a->locW && a->v2 &&
                a->REC0 && a->C0 && a->H0RAW && a->G0 && a->Q && a->S1 && a->AL1 && a->S2 &&
                a->ST && a->E && a->PART && a->QP && a->err,
                "sat_decoder_attention_fwd: null pointer");
  SAT_CHECK_ARG((a->mask_c == nullptr) == (a->mask_h == nullptr), "sat_decoder_attention_fwd: masks come in pairs");
  SAT_CHECK_ARG(aligned16(a->X0) && aligned16(a->G0) && aligned16(a->K1) && aligned16(a->V1) &&
                aligned16(a->W0r) && aligned16(a->Wq1) && aligned16(a->Wq2) && aligned16(a->REC0) &&
                aligned16(a->Q) && aligned16(a->E) && aligned16(a->PART) && aligned16(a->QP) &&
                aligned16(a->b1),
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
  p.B = a->B; p.N = a->N; p.T = a->T; p.ntiles = ntiles; p.UB = ceil_div(a->B, kG);
  p.u = a->u; p.zc = a->zc; p.zh = a->zh;
  p.X0 = a->X0; p.W0r = a->W0r; p.Wq1 = a->Wq1; p.Wq2 = a->Wq2;
  p.K1 = a->K1; p.V1 = a->V1; p.K2 = a->K2; p.V2 = a->V2; p.lengths = a->lengths;
  p.v1 = a->v1; p.b1 = a->b1; p.convW = a->convW; p.convb = a->convb; p.locW = a->locW;
  p.v2 = a->v2; p.mask_c = a->mask_c; p.mask_h = a->mask_h;
  p.REC0 = a->REC0; p.C0 = a->C0; p.H0RAW = a->H0RAW; p.G0 = a->G0; p.Q = a->Q;
  p.S1 = a->S1; p.AL1 = a->AL1; p.S2 = a->S2; p.ST = a->ST; p.LOC = a->LOC;
  p.HX = a->E;
  p.EH = a->E + hx_floats(a->B);
  p.AH = p.EH + eh_floats(a->B, ntiles);
  p.XID = reinterpret_cast<unsigned*>(p.AH + ah_floats(a->B, ntiles));
  p.PART = a->PART; p.QP = a->QP; p.err = a->err;
  p.flags = xcd_local_env();
  p.prof = reinterpret_cast<long long*>(a->prof);
  p.ZH = a->ZH;
  hipStream_t s = as_stream(stream);
  // every hand-off slot starts zeroed (tag 0 / LSB 0 never matches steps 0 and 1)
  const int64_t e_total = hx_floats(a->B) + eh_floats(a->B, ntiles) + ah_floats(a->B, ntiles) +
                        kXidWords;
  if (zero_ranges(s, a->E, e_total, a->PART, (int64_t)2 * a->B * ntiles * kPST, a->QP,
                  (int64_t)2 * a->B * kGW * kQ, a->err, 2) != hipSuccess) {
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
  if (e_floats) *e_floats = hx_floats(B) + eh_floats(B, ntiles) + ah_floats(B, ntiles) + kXidWords;
  if (part_floats) *part_floats = (int64_t)2 * B * ntiles * kPST;
  if (qp_floats) *qp_floats = (int64_t)2 * B * kGW * kQ;
  return kG * 64;   // counter words (unused by the tagged hand-offs; kept for the ABI)
}
