// Free-running decoding (PREDICT, BASELINE configs[4] = C5) as ONE persistent launch.
//
// The per-step launch path (inference.py) runs each decoder step as ~14 dependent kernels, each
// at the ~5-9 us floor of a dependent launch.  Here every step of the whole decode runs inside
// one launch: RNNTransformer's PREDICT branch (modules/module.py:766-784) =
// OutputAndStopTokenTransparentWrapper(TransformerWrapper(RNNStateHistoryWrapper(DecoderRNNV2)))
// (modules/rnn_wrappers.py:47-124, 188-214) under the tacotron2 StopTokenBasedInferenceHelper
// (analog modules/helpers.py:111-160): prenets on the fed frame, the attention RNN, forward +
// additive attention (modules/forward_attention.py:88-122), the two ZoneoutLSTMs, the causal
// self-attention head over a key/value cache, the mel / stop projections and the stop test.
//
// Layout: utterances 2g and 2g + 1 are decoded by group g = {g, g + 4, ..., g + 252} of 64
// workgroups (two XCDs under the dispatcher's round-robin).  Every weight slice a workgroup needs
// stays on chip for the whole decode -- per group one 10 MB replica of the decoder over 64 CUs:
// the LSTMs' input rows, the fed-frame / prenet / query / q-k-u columns in registers, the attention
// RNN's recurrent rows in LDS.  (One utterance per 32 workgroups would need a replica per XCD:
// 325 KB per CU, more than the register file and LDS leave around the working set.)  Utterances
// are independent until the stop test, so each step's ten hand-offs stay inside the group: each
// an all-gather of LSB-tagged floats (persistent.h: the data IS the flag, slots alternate by step
// parity; stores sc1, loads sc1).
//
// Per step t (workgroup w of the group owns LSTM units 4w..4w+3 and a few dense columns, both
// rows -- the group's two utterances -- at once):
//   P1  z_{t-1} -> mel|stop of step t-1 (outputs; stop granules to every group) and the first
//       prenet layer of step t (the fed frame is folded in: Wzp = W_out[:, fed] W_p0)
//   P2  prenet layer 2                          P3  attention RNN (ZoneoutLSTM 256)
//   P4  query layers of both attentions         P5  8 workgroups per utterance: energies of
//       their memory positions + flash-style tile records (max, sum e, sum a~ e, contexts)
//   P6  every workgroup: both utterances' alignments (forward recursion) and contexts
//   P7  LSTM1                                   P8  LSTM2
//   P9  q | k | u of the head (u = v W_o W_t per head: the value, output projection and transform
//       products folded into the cached rows, so the attention output IS the transform input)
//   P10 each workgroup scores its own cache rows (row j lives in workgroup j % 64): partial
//       softmax sums and partial outputs per head
//   P11 z = h2' + tanh(sum_h O_h / Z_h + b_z), the residual head output (TransformerWrapper,
//       modules/rnn_wrappers.py:87-124; self_attention.py:45-65 without dropout)
// An LSTM's K rows are split over two waves per unit (partials combined through LDS); the
// recurrent parts (h_{t-1}, contexts) are formed while the step's other hand-offs are in flight.
// The stop test of step t-1 (t > min_iters and sigmoid(stop) > 0.5 for every utterance) reads
// the B stop granules at the end of step t: every workgroup of every group sees the same values
// and leaves the loop at the same step.
#include "persistent.h"

#include <algorithm>

namespace sat {
namespace {

// ---- the LJSpeech / VCTK decoder (hparams.py; checked by the host entry)
constexpr int kG = 4;             // groups of two utterances (B <= 8)
constexpr int kW = 64;            // workgroups per group
constexpr int kTh = 512;          // threads per workgroup
constexpr int kAW = 8;            // attention workgroups per utterance (memory positions split)
constexpr int kPM = 32;           // memory positions per attention workgroup (N <= 256)
constexpr int kRM = 8;            // cache rows per workgroup and utterance (T <= 512)
constexpr int kNM = kAW * kPM;    // 256
constexpr int kMR = 160;          // mel values per step (80 x r=2)
constexpr int kMS = 164;          // MS row: mel | stop | pad
constexpr int kP0 = 256, kP1 = 128;
constexpr int kU = 256;           // attention RNN = LSTM1 = LSTM2 units
constexpr int kC1 = 256, kCtx = 288, kCtxP = 320;
constexpr int kD1 = 224, kQ = 256;
constexpr int kF = 5, kKW = 10, kPad = 4;
constexpr int kSD = 256, kSDH = 128, kQKU = 1024, kRow = 768;   // cached row = [k | u0 | u1]
constexpr int kRec = 8 + 2 * kPM + kCtx;                         // 360
constexpr int kSaRec = 8 + 2 * kSD;                              // 520
constexpr float kNeg = -3.0e38f;   // finite stand-in for -inf in tagged words
constexpr float kNegT = -1.0e38f;  // anything below is "no position"

// hand-off buffers of one group (float offsets; two slots per edge, slot = step & 1, then the
// two utterance rows)
constexpr int oZ = 0;
constexpr int oY0 = oZ + 2 * 2 * kSD;
constexpr int oP = oY0 + 2 * 2 * kP0;
constexpr int oH0 = oP + 2 * 2 * kP1;
constexpr int oQ = oH0 + 2 * 2 * 2 * kU;
constexpr int oREC = oQ + 2 * 2 * kQ;
constexpr int oH1 = oREC + 2 * 2 * kAW * kRec;
constexpr int oH2 = oH1 + 2 * 2 * 2 * kU;
constexpr int oQKU = oH2 + 2 * 2 * 2 * kU;
constexpr int oSA = oQKU + 2 * 2 * kQKU;
constexpr int kGroupFloats = oSA + 2 * kW * 2 * kSaRec;
// after the groups: stop granules [2][8] (uint2), then the caches
constexpr int64_t kZeroDwords = (int64_t)kG * kGroupFloats + 32;
constexpr int64_t kCacheFloats = (int64_t)kG * kW * 2 * kRM * kRow;

__device__ __forceinline__ float4 fma4(float x, float4 w, float4 a) {
  return make_float4(fmaf(x, w.x, a.x), fmaf(x, w.y, a.y), fmaf(x, w.z, a.z), fmaf(x, w.w, a.w));
}
__device__ __forceinline__ float rdl(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

// ZoneoutLSTM cell, eval mode (ext tacotron2 ZoneoutLSTMCell: c = (1-zc) c' + zc c, same for h),
// formed exactly as lstm.hip's step kernels; returns the raw output h'.
__device__ __forceinline__ float zlstm_cell(float gx, float gy, float gz, float gw, float4 b,
                                            float zc, float zh, float& c, float& h) {
  const float gi = sigmoid_fast(gx + b.x);
  const float gj = tanh_lstm(gy + b.y);
  const float gf = sigmoid_fast(gz + b.z + 1.0f);   // forget_bias = 1.0
  const float go = sigmoid_fast(gw + b.w);
  const float cn = gf * c + gi * gj;
  const float hn = go * tanh_lstm(cn);
  c = (1.f - zc) * cn + zc * c;
  h = (1.f - zh) * hn + zh * h;
  return hn;
}

// Poll-gather nrows x n4r tagged float4 words (row r at float4 index base4 + r * stride4) into
// LDS (row r at dst + r * dstride4): NPT loads per thread issued before the first check.
template <int NPT>
__device__ __forceinline__ void gather(__amdgpu_buffer_rsrc_t r, int base4, int stride4, int n4r,
                                       int nrows, float4* dst, int dstride4, unsigned bit,
                                       int* err) {
  const int n4 = n4r * nrows;
  float4 v[NPT];
  int src[NPT], dix[NPT];
#pragma unroll
  for (int q = 0; q < NPT; ++q) {
    const int i = min((int)threadIdx.x + q * kTh, n4 - 1);
    const int row = i / n4r, c = i - row * n4r;
    src[q] = base4 + row * stride4 + c;
    dix[q] = row * dstride4 + c;
    v[q] = ldc4(r, src[q]);
  }
#pragma unroll
  for (int q = 0; q < NPT; ++q) {
    const int i = threadIdx.x + q * kTh;
    if (i < n4) {
      unsigned spins = 0;
      while (!tag_ok4(v[q], bit)) {
        __builtin_amdgcn_s_sleep(1);
        if (poll_give_up(++spins, err)) break;
        v[q] = ldc4(r, src[q]);
      }
      dst[dix[q]] = v[q];
    }
  }
}
__device__ __forceinline__ float poll1(__amdgpu_buffer_rsrc_t r, int idx, unsigned bit, int* err) {
  float v = ldc(r, idx);
  unsigned spins = 0;
  while (!tag_ok(v, bit)) {
    __builtin_amdgcn_s_sleep(1);
    if (poll_give_up(++spins, err)) break;
    v = ldc(r, idx);
  }
  return v;
}
__device__ __forceinline__ void pub(__amdgpu_buffer_rsrc_t r, int idx, float v, unsigned bit) {
  stc(r, idx, tagf(v, bit));
}

struct DecLds {
  float4 bias4[3][4];
  float xz[2][kSD];
  float xy0[2][kP0];
  float xp[2][kP1];
  float xh0[2][2 * kU];     // per row [h0 | h0']
  float xh1[2][2 * kU];     // per row [h1 | h1']
  float xh2[2][2 * kU];     // per row [h2 | h2']
  float xctx[2][kCtxP];     // per row [c1 | c2 | 0 pad]
  float xq[kQ];
  float xqt[2][kQKU];       // per row [q | k | u0 | u1] of step t
  float SAG[2][kW][12];     // self-attention records: header | own dims of both heads
  float red8[4][8];         // K-half partials of the LSTMs
  float sprev[2][kNM + 40]; // s_{t-1} per row, kPad zeros left
  float abuf[2][2][kNM];    // [slot][row] alignments
  float fs[kPM][kF];
  float e1s[kPM], e2s[kPM], w1s[kPM], w2s[kPM];
  float locw[kF][kD1];
  float vv[kQ];             // [v1 | v2]
  float cw[kKW * kF + kF];  // conv kernel [KW][F] | bias
  float hdr[2][8], scs[2][2][kAW], sa_s[2 * 2 * kRM], sa_pe[2 * 2 * kRM], mine[2][4];
  float cbzp[4], cbp0[4], cbms[4], cbp1[2], cbqku[16], cbz[4];
  int flag;
  float REC[2][kAW][kRec] __attribute__((aligned(16)));   // both rows' tile records
  float VS[kPM][kCtx] __attribute__((aligned(16)));       // [V1 | V2] of own positions
  float4 W0E[9 * 4 * 64];                                 // attention RNN [c1 c2 | h0] rows
};

__global__ void __launch_bounds__(kTh) decode_persistent_kernel(SatDecodePersistent p) {
  const int g = blockIdx.x % kG, w = blockIdx.x / kG;
  const int nb = min(2, p.B - 2 * g);   // utterances 2g, 2g + 1 (rows 0, 1)
  if (nb <= 0) return;                  // no utterance: no partner outside this group
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int N = p.N, T = p.T;
  const int P = (N + kAW - 1) / kAW;     // positions per attention workgroup
  const int ntiles = (N + P - 1) / P;
  const int aul = w & 1, atile = w >> 1;  // attention role: utterance row, tile
  const bool attn = w < 2 * kAW && atile < ntiles && aul < nb;
  const int ab = 2 * g + aul;
  const int n0 = atile * P, nt = attn ? min(P, N - n0) : 0;
  const int len = attn ? (int)p.lengths[ab] : 0;
  const float zc = p.zc, zh = p.zh, uf = p.u, scale = p.scale;
  float* scr = reinterpret_cast<float*>(p.scratch);
  const __amdgpu_buffer_rsrc_t R = rsrc(scr + (size_t)g * kGroupFloats);
  unsigned* stopw = reinterpret_cast<unsigned*>(scr + (size_t)kG * kGroupFloats);
  float* cache = reinterpret_cast<float*>(stopw + 32) + ((size_t)g * kW + w) * 2 * kRM * kRow;
  const __amdgpu_buffer_rsrc_t RS = rsrc(stopw);
  const __amdgpu_buffer_rsrc_t RC = rsrc(cache);

  // LDS (one struct, so the hot small arrays sit in the first 64 KB where every access is one
  // lane address + an immediate offset; the big per-phase tables come last)
  __shared__ DecLds L;
  auto& xz = L.xz; auto& xy0 = L.xy0; auto& xp = L.xp; auto& xh0 = L.xh0; auto& xh1 = L.xh1;
  auto& xh2 = L.xh2; auto& xctx = L.xctx; auto& xq = L.xq; auto& xqt = L.xqt; auto& SAG = L.SAG;
  auto& sprev = L.sprev; auto& abuf = L.abuf; auto& fs = L.fs; auto& e1s = L.e1s;
  auto& e2s = L.e2s; auto& w1s = L.w1s; auto& w2s = L.w2s; auto& locw = L.locw; auto& vv = L.vv;
  auto& cw = L.cw; auto& bias4 = L.bias4; auto& red8 = L.red8; auto& hdr = L.hdr; auto& scs = L.scs;
  auto& sa_s = L.sa_s; auto& sa_pe = L.sa_pe; auto& mine = L.mine; auto& cbzp = L.cbzp;
  auto& cbp0 = L.cbp0; auto& cbms = L.cbms; auto& cbp1 = L.cbp1; auto& cbqku = L.cbqku;
  auto& cbz = L.cbz; auto& flag = L.flag; auto& REC = L.REC; auto& VS = L.VS; auto& W0E = L.W0E;

  // ---------------------------------------------------------------- one-time loads
  const int unit = wave & 3, kh = wave >> 2;   // LSTM roles: unit 4w + unit, K half kh
  const int uu = 4 * w + unit;
  const float4* W0_4 = reinterpret_cast<const float4*>(p.W0);
  const float4* W1_4 = reinterpret_cast<const float4*>(p.W1);
  const float4* W2_4 = reinterpret_cast<const float4*>(p.W2);
  // attention RNN rows [0:128) p (late: block kh), LSTM1 blocks b = 2i + kh of
  // [h0' (0-3) | h1 (4-7) | c1 c2 (8-12)], LSTM2 blocks 2i + kh of [h1' (0-3) | h2 (4-7)]
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  const float4 w0r = W0_4[(size_t)(lane + 64 * kh) * kU + uu];
  float4 w1r[7];
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    const int blk = 2 * i + kh;
    int row = -1;
    if (blk < 4) row = lane + 64 * blk;
    else if (blk < 8) row = kU + kCtx + lane + 64 * (blk - 4);
    else if (blk < 13 && lane + 64 * (blk - 8) < kCtx) row = kU + lane + 64 * (blk - 8);
    w1r[i] = row >= 0 ? W1_4[(size_t)row * kU + uu] : z4;
  }
  float4 w2r[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) w2r[i] = W2_4[(size_t)(lane + 64 * (2 * i + kh)) * kU + uu];
  // dense columns (both rows): P1 waves 0-3 prenet-1 col 4w+wave from z, waves 4-6 mel|stop col
  // w + 64 (wave-4); P2 waves 0-1 prenet-2 col 2w+wave; P4 waves 0-3 query col 4w+wave;
  // P9 q|k|u cols 16w + 2 wave + j
  const int cpre = 4 * w + wave, cmel = w + 64 * (wave - 4), cp1 = 2 * w + wave, cq = 4 * w + wave;
  const bool has_pre = wave < 4, has_mel = wave >= 4 && wave < 7 && cmel <= kMR;
  float wa[4], wp1[4], wq[4], wk[2][4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int k = lane + 64 * i;
    wa[i] = has_pre ? p.Wzp[(size_t)k * kP0 + cpre] : has_mel ? p.Wms[(size_t)k * kMS + cmel] : 0.f;
    wp1[i] = wave < 2 ? p.Wp1[(size_t)k * kP1 + cp1] : 0.f;
    wq[i] = wave < 4 ? p.Wq[(size_t)k * kQ + cq] : 0.f;
#pragma unroll
    for (int j = 0; j < 2; ++j) wk[j][i] = p.Wqku[(size_t)k * kQKU + 16 * w + 2 * wave + j];
  }
  // attention: K1 + b1 / K2 slices of this lane's position (16 lanes per position)
  const int anl = tid >> 4, apart = tid & 15;
  const bool apos = attn && anl < nt;
  float k1b[14], k2r[2];
  {
    const size_t rowp = (size_t)ab * N + n0 + (apos ? anl : 0);
#pragma unroll
    for (int j = 0; j < 14; ++j)
      k1b[j] = apos ? p.K1[rowp * kD1 + apart + 16 * j] + p.b1[apart + 16 * j] : 0.f;
#pragma unroll
    for (int j = 0; j < 2; ++j) k2r[j] = apos ? p.K2[rowp * 32 + apart + 16 * j] : 0.f;
  }
  for (int idx = tid; idx < 9 * 4 * 64; idx += kTh) {
    const int i = idx >> 8, un = (idx >> 6) & 3, ln = idx & 63;
    int row;
    if (i < 5) row = (ln + 64 * i < kCtx) ? kP1 + ln + 64 * i : -1;
    else row = kP1 + kCtx + ln + 64 * (i - 5);
    W0E[idx] = row >= 0 ? W0_4[(size_t)row * kU + 4 * w + un] : z4;
  }
  for (int idx = tid; idx < nt * kCtx; idx += kTh) {
    const int i = idx / kCtx, d = idx - i * kCtx;
    const size_t rowp = (size_t)ab * N + n0 + i;
    VS[i][d] = d < kC1 ? p.V1[rowp * kC1 + d] : p.V2[rowp * 32 + (d - kC1)];
  }
  for (int idx = tid; idx < kF * kD1; idx += kTh) locw[idx / kD1][idx % kD1] = p.locW[idx];
  if (tid < kQ) vv[tid] = tid < kD1 ? p.v1[tid] : p.v2[tid - kD1];
  if (tid < kKW * kF) cw[tid] = p.convW[tid];
  if (tid < kF) cw[kKW * kF + tid] = p.convb[tid];
  for (int idx = tid; idx < 2 * (kNM + 40); idx += kTh) (&sprev[0][0])[idx] = 0.f;
  for (int idx = tid; idx < 4 * kNM; idx += kTh) (&abuf[0][0][0])[idx] = 0.f;
  for (int idx = tid; idx < 4 * kU; idx += kTh) {
    (&xh0[0][0])[idx] = 0.f; (&xh1[0][0])[idx] = 0.f; (&xh2[0][0])[idx] = 0.f;
  }
  for (int idx = tid; idx < 2 * kCtxP; idx += kTh) (&xctx[0][0])[idx] = 0.f;
  if (tid < 4) {
    bias4[0][tid] = reinterpret_cast<const float4*>(p.b0)[4 * w + tid];
    bias4[1][tid] = reinterpret_cast<const float4*>(p.bl1)[4 * w + tid];
    bias4[2][tid] = reinterpret_cast<const float4*>(p.bl2)[4 * w + tid];
    cbzp[tid] = p.bzp[4 * w + tid];
    cbp0[tid] = p.bp0[4 * w + tid];
    cbz[tid] = p.bz[4 * w + tid];
    const int cm = w + 64 * tid;
    cbms[tid] = (tid < 3 && cm <= kMR) ? p.bms[cm] : 0.f;
    if (tid < 2) cbp1[tid] = p.bp1[2 * w + tid];
  }
  if (tid < 16) cbqku[tid] = p.bqku[16 * w + tid];
  __syncthreads();
  if (tid < 2) abuf[1][tid][0] = 1.f;   // a_{-1} = one-hot at position 0 (forward_attention.py:131-133)
  __syncthreads();

  // own units' states, one per row (uniform across the K-half pair; kept by both waves)
  float c0[2] = {0.f, 0.f}, h0[2] = {0.f, 0.f}, c1[2] = {0.f, 0.f}, h1[2] = {0.f, 0.f};
  float c2[2] = {0.f, 0.f}, h2[2] = {0.f, 0.f};
  float4 att_e[2] = {z4, z4}, l2_e[2] = {z4, z4};   // recurrent parts of the next step's products

  // LSTM step of unit uu for both rows: acc[r] (this wave's K half, summed over its lanes) +
  // the partner wave's half through LDS, then the cell; publishes [h | h'] of both rows.
  auto lstm_finish = [&](float4 acc0, float4 acc1, int which, float* cst, float* hst, int obase,
                         unsigned bit) {
    float v[8] = {acc0.x, acc0.y, acc0.z, acc0.w, acc1.x, acc1.y, acc1.z, acc1.w};
    transpose_reduce8(v, lane);   // lanes 8m..8m+7 hold output m
    if (kh == 1 && (lane & 7) == 0) red8[unit][lane >> 3] = v[0];
    lds_barrier();
    float gsum[8];
#pragma unroll
    for (int m = 0; m < 8; ++m) gsum[m] = rdl(v[0], 8 * m) + red8[unit][m];
    const float4 bb = bias4[which][unit];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const float hr = zlstm_cell(gsum[4 * r], gsum[4 * r + 1], gsum[4 * r + 2], gsum[4 * r + 3], bb,
                                  zc, zh, cst[r], hst[r]);
      if (kh == 0 && lane == 0) {
        pub(R, obase + r * 2 * kU + uu, hst[r], bit);
        pub(R, obase + r * 2 * kU + kU + uu, hr, bit);
      }
    }
  };

  for (int t = 0; t <= T; ++t) {
    // role indices re-derived every step from an opaque copy of the thread id, so the compiler
    // cannot hoist (and then spill) the dozens of loop-invariant lane addresses of the phases
    int tid_ = (int)threadIdx.x;
    asm volatile("" : "+v"(tid_));
    const int tid = tid_, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int unit = wave & 3, kh = wave >> 2;
    const int anl = tid >> 4, apart = tid & 15;
    const int cpre = 4 * w + wave, cmel = w + 64 * (wave - 4), cp1 = 2 * w + wave, cq = 4 * w + wave;
    const bool has_pre = wave < 4, has_mel = wave >= 4 && wave < 7 && cmel <= kMR;
    const int s = t & 1, sp = s ^ 1;
    const unsigned bt = lsb_tag(t), bp = lsb_tag(t - 1);
    // ================================================= P1: mel|stop of t-1, prenet layer 1 of t
    if (t > 0) {
      gather<1>(R, (oZ + sp * 2 * kSD) / 4, 0, 2 * kSD / 4, 1, reinterpret_cast<float4*>(&xz[0][0]), 0,
                bp, p.err);
      lds_barrier();
      if (has_mel) {
        float a0 = 0.f, a1 = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          a0 = fmaf(xz[0][lane + 64 * i], wa[i], a0);
          a1 = fmaf(xz[1][lane + 64 * i], wa[i], a1);
        }
        a0 = wave_sum_dpp(a0) + cbms[wave - 4];
        a1 = wave_sum_dpp(a1) + cbms[wave - 4];
        if (lane < nb) {
          const float v = lane == 0 ? a0 : a1;
          const int b = 2 * g + lane;
          p.MS[((size_t)(t - 1) * p.B + b) * kMS + cmel] = v;
          if (cmel == kMR) stg(RS, sp * 8 + b, v, (unsigned)t);   // {stop_{t-1}, t} to all groups
        }
      }
    }
    if (t == T) break;
    if (has_pre) {
      float a0, a1;
      if (t > 0) {
        a0 = 0.f; a1 = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          a0 = fmaf(xz[0][lane + 64 * i], wa[i], a0);
          a1 = fmaf(xz[1][lane + 64 * i], wa[i], a1);
        }
        a0 = wave_sum_dpp(a0) + cbzp[wave];
        a1 = wave_sum_dpp(a1) + cbzp[wave];
      } else {
        a0 = a1 = cbp0[wave];   // the go frame (zeros)
      }
      if (lane < 2) pub(R, oY0 + (s * 2 + lane) * kP0 + cpre, fmaxf(lane == 0 ? a0 : a1, 0.f), bt);
    }
    // ================================================= P2: prenet layer 2
    gather<1>(R, (oY0 + s * 2 * kP0) / 4, 0, 2 * kP0 / 4, 1, reinterpret_cast<float4*>(&xy0[0][0]), 0,
              bt, p.err);
    lds_barrier();
    if (wave < 2) {
      float a0 = 0.f, a1 = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        a0 = fmaf(xy0[0][lane + 64 * i], wp1[i], a0);
        a1 = fmaf(xy0[1][lane + 64 * i], wp1[i], a1);
      }
      a0 = fmaxf(wave_sum_dpp(a0) + cbp1[wave], 0.f);
      a1 = fmaxf(wave_sum_dpp(a1) + cbp1[wave], 0.f);
      if (lane < 2) pub(R, oP + (s * 2 + lane) * kP1 + cp1, lane == 0 ? a0 : a1, bt);
    }
    // ================================================= P3: attention RNN
    gather<1>(R, (oP + s * 2 * kP1) / 4, 0, 2 * kP1 / 4, 1, reinterpret_cast<float4*>(&xp[0][0]), 0, bt,
              p.err);
    lds_barrier();
    lstm_finish(fma4(xp[0][lane + 64 * kh], w0r, att_e[0]), fma4(xp[1][lane + 64 * kh], w0r, att_e[1]),
                0, c0, h0, oH0 + s * 2 * 2 * kU, bt);
    // ================================================= P4: query layers; LSTM1 recurrent part
    gather<1>(R, (oH0 + s * 2 * 2 * kU) / 4, 0, 2 * 2 * kU / 4, 1,
              reinterpret_cast<float4*>(&xh0[0][0]), 0, bt, p.err);
    lds_barrier();
    if (wave < 4) {
      float a0 = 0.f, a1 = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        a0 = fmaf(xh0[0][kU + lane + 64 * i], wq[i], a0);
        a1 = fmaf(xh0[1][kU + lane + 64 * i], wq[i], a1);
      }
      a0 = wave_sum_dpp(a0);
      a1 = wave_sum_dpp(a1);
      if (lane < 2) pub(R, oQ + (s * 2 + lane) * kQ + cq, lane == 0 ? a0 : a1, bt);
    }
    float4 l1_e[2] = {z4, z4};
#pragma unroll
    for (int i = 0; i < 4; ++i) {   // blocks 2i + kh < 8: h0' (0-3), h1 (4-7)
      const int blk = 2 * i + kh;
      const int col = blk < 4 ? kU + lane + 64 * blk : lane + 64 * (blk - 4);
#pragma unroll
      for (int r = 0; r < 2; ++r)
        l1_e[r] = fma4(blk < 4 ? xh0[r][col] : xh1[r][col], w1r[i], l1_e[r]);
    }
    // ================================================= P5: energies + tile records
    if (attn) {
      if (tid < kPM * kF) {   // location features f = Conv1D_SAME(s_{t-1}) + bias, own positions
        const int i = tid / kF, f = tid - i * kF;
        float acc = cw[kKW * kF + f];
#pragma unroll
        for (int j = 0; j < kKW; ++j) acc = fmaf(sprev[aul][n0 + i + j], cw[j * kF + f], acc);
        fs[i][f] = acc;
      }
      gather<1>(R, (oQ + (s * 2 + aul) * kQ) / 4, 0, kQ / 4, 1, reinterpret_cast<float4*>(xq), 0, bt,
                p.err);
      lds_barrier();
      {
        float acc = 0.f;
#pragma unroll
        for (int j = 0; j < 14; ++j) {
          const int d = apart + 16 * j;
          float pre = k1b[j] + xq[d];
#pragma unroll
          for (int f = 0; f < kF; ++f) pre = fmaf(fs[anl][f], locw[f][d], pre);
          acc = fmaf(vv[d], tanh_fast(pre), acc);
        }
        float acc2 = 0.f;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int d = kD1 + apart + 16 * j;
          acc2 = fmaf(vv[d], tanh_fast(k2r[j] + xq[d]), acc2);
        }
        acc = group16_sum(acc);
        acc2 = group16_sum(acc2);
        if (apart == 0) {
          const bool valid = anl < nt && n0 + anl < len;
          e1s[anl] = valid ? acc : -INFINITY;
          e2s[anl] = valid ? acc2 : -INFINITY;
        }
      }
      lds_barrier();
      const int rb = oREC + ((s * 2 + aul) * kAW + atile) * kRec;
      if (wave == 0) {
        const float e1v = lane < nt ? e1s[lane] : -INFINITY;
        const float e2v = lane < nt ? e2s[lane] : -INFINITY;
        const float m1 = wave_max_dpp(e1v), m2 = wave_max_dpp(e2v);
        const float pe = (e1v == -INFINITY) ? 0.f : expf(e1v - m1);
        const float pe2 = (e2v == -INFINITY) ? 0.f : expf(e2v - m2);
        float wg = 0.f;
        if (lane < nt) {
          const int n = n0 + lane;
          const float* ap = abuf[sp][aul];
          wg = ((1.f - uf) * ap[n] + uf * (n > 0 ? ap[n - 1] : 0.f) + 1e-7f) * pe;
        }
        if (lane < kPM) { w1s[lane] = wg; w2s[lane] = lane < nt ? pe2 : 0.f; }
        const float z1 = wave_sum_dpp(pe), a1 = wave_sum_dpp(wg), z2 = wave_sum_dpp(pe2);
        if (lane < 8) {
          float v = 0.f;
          if (lane == 0) v = m1 == -INFINITY ? kNeg : m1;
          else if (lane == 1) v = z1;
          else if (lane == 2) v = a1;
          else if (lane == 3) v = m2 == -INFINITY ? kNeg : m2;
          else if (lane == 4) v = z2;
          pub(R, rb + lane, v, bt);
        }
        if (lane < kPM) {
          pub(R, rb + 8 + lane, e1v == -INFINITY ? kNeg : e1v, bt);
          pub(R, rb + 8 + kPM + lane, e2v == -INFINITY ? kNeg : e2v, bt);
        }
      }
      lds_barrier();
      if (tid < kCtx) {   // unnormalised partial contexts of the tile
        const float* ws = tid < kC1 ? w1s : w2s;
        float c = 0.f;
        for (int i = 0; i < nt; ++i) c = fmaf(ws[i], VS[i][tid], c);
        pub(R, rb + 8 + 2 * kPM + tid, c, bt);
      }
    }
    // ================================================= P6: alignments + contexts (every workgroup)
    gather<3>(R, (oREC + s * 2 * kAW * kRec) / 4, kAW * kRec / 4, ntiles * kRec / 4, nb,
              reinterpret_cast<float4*>(&REC[0][0][0]), kAW * kRec / 4, bt, p.err);
    lds_barrier();
    if (wave < nb) {   // wave r: row r's tile headers
      const bool ok = lane < ntiles;
      const float* hr = REC[wave][ok ? lane : 0];
      const float m1j = ok ? hr[0] : kNeg, z1j = ok ? hr[1] : 0.f, a1j = ok ? hr[2] : 0.f;
      const float m2j = ok ? hr[3] : kNeg, z2j = ok ? hr[4] : 0.f;
      const float M1 = wave_max_dpp(m1j), M2 = wave_max_dpp(m2j);
      const float s1 = m1j > kNegT ? expf(m1j - M1) : 0.f;
      const float s2 = m2j > kNegT ? expf(m2j - M2) : 0.f;
      if (lane < kAW) { scs[wave][0][lane] = s1; scs[wave][1][lane] = s2; }
      const float Z1 = wave_sum_dpp(z1j * s1), A1 = wave_sum_dpp(a1j * s1);
      const float Z2 = wave_sum_dpp(z2j * s2);
      if (lane == 0) {
        hdr[wave][0] = M1; hdr[wave][1] = Z1; hdr[wave][2] = A1; hdr[wave][3] = M2;
        hdr[wave][4] = Z2;
      }
    }
    lds_barrier();
    {
      const int pr = tid >> 8, pn = tid & 255;
      if (pr < nb && pn < N) {
        const float M1 = hdr[pr][0], Z1 = hdr[pr][1], A1 = hdr[pr][2], M2 = hdr[pr][3];
        const float Z2 = hdr[pr][4];
        const int j = pn / P, nl = pn - j * P;
        const float e1 = REC[pr][j][8 + nl], e2 = REC[pr][j][8 + kPM + nl];
        const float pe = e1 > kNegT ? expf(e1 - M1) : 0.f;
        const float pq = e2 > kNegT ? expf(e2 - M2) : 0.f;
        const float* ap = abuf[sp][pr];
        const float a = ((1.f - uf) * ap[pn] + uf * (pn > 0 ? ap[pn - 1] : 0.f) + 1e-7f) * pe *
                        (1.f / A1);
        abuf[s][pr][pn] = a;
        sprev[pr][kPad + pn] = pe * (1.f / Z1);
        if (w == 0) {
          const int b = 2 * g + pr;
          p.AL1[((size_t)(t + 1) * p.B + b) * N + pn] = a;
          p.S2[((size_t)t * p.B + b) * N + pn] = pq * (1.f / Z2);
        }
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int item = tid + kTh * h, cr = item / kCtx, cd = item - cr * kCtx;
        if (cr < nb) {
          const float* sc = scs[cr][cd < kC1 ? 0 : 1];
          float acc = 0.f;
          for (int j = 0; j < ntiles; ++j) acc = fmaf(REC[cr][j][8 + 2 * kPM + cd], sc[j], acc);
          xctx[cr][cd] = acc * (cd < kC1 ? 1.f / hdr[cr][2] : 1.f / hdr[cr][4]);
        }
      }
    }
    lds_barrier();
    // ================================================= P7: LSTM1; attention RNN recurrent part
    {
      float4 acc[2] = {l1_e[0], l1_e[1]};
#pragma unroll
      for (int i = 4; i < 7; ++i) {   // blocks 2i + kh >= 8: contexts
        const int blk = 2 * i + kh;
        if (blk < 13) {
#pragma unroll
          for (int r = 0; r < 2; ++r) acc[r] = fma4(xctx[r][lane + 64 * (blk - 8)], w1r[i], acc[r]);
        }
      }
      lstm_finish(acc[0], acc[1], 1, c1, h1, oH1 + s * 2 * 2 * kU, bt);
    }
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      float4 a = z4;
#pragma unroll
      for (int i = 0; i < 5; ++i) {   // blocks i = kh, kh + 2, ... of [c1 c2 (0-4) | h0 (5-8)]
        const int blk = kh + 2 * i;
        if (blk < 9) {
          const float x = blk < 5 ? xctx[r][lane + 64 * blk] : xh0[r][lane + 64 * (blk - 5)];
          a = fma4(x, W0E[(blk * 4 + unit) * 64 + lane], a);
        }
      }
      att_e[r] = a;
    }
    // ================================================= P8: LSTM2
    gather<1>(R, (oH1 + s * 2 * 2 * kU) / 4, 0, 2 * 2 * kU / 4, 1,
              reinterpret_cast<float4*>(&xh1[0][0]), 0, bt, p.err);
    lds_barrier();
    {
      float4 acc[2] = {l2_e[0], l2_e[1]};
#pragma unroll
      for (int i = 0; i < 2; ++i) {   // blocks 2i + kh < 4: h1'
        const int blk = 2 * i + kh;
#pragma unroll
        for (int r = 0; r < 2; ++r) acc[r] = fma4(xh1[r][kU + lane + 64 * blk], w2r[i], acc[r]);
      }
      lstm_finish(acc[0], acc[1], 2, c2, h2, oH2 + s * 2 * 2 * kU, bt);
    }
    // ================================================= P9: q | k | u; LSTM2 recurrent part
    gather<1>(R, (oH2 + s * 2 * 2 * kU) / 4, 0, 2 * 2 * kU / 4, 1,
              reinterpret_cast<float4*>(&xh2[0][0]), 0, bt, p.err);
    lds_barrier();
    {
      float a[2][2] = {{0.f, 0.f}, {0.f, 0.f}};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int r = 0; r < 2; ++r) {
          const float x = xh2[r][kU + lane + 64 * i];
          a[r][0] = fmaf(x, wk[0][i], a[r][0]);
          a[r][1] = fmaf(x, wk[1][i], a[r][1]);
        }
      }
      float o[4];
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int j = 0; j < 2; ++j) o[2 * r + j] = wave_sum_dpp(a[r][j]) + cbqku[2 * wave + j];
      if (lane < 4) {
        const float v = lane == 0 ? o[0] : lane == 1 ? o[1] : lane == 2 ? o[2] : o[3];
        pub(R, oQKU + (s * 2 + (lane >> 1)) * kQKU + 16 * w + 2 * wave + (lane & 1), v, bt);
      }
    }
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      float4 a = z4;
#pragma unroll
      for (int i = 2; i < 4; ++i)   // blocks 2i + kh >= 4: h2
        a = fma4(xh2[r][lane + 64 * (2 * i + kh - 4)], w2r[i], a);
      l2_e[r] = a;
    }
    // ================================================= P10: own cache rows: scores, partial sums
    // rows j = w + 64 rr of each utterance; slot (r, rr) at cache + (r * kRM + rr) * kRow
    const int nrp = t > w ? (t - 1 - w) / kW + 1 : 0;   // own rows j <= t - 1 (per utterance)
    const bool owner = (t % kW) == w;                  // row t of both utterances is appended here
    const int nr = nrp + (owner ? 1 : 0);
    const int sr = tid >> 5, srow = sr >> 3, srr = sr & 7, sh = (tid >> 4) & 1, ssub = tid & 15;
    const int vh = tid >> 8, vd = tid & 255;            // value pass: head, dim (both rows)
    float kreg[8], ureg[2][kRM];
#pragma unroll
    for (int i = 0; i < 8; ++i)
      kreg[i] = srr < nrp ? ldc(RC, (srow * kRM + srr) * kRow + sh * kSDH + ssub + 16 * i) : 0.f;
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int rr = 0; rr < kRM; ++rr)
        ureg[r][rr] = rr < nrp ? ldc(RC, (r * kRM + rr) * kRow + kSD + vh * kSD + vd) : 0.f;
    if (owner)
      gather<1>(R, (oQKU + s * 2 * kQKU) / 4, 0, 2 * kQKU / 4, 1, reinterpret_cast<float4*>(&xqt[0][0]),
                0, bt, p.err);
    else
      gather<1>(R, (oQKU + s * 2 * kQKU) / 4, kQKU / 4, kQ / 4, 2, reinterpret_cast<float4*>(&xqt[0][0]),
                kQKU / 4, bt, p.err);
    lds_barrier();
    if (owner && tid < 2 * kRow / 4) {   // append row t (plain stores: read back by this CU only)
      const int r = tid / (kRow / 4), c4 = tid - r * (kRow / 4);
      reinterpret_cast<float4*>(cache + (size_t)(r * kRM + nrp) * kRow)[c4] =
          reinterpret_cast<const float4*>(&xqt[r][kQ])[c4];
    }
    {
      float acc = 0.f;
      if (srr < nr) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int d = sh * kSDH + ssub + 16 * i;
          const float kv = srr < nrp ? kreg[i] : xqt[srow][kQ + d];
          acc = fmaf(xqt[srow][d], kv, acc);
        }
      }
      acc = group16_sum(acc);
      if (ssub == 0 && srr < nr) sa_s[(srow * kRM + srr) * 2 + sh] = acc * scale;
    }
    lds_barrier();
    const int sab = oSA + (s * kW + w) * 2 * kSaRec;
    if (wave < 2) {   // wave r: row r's (slot, head) pairs in lanes 2 rr + h
      const int rr = lane >> 1, h = lane & 1;
      const bool ok = lane < 2 * kRM && rr < nr;
      const float sv = ok ? sa_s[wave * 2 * kRM + lane] : -INFINITY;
      const float m0 = wave_max_dpp(h == 0 ? sv : -INFINITY);
      const float m1 = wave_max_dpp(h == 1 ? sv : -INFINITY);
      const float pe = ok ? __expf(sv - (h ? m1 : m0)) : 0.f;
      if (lane < 2 * kRM) sa_pe[wave * 2 * kRM + lane] = pe;
      const float z0 = wave_sum_dpp(h == 0 ? pe : 0.f), z1 = wave_sum_dpp(h == 1 ? pe : 0.f);
      if (lane < 4) {
        const float v = lane == 0 ? (nr > 0 ? m0 : kNeg) : lane == 1 ? z0
                      : lane == 2 ? (nr > 0 ? m1 : kNeg) : z1;
        mine[wave][lane] = v;
        pub(R, sab + wave * kSaRec + lane, v, bt);
      }
    }
    lds_barrier();
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      float o = 0.f;
#pragma unroll
      for (int rr = 0; rr < kRM; ++rr) {
        if (rr < nr) {
          const float uv = rr < nrp ? ureg[r][rr] : xqt[r][kQ + kSD + vh * kSD + vd];
          o = fmaf(sa_pe[(r * kRM + rr) * 2 + vh], uv, o);
        }
      }
      pub(R, sab + r * kSaRec + 8 + vh * kSD + vd, o, bt);
    }
    // ================================================= P11: head output z (this workgroup's 4 dims)
    if (tid < kW * 2 * 3) {   // (producer j, row r, piece q): header | O0[4w..] | O1[4w..]
      const int j = tid / 6, rq = tid - j * 6, r = rq / 3, q = rq - r * 3;
      const int off = oSA + ((s * kW + j) * 2 + r) * kSaRec +
                      (q == 0 ? 0 : q == 1 ? 8 + 4 * w : 8 + kSD + 4 * w);
      float4 v = ldc4(R, off / 4);
      unsigned spins = 0;
      while (!tag_ok4(v, bt)) {
        __builtin_amdgcn_s_sleep(1);
        if (poll_give_up(++spins, p.err)) break;
        v = ldc4(R, off / 4);
      }
      *reinterpret_cast<float4*>(&SAG[r][j][4 * q]) = v;
    }
    lds_barrier();
    if (wave < 2) {   // wave r: row r; lane j = producer
      const int r = wave;
      const float m0j = SAG[r][lane][0], z0j = SAG[r][lane][1];
      const float m1j = SAG[r][lane][2], z1j = SAG[r][lane][3];
      const float M0 = wave_max_dpp(m0j), M1 = wave_max_dpp(m1j);
      const float sc0 = m0j > kNegT ? __expf(m0j - M0) : 0.f;
      const float sc1 = m1j > kNegT ? __expf(m1j - M1) : 0.f;
      const float Z0 = wave_sum_dpp(z0j * sc0), Z1 = wave_sum_dpp(z1j * sc1);
      float v[8];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        v[i] = SAG[r][lane][4 + i] * sc0;
        v[4 + i] = SAG[r][lane][8 + i] * sc1;
      }
      transpose_reduce8(v, lane);   // lanes 8m..8m+7 hold output m: head 0 dims m < 4, head 1 m >= 4
      const float o1 = __shfl(v[0], (lane + 32) & 63, 64);
      if (lane < 32 && (lane & 7) == 0) {
        const int m = lane >> 3, d = 4 * w + m;
        const float pre = v[0] / Z0 + o1 / Z1 + cbz[m];
        pub(R, oZ + (s * 2 + r) * kSD + d, xh2[r][kU + d] + tanhf(pre), bt);
      }
      // this step's probabilities of the own cache rows (PREDICT's decoder self-alignments)
      if (p.SA_P && r < nb && lane < 2 * kRM) {
        const int rr = lane >> 1, h = lane & 1;
        if (rr < nr) {
          const float pr = sa_pe[r * 2 * kRM + lane] * __expf(mine[r][2 * h] - (h ? M1 : M0)) /
                           (h ? Z1 : Z0);
          p.SA_P[(((size_t)(2 * g + r) * 2 + h) * T + t) * T + w + kW * rr] = pr;
        }
      }
    }
    // ================================================= stop test of step t-1, error exit
    if (tid == 0) {
      int fin = __hip_atomic_load(p.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0 ? 2 : 0;
      if (!fin && p.stop_mode && t >= 1 && t - 1 > p.min_iters) {
        bool all = true;
        for (int b = 0; b < p.B; ++b) {
          v2u gv = ldg(RS, sp * 8 + b);
          unsigned spins = 0;
          while (gv[1] != (unsigned)t) {
            __builtin_amdgcn_s_sleep(1);
            if (poll_give_up(++spins, p.err)) break;
            gv = ldg(RS, sp * 8 + b);
          }
          const float sg = 1.f / (1.f + expf(-__uint_as_float(gv[0])));
          if (!(sg > 0.5f)) all = false;
        }
        if (all) fin = 1;
      }
      flag = fin;
    }
    lds_barrier();
    if (flag != 0) {
      if (flag == 1 && g == 0 && w == 0 && tid == 0) p.state[0] = t - 1;
      break;
    }
  }
}

}  // namespace
}  // namespace sat

using namespace sat;

extern "C" int64_t sat_decode_persistent_scratch_bytes(void) {
  return (kZeroDwords + kCacheFloats) * 4;
}

extern "C" int sat_decode_persistent(const SatDecodePersistent* a, void* stream) {
  SAT_CHECK_ARG(a && a->B >= 1 && a->B <= 2 * kG && a->N >= 1 && a->N <= kNM && a->T >= 1 &&
                    a->T <= kW * kRM,
                "sat_decode_persistent: B <= 8, N <= 256, T <= 512 (got B=%d N=%d T=%d)",
                a ? a->B : 0, a ? a->N : 0, a ? a->T : 0);
  SAT_CHECK_ARG(a->lengths && a->K1 && a->V1 && a->K2 && a->V2 && a->Wzp && a->bzp && a->bp0 &&
                    a->Wp1 && a->bp1 && a->W0 && a->b0 && a->Wq && a->b1 && a->v1 && a->convW &&
                    a->convb && a->locW && a->v2 && a->W1 && a->bl1 && a->W2 && a->bl2 &&
                    a->Wqku && a->bqku && a->bz && a->Wms && a->bms && a->MS && a->AL1 &&
                    a->S2 && a->state && a->scratch && a->err,
                "sat_decode_persistent: null pointer");
  SAT_CHECK_ARG(a->scratch_bytes >= sat_decode_persistent_scratch_bytes(),
                "sat_decode_persistent: scratch too small");
  SAT_CHECK_ARG(aligned16(a->W0) && aligned16(a->W1) && aligned16(a->W2) && aligned16(a->b0) &&
                    aligned16(a->bl1) && aligned16(a->bl2) && aligned16(a->scratch),
                "sat_decode_persistent: LSTM weights / biases / scratch must be 16-byte aligned");
  int dev = 0, cus = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, decode_persistent_kernel, kTh, 0) !=
          hipSuccess) {
    set_error("sat_decode_persistent: device query failed");
    return SAT_ERR_HIP;
  }
  if ((int64_t)cus * per_cu < kG * kW) {
    set_error("sat_decode_persistent: fewer than 256 co-resident workgroups on this device");
    return SAT_ERR_UNSUPPORTED;
  }
  hipStream_t s = as_stream(stream);
  if (zero_ranges(s, a->scratch, kZeroDwords, a->err, 1) != hipSuccess) {
    set_error("sat_decode_persistent: scratch clear failed");
    return SAT_ERR_HIP;
  }
  hipLaunchKernelGGL(decode_persistent_kernel, dim3(kG * kW), dim3(kTh), 0, s, *a);
  SAT_LAUNCH_CHECK("sat_decode_persistent");
  return SAT_OK;
}
