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
// Layout: utterance b is decoded by group b = {b, b + 8, ..., b + 248} of 32 workgroups (one XCD
// under the dispatcher's round-robin; the store policy is chosen by the run-time placement check
// xcd_local_group, correctness never rests on it).  Utterances are independent until the stop
// test, so every hand-off inside a step stays inside the group: ten per step, each an all-gather
// of LSB-tagged floats (persistent.h: the data IS the flag, slots alternate by step parity).
// Every weight slice a workgroup needs sits on chip for the whole decode: the two decoder LSTMs,
// the fed-frame / prenet / query / q-k-u columns in registers, the attention RNN's recurrent rows
// in LDS -- per group a full 10 MB replica over 32 CUs.
//
// Per step t (group b, workgroup w owns LSTM units 8w..8w+7 and 8 / 4 / 32 dense columns):
//   P1  z_{t-1} -> mel|stop of step t-1 (outputs, stop granule to every group) and the first
//       prenet layer of step t (the fed frame is folded in: Wzp = W_out[:, fed] W_p0)
//   P2  prenet layer 2                         P3  attention RNN (ZoneoutLSTM 256)
//   P4  query layers of both attentions        P5  16 workgroups: energies of their memory
//       positions + flash-style tile records (max, sum e, sum a~ e, partial contexts)
//   P6  every workgroup: the full alignment (forward recursion) and both contexts from the records
//   P7  LSTM1                                  P8  LSTM2
//   P9  q | k | u of the head (u = v W_o W_t per head: the value, output projection and transform
//       products folded into the cached rows, so the attention output IS the transform input)
//   P10 each workgroup scores its own cache rows (row j lives in workgroup j % 32), partial
//       softmax sums and partial outputs
//   P11 z = h2' + tanh(sum_h O_h / Z_h + b_z): the residual head output (TransformerWrapper,
//       modules/rnn_wrappers.py:87-124; self_attention.py:45-65 without dropout)
// Recurrent parts of the LSTM products (h_{t-1}, contexts) are formed while the step's other
// hand-offs are in flight.  The stop test of step t-1 (t > min_iters and sigmoid(stop) > 0.5 for
// every utterance) reads the B stop granules at the end of step t: every workgroup of every group
// sees the same values and leaves the loop at the same step.
#include "persistent.h"

#include <algorithm>

// -DSAT_DP_TRACE=1 (a separate build: tools/probes/dp_profile.py): thread 0 of every workgroup
// sums the wall clock (100 MHz) spent in each phase segment into prof[blockIdx][24]
#ifndef SAT_DP_TRACE
#define SAT_DP_TRACE 0
#endif

namespace sat {
namespace {

// ---- the LJSpeech / VCTK decoder (hparams.py; checked by the host entry)
constexpr int kG = 8;             // groups = utterances (B <= 8)
constexpr int kW = 32;            // workgroups per group
constexpr int kTh = 512;          // threads per workgroup
constexpr int kAW = 32;           // attention workgroups per group (memory positions split)
constexpr int kPM = 8;            // memory positions per attention workgroup (N <= 256)
constexpr int kRM = 16;           // cache rows per workgroup (T <= 512)
constexpr int kNM = kAW * kPM;    // 256
constexpr int kMR = 160;          // mel values per step (80 x r=2)
constexpr int kMS = 164;          // MS row: mel | stop | pad
constexpr int kP0 = 256, kP1 = 128;
constexpr int kU = 256;           // attention RNN = LSTM1 = LSTM2 units
constexpr int kC1 = 256, kCtx = 288;
constexpr int kD1 = 224, kQ = 256;
constexpr int kF = 5, kKW = 10, kPad = 4;
constexpr int kSD = 256, kSDH = 128, kQKU = 1024, kRow = 768;   // cached row = [k | u0 | u1]
constexpr int kRec = 8 + 2 * kPM + kCtx;                         // 312
constexpr int kSaRec = 8 + 2 * kSD;                              // 520
constexpr float kNeg = -3.0e38f;   // finite stand-in for -inf in tagged words
constexpr float kNegT = -1.0e38f;  // anything below is "no position"

// hand-off buffers of one group (float offsets; two slots per edge, slot = step & 1)
constexpr int oZ = 0;
constexpr int oY0 = oZ + 2 * kSD;
constexpr int oP = oY0 + 2 * kP0;
constexpr int oH0 = oP + 2 * kP1;
constexpr int oQ = oH0 + 2 * 2 * kU;
constexpr int oREC = oQ + 2 * kQ;
constexpr int oH1 = oREC + 2 * kAW * kRec;
constexpr int oH2 = oH1 + 2 * 2 * kU;
constexpr int oQKU = oH2 + 2 * 2 * kU;
constexpr int oSA = oQKU + 2 * kQKU;
constexpr int kGroupFloats = oSA + 2 * kW * kSaRec;
// after the groups: stop granules [2][8] (uint2), placement words [256], then the caches
constexpr int64_t kZeroDwords = (int64_t)kG * kGroupFloats + 32 + 256;
constexpr int64_t kCacheFloats = (int64_t)kG * kW * kRM * kRow;

__device__ __forceinline__ float4 fma4(float x, float4 w, float4 a) {
  return make_float4(fmaf(x, w.x, a.x), fmaf(x, w.y, a.y), fmaf(x, w.z, a.z), fmaf(x, w.w, a.w));
}
// max / sum over each aligned group of 16 or 32 lanes (result in every lane of the group): the
// step's small reductions (<= 8 positions, <= 16 cache rows, <= 32 tiles / producers) need no
// full-wave chain with readlanes
__device__ __forceinline__ float rdl(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ float g16max(float v) {
  v = group8_max(v);
  return fmaxf(v, dpp<0x140>(v));
}
__device__ __forceinline__ float g32max(float v) {
  v = g16max(v);
  return fmaxf(v, __shfl_xor(v, 16, 64));
}
__device__ __forceinline__ float4 wave_sum4(float4 v) {
  return make_float4(wave_sum_dpp(v.x), wave_sum_dpp(v.y), wave_sum_dpp(v.z), wave_sum_dpp(v.w));
}

// ZoneoutLSTM cell, eval mode (ext tacotron2 ZoneoutLSTMCell: c = (1-zc) c' + zc c, same for h),
// formed exactly as lstm.hip's step kernels; returns the raw output h'.
__device__ __forceinline__ float zlstm_cell(float4 g, float4 b, float zc, float zh, float& c,
                                            float& h) {
  const float gi = sigmoid_fast(g.x + b.x);
  const float gj = tanh_lstm(g.y + b.y);
  const float gf = sigmoid_fast(g.z + b.z + 1.0f);   // forget_bias = 1.0
  const float go = sigmoid_fast(g.w + b.w);
  const float cn = gf * c + gi * gj;
  const float hn = go * tanh_lstm(cn);
  c = (1.f - zc) * cn + zc * c;
  h = (1.f - zh) * hn + zh * h;
  return hn;
}

// Poll-gather n4 tagged float4 words starting at float4 index base4 into LDS: NPT loads per
// thread issued before the first check (one round trip when the producers are done).
template <int NPT>
__device__ __forceinline__ void gather(__amdgpu_buffer_rsrc_t r, int base4, int n4, float4* dst,
                                       unsigned bit, int* err) {
  float4 v[NPT];
#pragma unroll
  for (int q = 0; q < NPT; ++q) {
    const int i = threadIdx.x + q * kTh;
    v[q] = ldc4(r, base4 + min(i, n4 - 1));
  }
#pragma unroll
  for (int q = 0; q < NPT; ++q) {
    const int i = threadIdx.x + q * kTh;
    if (i < n4) {
      unsigned spins = 0;
      while (!tag_ok4(v[q], bit)) {
        __builtin_amdgcn_s_sleep(1);
        if (poll_give_up(++spins, err)) break;
        v[q] = ldc4(r, base4 + i);
      }
      dst[i] = v[q];
    }
  }
}

__global__ void __launch_bounds__(kTh) decode_persistent_kernel(SatDecodePersistent p) {
  const int g = blockIdx.x % kG, w = blockIdx.x / kG;
  if (g >= p.B) return;   // no utterance: no partner outside this group
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int N = p.N, T = p.T;
  const int P = (N + kAW - 1) / kAW;            // positions per attention workgroup
  const int ntiles = (N + P - 1) / P;
  const bool attn = w < ntiles;
  const int n0 = w * P, nt = attn ? min(P, N - n0) : 0;
  const int len = (int)p.lengths[g];
  const float zc = p.zc, zh = p.zh, uf = p.u;
  float* scr = reinterpret_cast<float*>(p.scratch);
  const __amdgpu_buffer_rsrc_t R = rsrc(scr + (size_t)g * kGroupFloats);
  unsigned* stopw = reinterpret_cast<unsigned*>(scr + (size_t)kG * kGroupFloats);
  unsigned* xid = stopw + 32;
  float* cache = reinterpret_cast<float*>(xid + 256) + ((size_t)g * kW + w) * kRM * kRow;
  const __amdgpu_buffer_rsrc_t RS = rsrc(stopw);
  const __amdgpu_buffer_rsrc_t RC = rsrc(cache);

  __shared__ __attribute__((aligned(16))) float4 W0E[9 * 8 * 64];   // attention RNN [c1 c2 | h0] rows
  __shared__ __attribute__((aligned(16))) float VS[kPM][kCtx];      // [V1 | V2] of own positions
  __shared__ __attribute__((aligned(16))) float locw[kF][kD1];
  __shared__ __attribute__((aligned(16))) float vv[kQ];             // [v1 | v2]
  __shared__ float cw[kKW * kF + kF];                               // conv kernel [KW][F] | bias
  __shared__ float sprev[kNM + 16];                                 // s_{t-1}, kPad zeros left
  __shared__ float abuf[2][kNM];                                    // alignments, slot = step & 1
  __shared__ float fs[kPM][kF];
  __shared__ float e1s[kPM], e2s[kPM], w1s[kPM], w2s[kPM];
  __shared__ __attribute__((aligned(16))) float REC[kAW][kRec];
  __shared__ __attribute__((aligned(16))) float xz[kSD];
  __shared__ __attribute__((aligned(16))) float xy0[kP0];
  __shared__ __attribute__((aligned(16))) float xp[kP1];
  __shared__ __attribute__((aligned(16))) float xh0[2 * kU];   // [h0 | h0']
  __shared__ __attribute__((aligned(16))) float xh1[2 * kU];   // [h1 | h1']
  __shared__ __attribute__((aligned(16))) float xh2[2 * kU];   // [h2 | h2']
  __shared__ __attribute__((aligned(16))) float xctx[320];     // [c1 | c2 | 0 pad]
  __shared__ __attribute__((aligned(16))) float xq[kQ];
  __shared__ __attribute__((aligned(16))) float xqt[kQKU];     // [q | k | u0 | u1] of step t
  __shared__ __attribute__((aligned(16))) float SAG[kW][20];
  __shared__ __attribute__((aligned(16))) float4 bias4[3][8];
  __shared__ float hdr[8], scs1[kAW], scs2[kAW], sa_s[2 * kRM], sa_pe[2 * kRM], mine[4];
  __shared__ float cbzp[8], cbp0[8], cbms[8], cbp1[4], cbqku[32], cbz[8];
  __shared__ int flag;

  // ---------------------------------------------------------------- one-time loads
  const int uu = 8 * w + wave;   // the LSTM unit of this wave (all three LSTMs)
  const float4* W0_4 = reinterpret_cast<const float4*>(p.W0);
  const float4* W1_4 = reinterpret_cast<const float4*>(p.W1);
  const float4* W2_4 = reinterpret_cast<const float4*>(p.W2);
  float4 w0r[2];    // attention RNN rows of the prenet output (late part)
#pragma unroll
  for (int i = 0; i < 2; ++i) w0r[i] = W0_4[(size_t)(lane + 64 * i) * kU + uu];
  // LSTM1 rows [0:256) h0', [256:544) c1 c2, [544:800) h1: i < 4 h0', 4..7 h1, 8..12 contexts
  float4 w1r[13];
#pragma unroll
  for (int i = 0; i < 13; ++i) {
    int row;
    if (i < 4) row = lane + 64 * i;
    else if (i < 8) row = kU + kCtx + lane + 64 * (i - 4);
    else row = (lane + 64 * (i - 8) < kCtx) ? kU + lane + 64 * (i - 8) : -1;
    w1r[i] = row >= 0 ? W1_4[(size_t)row * kU + uu] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  float4 w2r[8];    // LSTM2 rows [0:256) h1', [256:512) h2
#pragma unroll
  for (int i = 0; i < 8; ++i) w2r[i] = W2_4[(size_t)(lane + 64 * i) * kU + uu];
  // dense columns: prenet-1 col 8w+wave from z, mel|stop col w+32 wave, prenet-2 col 4w+wave,
  // query col 8w+wave, q|k|u cols 32w + 4 wave + j
  const int cpre = 8 * w + wave, cmel = w + 32 * wave, cp1 = 4 * w + wave, cq = 8 * w + wave;
  const bool has_mel = wave < 6 && cmel <= kMR;
  float wzp[4], wms[4], wp1[4], wq[4], wk[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int k = lane + 64 * i;
    wzp[i] = p.Wzp[(size_t)k * kP0 + cpre];
    wms[i] = has_mel ? p.Wms[(size_t)k * kMS + cmel] : 0.f;
    wp1[i] = wave < 4 ? p.Wp1[(size_t)k * kP1 + cp1] : 0.f;
    wq[i] = p.Wq[(size_t)k * kQ + cq];
#pragma unroll
    for (int j = 0; j < 4; ++j) wk[j][i] = p.Wqku[(size_t)k * kQKU + 32 * w + 4 * wave + j];
  }
  // attention: K1 + b1 / K2 slices of this lane's position (32 lanes per position)
  // (one wave per position, lane = energy dims lane + 64 j)
  const int anl = tid >> 6, apart = tid & 63;
  const bool apos = attn && anl < nt;
  float k1b[4], k2r = 0.f;
  {
    const size_t rowp = (size_t)g * N + n0 + (apos ? anl : 0);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int d = apart + 64 * j;
      k1b[j] = (apos && d < kD1) ? p.K1[rowp * kD1 + d] + p.b1[d] : 0.f;
    }
    if (apos && apart < 32) k2r = p.K2[rowp * 32 + apart];
  }
  for (int idx = tid; idx < 9 * 8 * 64; idx += kTh) {
    const int i = idx >> 9, wv = (idx >> 6) & 7, ln = idx & 63;
    int row;
    if (i < 5) row = (ln + 64 * i < kCtx) ? kP1 + ln + 64 * i : -1;
    else row = kP1 + kCtx + ln + 64 * (i - 5);
    W0E[idx] = row >= 0 ? W0_4[(size_t)row * kU + 8 * w + wv] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  for (int idx = tid; idx < nt * kCtx; idx += kTh) {
    const int i = idx / kCtx, d = idx - i * kCtx;
    const size_t rowp = (size_t)g * N + n0 + i;
    VS[i][d] = d < kC1 ? p.V1[rowp * kC1 + d] : p.V2[rowp * 32 + (d - kC1)];
  }
  for (int idx = tid; idx < kF * kD1; idx += kTh) locw[idx / kD1][idx % kD1] = p.locW[idx];
  if (tid < kQ) vv[tid] = tid < kD1 ? p.v1[tid] : p.v2[tid - kD1];
  if (tid < kKW * kF) cw[tid] = p.convW[tid];
  if (tid < kF) cw[kKW * kF + tid] = p.convb[tid];
  for (int idx = tid; idx < kNM + 16; idx += kTh) sprev[idx] = 0.f;
  for (int idx = tid; idx < 2 * kNM; idx += kTh) (&abuf[0][0])[idx] = 0.f;
  for (int idx = tid; idx < 2 * kU; idx += kTh) { xh0[idx] = 0.f; xh1[idx] = 0.f; xh2[idx] = 0.f; }
  if (tid < 320) xctx[tid] = 0.f;
  if (tid < 8) {
    bias4[0][tid] = reinterpret_cast<const float4*>(p.b0)[8 * w + tid];
    bias4[1][tid] = reinterpret_cast<const float4*>(p.bl1)[8 * w + tid];
    bias4[2][tid] = reinterpret_cast<const float4*>(p.bl2)[8 * w + tid];
    cbzp[tid] = p.bzp[8 * w + tid];
    cbp0[tid] = p.bp0[8 * w + tid];
    cbz[tid] = p.bz[8 * w + tid];
    const int cm = w + 32 * tid;
    cbms[tid] = (tid < 6 && cm <= kMR) ? p.bms[cm] : 0.f;
    if (tid < 4) cbp1[tid] = p.bp1[4 * w + tid];
  }
  if (tid < 32) cbqku[tid] = p.bqku[32 * w + tid];
  __syncthreads();
  if (tid == 0) abuf[1][0] = 1.f;   // a_{-1} = one-hot at position 0 (forward_attention.py:131-133)
  const bool xl = xcd_local_group(xid, g, kG, kW, p.err);   // ends in a barrier

  float c0 = 0.f, h0 = 0.f, c1 = 0.f, h1 = 0.f, c2 = 0.f, h2 = 0.f;   // own unit's states
  float4 att_early = make_float4(0.f, 0.f, 0.f, 0.f);   // recurrent part of the next attention RNN step
  float4 l2_early = make_float4(0.f, 0.f, 0.f, 0.f);    // recurrent part of the next LSTM2 step
  const float scale = p.scale;

#if SAT_DP_TRACE
  __shared__ long long tacc[28], tabs[28];   // thread 0's segment clocks (LDS: no registers)
  if (threadIdx.x < 28) { tacc[threadIdx.x] = 0; tabs[threadIdx.x] = 0; }
  long long tlast = wall_clock64();
#define TP(k)                                   \
  if (threadIdx.x == 0) {                       \
    const long long tnow = wall_clock64();      \
    tacc[k] += tnow - tlast;                    \
    tlast = tnow;                               \
    if (t == 300) tabs[k] = tnow;               \
  }
#else
#define TP(k)
#endif
  int t = 0;
  for (; t <= T; ++t) {
    int tid_ = (int)threadIdx.x;
    asm volatile("" : "+v"(tid_));
    const int tid = tid_, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int uu = 8 * w + wave;
    const int anl = tid >> 6, apart = tid & 63;
    const int cpre = 8 * w + wave, cmel = w + 32 * wave, cp1 = 4 * w + wave, cq = 8 * w + wave;
    const bool has_mel = wave < 6 && cmel <= kMR;
    const int s = t & 1, sp = s ^ 1;
    const unsigned bt = lsb_tag(t), bp = lsb_tag(t - 1);
    // ================================================= P1: mel|stop of t-1, prenet layer 1 of t
    if (t > 0) {
      gather<1>(R, (oZ + sp * kSD) / 4, kSD / 4, reinterpret_cast<float4*>(xz), bp, p.err);
      lds_barrier();
      TP(1)
      if (wave < 6) {
        float a = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) a = fmaf(xz[lane + 64 * i], wms[i], a);
        a = wave_sum_dpp(a);
        if (has_mel && lane == 0) {
          const float v = a + cbms[wave];
          p.MS[((size_t)(t - 1) * p.B + g) * kMS + cmel] = v;
          if (cmel == kMR) stg(RS, sp * 8 + g, v, (unsigned)t);   // {stop_{t-1}, t} to every group
        }
      }
    }
    if (t == T) break;
    TP(2)
    {
      float a;
      if (t > 0) {
        a = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) a = fmaf(xz[lane + 64 * i], wzp[i], a);
        a = wave_sum_dpp(a) + cbzp[wave];
      } else {
        a = cbp0[wave];   // the go frame (zeros)
      }
      a = fmaxf(a, 0.f);
      if (lane == 0) stcx(xl, R, oY0 + s * kP0 + cpre, tagf(a, bt));
    }
    TP(3)
    // ================================================= P2: prenet layer 2
    gather<1>(R, (oY0 + s * kP0) / 4, kP0 / 4, reinterpret_cast<float4*>(xy0), bt, p.err);
    lds_barrier();
    TP(4)
    if (wave < 4) {
      float a = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) a = fmaf(xy0[lane + 64 * i], wp1[i], a);
      a = fmaxf(wave_sum_dpp(a) + cbp1[wave], 0.f);
      if (lane == 0) stcx(xl, R, oP + s * kP1 + cp1, tagf(a, bt));
    }
    TP(5)
    // ================================================= P3: attention RNN
    gather<1>(R, (oP + s * kP1) / 4, kP1 / 4, reinterpret_cast<float4*>(xp), bt, p.err);
    lds_barrier();
    TP(6)
    {
      float4 acc = att_early;
#pragma unroll
      for (int i = 0; i < 2; ++i) acc = fma4(xp[lane + 64 * i], w0r[i], acc);
      acc = wave_sum4(acc);
      const float hr = zlstm_cell(acc, bias4[0][wave], zc, zh, c0, h0);
      if (lane == 0) {
        stcx(xl, R, oH0 + s * 2 * kU + uu, tagf(h0, bt));
        stcx(xl, R, oH0 + s * 2 * kU + kU + uu, tagf(hr, bt));
      }
    }
    TP(7)
    // ================================================= P4: query layers; LSTM1 recurrent part
    gather<1>(R, (oH0 + s * 2 * kU) / 4, 2 * kU / 4, reinterpret_cast<float4*>(xh0), bt, p.err);
    lds_barrier();
    TP(8)
    {
      float a = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) a = fmaf(xh0[kU + lane + 64 * i], wq[i], a);
      a = wave_sum_dpp(a);
      if (lane == 0) stcx(xl, R, oQ + s * kQ + cq, tagf(a, bt));
    }
    float4 l1_early = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int i = 0; i < 4; ++i) l1_early = fma4(xh0[kU + lane + 64 * i], w1r[i], l1_early);
#pragma unroll
    for (int i = 4; i < 8; ++i) l1_early = fma4(xh1[lane + 64 * (i - 4)], w1r[i], l1_early);
    TP(9)
    // ================================================= P5: energies + tile records
    if (attn) {
      if (tid < kPM * kF) {   // location features f = Conv1D_SAME(s_{t-1}) + bias, own positions
        const int i = tid / kF, f = tid - i * kF;
        float acc = cw[kKW * kF + f];
#pragma unroll
        for (int j = 0; j < kKW; ++j) acc = fmaf(sprev[n0 + i + j], cw[j * kF + f], acc);
        fs[i][f] = acc;
      }
      gather<1>(R, (oQ + s * kQ) / 4, kQ / 4, reinterpret_cast<float4*>(xq), bt, p.err);
      lds_barrier();
      TP(10)
      {
        float acc = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int d = min(apart + 64 * j, kD1 - 1);   // j = 3: lanes >= 32 carry zero weight
          float pre = k1b[j] + xq[d];
#pragma unroll
          for (int f = 0; f < kF; ++f) pre = fmaf(fs[anl][f], locw[f][d], pre);
          const float vw = (j < 3 || apart < 32) ? vv[d] : 0.f;
          acc = fmaf(vw, tanh_fast(pre), acc);
        }
        const int d2 = kD1 + (apart & 31);
        const float acc2 = apart < 32 ? vv[d2] * tanh_fast(k2r + xq[d2]) : 0.f;
        acc = wave_sum_dpp(acc);
        const float acc2s = wave_sum_dpp(acc2);
        if (apart == 0) {
          const bool valid = anl < nt && n0 + anl < len;
          e1s[anl] = valid ? acc : -INFINITY;
          e2s[anl] = valid ? acc2s : -INFINITY;
        }
      }
      lds_barrier();
      TP(24)
      const int rb = oREC + (s * kAW + w) * kRec;
      if (wave == 0) {
        const float e1v = lane < nt ? e1s[lane] : -INFINITY;
        const float e2v = lane < nt ? e2s[lane] : -INFINITY;
        const float m1 = group8_max(e1v), m2 = group8_max(e2v);   // lanes 0-7 = positions
        const float pe = (e1v == -INFINITY) ? 0.f : expf(e1v - m1);
        const float pe2 = (e2v == -INFINITY) ? 0.f : expf(e2v - m2);
        float wg = 0.f;
        if (lane < nt) {
          const int n = n0 + lane;
          const float* ap = abuf[sp];
          wg = ((1.f - uf) * ap[n] + uf * (n > 0 ? ap[n - 1] : 0.f) + 1e-7f) * pe;
        }
        if (lane < kPM) { w1s[lane] = wg; w2s[lane] = lane < nt ? pe2 : 0.f; }
        const float z1 = group8_sum(pe), a1 = group8_sum(wg), z2 = group8_sum(pe2);
        if (lane < 8) {
          float v = 0.f;
          if (lane == 0) v = m1 == -INFINITY ? kNeg : m1;
          else if (lane == 1) v = z1;
          else if (lane == 2) v = a1;
          else if (lane == 3) v = m2 == -INFINITY ? kNeg : m2;
          else if (lane == 4) v = z2;
          stcx(xl, R, rb + lane, tagf(v, bt));
        }
        if (lane < kPM) {
          stcx(xl, R, rb + 8 + lane, tagf(e1v == -INFINITY ? kNeg : e1v, bt));
          stcx(xl, R, rb + 8 + kPM + lane, tagf(e2v == -INFINITY ? kNeg : e2v, bt));
        }
      }
      lds_barrier();
      TP(25)
      if (tid < kCtx) {   // unnormalised partial contexts of the tile
        const float* ws = tid < kC1 ? w1s : w2s;
        float c = 0.f;
        for (int i = 0; i < nt; ++i) c = fmaf(ws[i], VS[i][tid], c);
        stcx(xl, R, rb + 8 + 2 * kPM + tid, tagf(c, bt));
      }
    }
    TP(11)
    // ================================================= P6: alignment + contexts (every workgroup)
    gather<5>(R, (oREC + s * kAW * kRec) / 4, ntiles * kRec / 4, reinterpret_cast<float4*>(&REC[0][0]),
              bt, p.err);
    lds_barrier();
    TP(12)
    if (wave == 0) {
      const bool ok = lane < ntiles;
      const float m1j = ok ? REC[lane][0] : kNeg, z1j = ok ? REC[lane][1] : 0.f;
      const float a1j = ok ? REC[lane][2] : 0.f, m2j = ok ? REC[lane][3] : kNeg;
      const float z2j = ok ? REC[lane][4] : 0.f;
      const float M1 = g32max(m1j), M2 = g32max(m2j);   // lanes 0-31 = tiles
      const float s1 = m1j > kNegT ? expf(m1j - M1) : 0.f;
      const float s2 = m2j > kNegT ? expf(m2j - M2) : 0.f;
      if (lane < kAW) { scs1[lane] = s1; scs2[lane] = s2; }
      const float Z1 = group32_sum(z1j * s1), A1 = group32_sum(a1j * s1);
      const float Z2 = group32_sum(z2j * s2);
      if (lane == 0) { hdr[0] = M1; hdr[1] = Z1; hdr[2] = A1; hdr[3] = M2; hdr[4] = Z2; }
    }
    lds_barrier();
    TP(26)
    {
      const float M1 = hdr[0], Z1 = hdr[1], A1 = hdr[2], M2 = hdr[3], Z2 = hdr[4];
      const float inv1 = 1.f / A1, invz1 = 1.f / Z1, invz2 = 1.f / Z2;
      if (tid < N) {
        const int n = tid, j = n / P, nl = n - j * P;
        const float e = REC[j][8 + nl], e2 = REC[j][8 + kPM + nl];
        const float pe = e > kNegT ? expf(e - M1) : 0.f;
        const float pe2 = e2 > kNegT ? expf(e2 - M2) : 0.f;
        const float* ap = abuf[sp];
        const float a = ((1.f - uf) * ap[n] + uf * (n > 0 ? ap[n - 1] : 0.f) + 1e-7f) * pe * inv1;
        const float s2v = pe2 * invz2;
        abuf[s][n] = a;
        sprev[kPad + n] = pe * invz1;
        if (w == 0) {
          p.AL1[((size_t)(t + 1) * p.B + g) * N + n] = a;
          p.S2[((size_t)t * p.B + g) * N + n] = s2v;
        }
      }
      if (tid < kCtx) {
        const float* sc = tid < kC1 ? scs1 : scs2;
        float acc = 0.f;
        for (int j = 0; j < ntiles; ++j) acc = fmaf(REC[j][8 + 2 * kPM + tid], sc[j], acc);
        xctx[tid] = acc * (tid < kC1 ? inv1 : invz2);
      }
    }
    lds_barrier();
    TP(13)
    // ================================================= P7: LSTM1; attention RNN recurrent part
    {
      float4 acc = l1_early;
#pragma unroll
      for (int i = 8; i < 13; ++i) acc = fma4(xctx[lane + 64 * (i - 8)], w1r[i], acc);
      acc = wave_sum4(acc);
      const float hr = zlstm_cell(acc, bias4[1][wave], zc, zh, c1, h1);
      if (lane == 0) {
        stcx(xl, R, oH1 + s * 2 * kU + uu, tagf(h1, bt));
        stcx(xl, R, oH1 + s * 2 * kU + kU + uu, tagf(hr, bt));
      }
    }
    att_early = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int i = 0; i < 5; ++i)
      att_early = fma4(xctx[lane + 64 * i], W0E[(i * 8 + wave) * 64 + lane], att_early);
#pragma unroll
    for (int i = 5; i < 9; ++i)
      att_early = fma4(xh0[lane + 64 * (i - 5)], W0E[(i * 8 + wave) * 64 + lane], att_early);
    TP(14)
    // ================================================= P8: LSTM2
    gather<1>(R, (oH1 + s * 2 * kU) / 4, 2 * kU / 4, reinterpret_cast<float4*>(xh1), bt, p.err);
    lds_barrier();
    TP(15)
    {
      float4 acc = l2_early;
#pragma unroll
      for (int i = 0; i < 4; ++i) acc = fma4(xh1[kU + lane + 64 * i], w2r[i], acc);
      acc = wave_sum4(acc);
      const float hr = zlstm_cell(acc, bias4[2][wave], zc, zh, c2, h2);
      if (lane == 0) {
        stcx(xl, R, oH2 + s * 2 * kU + uu, tagf(h2, bt));
        stcx(xl, R, oH2 + s * 2 * kU + kU + uu, tagf(hr, bt));
      }
    }
    TP(16)
    // ================================================= P9: q | k | u; LSTM2 recurrent part
    gather<1>(R, (oH2 + s * 2 * kU) / 4, 2 * kU / 4, reinterpret_cast<float4*>(xh2), bt, p.err);
    lds_barrier();
    TP(17)
    {
      float a[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float x = xh2[kU + lane + 64 * i];
#pragma unroll
        for (int j = 0; j < 4; ++j) a[j] = fmaf(x, wk[j][i], a[j]);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) a[j] = wave_sum_dpp(a[j]) + cbqku[4 * wave + j];
      if (lane < 4) {
        const float v = lane == 0 ? a[0] : lane == 1 ? a[1] : lane == 2 ? a[2] : a[3];
        stcx(xl, R, oQKU + s * kQKU + 32 * w + 4 * wave + lane, tagf(v, bt));
      }
    }
    l2_early = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int i = 4; i < 8; ++i) l2_early = fma4(xh2[lane + 64 * (i - 4)], w2r[i], l2_early);
    TP(18)
    // ================================================= P10: own cache rows: scores, partial sums
    const int nrp = t > w ? (t - 1 - w) / kW + 1 : 0;   // own rows j = w + 32 r <= t - 1
    const bool owner = (t % kW) == w;                  // row t is appended here
    const int nr = nrp + (owner ? 1 : 0);
    const int sr = tid >> 5, sh = (tid >> 4) & 1, ssub = tid & 15;   // score pass roles
    const int vh = tid >> 8, vd = tid & 255;                          // value pass roles
    float kreg[8], ureg[kRM];
#pragma unroll
    for (int i = 0; i < 8; ++i)
      kreg[i] = sr < nrp ? ldc(RC, sr * kRow + sh * kSDH + ssub + 16 * i) : 0.f;
#pragma unroll
    for (int r = 0; r < kRM; ++r) ureg[r] = r < nrp ? ldc(RC, r * kRow + kSD + vh * kSD + vd) : 0.f;
    gather<1>(R, (oQKU + s * kQKU) / 4, owner ? kQKU / 4 : kQ / 4, reinterpret_cast<float4*>(xqt), bt,
              p.err);
    lds_barrier();
    TP(19)
    if (owner && tid < kRow / 4)   // append row t = [k | u0 | u1] (plain stores: read back by this CU)
      reinterpret_cast<float4*>(cache + (size_t)nrp * kRow)[tid] =
          reinterpret_cast<const float4*>(xqt + kQ)[tid];
    {
      float acc = 0.f;
      if (sr < nr) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int d = sh * kSDH + ssub + 16 * i;
          const float kv = sr < nrp ? kreg[i] : xqt[kQ + d];
          acc = fmaf(xqt[d], kv, acc);
        }
      }
      acc = group16_sum(acc);
      if (ssub == 0 && sr < nr) sa_s[sh * kRM + sr] = acc * scale;
    }
    lds_barrier();
    const int sab = oSA + (s * kW + w) * kSaRec;
    if (wave == 0) {
      const int r = lane & 15;   // lanes 0-15 head 0, 16-31 head 1 (row r)
      const bool ok = lane < 2 * kRM && r < nr;
      const float sv = ok ? sa_s[lane] : -INFINITY;
      const float mh = g16max(sv);
      const float pe = ok ? __expf(sv - mh) : 0.f;
      if (lane < 2 * kRM) sa_pe[lane] = pe;
      const float zg = group16_sum(pe);
      const float m0 = rdl(mh, 0), m1 = rdl(mh, 16), z0 = rdl(zg, 0), z1 = rdl(zg, 16);
      if (lane < 4) {
        const float v = lane == 0 ? (nr > 0 ? m0 : kNeg) : lane == 1 ? z0
                      : lane == 2 ? (nr > 0 ? m1 : kNeg) : z1;
        mine[lane] = v;
        stcx(xl, R, sab + lane, tagf(v, bt));
      }
    }
    lds_barrier();
    {
      float o = 0.f;
#pragma unroll
      for (int r = 0; r < kRM; ++r) {
        if (r < nr) {
          const float uv = r < nrp ? ureg[r] : xqt[kQ + kSD + vh * kSD + vd];
          o = fmaf(sa_pe[vh * kRM + r], uv, o);
        }
      }
      stcx(xl, R, sab + 8 + vh * kSD + vd, tagf(o, bt));
    }
    TP(20)
    // ================================================= P11: head output z (this workgroup's 8 dims)
    if (tid < kW * 5) {
      const int j = tid / 5, q = tid - j * 5;
      const int off = oSA + (s * kW + j) * kSaRec +
                      (q == 0 ? 0 : q <= 2 ? 8 + 8 * w + 4 * (q - 1) : 8 + kSD + 8 * w + 4 * (q - 3));
      float4 v = ldc4(R, off / 4);
      unsigned spins = 0;
      while (!tag_ok4(v, bt)) {
        __builtin_amdgcn_s_sleep(1);
        if (poll_give_up(++spins, p.err)) break;
        v = ldc4(R, off / 4);
      }
      *reinterpret_cast<float4*>(&SAG[j][4 * q]) = v;
    }
    lds_barrier();
    TP(21)
    if (wave == 0) {
      const bool ok = lane < kW;
      const float m0j = ok ? SAG[lane][0] : kNeg, z0j = ok ? SAG[lane][1] : 0.f;
      const float m1j = ok ? SAG[lane][2] : kNeg, z1j = ok ? SAG[lane][3] : 0.f;
      const float M0 = rdl(g32max(m0j), 0), M1 = rdl(g32max(m1j), 0);
      const float sc0 = m0j > kNegT ? __expf(m0j - M0) : 0.f;
      const float sc1 = m1j > kNegT ? __expf(m1j - M1) : 0.f;
      const float Z0 = rdl(group32_sum(z0j * sc0), 0), Z1 = rdl(group32_sum(z1j * sc1), 0);
      float v[16];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        v[i] = ok ? SAG[lane][4 + i] * sc0 : 0.f;
        v[8 + i] = ok ? SAG[lane][12 + i] * sc1 : 0.f;
      }
      transpose_reduce16(v, lane);   // lane 4m holds output m: head 0 dims m < 8, head 1 m >= 8
      const float o1 = __shfl(v[0], (lane + 32) & 63, 64);
      if (lane < 32 && (lane & 3) == 0) {
        const int m = lane >> 2, d = 8 * w + m;
        const float pre = v[0] / Z0 + o1 / Z1 + cbz[m];
        const float z = xh2[kU + d] + tanhf(pre);
        stcx(xl, R, oZ + s * kSD + d, tagf(z, bt));
      }
      // this step's probability row of the own cache rows (PREDICT's decoder self-alignments)
      if (p.SA_P && lane < 2 * kRM) {
        const int r = lane & 15, h = lane >> 4;
        if (r < nr) {
          const float pr = sa_pe[lane] * __expf(mine[2 * h] - (h ? M1 : M0)) / (h ? Z1 : Z0);
          p.SA_P[(((size_t)g * 2 + h) * T + t) * T + w + kW * r] = pr;
        }
      }
    }
    TP(22)
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
    TP(23)
    if (flag != 0) {
      if (flag == 1 && g == 0 && w == 0 && tid == 0) p.state[0] = t - 1;
      break;
    }
  }
#if SAT_DP_TRACE
  if (threadIdx.x == 0 && p.prof) {
    for (int k = 0; k < 28; ++k) p.prof[blockIdx.x * 28 + k] = tacc[k];
    p.prof[256 * 28 + blockIdx.x] = t;
    for (int k = 0; k < 28; ++k) p.prof[256 * 29 + blockIdx.x * 28 + k] = tabs[k];
  }
#endif
#undef TP
}

}  // namespace
}  // namespace sat

using namespace sat;

extern "C" int64_t sat_decode_persistent_scratch_bytes(void) {
  return (kZeroDwords + kCacheFloats) * 4;
}

extern "C" int sat_decode_persistent(const SatDecodePersistent* a, void* stream) {
  SAT_CHECK_ARG(a && a->B >= 1 && a->B <= kG && a->N >= 1 && a->N <= kNM && a->T >= 1 &&
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
