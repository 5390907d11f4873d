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
// group barrier plus on-chip arithmetic.
//
// Layout (same as the attention chain): 8 groups x 32 workgroups (256, one per CU).  Group
// g = blockIdx % 8 owns utterances b = g + 8*ub (ub < B/8 <= 4); workgroup j = blockIdx / 8 owns
// units [8j, 8j+8) of BOTH layers.  The LSTMs couple units, never utterances, so a group's
// hand-offs never leave the group.
//   forward, iteration i (0..T'):   LSTM1 step i  and  LSTM2 step i-1  (one barrier)
//     LSTM1 step i   needs h1_{i-1} (all units)                       -> H1S[i]
//     LSTM2 step i-1 needs h1'_{i-1} (raw output, its input) and h2_{i-2} -> H1RAW[i-1], H2S[i-1]
//   backward, iteration j (0..T'):  LSTM2 step T'-1-j  and  LSTM1 step T'-j  (one barrier)
//     LSTM2 step t   needs dgates2_{t+1} (its recurrent product)
//     LSTM1 step t+1 needs dgates2_{t+1} (its output gradient through LSTM2's input rows)
//                    and  dgates1_{t+2} (its recurrent product)
// Hand-offs: the histories themselves (sc1 stores / sc1 loads, persistent.h); every spin is
// bounded and a timeout raises err[0] so the grid always drains.
#include "sat_common.h"
#include "persistent.h"

namespace sat {
namespace {

constexpr int kG = 8;              // groups
constexpr int kGW = 32;            // workgroups per group
constexpr int kU = 256;            // units per layer
constexpr int kUW = kU / kGW;      // units per workgroup per layer (8)
constexpr int kUBmax = 4;          // utterances per group
constexpr int kC = 4 * kUW;        // gate columns per workgroup per layer (32)
constexpr int kX = 3 * kU;         // forward staging row: [h1_{i-1} | h1'_{i-1} | h2_{i-2}]
constexpr int kI1 = kU / 32;       // LSTM1 recurrent float4 per thread (8)
constexpr int kI2 = 2 * kU / 32;   // LSTM2 [input | recurrent] float4 per thread (16)
constexpr int kIB = 4 * kU / 128;  // backward float4 per thread per weight row (8)

struct DecLstmFwdP {
  int B, T, UB;
  float zc, zh;
  const float* X1;                                    // [T][B][4U]
  const float* W1r;                                   // [U][U][4]
  const float* W2;                                    // [2U][U][4]
  const float* b2;                                    // [4U]
  const float* m1c; const float* m1h; const float* m2c; const float* m2h;   // [T][B][U] | null
  float* H1RAW; float* C1S; float* H1S; float* G1;
  float* H2RAW; float* C2S; float* H2S; float* G2;
  unsigned* ctr; int* err;
  long long* prof;                                    // [256][4] segment clocks (nullable)
};

__device__ __forceinline__ float dot4(float4 a, float4 b, float acc) {
  acc = fmaf(a.x, b.x, acc);
  acc = fmaf(a.y, b.y, acc);
  acc = fmaf(a.z, b.z, acc);
  return fmaf(a.w, b.w, acc);
}

// Forward.  Dot role: thread = (gate column c = unit_local*4 + gate, k-slice ks of 8); its
// weights are the float4 runs k = 32i + 4ks .. +3 of column c (LSTM1: 8 runs of the recurrent
// kernel, LSTM2: 16 runs of [input | recurrent]), loaded once into registers.  Pointwise role:
// threads 0..63 = (layer, ub, unit); each keeps its unit's (c, h) state in registers.
__global__ void __launch_bounds__(256) dec_lstm_fwd_kernel(DecLstmFwdP p) {
  __shared__ __attribute__((aligned(16))) float xs[kUBmax][kX];
  __shared__ float gs[2][kUBmax][kC];
  const int tid = threadIdx.x;
  const int g = blockIdx.x % kG, j = blockIdx.x / kG;
  const int u0 = j * kUW;
  const int B = p.B, T = p.T, UB = p.UB;
  unsigned* ctr = p.ctr + 64 * g;

  const int c = tid >> 3, ks = tid & 7;
  const int ucol = u0 + (c >> 2), gcol = c & 3;
  float4 w1[kI1], w2[kI2];
#pragma unroll
  for (int i = 0; i < kI1; ++i) {
    const int k = 32 * i + 4 * ks;
    const float* src = p.W1r + ((int64_t)k * kU + ucol) * 4 + gcol;
    w1[i] = make_float4(src[0], src[4 * kU], src[8 * kU], src[12 * kU]);
  }
#pragma unroll
  for (int i = 0; i < kI2; ++i) {
    const int k = 32 * i + 4 * ks;
    const float* src = p.W2 + ((int64_t)k * kU + ucol) * 4 + gcol;
    w2[i] = make_float4(src[0], src[4 * kU], src[8 * kU], src[12 * kU]);
  }

  // pointwise role
  const bool pw = tid < 64;
  const int layer = (tid >> 5) & 1, pub = (tid >> 3) & 3, pul = tid & 7;
  const bool pw_on = pw && pub < UB;
  const int pb = g + kG * pub, pu = u0 + pul;
  float cst = 0.f, hst = 0.f;
  float4 bias2 = make_float4(0.f, 0.f, 0.f, 0.f);
  if (pw_on) {
    const int64_t i0 = (int64_t)pb * kU + pu;
    cst = layer == 0 ? p.C1S[i0] : p.C2S[i0];
    hst = layer == 0 ? p.H1S[i0] : p.H2S[i0];
    if (layer == 1) bias2 = reinterpret_cast<const float4*>(p.b2)[pu];
  }
  const bool masked = p.m1c != nullptr;
  const auto rH1S = rsrc(p.H1S), rH1R = rsrc(p.H1RAW), rH2S = rsrc(p.H2S);

  // optional segment clocks (thread 0): barrier wait, staging loads, dots, pointwise
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
    const bool pw_step = pw_on && (layer == 0 ? do1 : do2);
    // pointwise operands of this step (forward inputs: plain loads, issued first)
    float4 xp = bias2;
    float mc = 1.f - p.zc, mh = 1.f - p.zh;
    if (pw_step) {
      const int64_t bu = ((int64_t)t * B + pb) * kU + pu;
      if (layer == 0) xp = reinterpret_cast<const float4*>(p.X1)[bu];
      if (masked) {
        mc = layer == 0 ? p.m1c[bu] : p.m2c[bu];
        mh = layer == 0 ? p.m1h[bu] : p.m2h[bu];
      }
    }
    // stage the group's recurrent/input rows (other workgroups' outputs: sc1 loads)
    for (int idx = tid; idx < UB * (kX / 4); idx += 256) {
      const int ub = idx / (kX / 4), q = idx - ub * (kX / 4);
      const int b = g + kG * ub;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (q < kU / 4) {
        if (do1) v = ldc4(rH1S, ((i * B + b) * kU) / 4 + q);
      } else if (do2) {
        if (q < kU / 2) v = ldc4(rH1R, (((i - 1) * B + b) * kU) / 4 + q - kU / 4);
        else v = ldc4(rH2S, (((i - 1) * B + b) * kU) / 4 + q - kU / 2);
      }
      *reinterpret_cast<float4*>(&xs[ub][4 * q]) = v;
    }
    __syncthreads();
    tick(1);
    float a1[kUBmax], a2[kUBmax];
#pragma unroll
    for (int ub = 0; ub < kUBmax; ++ub) {
      a1[ub] = 0.f;
      a2[ub] = 0.f;
      if (ub < UB) {
        const float4* x4 = reinterpret_cast<const float4*>(xs[ub]);
        if (do1) {
#pragma unroll
          for (int q = 0; q < kI1; ++q) a1[ub] = dot4(x4[8 * q + ks], w1[q], a1[ub]);
        }
        if (do2) {
#pragma unroll
          for (int q = 0; q < kI2; ++q) a2[ub] = dot4(x4[kU / 4 + 8 * q + ks], w2[q], a2[ub]);
        }
      }
    }
#pragma unroll
    for (int o = 1; o < 8; o <<= 1)
#pragma unroll
      for (int ub = 0; ub < kUBmax; ++ub) {
        a1[ub] += __shfl_xor(a1[ub], o, 64);
        a2[ub] += __shfl_xor(a2[ub], o, 64);
      }
    if (ks == 0) {
#pragma unroll
      for (int ub = 0; ub < kUBmax; ++ub) {
        gs[0][ub][c] = a1[ub];
        gs[1][ub][c] = a2[ub];
      }
    }
    __syncthreads();
    tick(2);
    if (pw_step) {
      const float* gg = gs[layer][pub] + 4 * pul;
      const float gi = sigmf(gg[0] + xp.x);
      const float gj = tanhf(gg[1] + xp.y);
      const float gf = sigmf(gg[2] + xp.z + 1.0f);   // forget_bias = 1.0
      const float go = sigmf(gg[3] + xp.w);
      const float cn = gf * cst + gi * gj;
      const float hn = go * tanhf(cn);
      const float c2 = mc * cn + (1.f - mc) * cst;
      const float h2 = mh * hn + (1.f - mh) * hst;
      cst = c2;
      hst = h2;
      const int64_t bu = ((int64_t)t * B + pb) * kU + pu;
      const int64_t bn = bu + (int64_t)B * kU;       // [t + 1]
      if (layer == 0) {
        stc(rH1R, (int)bu, hn);
        stc(rH1S, (int)bn, h2);
        p.C1S[bn] = c2;
        reinterpret_cast<float4*>(p.G1)[bu] = make_float4(gi, gj, gf, go);
      } else {
        p.H2RAW[bu] = hn;
        stc(rH2S, (int)bn, h2);
        p.C2S[bn] = c2;
        reinterpret_cast<float4*>(p.G2)[bu] = make_float4(gi, gj, gf, go);
      }
    }
    tick(3);
    if (i < T) group_barrier(ctr, (unsigned)(i + 1) * kGW, p.err);
    tick(0);
  }
  if (p.prof && tid == 0)
    for (int i = 0; i < 4; ++i) p.prof[blockIdx.x * 4 + i] = tp[i];
}

struct DecLstmBwdP {
  int B, T, UB;
  float zc, zh;
  const float* W1r;                                   // [U][U][4]
  const float* W2;                                    // [2U][U][4]
  const float* G1; const float* C1S; const float* G2; const float* C2S;
  const float* DH2;                                   // [T][B][U]
  const float* m1c; const float* m1h; const float* m2c; const float* m2h;
  float* DG1; float* DG2;                             // [T][B][4U]
  unsigned* ctr; int* err;
  long long* prof;                                    // [256][4] segment clocks (nullable)
};

// TF LSTMCell + zoneout backward of one (utterance, unit) (lstm.hip lstm_bwd_block's pointwise):
// returns dgates and updates the (dh, dc) carries.
__device__ __forceinline__ float4 lstm_cell_bwd(float4 g4, float cp, float dy, float rec,
                                                float mc, float mh, float& dhc, float& dcc) {
  const float gi = g4.x, gj = g4.y, gf = g4.z, go = g4.w;
  const float cn = gf * cp + gi * gj;
  const float tc = tanhf(cn);
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

// Backward.  Dot role: thread = (own unit ul = tid/32, k-slice ks = tid%32); its weights are the
// float4 runs 4ks + 128i of three 4U-long rows of unit u: LSTM2's recurrent row W2[U+u],
// LSTM2's input row W2[u] (LSTM1's output gradient) and LSTM1's recurrent row W1r[u].
// Pointwise role: lanes ks < 8 of each unit's 32 lanes = (layer, ub); carries in registers.
__global__ void __launch_bounds__(256) dec_lstm_bwd_kernel(DecLstmBwdP p) {
  __shared__ __attribute__((aligned(16))) float dg2s[kUBmax][4 * kU];
  __shared__ __attribute__((aligned(16))) float dg1s[kUBmax][4 * kU];
  const int tid = threadIdx.x;
  const int g = blockIdx.x % kG, j = blockIdx.x / kG;
  const int u0 = j * kUW;
  const int B = p.B, T = p.T, UB = p.UB;
  unsigned* ctr = p.ctr + 64 * g;

  const int ul = tid >> 5, ks = tid & 31;
  const int u = u0 + ul;
  float4 wa[kIB], wb[kIB], wc[kIB];
  {
    const float4* ra = reinterpret_cast<const float4*>(p.W2 + (int64_t)(kU + u) * 4 * kU);
    const float4* rb = reinterpret_cast<const float4*>(p.W2 + (int64_t)u * 4 * kU);
    const float4* rc = reinterpret_cast<const float4*>(p.W1r + (int64_t)u * 4 * kU);
#pragma unroll
    for (int i = 0; i < kIB; ++i) {
      wa[i] = ra[ks + 32 * i];
      wb[i] = rb[ks + 32 * i];
      wc[i] = rc[ks + 32 * i];
    }
  }
  // pointwise role: lanes 0..3 -> LSTM2 of utterance ub = ks, lanes 4..7 -> LSTM1 of ub = ks-4
  const bool pw = ks < 8;
  const int layer = ks < 4 ? 2 : 1, pub = ks & 3;
  const bool pw_on = pw && pub < UB;
  const int pb = g + kG * pub;
  float dhc = 0.f, dcc = 0.f;
  const bool masked = p.m1c != nullptr;
  const auto rDG1 = rsrc(p.DG1), rDG2 = rsrc(p.DG2);

  // optional segment clocks (thread 0): barrier wait, staging loads, dots, pointwise
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
    const bool pw_step = pw_on && (layer == 2 ? has2 : has1);
    // pointwise operands (forward histories and the head's gradient: plain loads, issued first)
    float4 g4 = make_float4(0.f, 0.f, 0.f, 0.f);
    float cp = 0.f, dyv = 0.f, mc = 1.f - p.zc, mh = 1.f - p.zh;
    if (pw_step) {
      const int64_t bu = ((int64_t)t * B + pb) * kU + u;
      if (layer == 2) {
        g4 = reinterpret_cast<const float4*>(p.G2)[bu];
        cp = p.C2S[bu];
        dyv = p.DH2[bu];
      } else {
        g4 = reinterpret_cast<const float4*>(p.G1)[bu];
        cp = p.C1S[bu];
      }
      if (masked) {
        mc = layer == 2 ? p.m2c[bu] : p.m1c[bu];
        mh = layer == 2 ? p.m2h[bu] : p.m1h[bu];
      }
    }
    // stage dgates2_{t2+1} and dgates1_{t1+1} of the group's utterances (sc1 loads)
    for (int idx = tid; idx < UB * 2 * kU; idx += 256) {
      const int ub = idx / (2 * kU), q = idx - ub * (2 * kU);
      const int b = g + kG * ub;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (q < kU) {
        if (stage2) v = ldc4(rDG2, (((t2 + 1) * B + b) * 4 * kU) / 4 + q);
        *reinterpret_cast<float4*>(&dg2s[ub][4 * q]) = v;
      } else {
        if (stage1) v = ldc4(rDG1, (((t1 + 1) * B + b) * 4 * kU) / 4 + q - kU);
        *reinterpret_cast<float4*>(&dg1s[ub][4 * (q - kU)]) = v;
      }
    }
    __syncthreads();
    tick(1);
    float r2[kUBmax], y1[kUBmax], r1[kUBmax];
#pragma unroll
    for (int ub = 0; ub < kUBmax; ++ub) {
      r2[ub] = 0.f;
      y1[ub] = 0.f;
      r1[ub] = 0.f;
      if (ub < UB) {
        const float4* d2 = reinterpret_cast<const float4*>(dg2s[ub]);
        const float4* d1 = reinterpret_cast<const float4*>(dg1s[ub]);
        if (stage2) {
#pragma unroll
          for (int q = 0; q < kIB; ++q) {
            const float4 x = d2[ks + 32 * q];
            r2[ub] = dot4(x, wa[q], r2[ub]);
            y1[ub] = dot4(x, wb[q], y1[ub]);
          }
        }
        if (stage1) {
#pragma unroll
          for (int q = 0; q < kIB; ++q) r1[ub] = dot4(d1[ks + 32 * q], wc[q], r1[ub]);
        }
      }
    }
#pragma unroll
    for (int o = 1; o < 32; o <<= 1)
#pragma unroll
      for (int ub = 0; ub < kUBmax; ++ub) {
        r2[ub] += __shfl_xor(r2[ub], o, 64);
        y1[ub] += __shfl_xor(y1[ub], o, 64);
        r1[ub] += __shfl_xor(r1[ub], o, 64);
      }
    tick(2);
    if (pw_step) {
      float rec = 0.f, dy = dyv;
#pragma unroll
      for (int ub = 0; ub < kUBmax; ++ub)
        if (ub == pub) {
          if (layer == 2) rec = r2[ub];
          else { rec = r1[ub]; dy = y1[ub]; }
        }
      const float4 dg = lstm_cell_bwd(g4, cp, dy, rec, mc, mh, dhc, dcc);
      const int64_t bu = ((int64_t)t * B + pb) * kU + u;
      stc4(layer == 2 ? rDG2 : rDG1, (int)bu, dg);
    }
    tick(3);
    if (jj < T) group_barrier(ctr, (unsigned)(jj + 1) * kGW, p.err);
    else __syncthreads();
    tick(0);
  }
  if (p.prof && tid == 0)
    for (int i = 0; i < 4; ++i) p.prof[blockIdx.x * 4 + i] = tp[i];
}

int check_coresident(const void* kernel, const char* name) {
  int dev = 0, cus = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, 256, 0) != hipSuccess) {
    set_error("%s: device query failed", name);
    return SAT_ERR_HIP;
  }
  SAT_CHECK_ARG((int64_t)cus * per_cu >= kG * kGW,
                "%s: fewer than 256 co-resident workgroups on this device", name);
  return SAT_OK;
}

int reset_sync(uint32_t* ctr, int32_t* err, hipStream_t s, const char* name) {
  if (hipMemsetAsync(ctr, 0, kG * 64 * sizeof(unsigned), s) != hipSuccess ||
      hipMemsetAsync(err, 0, 2 * sizeof(int), s) != hipSuccess) {
    set_error("%s: memset failed", name);
    return SAT_ERR_HIP;
  }
  return SAT_OK;
}

}  // namespace
}  // namespace sat

using namespace sat;

extern "C" int sat_decoder_lstms_fwd(const SatDecLstmFwd* a, void* stream) {
  const char* nm = "sat_decoder_lstms_fwd";
  SAT_CHECK_ARG(a && a->B > 0 && a->T > 0, "%s: bad sizes", nm);
  SAT_CHECK_ARG(a->U == kU, "%s: compiled for U=256 (the self-attention-tacotron configs)", nm);
  SAT_CHECK_ARG(a->B % kG == 0 && a->B / kG <= kUBmax, "%s: B in {8,16,24,32}", nm);
  SAT_CHECK_ARG(a->X1 && a->W1r && a->W2 && a->b2 && a->H1RAW && a->C1S && a->H1S && a->G1 &&
                a->H2RAW && a->C2S && a->H2S && a->G2 && a->ctr && a->err, "%s: null pointer", nm);
  SAT_CHECK_ARG((a->mask1_c == nullptr) == (a->mask1_h == nullptr) &&
                (a->mask1_c == nullptr) == (a->mask2_c == nullptr) &&
                (a->mask2_c == nullptr) == (a->mask2_h == nullptr),
                "%s: the four zoneout masks are all given or all NULL", nm);
  SAT_CHECK_ARG(aligned16(a->X1) && aligned16(a->b2) && aligned16(a->G1) && aligned16(a->G2) &&
                aligned16(a->H1S) && aligned16(a->H1RAW) && aligned16(a->H2S),
                "%s: 16-byte aligned operands", nm);
  SAT_CHECK_ARG((int64_t)(a->T + 1) * a->B * 4 * kU < (1ll << 29), "%s: histories too long", nm);
  int rc = check_coresident(reinterpret_cast<const void*>(dec_lstm_fwd_kernel), nm);
  if (rc != SAT_OK) return rc;
  DecLstmFwdP p;
  p.B = a->B; p.T = a->T; p.UB = a->B / kG; p.zc = a->zc; p.zh = a->zh;
  p.X1 = a->X1; p.W1r = a->W1r; p.W2 = a->W2; p.b2 = a->b2;
  p.m1c = a->mask1_c; p.m1h = a->mask1_h; p.m2c = a->mask2_c; p.m2h = a->mask2_h;
  p.H1RAW = a->H1RAW; p.C1S = a->C1S; p.H1S = a->H1S; p.G1 = a->G1;
  p.H2RAW = a->H2RAW; p.C2S = a->C2S; p.H2S = a->H2S; p.G2 = a->G2;
  p.ctr = a->ctr; p.err = a->err;
  p.prof = reinterpret_cast<long long*>(a->prof);
  hipStream_t s = as_stream(stream);
  rc = reset_sync(a->ctr, a->err, s, nm);
  if (rc != SAT_OK) return rc;
  hipLaunchKernelGGL(dec_lstm_fwd_kernel, dim3(kG * kGW), dim3(256), 0, s, p);
  SAT_LAUNCH_CHECK(nm);
  return SAT_OK;
}

extern "C" int sat_decoder_lstms_bwd(const SatDecLstmBwd* a, void* stream) {
  const char* nm = "sat_decoder_lstms_bwd";
  SAT_CHECK_ARG(a && a->B > 0 && a->T > 0, "%s: bad sizes", nm);
  SAT_CHECK_ARG(a->U == kU, "%s: compiled for U=256 (the self-attention-tacotron configs)", nm);
  SAT_CHECK_ARG(a->B % kG == 0 && a->B / kG <= kUBmax, "%s: B in {8,16,24,32}", nm);
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
  p.B = a->B; p.T = a->T; p.UB = a->B / kG; p.zc = a->zc; p.zh = a->zh;
  p.W1r = a->W1r; p.W2 = a->W2; p.G1 = a->G1; p.C1S = a->C1S; p.G2 = a->G2; p.C2S = a->C2S;
  p.DH2 = a->DH2;
  p.m1c = a->mask1_c; p.m1h = a->mask1_h; p.m2c = a->mask2_c; p.m2h = a->mask2_h;
  p.DG1 = a->DG1; p.DG2 = a->DG2; p.ctr = a->ctr; p.err = a->err;
  p.prof = reinterpret_cast<long long*>(a->prof);
  hipStream_t s = as_stream(stream);
  rc = reset_sync(a->ctr, a->err, s, nm);
  if (rc != SAT_OK) return rc;
  hipLaunchKernelGGL(dec_lstm_bwd_kernel, dim3(kG * kGW), dim3(256), 0, s, p);
  SAT_LAUNCH_CHECK(nm);
  return SAT_OK;
}
