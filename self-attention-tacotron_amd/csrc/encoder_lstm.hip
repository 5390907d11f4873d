// Persistent encoder BiLSTM: ALL N steps of both directions of ZoneoutCBHG's bidirectional
// ZoneoutLSTM (modules/module.py:93-110: bidirectional_dynamic_rnn(ZoneoutLSTMCell fw, bw,
// sequence_length=input_lengths); zoneout cell of ext tacotron2) in ONE launch forward and
// ONE launch backward.  The arithmetic is lstm.hip's per-step kernels' restated (TF LSTMCell
// gate order i j f o, forget_bias 1.0, zoneout masks as inputs or the eval blend, steps at or
// beyond the utterance length copy the state and emit 0); only the schedule differs.
//
// Why: the per-step path is N = 200 launches each way (fw step n and bw step N-1-n share one
// multi-problem launch), each paying a kernel boundary and a cold reload of the recurrent
// weights.  The recurrent matrix of one direction is U x 4U = 128 x 512 floats = exactly 64
// floats per thread of a 1024-thread workgroup, so ONE workgroup per (direction, utterance)
// keeps it in registers for the whole sequence and a step needs no inter-workgroup hand-off at
// all: two LDS barriers per step forward, one backward.  2B workgroups, no co-residency
// requirement.
#include "sat_common.h"
#include "persistent.h"

namespace sat {
namespace {

constexpr int kU = 128;            // units per direction
constexpr int kG4 = 4 * kU;        // gate columns (512)
constexpr int kTh = 1024;
// BPTT workgroup: SAT_ENC_BWD8 (default) 8 waves, each 16 units x 8 gate columns per lane (128
// weights); otherwise 16 waves of 8 units x 8 columns.  The step is issue-bound: the 16-wave
// form spent ~3/4 of its instructions on per-wave overhead (the cell on 8 of 64 lanes, the
// 64-lane reduce, addresses) that every wave repeats.
#ifndef SAT_ENC_BWD8
#define SAT_ENC_BWD8 1
#endif
// SAT_ENC_BWD_DMA: the cell operands (G, c_{t-1}, dL/dh, zoneout masks: 4 KB per step) stream
// into LDS by asm LDS-DMA a chunk of 8 steps ahead (wave w loads step w of the next chunk,
// double-buffered), waited for once per chunk; the per-step register prefetch exposed its
// load latency (no operand loads at all: 229 -> 148 us, profiles/r06z_enc_bwd_dma_ab.txt)
#ifndef SAT_ENC_BWD_DMA
#define SAT_ENC_BWD_DMA 1
#endif
constexpr int kRowsB = SAT_ENC_BWD8 ? 16 : 8;      // units per wave
constexpr int kThB = 64 * (kU / kRowsB);
typedef float f2 __attribute__((ext_vector_type(2)));

struct EncFwdP {
  int B, N;
  float zc, zh;
  const float* X[2]; int64_t x_sb, x_sn;
  const float* W[2];
  const float* mc[2]; const float* mh[2];
  const int64_t* lengths;
  float* H; int64_t h_sb, h_sn;
  float* CS[2]; float* HS[2]; float* G[2];
};

struct EncBwdP {
  int B, N;
  float zc, zh;
  const float* W[2]; const float* G[2]; const float* CS[2];
  const float* mc[2]; const float* mh[2];
  const int64_t* lengths;
  const float* DY; int64_t dy_sb, dy_sn;
  float* DG[2];
};

// Forward.  Dot role (SAT_ENC_FWD_T, default): thread t owns gate columns 4cb .. 4cb+3
// (cb = t >> 3) over recurrent rows 16rg .. 16rg+15 (rg = t & 7): 64 weights in registers, 16
// state values read from LDS per step (4 ds_read_b128; the former layout -- one column, 64
// rows per thread -- read 64, and 1024 threads x 256 B of LDS reads per step bound the step at
// the LDS data path); the 8 row groups' partial sums of the 4 columns meet by a DPP
// transpose-reduce, after which lanes 2m of each 8-lane group hold column 4cb + m.
// Cell role: threads u < 128 own unit u's (c, h) state in registers.
// SAT_ENC_DRAIN_CELL: wait for the step's operand prefetch right before the cell (whose stores
// then stay in flight into the next step) instead of at the loop's back edge, where the
// compiler's vmcnt(0) also waits for the cell's stores
#ifndef SAT_ENC_DRAIN_CELL
#define SAT_ENC_DRAIN_CELL 1
#endif
#ifndef SAT_ENC_FWD_T
#define SAT_ENC_FWD_T 1
#endif
__global__ void __launch_bounds__(kTh) enc_lstm_fwd_kernel(EncFwdP p) {
  __shared__ __attribute__((aligned(16))) float hs[kU];
  __shared__ __attribute__((aligned(16))) float gp[kG4];
  const int tid = threadIdx.x;
  const int d = blockIdx.x & 1, b = blockIdx.x >> 1;
  const int N = p.N, B = p.B;
#if SAT_ENC_FWD_T
  const int lane = tid & 63;
  const int cb = tid >> 3, rg = tid & 7;
  const int c = 4 * cb + 2 * ((lane >> 2) & 1) + ((lane >> 1) & 1);   // column after the reduce
  const bool hf = (lane & 1) != 0;                                    // false: the writer lane
  f2 w[16][2];
  {
    const float* W = p.W[d];
#pragma unroll
    for (int r = 0; r < 16; ++r)
#pragma unroll
      for (int cp = 0; cp < 2; ++cp) {
        const float* src = W + (int64_t)(16 * rg + r) * kG4 + 4 * cb + 2 * cp;
        w[r][cp] = f2{src[0], src[1]};
      }
  }
#else
  const int c = tid >> 1, hf = tid & 1;
  f2 w[32];
  {
    const float* W = p.W[d];
#pragma unroll
    for (int i = 0; i < 32; ++i)
      w[i] = f2{W[(int64_t)(64 * hf + 2 * i) * kG4 + c], W[(int64_t)(64 * hf + 2 * i + 1) * kG4 + c]};
  }
#endif
  const int len = (int)p.lengths[b];
  const bool cell = tid < kU;
  const int u = tid;
  const int r0 = d ? N : 0;                 // initial state row
  float cst = 0.f, hst = 0.f;
  if (cell) {
    cst = p.CS[d][((int64_t)r0 * B + b) * kU + u];
    hst = p.HS[d][((int64_t)r0 * B + b) * kU + u];
    hs[u] = hst;
  }
  const bool masked = p.mc[0] != nullptr;
  // operands of processing step i (plain loads), prefetched one step ahead
  auto load_x = [&](int i) {
    const int n = d ? N - 1 - i : i;
    return (hf == 0 && i < N) ? p.X[d][(int64_t)b * p.x_sb + (int64_t)n * p.x_sn + c] : 0.f;
  };
  auto load_m = [&](int i, float& mc_, float& mh_) {
    mc_ = 1.f - p.zc;
    mh_ = 1.f - p.zh;
    if (cell && masked && i < N) {
      const int n = d ? N - 1 - i : i;
      const int64_t r = ((int64_t)n * B + b) * kU + u;
      mc_ = p.mc[d][r];
      mh_ = p.mh[d][r];
    }
  };
  float xn = load_x(0), mcn, mhn;
  load_m(0, mcn, mhn);
  // the register-resident weights (and the first operands) land before the step loop, in the
  // compiler-visible form: left pending at the loop header, the waits for them are placed at
  // their first use INSIDE the loop, where every later iteration's counts then also wait for
  // that step's just-issued operand prefetch (and the previous step's history stores)
  vm_drain();
  __syncthreads();
  for (int i = 0; i < N; ++i) {
    const int n = d ? N - 1 - i : i;
    const int nx = d ? n : n + 1;           // state row written
    const float xv = xn, mc = mcn, mh = mhn;
    xn = load_x(i + 1);
    load_m(i + 1, mcn, mhn);
#if SAT_ENC_FWD_T
    {
      const float4* h4 = reinterpret_cast<const float4*>(&hs[16 * rg]);
      f2 a0 = {0.f, 0.f}, a1 = {0.f, 0.f}, b0 = {0.f, 0.f}, b1 = {0.f, 0.f};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 h = h4[q];
        a0 = __builtin_elementwise_fma(f2{h.x, h.x}, w[4 * q][0], a0);
        a1 = __builtin_elementwise_fma(f2{h.x, h.x}, w[4 * q][1], a1);
        b0 = __builtin_elementwise_fma(f2{h.y, h.y}, w[4 * q + 1][0], b0);
        b1 = __builtin_elementwise_fma(f2{h.y, h.y}, w[4 * q + 1][1], b1);
        a0 = __builtin_elementwise_fma(f2{h.z, h.z}, w[4 * q + 2][0], a0);
        a1 = __builtin_elementwise_fma(f2{h.z, h.z}, w[4 * q + 2][1], a1);
        b0 = __builtin_elementwise_fma(f2{h.w, h.w}, w[4 * q + 3][0], b0);
        b1 = __builtin_elementwise_fma(f2{h.w, h.w}, w[4 * q + 3][1], b1);
      }
      const f2 s0 = a0 + b0, s1 = a1 + b1;
      float v[4] = {s0.x, s0.y, s1.x, s1.y};
      tr_dpp<4, 2>(v, lane);               // lane bit 2: columns {0, 1} | {2, 3}
      tr_dpp<2, 1>(v, lane);               // lane bit 1: the column within the pair
      v[0] += dpp_mov<0xB1>(v[0]);         // lane bit 0: the last pair of row groups
      if (!hf) gp[c] = v[0] + xv;
    }
#else
    // ---- gate pre-activations: column c, rows 64 hf .. 64 hf + 63
    {
      const float4* h4 = reinterpret_cast<const float4*>(&hs[64 * hf]);
      f2 a0 = {0.f, 0.f}, a1 = {0.f, 0.f};
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const float4 h = h4[q];
        a0 = __builtin_elementwise_fma(f2{h.x, h.y}, w[2 * q], a0);
        a1 = __builtin_elementwise_fma(f2{h.z, h.w}, w[2 * q + 1], a1);
      }
      float acc = (a0.x + a0.y) + (a1.x + a1.y);
      acc += dpp<0xB1>(acc);                // the pair (lanes t, t ^ 1) of column c
      if (hf == 0) gp[c] = acc + xv;
    }
#endif
    // LDS-only barriers: a __syncthreads would also drain the prefetch and the history stores
    lds_barrier();
#if SAT_ENC_DRAIN_CELL
    vm_drain();   // this step's operand prefetch landed; the cell's stores then stay in flight
#endif
    // ---- cell
    if (cell) {
      const float4 g = *reinterpret_cast<const float4*>(&gp[4 * u]);
      const int64_t bu = (int64_t)b * kU + u;
      float* Hd = p.H + (int64_t)b * p.h_sb + (int64_t)n * p.h_sn + d * kU + u;
      if (n < len) {
        // one v_exp + one v_rcp per activation (decoder_lstm_persistent.hip: same forms)
        const float gi = sigmoid_fast(g.x);
        const float gj = tanh_lstm(g.y);
        const float gf = sigmoid_fast(g.z + 1.0f);   // forget_bias = 1.0
        const float go = sigmoid_fast(g.w);
        const float cn = gf * cst + gi * gj;
        const float hn = go * tanh_lstm(cn);
        cst = mc * cn + (1.f - mc) * cst;
        hst = mh * hn + (1.f - mh) * hst;
        *Hd = hn;
        reinterpret_cast<float4*>(p.G[d])[(int64_t)n * B * kU + bu] = make_float4(gi, gj, gf, go);
      } else {   // bidirectional_dynamic_rnn(sequence_length): state copied, output 0
        *Hd = 0.f;
        reinterpret_cast<float4*>(p.G[d])[(int64_t)n * B * kU + bu] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
      p.CS[d][(int64_t)nx * B * kU + bu] = cst;
      p.HS[d][(int64_t)nx * B * kU + bu] = hst;
      hs[u] = hst;
    }
    lds_barrier();
  }
}

// Backward.  Recurrent product, wave-transposed: wave w owns rows R w .. R w + R-1 (units; R =
// kRowsB, 16 in the 8-wave form), lane l gate columns 8l .. 8l+7 of them (8R weights in
// registers), so a step reads 8 floats of the previous step's gate gradients per lane; the R
// partial row sums are transpose-reduced across the wave and lane (64/R) m runs unit R w + m's
// reverse step with its carries in registers.  The gate gradients of the previously processed
// step sit in LDS (double buffer: one barrier per step).
__global__ void __launch_bounds__(kThB) enc_lstm_bwd_kernel(EncBwdP p) {
  __shared__ __attribute__((aligned(16))) float dgn[2][kG4];
#if SAT_ENC_BWD_DMA
  static_assert(kThB == 512, "one wave per step of an 8-step chunk");
  // [buffer][step of the chunk][G 4U | c_{t-1} U | dL/dh U | mask c U | mask h U]
  __shared__ __attribute__((aligned(16))) float opsb[2][8][8 * kU];
#endif
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int d = blockIdx.x & 1, b = blockIdx.x >> 1;
  const int N = p.N, B = p.B;
  f2 w[kRowsB][4];                         // row kRowsB w + r, column pairs 8l + 2cp, +1
  {
#pragma unroll
    for (int r = 0; r < kRowsB; ++r) {
      const float4* src = reinterpret_cast<const float4*>(p.W[d] + (int64_t)(kRowsB * wave + r) * kG4 + 8 * lane);
      const float4 a0 = src[0], a1 = src[1];
      w[r][0] = f2{a0.x, a0.y}; w[r][1] = f2{a0.z, a0.w};
      w[r][2] = f2{a1.x, a1.y}; w[r][3] = f2{a1.z, a1.w};
    }
  }
  for (int i = tid; i < kG4; i += kThB) dgn[0][i] = 0.f;
  const int len = (int)p.lengths[b];
  // after the transpose-reduce, lanes (64 / kRowsB) m .. hold unit kRowsB w + m
  constexpr int kLPU = 64 / kRowsB;
  const bool lead = (lane & (kLPU - 1)) == 0;
  const int u = kRowsB * wave + lane / kLPU;
  const bool masked = p.mc[0] != nullptr;
  struct Ops { float4 g; float cp, dy, mc, mh; };
  auto load_ops = [&](int i) {
    Ops o{make_float4(0.f, 0.f, 0.f, 0.f), 0.f, 0.f, 1.f - p.zc, 1.f - p.zh};
#if SAT_ENC_PROBE_NOLOAD
    if (i >= 0) return o;   // timing probe only: no operand loads (wrong results)
#endif
    if (lead && i < N) {
      const int n = d ? i : N - 1 - i;
      const int cprow = d ? n + 1 : n;      // c_{t-1} in processing order of the direction
      const int64_t bu = (int64_t)b * kU + u;
      o.g = reinterpret_cast<const float4*>(p.G[d])[(int64_t)n * B * kU + bu];
      o.cp = p.CS[d][(int64_t)cprow * B * kU + bu];
      o.dy = p.DY[(int64_t)b * p.dy_sb + (int64_t)n * p.dy_sn + d * kU + u];
      if (masked) {
        const int64_t r = ((int64_t)n * B + b) * kU + u;
        o.mc = p.mc[d][r];
        o.mh = p.mh[d][r];
      }
    }
    return o;
  };
#if SAT_ENC_BWD_DMA
  (void)load_ops;   // the register path of SAT_ENC_BWD_DMA=0
  // step ii's operands (clamped to a valid step past N: loaded, never used) into opsb[buf][w]
  auto dma_step = [&](int ii, int buf) {
    const int ic = min(ii, N - 1);
    const int n = d ? ic : N - 1 - ic;
    const int cprow = d ? n + 1 : n;
    const uint32_t base = lds_addr_of(&opsb[buf][wave][0]);
    const float* g = p.G[d] + ((int64_t)n * B + b) * kU * 4;
    lds_dma16(g + 4 * lane, base);
    lds_dma16(g + 4 * kU / 2 + 4 * lane, base + 1024);
    if (lane < kU / 4) {
      lds_dma16(p.CS[d] + ((int64_t)cprow * B + b) * kU + 4 * lane, base + 2048);
      lds_dma16(p.DY + (int64_t)b * p.dy_sb + (int64_t)n * p.dy_sn + d * kU + 4 * lane, base + 2560);
      if (masked) {
        const int64_t r = ((int64_t)n * B + b) * kU + 4 * lane;
        lds_dma16(p.mc[d] + r, base + 3072);
        lds_dma16(p.mh[d] + r, base + 3584);
      }
    }
  };
  dma_step(wave, 0);                       // chunk 0
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#elif SAT_ENC_BWD_PF2
  // operands prefetched two steps ahead (one step ahead, their load latency showed in the step)
  Ops nxt = load_ops(0), nxt2 = load_ops(1);
#else
  Ops nxt = load_ops(0);
#endif
  float dh_c = 0.f, dc_c = 0.f;
  vm_drain();                              // (see the forward: weights landed before the loop)
  __syncthreads();
  for (int i = 0; i < N; ++i) {
    const int n = d ? i : N - 1 - i;
#if SAT_ENC_BWD_DMA
    if ((i & 7) == 0) dma_step(i + 8 + wave, ((i >> 3) + 1) & 1);   // the next chunk
    Ops o{make_float4(0.f, 0.f, 0.f, 0.f), 0.f, 0.f, 1.f - p.zc, 1.f - p.zh};
    if (lead) {
      const float* ob = &opsb[(i >> 3) & 1][i & 7][0];
      o.g = *reinterpret_cast<const float4*>(&ob[4 * u]);
      o.cp = ob[4 * kU + u];
      o.dy = ob[5 * kU + u];
      if (masked) {
        o.mc = ob[6 * kU + u];
        o.mh = ob[7 * kU + u];
      }
    }
#else
    const Ops o = nxt;
#if SAT_ENC_BWD_PF2
    nxt = nxt2;
    nxt2 = load_ops(i + 2);
#else
    nxt = load_ops(i + 1);
#endif
#endif
    // ---- recurrent product of the previously processed step's gate gradients
    float v[kRowsB];
    {
      const float4* g4 = reinterpret_cast<const float4*>(&dgn[i & 1][8 * lane]);
      const float4 ga = g4[0], gb = g4[1];
      const f2 g[4] = {f2{ga.x, ga.y}, f2{ga.z, ga.w}, f2{gb.x, gb.y}, f2{gb.z, gb.w}};
#pragma unroll
      for (int r = 0; r < kRowsB; ++r) {
        f2 a = g[0] * w[r][0];
        a = __builtin_elementwise_fma(g[1], w[r][1], a);
        a = __builtin_elementwise_fma(g[2], w[r][2], a);
        a = __builtin_elementwise_fma(g[3], w[r][3], a);
        v[r] = a.x + a.y;
      }
    }
#if SAT_ENC_BWD8
    transpose_reduce16(v, lane);
#else
    transpose_reduce8(v, lane);
#endif
#if SAT_ENC_DRAIN_CELL && !SAT_ENC_BWD_DMA
    vm_drain();   // (see the forward)
#endif
    if (lead) {
      const float dh_t = v[0] + dh_c;
      const float dc_t = dc_c;
      const int64_t bu = (int64_t)b * kU + u;
      float4 dg = make_float4(0.f, 0.f, 0.f, 0.f);
      if (n < len) {
        const float gi = o.g.x, gj = o.g.y, gf = o.g.z, go = o.g.w;
        const float cn = gf * o.cp + gi * gj;
        const float tc = tanh_lstm(cn);   // formed exactly as the forward formed it
        const float dhn = o.dy + o.mh * dh_t;               // dL/dh'
        const float dcn = o.mc * dc_t + dhn * go * (1.f - tc * tc);
        dg = make_float4(dcn * gj * gi * (1.f - gi), dcn * gi * (1.f - gj * gj),
                         dcn * o.cp * gf * (1.f - gf), dhn * tc * go * (1.f - go));
        dc_c = dcn * gf + (1.f - o.mc) * dc_t;
        dh_c = (1.f - o.mh) * dh_t;
      } else {   // beyond the length: the carries pass through unchanged
        dh_c = dh_t;
        dc_c = dc_t;
      }
      reinterpret_cast<float4*>(p.DG[d])[(int64_t)n * B * kU + bu] = dg;
      *reinterpret_cast<float4*>(&dgn[(i + 1) & 1][4 * u]) = dg;
    }
#if SAT_ENC_BWD_DMA
    // the chunk's last step: this wave's DMA of the next chunk has landed before the barrier
    if ((i & 7) == 7) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    lds_barrier();   // LDS only: a __syncthreads would drain the DG store and the prefetch
  }
}

}  // namespace
}  // namespace sat

using namespace sat;

extern "C" int sat_encoder_lstm_fwd(const SatEncLstmFwd* a, void* stream) {
  SAT_CHECK_ARG(a && a->B > 0 && a->N > 0, "sat_encoder_lstm_fwd: bad sizes");
  SAT_CHECK_ARG(a->U == kU, "sat_encoder_lstm_fwd: compiled for U = 128 (cbhg_out_units 256)");
  SAT_CHECK_ARG(a->X_fw && a->X_bw && a->W_fw && a->W_bw && a->lengths && a->H && a->CS_fw &&
                a->HS_fw && a->CS_bw && a->HS_bw && a->G_fw && a->G_bw,
                "sat_encoder_lstm_fwd: null pointer");
  const bool m0 = a->mc_fw != nullptr;
  SAT_CHECK_ARG((a->mh_fw != nullptr) == m0 && (a->mc_bw != nullptr) == m0 && (a->mh_bw != nullptr) == m0,
                "sat_encoder_lstm_fwd: zoneout masks come all four or none");
  SAT_CHECK_ARG(aligned16(a->G_fw) && aligned16(a->G_bw) && aligned16(a->W_fw) && aligned16(a->W_bw) &&
                aligned16(a->X_fw) && aligned16(a->X_bw) && a->x_sb % 4 == 0 && a->x_sn % 4 == 0,
                "sat_encoder_lstm_fwd: 16-byte aligned operands");
  EncFwdP p;
  p.B = a->B; p.N = a->N; p.zc = a->zc; p.zh = a->zh;
  p.X[0] = a->X_fw; p.X[1] = a->X_bw; p.x_sb = a->x_sb; p.x_sn = a->x_sn;
  p.W[0] = a->W_fw; p.W[1] = a->W_bw;
  p.mc[0] = a->mc_fw; p.mh[0] = a->mh_fw; p.mc[1] = a->mc_bw; p.mh[1] = a->mh_bw;
  p.lengths = a->lengths;
  p.H = a->H; p.h_sb = a->h_sb; p.h_sn = a->h_sn;
  p.CS[0] = a->CS_fw; p.HS[0] = a->HS_fw; p.CS[1] = a->CS_bw; p.HS[1] = a->HS_bw;
  p.G[0] = a->G_fw; p.G[1] = a->G_bw;
  hipLaunchKernelGGL(enc_lstm_fwd_kernel, dim3(2 * a->B), dim3(kTh), 0, as_stream(stream), p);
  SAT_LAUNCH_CHECK("sat_encoder_lstm_fwd");
  return SAT_OK;
}

extern "C" int sat_encoder_lstm_bwd(const SatEncLstmBwd* a, void* stream) {
  SAT_CHECK_ARG(a && a->B > 0 && a->N > 0, "sat_encoder_lstm_bwd: bad sizes");
  SAT_CHECK_ARG(a->U == kU, "sat_encoder_lstm_bwd: compiled for U = 128 (cbhg_out_units 256)");
  SAT_CHECK_ARG(a->W_fw && a->W_bw && a->G_fw && a->G_bw && a->CS_fw && a->CS_bw && a->lengths &&
                a->DY && a->DG_fw && a->DG_bw, "sat_encoder_lstm_bwd: null pointer");
  const bool m0 = a->mc_fw != nullptr;
  SAT_CHECK_ARG((a->mh_fw != nullptr) == m0 && (a->mc_bw != nullptr) == m0 && (a->mh_bw != nullptr) == m0,
                "sat_encoder_lstm_bwd: zoneout masks come all four or none");
  SAT_CHECK_ARG(aligned16(a->W_fw) && aligned16(a->W_bw) && aligned16(a->G_fw) && aligned16(a->G_bw) &&
                aligned16(a->DG_fw) && aligned16(a->DG_bw),
                "sat_encoder_lstm_bwd: 16-byte aligned operands");
  EncBwdP p;
  p.B = a->B; p.N = a->N; p.zc = a->zc; p.zh = a->zh;
  p.W[0] = a->W_fw; p.W[1] = a->W_bw; p.G[0] = a->G_fw; p.G[1] = a->G_bw;
  p.CS[0] = a->CS_fw; p.CS[1] = a->CS_bw;
  p.mc[0] = a->mc_fw; p.mh[0] = a->mh_fw; p.mc[1] = a->mc_bw; p.mh[1] = a->mh_bw;
  p.lengths = a->lengths;
  p.DY = a->DY; p.dy_sb = a->dy_sb; p.dy_sn = a->dy_sn;
  p.DG[0] = a->DG_fw; p.DG[1] = a->DG_bw;
  hipLaunchKernelGGL(enc_lstm_bwd_kernel, dim3(2 * a->B), dim3(kThB), 0, as_stream(stream), p);
  SAT_LAUNCH_CHECK("sat_encoder_lstm_bwd");
  return SAT_OK;
}
