// Dual-source attention step of the decoder (the north-star kernel), forward.
//
// Per decoder step t and utterance b (modules/forward_attention.py:88-122 + TF BahdanauAttention,
// AttentionWrapper._compute_attention):
//   source 1, ForwardAttention(224):  f = Conv1D_SAME(s_{t-1}) (5 filters, k=10) ; l = f @ W_loc
//       e[n] = sum_d v[d] tanh(K1[n,d] + q[d] + l[n,d] + b[d]),  s = softmax_masked(e)
//       a~[n] = ((1-u) a_{t-1}[n] + u a_{t-1}[n-1] + 1e-7) s[n],  a = a~ / sum(a~),  c1 = a @ V1
//   source 2, BahdanauAttention(32): e2[n] = sum_d v2[d] tanh(K2[n,d] + q2[d]), s2 = softmax, c2 = s2 @ V2
//
// Split over (utterance, tile of NT memory positions) workgroups so the step streams K1/V1/K2/V2
// from all CUs (~14 MB per step at B=32, N=200).  Softmax normalisers factor out of the contexts,
// so each tile emits flash-style partials (tile max m, sum exp, sum a~-weight, unnormalised
// partial contexts) and a per-utterance combine kernel finishes s, a, c1, c2:
//   a[n] = g[n] e^{e[n]-M} / sum_j A_j e^{m_j-M},  c1 = sum_j C_j e^{m_j-M} / sum_j A_j e^{m_j-M}.
// Energy reduction over d: lanes own d (coalesced 896-B rows of K1), wave_sum per position.
#include "sat_common.h"

namespace sat {
namespace {

constexpr int kMaxD = 256, kMaxF = 16, kMaxKW = 32, kMaxNT = 64;

struct AttnFwdP {
  int B, N, D1, M1, D2, M2, F, KW, NT, ntiles, att1_forward;
  const float* q; int64_t q_sb;          // [B][D1 + D2]
  const float* K1; const float* V1;      // [B][N][D1], [B][N][M1]
  const float* K2; const float* V2;      // [B][N][D2], [B][N][M2]
  const int64_t* lengths;
  const float* s_prev; const float* a_prev;   // [B][N]
  const float* v1; const float* b1;      // [D1]
  const float* convW; const float* convb;     // [KW][F] (Conv1D kernel [KW,1,F]), [F]
  const float* locW;                     // [F][D1]
  const float* v2;                       // [D2]
  float u;
  float* e1; float* e2;                  // [B][N]
  float* part; int64_t part_stride;      // [B][ntiles][part_stride]
};

// partial record: [0]=m1 [1]=Z1 [2]=A1 [3]=m2 [4]=Z2 [5..7]=pad [8..8+M1) C1 [8+M1..) C2
constexpr int kPartHdr = 8;

__global__ void __launch_bounds__(256) attn_energy_kernel(AttnFwdP p) {
  __shared__ float qb[kMaxD], vv[kMaxD], q2s[kMaxD], v2s[kMaxD];
  __shared__ float locw[kMaxF * kMaxD];
  __shared__ float fs[kMaxNT][kMaxF];
  __shared__ float sp[kMaxNT + kMaxKW];
  __shared__ float e1s[kMaxNT], e2s[kMaxNT], w1s[kMaxNT], w2s[kMaxNT];
  __shared__ float red[8];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = blockIdx.y, tile = blockIdx.x;
  const int n0 = tile * p.NT;
  const int nt = min(p.NT, p.N - n0);
  const int len = (int)p.lengths[b];
  const float* q = p.q + (int64_t)b * p.q_sb;

  for (int d = tid; d < p.D1; d += 256) {
    qb[d] = q[d] + (p.b1 ? p.b1[d] : 0.f);
    vv[d] = p.v1[d];
  }
  for (int d = tid; d < p.D2; d += 256) {
    q2s[d] = q[p.D1 + d];
    v2s[d] = p.v2[d];
  }
  const int padl = (p.KW - 1) / 2;
  if (p.att1_forward) {
    for (int i = tid; i < p.F * p.D1; i += 256) locw[i] = p.locW[i];
    // s_{t-1} over [n0 - padl, n0 + nt + (KW-1-padl)) (zero outside [0, N))
    const int span = nt + p.KW - 1;
    for (int i = tid; i < span; i += 256) {
      const int n = n0 - padl + i;
      sp[i] = (n >= 0 && n < p.N) ? p.s_prev[(int64_t)b * p.N + n] : 0.f;
    }
  }
  __syncthreads();
  if (p.att1_forward) {
    for (int i = tid; i < nt * p.F; i += 256) {
      const int nl = i / p.F, f = i - nl * p.F;
      float acc = p.convb[f];
      for (int j = 0; j < p.KW; ++j) acc = fmaf(sp[nl + j], p.convW[j * p.F + f], acc);
      fs[nl][f] = acc;
    }
    __syncthreads();
  }

  // energies: one wave per position, lanes over d
  for (int nl = wave; nl < nt; nl += 4) {
    const int n = n0 + nl;
    const float* k1 = p.K1 + ((int64_t)b * p.N + n) * p.D1;
    float acc = 0.f;
    for (int d = lane; d < p.D1; d += 64) {
      float pre = k1[d] + qb[d];
      if (p.att1_forward) {
        for (int f = 0; f < p.F; ++f) pre = fmaf(fs[nl][f], locw[f * p.D1 + d], pre);
      }
      acc = fmaf(vv[d], tanhf(pre), acc);
    }
    const float* k2 = p.K2 + ((int64_t)b * p.N + n) * p.D2;
    float acc2 = 0.f;
    for (int d = lane; d < p.D2; d += 64) acc2 = fmaf(v2s[d], tanhf(k2[d] + q2s[d]), acc2);
    acc = wave_sum(acc);
    acc2 = wave_sum(acc2);
    if (lane == 0) {
      const bool valid = n < len;
      e1s[nl] = valid ? acc : -INFINITY;
      e2s[nl] = valid ? acc2 : -INFINITY;
    }
  }
  __syncthreads();

  // tile statistics (wave 0)
  if (wave == 0) {
    float m1 = -INFINITY, m2 = -INFINITY;
    for (int i = lane; i < nt; i += 64) { m1 = fmaxf(m1, e1s[i]); m2 = fmaxf(m2, e2s[i]); }
    m1 = wave_max(m1);
    m2 = wave_max(m2);
    float z1 = 0.f, a1 = 0.f, z2 = 0.f;
    for (int i = lane; i < nt; i += 64) {
      const int n = n0 + i;
      const float pe = (e1s[i] == -INFINITY) ? 0.f : expf(e1s[i] - m1);
      float w = pe;
      if (p.att1_forward) {
        const float ap = p.a_prev[(int64_t)b * p.N + n];
        const float am = n > 0 ? p.a_prev[(int64_t)b * p.N + n - 1] : 0.f;
        w = ((1.f - p.u) * ap + p.u * am + 1e-7f) * pe;
      }
      const float pe2 = (e2s[i] == -INFINITY) ? 0.f : expf(e2s[i] - m2);
      w1s[i] = w;
      w2s[i] = pe2;
      z1 += pe; a1 += w; z2 += pe2;
    }
    z1 = wave_sum(z1); a1 = wave_sum(a1); z2 = wave_sum(z2);
    if (lane == 0) { red[0] = m1; red[1] = z1; red[2] = a1; red[3] = m2; red[4] = z2; }
  }
  __syncthreads();

  float* part = p.part + ((int64_t)b * p.ntiles + tile) * p.part_stride;
  if (tid < kPartHdr) part[tid] = tid < 5 ? red[tid] : 0.f;
  for (int i = tid; i < nt; i += 256) {
    p.e1[(int64_t)b * p.N + n0 + i] = e1s[i];
    p.e2[(int64_t)b * p.N + n0 + i] = e2s[i];
  }
  // unnormalised partial contexts; threads over the value width (coalesced rows)
  for (int d = tid; d < p.M1 + p.M2; d += 256) {
    float acc = 0.f;
    if (d < p.M1) {
      const float* v1 = p.V1 + ((int64_t)b * p.N + n0) * p.M1 + d;
      for (int i = 0; i < nt; ++i) acc = fmaf(w1s[i], v1[(int64_t)i * p.M1], acc);
    } else {
      const int d2 = d - p.M1;
      const float* v2 = p.V2 + ((int64_t)b * p.N + n0) * p.M2 + d2;
      for (int i = 0; i < nt; ++i) acc = fmaf(w2s[i], v2[(int64_t)i * p.M2], acc);
    }
    part[kPartHdr + d] = acc;
  }
}

struct AttnCombineP {
  int B, N, M1, M2, ntiles, att1_forward;
  float u;
  const float* e1; const float* e2; const float* part; int64_t part_stride;
  const float* a_prev;
  float* s_out; float* a_out; float* s2_out;   // [B][N]
  float* ctx; int64_t ctx_sb;                  // [B][M1 + M2] (row stride ctx_sb)
  float* stats;                                // [B][4]: M1, Z1, A1/Z1 (= sum g s), Z2 ... for bwd
};

__global__ void __launch_bounds__(256) attn_combine_kernel(AttnCombineP p) {
  __shared__ float sc1[256], sc2[256];
  __shared__ float hdr[6];
  const int tid = threadIdx.x;
  const int b = blockIdx.x;
  const float* part = p.part + (int64_t)b * p.ntiles * p.part_stride;
  if (tid == 0) {
    float M1 = -INFINITY, M2 = -INFINITY;
    for (int j = 0; j < p.ntiles; ++j) {
      M1 = fmaxf(M1, part[j * p.part_stride + 0]);
      M2 = fmaxf(M2, part[j * p.part_stride + 3]);
    }
    float Z1 = 0.f, A1 = 0.f, Z2 = 0.f;
    for (int j = 0; j < p.ntiles; ++j) {
      const float* r = part + j * p.part_stride;
      const float s1 = (r[0] == -INFINITY) ? 0.f : expf(r[0] - M1);
      const float s2 = (r[3] == -INFINITY) ? 0.f : expf(r[3] - M2);
      sc1[j] = s1;
      sc2[j] = s2;
      Z1 += r[1] * s1; A1 += r[2] * s1; Z2 += r[4] * s2;
    }
    hdr[0] = M1; hdr[1] = Z1; hdr[2] = A1; hdr[3] = Z2; hdr[4] = M2;
    if (p.stats) {  // sum_n g[n] s[n] = A1 / Z1 (the forward-attention normaliser) for the bwd
      p.stats[b * 4 + 0] = M1; p.stats[b * 4 + 1] = Z1; p.stats[b * 4 + 2] = A1 / Z1;
      p.stats[b * 4 + 3] = Z2;
    }
  }
  __syncthreads();
  const float M1 = hdr[0], Z1 = hdr[1], A1 = hdr[2], Z2 = hdr[3], M2 = hdr[4];
  const float inv1 = 1.f / (p.att1_forward ? A1 : Z1);
  const float invz1 = 1.f / Z1, invz2 = 1.f / Z2;
  float* ctx = p.ctx + (int64_t)b * p.ctx_sb;
  for (int d = tid; d < p.M1 + p.M2; d += 256) {
    float acc = 0.f;
    const bool first = d < p.M1;
    for (int j = 0; j < p.ntiles; ++j)
      acc = fmaf(part[j * p.part_stride + kPartHdr + d], first ? sc1[j] : sc2[j], acc);
    ctx[d] = acc * (first ? inv1 : invz2);
  }
  for (int n = tid; n < p.N; n += 256) {
    const int64_t i = (int64_t)b * p.N + n;
    const float e = p.e1[i], e2 = p.e2[i];
    const float pe = (e == -INFINITY) ? 0.f : expf(e - M1);
    const float pe2 = (e2 == -INFINITY) ? 0.f : expf(e2 - M2);
    const float s = pe * invz1;
    p.s_out[i] = s;
    p.s2_out[i] = pe2 * invz2;
    if (p.att1_forward) {
      const float ap = p.a_prev[i];
      const float am = n > 0 ? p.a_prev[i - 1] : 0.f;
      p.a_out[i] = ((1.f - p.u) * ap + p.u * am + 1e-7f) * pe * inv1;
    } else {
      p.a_out[i] = s;
    }
  }
}

// q[b, :] = x[b, :] @ [W1 | W2]   (query layers of both mechanisms, no bias)
__global__ void __launch_bounds__(256) query_kernel(int B, int K, int N1, int N2, const float* x,
                                                   int64_t x_sb, const float* W1, const float* W2,
                                                   float* q, int64_t q_sb) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + lane;
  const int b0 = blockIdx.y * 8 + wave * 2;
  extern __shared__ float xs[];   // [8][K]
  for (int i = threadIdx.x; i < 8 * K; i += 256) {
    const int r = i / K, k = i - r * K;
    const int bb = blockIdx.y * 8 + r;
    xs[i] = bb < B ? x[(int64_t)bb * x_sb + k] : 0.f;
  }
  __syncthreads();
  if (col >= N1 + N2) return;
  const float* W = col < N1 ? W1 + col : W2 + (col - N1);
  const int ld = col < N1 ? N1 : N2;
  const int r0 = wave * 2;
  float a0 = 0.f, a1 = 0.f;
#pragma unroll 8
  for (int k = 0; k < K; ++k) {
    const float w = W[(int64_t)k * ld];
    a0 = fmaf(xs[r0 * K + k], w, a0);
    a1 = fmaf(xs[(r0 + 1) * K + k], w, a1);
  }
  if (b0 < B) q[(int64_t)b0 * q_sb + col] = a0;
  if (b0 + 1 < B) q[(int64_t)(b0 + 1) * q_sb + col] = a1;
}

}  // namespace
}  // namespace sat

using namespace sat;

extern "C" int sat_attn_part_stride(int32_t M1, int32_t M2) {
  return (kPartHdr + M1 + M2 + 3) / 4 * 4;
}

extern "C" int sat_attn_query(int32_t B, int32_t K, int32_t N1, int32_t N2, const float* x,
                              int64_t x_sb, const float* W1, const float* W2, float* q,
                              int64_t q_sb, void* stream) {
  SAT_CHECK_ARG(B > 0 && K > 0 && N1 >= 0 && N2 >= 0, "sat_attn_query: bad sizes");
  SAT_CHECK_ARG(x && W1 && (N2 == 0 || W2) && q, "sat_attn_query: null pointer");
  SAT_CHECK_ARG(8 * K * 4 <= 65536, "sat_attn_query: K too large");
  dim3 grid(ceil_div(N1 + N2, 64), ceil_div(B, 8));
  hipLaunchKernelGGL(query_kernel, grid, dim3(256), 8 * K * sizeof(float), as_stream(stream), B,
                     K, N1, N2, x, x_sb, W1, W2, q, q_sb);
  SAT_LAUNCH_CHECK("sat_attn_query");
  return SAT_OK;
}

extern "C" int sat_attn_step_fwd(const SatAttnStep* a, void* stream) {
  SAT_CHECK_ARG(a && a->B > 0 && a->N > 0, "sat_attn_step_fwd: bad sizes");
  SAT_CHECK_ARG(a->D1 <= kMaxD && a->D2 <= kMaxD && a->M2 >= 0, "sat_attn_step_fwd: D > 256");
  SAT_CHECK_ARG(a->NT > 0 && a->NT <= kMaxNT, "sat_attn_step_fwd: tile size must be in [1, 64]");
  SAT_CHECK_ARG(!a->att1_forward || (a->F <= kMaxF && a->KW <= kMaxKW && a->F * a->D1 <= kMaxF * kMaxD),
                "sat_attn_step_fwd: location conv too large");
  SAT_CHECK_ARG(a->part_stride >= sat_attn_part_stride(a->M1, a->M2), "sat_attn_step_fwd: part stride");
  SAT_CHECK_ARG(a->ntiles <= 256 && a->ntiles == ceil_div(a->N, a->NT), "sat_attn_step_fwd: ntiles");
  SAT_CHECK_ARG(a->q && a->K1 && a->V1 && a->K2 && a->V2 && a->lengths && a->v1 && a->v2 &&
                a->e1 && a->e2 && a->part && a->s_out && a->a_out && a->s2_out && a->ctx,
                "sat_attn_step_fwd: null pointer");
  SAT_CHECK_ARG(!a->att1_forward || (a->s_prev && a->a_prev && a->convW && a->convb && a->locW),
                "sat_attn_step_fwd: forward attention needs state and location weights");
  AttnFwdP p;
  p.B = a->B; p.N = a->N; p.D1 = a->D1; p.M1 = a->M1; p.D2 = a->D2; p.M2 = a->M2;
  p.F = a->F; p.KW = a->KW; p.NT = a->NT; p.ntiles = a->ntiles; p.att1_forward = a->att1_forward;
  p.q = a->q; p.q_sb = a->q_sb; p.K1 = a->K1; p.V1 = a->V1; p.K2 = a->K2; p.V2 = a->V2;
  p.lengths = a->lengths; p.s_prev = a->s_prev; p.a_prev = a->a_prev;
  p.v1 = a->v1; p.b1 = a->b1; p.convW = a->convW; p.convb = a->convb; p.locW = a->locW;
  p.v2 = a->v2; p.u = a->u; p.e1 = a->e1; p.e2 = a->e2; p.part = a->part;
  p.part_stride = a->part_stride;
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL(attn_energy_kernel, dim3(a->ntiles, a->B), dim3(256), 0, s, p);
  SAT_LAUNCH_CHECK("sat_attn_step_fwd(energy)");
  AttnCombineP c;
  c.B = a->B; c.N = a->N; c.M1 = a->M1; c.M2 = a->M2; c.ntiles = a->ntiles;
  c.att1_forward = a->att1_forward; c.u = a->u;
  c.e1 = a->e1; c.e2 = a->e2; c.part = a->part; c.part_stride = a->part_stride;
  c.a_prev = a->a_prev; c.s_out = a->s_out; c.a_out = a->a_out; c.s2_out = a->s2_out;
  c.ctx = a->ctx; c.ctx_sb = a->ctx_sb; c.stats = a->stats;
  hipLaunchKernelGGL(attn_combine_kernel, dim3(a->B), dim3(256), 0, s, c);
  SAT_LAUNCH_CHECK("sat_attn_step_fwd(combine)");
  return SAT_OK;
}
