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
  const int phases = a->phases == 0 ? 3 : a->phases;
  if (phases & 1) {
    hipLaunchKernelGGL(attn_energy_kernel, dim3(a->ntiles, a->B), dim3(256), 0, s, p);
    SAT_LAUNCH_CHECK("sat_attn_step_fwd(energy)");
  }
  if (!(phases & 2)) return SAT_OK;
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

// ============================================================================ backward
// Reverse step t of the dual-source attention (see the forward formulas at the top).
// K_b1 (per utterance x tile):  dA[n] = dA_next[n] + dc1 . V1[n],  dS2[n] = dc2 . V2[n]
// K_b2 (per utterance x tile):  the normaliser sums over all n (cheap: [N] vectors), then for the
//   tile: de, de2, dA_prev (recursion), the energies' tanh recomputed from K1 (no [T',B,N,224]
//   tensor is ever stored), dK1/dK2 accumulated in place (each element owned by one thread),
//   per-tile dq partials, location-conv grads df (conv-transposed by the NEXT reverse step into
//   dS_prev), and the small parameter grads accumulated per (utterance, tile) without atomics.
// Utterance b's tiles are mapped to blocks b, b+B, b+2B, ... so (B % 8 == 0) all of b's tiles
// run on one XCD every step and K1[b], V1[b], dK1[b] stay in that XCD's L2.
namespace sat {
namespace {

constexpr int kMaxN = 1024, kMaxFb = 8;

struct AttnBwdP {
  int B, N, D1, M1, D2, M2, F, KW, NT, ntiles, att1_forward;
  float u;
  const float* dctx; int64_t dctx_sb;
  const float* dalpha_next;
  const float* V1; const float* V2;
  float* DA; float* DS2;
  const float* s_t; const float* a_t; const float* a_prev; const float* s_prev; const float* s2_t;
  const float* stats;
  const float* df_next;
  const int64_t* lengths;
  const float* q; int64_t q_sb;
  const float* K1; const float* K2;
  const float* v1; const float* b1; const float* convW; const float* convb; const float* locW;
  const float* v2;
  float* dalpha_prev;
  float* df_out;
  float* dK1; float* dK2;
  float* dqp;
  float* pg; int64_t pg_stride;
};

__global__ void __launch_bounds__(256) attn_bwd_ctx_kernel(AttnBwdP p) {
  __shared__ float dc[2 * kMaxD + kMaxD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = blockIdx.x % p.B, tile = blockIdx.x / p.B;
  const int n0 = tile * p.NT, nt = min(p.NT, p.N - n0);
  const float* g = p.dctx + (int64_t)b * p.dctx_sb;
  for (int i = tid; i < p.M1 + p.M2; i += 256) dc[i] = g[i];
  __syncthreads();
  for (int nl = wave; nl < nt; nl += 4) {
    const int n = n0 + nl;
    const float* v1 = p.V1 + ((int64_t)b * p.N + n) * p.M1;
    const float* v2 = p.V2 + ((int64_t)b * p.N + n) * p.M2;
    float a = 0.f, c = 0.f;
    for (int d = lane; d < p.M1; d += 64) a = fmaf(dc[d], v1[d], a);
    for (int d = lane; d < p.M2; d += 64) c = fmaf(dc[p.M1 + d], v2[d], c);
    a = wave_sum(a);
    c = wave_sum(c);
    if (lane == 0) {
      const int64_t i = (int64_t)b * p.N + n;
      p.DA[i] = a + (p.dalpha_next ? p.dalpha_next[i] : 0.f);
      p.DS2[i] = c;
    }
  }
}

__global__ void __launch_bounds__(256) attn_bwd_energy_kernel(AttnBwdP p) {
  __shared__ float dst[kMaxN], dat[kMaxN];
  __shared__ float qb[kMaxD], vv[kMaxD], q2s[kMaxD], v2s[kMaxD];
  __shared__ float locw[kMaxFb * kMaxD];
  __shared__ float fs[kMaxNT][kMaxFb], dfs[kMaxNT][kMaxFb];
  __shared__ float sp[kMaxNT + kMaxKW];
  __shared__ float de1[kMaxNT], de2[kMaxNT];
  __shared__ float red[16];
  __shared__ float racc[4][kMaxD * (2 + kMaxFb) + 128];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = blockIdx.x % p.B, tile = blockIdx.x / p.B;
  const int n0 = tile * p.NT, nt = min(p.NT, p.N - n0);
  const int64_t rb = (int64_t)b * p.N;
  const int padl = (p.KW - 1) / 2;
  const bool fwd = p.att1_forward != 0;
  const float u = p.u;

  // ---- normaliser sums over the whole utterance
  float s1 = 0.f, s3 = 0.f;
  for (int n = tid; n < p.N; n += 256) {
    if (fwd) s1 += p.DA[rb + n] * p.a_t[rb + n];
    s3 += p.s2_t[rb + n] * p.DS2[rb + n];
  }
  s1 = block_sum(s1, red);
  s3 = block_sum(s3, red + 4);
  const float Sa = fwd ? p.stats[b * 4 + 2] : 1.f;
  float s2sum = 0.f;
  for (int n = tid; n < p.N; n += 256) {
    float ds;
    if (fwd) {
      const float da = (p.DA[rb + n] - s1) / Sa;
      const float g = (1.f - u) * p.a_prev[rb + n] + (n > 0 ? u * p.a_prev[rb + n - 1] : 0.f) + 1e-7f;
      float dsn = 0.f;
      if (p.df_next) {  // conv-transpose of the next step's location-feature grads
        for (int j = 0; j < p.KW; ++j) {
          const int m = n - j + padl;
          if (m < 0 || m >= p.N) continue;
          const float* dfr = p.df_next + (rb + m) * p.F;
          for (int f = 0; f < p.F; ++f) dsn = fmaf(dfr[f], p.convW[j * p.F + f], dsn);
        }
      }
      dat[n] = da;
      ds = dsn + da * g;
    } else {
      ds = p.DA[rb + n];
    }
    dst[n] = ds;
    s2sum += p.s_t[rb + n] * ds;
  }
  s2sum = block_sum(s2sum, red + 8);   // (block_sum syncs: dst/dat visible after)

  // ---- tile: de, de2, dA_prev
  for (int i = tid; i < nt; i += 256) {
    const int n = n0 + i;
    de1[i] = p.s_t[rb + n] * (dst[n] - s2sum);
    de2[i] = p.s2_t[rb + n] * (p.DS2[rb + n] - s3);
    if (fwd) {
      float v = (1.f - u) * dat[n] * p.s_t[rb + n];
      if (n + 1 < p.N) v += u * dat[n + 1] * p.s_t[rb + n + 1];
      p.dalpha_prev[rb + n] = v;
    }
  }
  const float* q = p.q + (int64_t)b * p.q_sb;
  for (int d = tid; d < p.D1; d += 256) {
    qb[d] = q[d] + (p.b1 ? p.b1[d] : 0.f);
    vv[d] = p.v1[d];
  }
  for (int d = tid; d < p.D2; d += 256) {
    q2s[d] = q[p.D1 + d];
    v2s[d] = p.v2[d];
  }
  if (fwd) {
    for (int i = tid; i < p.F * p.D1; i += 256) locw[i] = p.locW[i];
    const int span = nt + p.KW - 1;
    for (int i = tid; i < span; i += 256) {
      const int n = n0 - padl + i;
      sp[i] = (n >= 0 && n < p.N) ? p.s_prev[rb + n] : 0.f;
    }
  }
  __syncthreads();
  if (fwd) {
    for (int i = tid; i < nt * p.F; i += 256) {
      const int nl = i / p.F, f = i - nl * p.F;
      float acc = p.convb[f];
      for (int j = 0; j < p.KW; ++j) acc = fmaf(sp[nl + j], p.convW[j * p.F + f], acc);
      fs[nl][f] = acc;
    }
  }
  __syncthreads();

  // ---- recompute energies of the tile and back-propagate through tanh
  float aq[4] = {0, 0, 0, 0}, av[4] = {0, 0, 0, 0};
  float aw[4][kMaxFb];
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int f = 0; f < kMaxFb; ++f) aw[k][f] = 0.f;
  float aq2 = 0.f, av2 = 0.f;   // lane owns d2 = lane (D2 <= 64, checked on the host)
  for (int nl = wave; nl < nt; nl += 4) {
    const int n = n0 + nl;
    const float e = de1[nl];
    const float* k1 = p.K1 + (rb + n) * p.D1;
    float* dk1 = p.dK1 + (rb + n) * p.D1;
    float dfp[kMaxFb];
#pragma unroll
    for (int f = 0; f < kMaxFb; ++f) dfp[f] = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int d = lane + 64 * k;
      if (d < p.D1) {
        float pre = k1[d] + qb[d];
        if (fwd) {
#pragma unroll
          for (int f = 0; f < kMaxFb; ++f)
            if (f < p.F) pre = fmaf(fs[nl][f], locw[f * p.D1 + d], pre);
        }
        const float z = tanhf(pre);
        const float dp = e * vv[d] * (1.f - z * z);
        dk1[d] += dp;
        aq[k] += dp;
        av[k] = fmaf(e, z, av[k]);
        if (fwd) {
#pragma unroll
          for (int f = 0; f < kMaxFb; ++f)
            if (f < p.F) {
              aw[k][f] = fmaf(fs[nl][f], dp, aw[k][f]);
              dfp[f] = fmaf(dp, locw[f * p.D1 + d], dfp[f]);
            }
        }
      }
    }
    if (fwd) {
#pragma unroll
      for (int f = 0; f < kMaxFb; ++f) {
        if (f < p.F) {
          const float s = wave_sum(dfp[f]);
          if (lane == 0) dfs[nl][f] = s;
        }
      }
    }
    const float e2v = de2[nl];
    const float* k2 = p.K2 + (rb + n) * p.D2;
    float* dk2 = p.dK2 + (rb + n) * p.D2;
    if (lane < p.D2) {
      const int d = lane;
      const float z = tanhf(k2[d] + q2s[d]);
      const float dp = e2v * v2s[d] * (1.f - z * z);
      dk2[d] += dp;
      aq2 += dp;
      av2 = fmaf(e2v, z, av2);
    }
  }
  // ---- reduce the per-lane accumulators of the 4 waves
  // layout per wave: [dq D1][dv1 D1][dWloc F*D1][dq2 64][dv2 64]
  float* r = racc[wave];
  const int W = p.D1, F = fwd ? p.F : 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int d = lane + 64 * k;
    if (d < W) {
      r[d] = aq[k];
      r[W + d] = av[k];
#pragma unroll
      for (int f = 0; f < kMaxFb; ++f)
        if (f < F) r[2 * W + f * W + d] = aw[k][f];
    }
  }
  const int off2 = (2 + F) * W;
  if (lane < 64) {
    r[off2 + lane] = aq2;
    r[off2 + 64 + lane] = av2;
  }
  __syncthreads();
  float* dqp = p.dqp + ((int64_t)b * p.ntiles + tile) * (p.D1 + p.D2);
  float* pg = p.pg + ((int64_t)b * p.ntiles + tile) * p.pg_stride;
  // pg layout: [dv1 D1][dWloc F*D1][dconvW KW*F][dconvb F][dv2 D2]
  const int total = off2;
  for (int i = tid; i < total; i += 256) {
    const float v = racc[0][i] + racc[1][i] + racc[2][i] + racc[3][i];
    if (i < W) dqp[i] = v;
    else pg[i - W] += v;        // dv1 then dWloc
  }
  for (int i = tid; i < p.D2; i += 256) {
    float vq = 0.f, vv2 = 0.f;
    for (int w = 0; w < 4; ++w) { vq += racc[w][off2 + i]; vv2 += racc[w][off2 + 64 + i]; }
    dqp[p.D1 + i] = vq;
    pg[(1 + p.F) * W + p.KW * p.F + p.F + i] += vv2;
  }
  if (fwd) {
    // location conv grads: dconvW[j,f] = sum_n s_prev[n+j-padl] df[n,f], dconvb[f] = sum_n df
    for (int i = tid; i < p.KW * p.F + p.F; i += 256) {
      float acc = 0.f;
      if (i < p.KW * p.F) {
        const int j = i / p.F, f = i - j * p.F;
        for (int nl = 0; nl < nt; ++nl) acc = fmaf(sp[nl + j], dfs[nl][f], acc);
      } else {
        const int f = i - p.KW * p.F;
        for (int nl = 0; nl < nt; ++nl) acc += dfs[nl][f];
      }
      pg[(1 + p.F) * W + i] += acc;
    }
    for (int i = tid; i < nt * p.F; i += 256) {
      const int nl = i / p.F, f = i - nl * p.F;
      p.df_out[(rb + n0 + nl) * p.F + f] = dfs[nl][f];
    }
  }
}

}  // namespace
}  // namespace sat

using namespace sat;

extern "C" int sat_attn_pg_stride(int32_t D1, int32_t D2, int32_t F, int32_t KW) {
  return (D1 + F * D1 + KW * F + F + D2 + 3) / 4 * 4;
}

extern "C" int sat_attn_step_bwd(const SatAttnStepBwd* a, void* stream) {
  SAT_CHECK_ARG(a && a->B > 0 && a->N > 0 && a->N <= kMaxN, "sat_attn_step_bwd: bad sizes (N <= 1024)");
  SAT_CHECK_ARG(a->D1 <= kMaxD && a->D2 <= 64 && a->M1 + a->M2 <= 3 * kMaxD,
                "sat_attn_step_bwd: D1 <= 256, D2 <= 64");
  SAT_CHECK_ARG(a->NT > 0 && a->NT <= kMaxNT && a->ntiles == ceil_div(a->N, a->NT),
                "sat_attn_step_bwd: tiles");
  SAT_CHECK_ARG(!a->att1_forward || (a->F <= kMaxFb && a->KW <= kMaxKW),
                "sat_attn_step_bwd: location conv too large (F <= 8)");
  SAT_CHECK_ARG(a->pg_stride >= sat_attn_pg_stride(a->D1, a->D2, a->F, a->KW), "sat_attn_step_bwd: pg stride");
  SAT_CHECK_ARG(a->dctx && a->V1 && a->V2 && a->DA && a->DS2 && a->s_t && a->s2_t && a->q &&
                a->K1 && a->K2 && a->v1 && a->v2 && a->dK1 && a->dK2 && a->dqp && a->pg,
                "sat_attn_step_bwd: null pointer");
  SAT_CHECK_ARG(!a->att1_forward || (a->a_t && a->a_prev && a->s_prev && a->stats && a->convW &&
                                     a->convb && a->locW && a->dalpha_prev && a->df_out),
                "sat_attn_step_bwd: forward attention state missing");
  AttnBwdP p;
  p.B = a->B; p.N = a->N; p.D1 = a->D1; p.M1 = a->M1; p.D2 = a->D2; p.M2 = a->M2; p.F = a->F;
  p.KW = a->KW; p.NT = a->NT; p.ntiles = a->ntiles; p.att1_forward = a->att1_forward; p.u = a->u;
  p.dctx = a->dctx; p.dctx_sb = a->dctx_sb; p.dalpha_next = a->dalpha_next;
  p.V1 = a->V1; p.V2 = a->V2; p.DA = a->DA; p.DS2 = a->DS2;
  p.s_t = a->s_t; p.a_t = a->a_t; p.a_prev = a->a_prev; p.s_prev = a->s_prev; p.s2_t = a->s2_t;
  p.stats = a->stats; p.df_next = a->df_next; p.lengths = a->lengths; p.q = a->q; p.q_sb = a->q_sb;
  p.K1 = a->K1; p.K2 = a->K2; p.v1 = a->v1; p.b1 = a->b1; p.convW = a->convW; p.convb = a->convb;
  p.locW = a->locW; p.v2 = a->v2; p.dalpha_prev = a->dalpha_prev; p.df_out = a->df_out;
  p.dK1 = a->dK1; p.dK2 = a->dK2; p.dqp = a->dqp; p.pg = a->pg; p.pg_stride = a->pg_stride;
  hipStream_t s = as_stream(stream);
  const int blocks = a->B * a->ntiles;
  hipLaunchKernelGGL(attn_bwd_ctx_kernel, dim3(blocks), dim3(256), 0, s, p);
  SAT_LAUNCH_CHECK("sat_attn_step_bwd(ctx)");
  hipLaunchKernelGGL(attn_bwd_energy_kernel, dim3(blocks), dim3(256), 0, s, p);
  SAT_LAUNCH_CHECK("sat_attn_step_bwd(energy)");
  return SAT_OK;
}
