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

constexpr int kMaxD = 256, kMaxF = 16, kMaxKW = 32;

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
  float* loc_out;                        // [B][N][F] location features (history for the bwd), nullable
};

// partial record: [0]=m1 [1]=Z1 [2]=A1 [3]=m2 [4]=Z2 [5..7]=pad [8..8+M1) C1 [8+M1..) C2
constexpr int kPartHdr = 8;

struct AttnCombineP {
  int B, N, M1, M2, ntiles, att1_forward;
  float u;
  const float* e1; const float* e2; const float* part; int64_t part_stride;
  const float* a_prev;
  float* s_out; float* a_out; float* s2_out;   // [B][N]
  float* ctx; int64_t ctx_sb;                  // [B][M1 + M2] (row stride ctx_sb)
  float* stats;                                // [B][4]: M1, Z1, A1/Z1 (= sum g s), Z2 for the bwd
};

// Per-utterance combine: all loads issued at entry, tile headers reduced by one wave.
// (A last-tile-block fusion into the tile kernel was measured slower: the device-scope fence it
// needs writes back the XCD's L2, 12 -> 29 us per step.)
__device__ __forceinline__ void combine_utterance(const AttnCombineP& p, int b) {
  __shared__ float sc1[64], sc2[64];
  __shared__ float hdr[6];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t rb = (int64_t)b * p.N;
  const float* part = p.part + (int64_t)b * p.ntiles * p.part_stride;
  const int W = p.M1 + p.M2;
  constexpr int kMaxPos = 4;
  float ev[kMaxPos], e2v[kMaxPos], apv[kMaxPos], amv[kMaxPos];
#pragma unroll
  for (int i = 0; i < kMaxPos; ++i) {
    const int n = tid + 256 * i;
    const bool ok = n < p.N;
    ev[i] = ok ? p.e1[rb + n] : -INFINITY;
    e2v[i] = ok ? p.e2[rb + n] : -INFINITY;
    apv[i] = (ok && p.att1_forward) ? p.a_prev[rb + n] : 0.f;
    amv[i] = (ok && p.att1_forward && n > 0) ? p.a_prev[rb + n - 1] : 0.f;
  }
  float cpart[2][16];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int d = tid + 256 * h;
#pragma unroll
    for (int j = 0; j < 16; ++j)
      cpart[h][j] = (d < W && j < p.ntiles) ? part[j * p.part_stride + kPartHdr + d] : 0.f;
  }
  if (wave == 0) {
    float hm1 = -INFINITY, hz1 = 0.f, ha1 = 0.f, hm2 = -INFINITY, hz2 = 0.f;
    if (lane < p.ntiles) {
      const float* r = part + lane * p.part_stride;
      hm1 = r[0]; hz1 = r[1]; ha1 = r[2]; hm2 = r[3]; hz2 = r[4];
    }
    const float M1 = wave_max(hm1), M2 = wave_max(hm2);
    const float s1 = (hm1 == -INFINITY) ? 0.f : expf(hm1 - M1);
    const float s2 = (hm2 == -INFINITY) ? 0.f : expf(hm2 - M2);
    if (lane < p.ntiles) { sc1[lane] = s1; sc2[lane] = s2; }
    const float Z1 = wave_sum(hz1 * s1), A1 = wave_sum(ha1 * s1), Z2 = wave_sum(hz2 * s2);
    if (lane == 0) {
      hdr[0] = M1; hdr[1] = Z1; hdr[2] = A1; hdr[3] = Z2; hdr[4] = M2;
      if (p.stats) {  // sum_n g[n] s[n] = A1 / Z1 (the forward-attention normaliser) for the bwd
        p.stats[b * 4 + 0] = M1; p.stats[b * 4 + 1] = Z1; p.stats[b * 4 + 2] = A1 / Z1;
        p.stats[b * 4 + 3] = Z2;
      }
    }
  }
  __syncthreads();
  const float M1 = hdr[0], Z1 = hdr[1], A1 = hdr[2], Z2 = hdr[3], M2 = hdr[4];
  const float inv1 = 1.f / (p.att1_forward ? A1 : Z1);
  const float invz1 = 1.f / Z1, invz2 = 1.f / Z2;
  float* ctx = p.ctx + (int64_t)b * p.ctx_sb;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int d = tid + 256 * h;
    if (d < W) {
      const bool first = d < p.M1;
      float acc = 0.f;
#pragma unroll
      for (int j = 0; j < 16; ++j)
        if (j < p.ntiles) acc = fmaf(cpart[h][j], first ? sc1[j] : sc2[j], acc);
      ctx[d] = acc * (first ? inv1 : invz2);
    }
  }
#pragma unroll
  for (int i = 0; i < kMaxPos; ++i) {
    const int n = tid + 256 * i;
    if (n >= p.N) break;
    const float pe = (ev[i] == -INFINITY) ? 0.f : expf(ev[i] - M1);
    const float pe2 = (e2v[i] == -INFINITY) ? 0.f : expf(e2v[i] - M2);
    const float s = pe * invz1;
    p.s_out[rb + n] = s;
    p.s2_out[rb + n] = pe2 * invz2;
    p.a_out[rb + n] = p.att1_forward ? ((1.f - p.u) * apv[i] + p.u * amv[i] + 1e-7f) * pe * inv1 : s;
  }
}

__global__ void __launch_bounds__(256) attn_combine_kernel(AttnCombineP p) {
  combine_utterance(p, blockIdx.x);
}

// Tile kernel (NT = 32 memory positions per workgroup, 256 threads = 32 positions x 8 lanes).
// Each lane owns 4*DW4 consecutive energy dims of one position: its K1 slice arrives as DW4
// 16-byte loads issued at entry (indices clamped so no load sits behind a branch), the energy
// is reduced over the 8 lanes with DPP, and the value rows are read as float4 columns (64 lanes
// x 16 B = one 1 KiB row per wave-instruction) for the unnormalised partial contexts.
// Shapes are compile-time: <F=5, DW4=7, D2W4=1> is LJSpeech/VCTK (D1=224, D2=32); <8, 8, 2> is
// the zero-padded generic form (padding lanes carry zero weights, so no guard in the loop).
// Block -> (b, tile): b = blockIdx % B keeps all tiles of an utterance on one XCD.
constexpr int kNT = 32;

template <int F, int DW4, int D2W4, bool FWD>
__global__ void __launch_bounds__(256) attn_energy_kernel(AttnFwdP p) {
  constexpr int NT = kNT;
  constexpr int LD = DW4 * 32;                    // padded energy width
  constexpr int LD2 = D2W4 * 32;
  __shared__ __attribute__((aligned(16))) float qb[LD];
  __shared__ __attribute__((aligned(16))) float vv[LD];
  __shared__ __attribute__((aligned(16))) float locw[(F > 0 ? F : 1) * LD];
  __shared__ __attribute__((aligned(16))) float q2s[LD2];
  __shared__ __attribute__((aligned(16))) float v2s[LD2];
  __shared__ float cw[kMaxKW * kMaxF + kMaxF];
  __shared__ float fs[NT][F > 0 ? F : 1];
  __shared__ float sp[NT + kMaxKW], ap[NT + 1];
  __shared__ float e1s[NT], e2s[NT], w1s[NT], w2s[NT];
  __shared__ __attribute__((aligned(16))) float4 cred[4][64];
  __shared__ __attribute__((aligned(16))) float4 c2red[NT][16];
  __shared__ float red[8];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = blockIdx.x % p.B, tile = blockIdx.x / p.B;
  const int n0 = tile * NT;
  const int nt = min(NT, p.N - n0);
  const int64_t rb = (int64_t)b * p.N;
  const int padl = (p.KW - 1) / 2;
  const int D1 = p.D1;
  const int nl = tid >> 3, part = tid & 7;
  const int nc = min(n0 + nl, p.N - 1);       // clamped position for this lane's loads

  // ---- burst: K1 / K2 slices of this lane's position (registers)
  float4 k1r[DW4];
  {
    const int d1q = D1 / 4;
    const float4* k1p = reinterpret_cast<const float4*>(p.K1 + (rb + nc) * D1);
#pragma unroll
    for (int j = 0; j < DW4; ++j) k1r[j] = k1p[min(part * DW4 + j, d1q - 1)];
  }
  float4 k2r[D2W4];
  {
    const int d2q = p.D2 / 4;
    const float4* k2p = reinterpret_cast<const float4*>(p.K2 + (rb + nc) * p.D2);
#pragma unroll
    for (int j = 0; j < D2W4; ++j) k2r[j] = k2p[min(part * D2W4 + j, d2q - 1)];
  }
  const int c4 = tid & 63, g = tid >> 6;
  const int M1q = p.M1 / 4, M2q = p.M2 / 4;
  float4 v1r[NT / 4];
#pragma unroll
  for (int i = 0; i < NT / 4; ++i) {
    const int n = min(n0 + g * (NT / 4) + i, p.N - 1);
    v1r[i] = reinterpret_cast<const float4*>(p.V1 + (rb + n) * p.M1)[min(c4, M1q - 1)];
  }
  const float4 v2r = reinterpret_cast<const float4*>(p.V2 + (rb + nc) * p.M2)[min(part, M2q - 1)];
  // ---- burst: small per-step vectors and weights (LDS, zero padded)
  const float* q = p.q + (int64_t)b * p.q_sb;
  for (int d = tid; d < LD; d += 256) {
    const bool ok = d < D1;
    qb[d] = ok ? q[d] + (p.b1 ? p.b1[d] : 0.f) : 0.f;
    vv[d] = ok ? p.v1[d] : 0.f;
  }
  for (int d = tid; d < LD2; d += 256) {
    const bool ok = d < p.D2;
    q2s[d] = ok ? q[D1 + d] : 0.f;
    v2s[d] = ok ? p.v2[d] : 0.f;
  }
  if (FWD) {
    for (int i = tid; i < F * LD; i += 256) {
      const int f = i / LD, d = i - f * LD;
      locw[i] = (f < p.F && d < D1) ? p.locW[f * D1 + d] : 0.f;
    }
    for (int i = tid; i < p.KW * p.F; i += 256) cw[i] = p.convW[i];
    if (tid < p.F) cw[p.KW * p.F + tid] = p.convb[tid];
    const int span = nt + p.KW - 1;
    for (int i = tid; i < span; i += 256) {
      const int n = n0 - padl + i;
      sp[i] = (n >= 0 && n < p.N) ? p.s_prev[rb + n] : 0.f;
    }
    if (tid <= nt) ap[tid] = (n0 - 1 + tid >= 0) ? p.a_prev[rb + n0 - 1 + tid] : 0.f;
  }
  const int len = (int)p.lengths[b];
  __syncthreads();
  if (FWD) {  // location features f = Conv1D_SAME(s_{t-1}) + bias (padded filters = 0)
    if (tid < NT * F) {
      const int i = tid / F, f = tid - i * F;
      float acc = 0.f;
      if (f < p.F) {
        acc = cw[p.KW * p.F + f];
        for (int j = 0; j < p.KW; ++j) acc = fmaf(sp[i + j], cw[j * p.F + f], acc);
      }
      fs[i][f] = acc;
      if (p.loc_out && i < nt && f < p.F) p.loc_out[(rb + n0 + i) * p.F + f] = acc;
    }
    __syncthreads();
  }
  // ---- energies: 4*DW4 dims per lane, 8-lane DPP reduction
  float fl[F > 0 ? F : 1];
#pragma unroll
  for (int f = 0; f < F; ++f) fl[f] = fs[nl][f];
  float acc = 0.f;
  const int d0 = part * DW4 * 4;
#pragma unroll
  for (int j = 0; j < DW4; ++j) {
    const int d = d0 + 4 * j;
    const float4 qv = *reinterpret_cast<const float4*>(&qb[d]);
    const float4 vw = *reinterpret_cast<const float4*>(&vv[d]);
    float4 pre = make_float4(k1r[j].x + qv.x, k1r[j].y + qv.y, k1r[j].z + qv.z, k1r[j].w + qv.w);
    if (FWD) {
#pragma unroll
      for (int f = 0; f < F; ++f) {
        const float4 lw = *reinterpret_cast<const float4*>(&locw[f * LD + d]);
        pre.x = fmaf(fl[f], lw.x, pre.x); pre.y = fmaf(fl[f], lw.y, pre.y);
        pre.z = fmaf(fl[f], lw.z, pre.z); pre.w = fmaf(fl[f], lw.w, pre.w);
      }
    }
    acc = fmaf(vw.x, tanh_fast(pre.x), acc);
    acc = fmaf(vw.y, tanh_fast(pre.y), acc);
    acc = fmaf(vw.z, tanh_fast(pre.z), acc);
    acc = fmaf(vw.w, tanh_fast(pre.w), acc);
  }
  float acc2 = 0.f;
#pragma unroll
  for (int j = 0; j < D2W4; ++j) {
    const int d = (part * D2W4 + j) * 4;
    const float4 qv = *reinterpret_cast<const float4*>(&q2s[d]);
    const float4 vw = *reinterpret_cast<const float4*>(&v2s[d]);
    acc2 = fmaf(vw.x, tanh_fast(k2r[j].x + qv.x), acc2);
    acc2 = fmaf(vw.y, tanh_fast(k2r[j].y + qv.y), acc2);
    acc2 = fmaf(vw.z, tanh_fast(k2r[j].z + qv.z), acc2);
    acc2 = fmaf(vw.w, tanh_fast(k2r[j].w + qv.w), acc2);
  }
  acc = group8_sum(acc);
  acc2 = group8_sum(acc2);
  if (part == 0 && nl < nt) {
    const bool valid = n0 + nl < len;
    e1s[nl] = valid ? acc : -INFINITY;
    e2s[nl] = valid ? acc2 : -INFINITY;
  }
  __syncthreads();
  // ---- tile statistics (wave 0)
  if (wave == 0) {
    const float e1v = lane < nt ? e1s[lane] : -INFINITY;
    const float e2v = lane < nt ? e2s[lane] : -INFINITY;
    const float m1 = wave_max(e1v), m2 = wave_max(e2v);
    const float pe = (e1v == -INFINITY) ? 0.f : expf(e1v - m1);
    const float pe2 = (e2v == -INFINITY) ? 0.f : expf(e2v - m2);
    float w = pe;
    if (FWD && lane < nt) w = ((1.f - p.u) * ap[lane + 1] + p.u * ap[lane] + 1e-7f) * pe;
    if (lane < NT) { w1s[lane] = lane < nt ? w : 0.f; w2s[lane] = lane < nt ? pe2 : 0.f; }
    const float z1 = wave_sum_dpp(pe), a1 = wave_sum_dpp(lane < nt ? w : 0.f),
                z2 = wave_sum_dpp(pe2);
    if (lane == 0) { red[0] = m1; red[1] = z1; red[2] = a1; red[3] = m2; red[4] = z2; }
  }
  __syncthreads();
  float* part_out = p.part + ((int64_t)b * p.ntiles + tile) * p.part_stride;
  if (tid < kPartHdr) part_out[tid] = tid < 5 ? red[tid] : 0.f;
  if (tid < nt) {
    p.e1[rb + n0 + tid] = e1s[tid];
    p.e2[rb + n0 + tid] = e2s[tid];
  }
  // ---- unnormalised partial contexts
  float4 c = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int i = 0; i < NT / 4; ++i) {
    const float w = w1s[g * (NT / 4) + i];
    c.x = fmaf(w, v1r[i].x, c.x); c.y = fmaf(w, v1r[i].y, c.y);
    c.z = fmaf(w, v1r[i].z, c.z); c.w = fmaf(w, v1r[i].w, c.w);
  }
  cred[g][c4] = c;
  {
    const float w = w2s[nl];
    c2red[nl][part] = make_float4(w * v2r.x, w * v2r.y, w * v2r.z, w * v2r.w);
  }
  __syncthreads();
  if (tid < M1q) {
    const float4 a0 = cred[0][tid], a1 = cred[1][tid], a2 = cred[2][tid], a3 = cred[3][tid];
    reinterpret_cast<float4*>(part_out + kPartHdr)[tid] =
        make_float4((a0.x + a1.x) + (a2.x + a3.x), (a0.y + a1.y) + (a2.y + a3.y),
                    (a0.z + a1.z) + (a2.z + a3.z), (a0.w + a1.w) + (a2.w + a3.w));
  } else if (tid >= 64 && tid < 64 + M2q) {
    const int j = tid - 64;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 8
    for (int i = 0; i < NT; ++i) {
      const float4 v = c2red[i][j];
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    reinterpret_cast<float4*>(part_out + kPartHdr + p.M1)[j] = s;
  }
}

// Wide tile kernel: the same step with LPP lanes per memory position (NT * LPP threads, 512 or
// 1024), so each lane's serial chain is 64 / LPP float4 of the (zero padded to 256) energy row;
// the step is latency-bound, and more, shorter chains per block hide the exp / rcp / LDS
// latencies.  Source 2 (D2 <= 4 * LPP) takes one float4 per lane.  Same partial record.
template <int F, int LPP, bool FWD>
__global__ void __launch_bounds__(kNT * LPP) attn_energy_wide_kernel(AttnFwdP p) {
  constexpr int NT = kNT, NTH = NT * LPP, NW = NTH / 64;
  constexpr int J = 64 / LPP;                      // float4 of the padded energy row per lane
  constexpr int G = NTH / 64;                      // position groups of the context phase
  constexpr int PG = NT / G;                       // positions per group
  constexpr int FL = F > 0 ? F : 1;
  __shared__ __attribute__((aligned(16))) float qb[kMaxD];
  __shared__ __attribute__((aligned(16))) float vv[kMaxD];
  __shared__ __attribute__((aligned(16))) float locw[FL * kMaxD];
  __shared__ __attribute__((aligned(16))) float q2s[64];
  __shared__ __attribute__((aligned(16))) float v2s[64];
  __shared__ float cw[kMaxKW * kMaxF + kMaxF];
  __shared__ float fs[NT][FL];
  __shared__ float sp[NT + kMaxKW], ap[NT + 1];
  __shared__ float e1s[NT], e2s[NT], w1s[NT], w2s[NT];
  __shared__ __attribute__((aligned(16))) float4 cred[G][64];
  __shared__ __attribute__((aligned(16))) float4 c2red[NT][16];
  __shared__ float red[8];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = blockIdx.x % p.B, tile = blockIdx.x / p.B;
  const int n0 = tile * NT;
  const int nt = min(NT, p.N - n0);
  const int64_t rb = (int64_t)b * p.N;
  const int padl = (p.KW - 1) / 2;
  const int D1 = p.D1;
  const int nl = tid / LPP, part = tid - nl * LPP;
  const int nc = min(n0 + nl, p.N - 1);       // clamped position for this lane's loads

  // ---- burst: K1 / K2 slices of this lane's position, V1 / V2 rows of the context phase
  float4 k1r[J];
  {
    const int d1q = D1 / 4;
    const float4* k1p = reinterpret_cast<const float4*>(p.K1 + (rb + nc) * D1);
#pragma unroll
    for (int j = 0; j < J; ++j) k1r[j] = k1p[min(part + LPP * j, d1q - 1)];
  }
  const int d2q = p.D2 / 4;
  const float4 k2r = reinterpret_cast<const float4*>(p.K2 + (rb + nc) * p.D2)[min(part, d2q - 1)];
  const int c4 = lane, g = wave;               // context phase: group g, float4 column c4
  const int M1q = p.M1 / 4, M2q = p.M2 / 4;
  float4 v1r[PG];
#pragma unroll
  for (int i = 0; i < PG; ++i) {
    const int n = min(n0 + g * PG + i, p.N - 1);
    v1r[i] = reinterpret_cast<const float4*>(p.V1 + (rb + n) * p.M1)[min(c4, M1q - 1)];
  }
  const float4 v2r = reinterpret_cast<const float4*>(p.V2 + (rb + nc) * p.M2)[min(part, M2q - 1)];
  // ---- burst: small per-step vectors and weights (LDS, zero padded)
  const float* q = p.q + (int64_t)b * p.q_sb;
  if (tid < kMaxD) {
    const int d = tid;
    const bool ok = d < D1;
    qb[d] = ok ? q[d] + (p.b1 ? p.b1[d] : 0.f) : 0.f;
    vv[d] = ok ? p.v1[d] : 0.f;
    if (d < 64) {
      q2s[d] = d < p.D2 ? q[D1 + d] : 0.f;
      v2s[d] = d < p.D2 ? p.v2[d] : 0.f;
    }
    if (FWD) {
#pragma unroll
      for (int f = 0; f < F; ++f) locw[f * kMaxD + d] = (ok && f < p.F) ? p.locW[f * D1 + d] : 0.f;
    }
  }
  if (FWD) {
    if (tid < p.KW * p.F) cw[tid] = p.convW[tid];
    if (tid < p.F) cw[p.KW * p.F + tid] = p.convb[tid];
    const int span = nt + p.KW - 1;
    if (tid < span) {
      const int n = n0 - padl + tid;
      sp[tid] = (n >= 0 && n < p.N) ? p.s_prev[rb + n] : 0.f;
    }
    if (tid <= nt) ap[tid] = (n0 - 1 + tid >= 0) ? p.a_prev[rb + n0 - 1 + tid] : 0.f;
  }
  const int len = (int)p.lengths[b];
  __syncthreads();
  if (FWD) {  // location features f = Conv1D_SAME(s_{t-1}) + bias
    if (tid < NT * F) {
      const int i = tid / F, f = tid - i * F;    // padded filters (f >= p.F) are zero
      float acc = 0.f;
      if (f < p.F) {
        acc = cw[p.KW * p.F + f];
        for (int j = 0; j < p.KW; ++j) acc = fmaf(sp[i + j], cw[j * p.F + f], acc);
        if (p.loc_out && i < nt) p.loc_out[(rb + n0 + i) * p.F + f] = acc;
      }
      fs[i][f] = acc;
    }
    __syncthreads();
  }
  // ---- energies: J float4 per lane, LPP-lane reduction
  float fl[FL];
#pragma unroll
  for (int f = 0; f < FL; ++f) fl[f] = FWD ? fs[nl][f] : 0.f;
  float acc = 0.f;
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int d = 4 * (part + LPP * j);
    const float4 qv = *reinterpret_cast<const float4*>(&qb[d]);
    const float4 vw = *reinterpret_cast<const float4*>(&vv[d]);
    float4 pre = make_float4(k1r[j].x + qv.x, k1r[j].y + qv.y, k1r[j].z + qv.z, k1r[j].w + qv.w);
    if (FWD) {
#pragma unroll
      for (int f = 0; f < F; ++f) {
        const float4 lw = *reinterpret_cast<const float4*>(&locw[f * kMaxD + d]);
        pre.x = fmaf(fl[f], lw.x, pre.x); pre.y = fmaf(fl[f], lw.y, pre.y);
        pre.z = fmaf(fl[f], lw.z, pre.z); pre.w = fmaf(fl[f], lw.w, pre.w);
      }
    }
    acc = fmaf(vw.x, tanh_fast(pre.x), acc);
    acc = fmaf(vw.y, tanh_fast(pre.y), acc);
    acc = fmaf(vw.z, tanh_fast(pre.z), acc);
    acc = fmaf(vw.w, tanh_fast(pre.w), acc);
  }
  float acc2 = 0.f;
  if (part < 16) {
    const int d = 4 * part;
    const float4 qv = *reinterpret_cast<const float4*>(&q2s[d]);
    const float4 vw = *reinterpret_cast<const float4*>(&v2s[d]);
    acc2 = fmaf(vw.x, tanh_fast(k2r.x + qv.x), acc2);
    acc2 = fmaf(vw.y, tanh_fast(k2r.y + qv.y), acc2);
    acc2 = fmaf(vw.z, tanh_fast(k2r.z + qv.z), acc2);
    acc2 = fmaf(vw.w, tanh_fast(k2r.w + qv.w), acc2);
  }
  if (LPP == 16) { acc = group16_sum(acc); acc2 = group16_sum(acc2); }
  else { acc = group32_sum(acc); acc2 = group32_sum(acc2); }
  if (part == 0 && nl < nt) {
    const bool valid = n0 + nl < len;
    e1s[nl] = valid ? acc : -INFINITY;
    e2s[nl] = valid ? acc2 : -INFINITY;
  }
  __syncthreads();
  // ---- tile statistics (wave 0)
  if (wave == 0) {
    const float e1v = lane < nt ? e1s[lane] : -INFINITY;
    const float e2v = lane < nt ? e2s[lane] : -INFINITY;
    const float m1 = wave_max(e1v), m2 = wave_max(e2v);
    const float pe = (e1v == -INFINITY) ? 0.f : expf(e1v - m1);
    const float pe2 = (e2v == -INFINITY) ? 0.f : expf(e2v - m2);
    float w = pe;
    if (FWD && lane < nt) w = ((1.f - p.u) * ap[lane + 1] + p.u * ap[lane] + 1e-7f) * pe;
    if (lane < NT) { w1s[lane] = lane < nt ? w : 0.f; w2s[lane] = lane < nt ? pe2 : 0.f; }
    const float z1 = wave_sum_dpp(pe), a1 = wave_sum_dpp(lane < nt ? w : 0.f),
                z2 = wave_sum_dpp(pe2);
    if (lane == 0) { red[0] = m1; red[1] = z1; red[2] = a1; red[3] = m2; red[4] = z2; }
  }
  __syncthreads();
  float* part_out = p.part + ((int64_t)b * p.ntiles + tile) * p.part_stride;
  if (tid < kPartHdr) part_out[tid] = tid < 5 ? red[tid] : 0.f;
  if (tid < nt) {
    p.e1[rb + n0 + tid] = e1s[tid];
    p.e2[rb + n0 + tid] = e2s[tid];
  }
  // ---- unnormalised partial contexts
  float4 c = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int i = 0; i < PG; ++i) {
    const float w = w1s[g * PG + i];
    c.x = fmaf(w, v1r[i].x, c.x); c.y = fmaf(w, v1r[i].y, c.y);
    c.z = fmaf(w, v1r[i].z, c.z); c.w = fmaf(w, v1r[i].w, c.w);
  }
  cred[g][c4] = c;
  if (part < 16) {
    const float w = w2s[nl];
    c2red[nl][part] = make_float4(w * v2r.x, w * v2r.y, w * v2r.z, w * v2r.w);
  }
  __syncthreads();
  if (tid < M1q) {
    float4 sum = cred[0][tid];
#pragma unroll
    for (int j = 1; j < G; ++j) {
      const float4 v = cred[j][tid];
      sum.x += v.x; sum.y += v.y; sum.z += v.z; sum.w += v.w;
    }
    reinterpret_cast<float4*>(part_out + kPartHdr)[tid] = sum;
  } else if (tid >= 64 && tid < 64 + M2q) {
    const int j = tid - 64;
    float4 sum = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 8
    for (int i = 0; i < NT; ++i) {
      const float4 v = c2red[i][j];
      sum.x += v.x; sum.y += v.y; sum.z += v.z; sum.w += v.w;
    }
    reinterpret_cast<float4*>(part_out + kPartHdr + p.M1)[j] = sum;
  }
  (void)NW;
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
  SAT_CHECK_ARG(a->NT == kNT, "sat_attn_step_fwd: tile size must be 32");
  SAT_CHECK_ARG(a->N <= 1024 && a->M1 <= 256 && a->M1 % 4 == 0 && a->M2 <= 32 && a->M2 % 4 == 0,
                "sat_attn_step_fwd: N <= 1024, M1 <= 256, M2 <= 32 (multiples of 4)");
  SAT_CHECK_ARG(a->D1 % 32 == 0 && a->D1 <= 256 && a->D2 % 32 == 0 && a->D2 <= 64,
                "sat_attn_step_fwd: D1 % 32 == 0 (<= 256), D2 in {32, 64}");
  SAT_CHECK_ARG(!a->att1_forward || a->F <= 8, "sat_attn_step_fwd: F <= 8");
  SAT_CHECK_ARG(!a->att1_forward || (a->F <= kMaxF && a->KW <= kMaxKW && a->F * a->D1 <= kMaxF * kMaxD),
                "sat_attn_step_fwd: location conv too large");
  SAT_CHECK_ARG(a->part_stride >= sat_attn_part_stride(a->M1, a->M2), "sat_attn_step_fwd: part stride");
  SAT_CHECK_ARG(a->ntiles <= 16 && a->ntiles == ceil_div(a->N, a->NT), "sat_attn_step_fwd: ntiles must be <= 16");
  SAT_CHECK_ARG(a->D2 <= 64, "sat_attn_step_fwd: D2 <= 64");
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
  p.loc_out = a->att1_forward ? a->loc_out : nullptr;
  hipStream_t s = as_stream(stream);
  const int phases = a->phases == 0 ? 3 : a->phases;
  if (phases & 1) {
    const dim3 grid(a->ntiles * a->B);
    const int lpp = a->lpp == 0 ? 16 : a->lpp;
    SAT_CHECK_ARG(lpp == 8 || lpp == 16 || lpp == 32, "sat_attn_step_fwd: lpp in {8, 16, 32}");
    if (lpp == 16 && a->att1_forward && a->F == 5)
      hipLaunchKernelGGL((attn_energy_wide_kernel<5, 16, true>), grid, dim3(kNT * 16), 0, s, p);
    else if (lpp == 32 && a->att1_forward && a->F == 5)
      hipLaunchKernelGGL((attn_energy_wide_kernel<5, 32, true>), grid, dim3(kNT * 32), 0, s, p);
    else if (lpp != 8 && a->att1_forward)
      hipLaunchKernelGGL((attn_energy_wide_kernel<8, 16, true>), grid, dim3(kNT * 16), 0, s, p);
    else if (lpp != 8)
      hipLaunchKernelGGL((attn_energy_wide_kernel<0, 16, false>), grid, dim3(kNT * 16), 0, s, p);
    else if (a->att1_forward && a->F == 5 && a->D1 == 224 && a->D2 == 32)
      hipLaunchKernelGGL((attn_energy_kernel<5, 7, 1, true>), grid, dim3(256), 0, s, p);
    else if (a->att1_forward)
      hipLaunchKernelGGL((attn_energy_kernel<8, 8, 2, true>), grid, dim3(256), 0, s, p);
    else
      hipLaunchKernelGGL((attn_energy_kernel<0, 8, 2, false>), grid, dim3(256), 0, s, p);
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
// Reverse step t of the dual-source attention (see the forward formulas at the top), ONE
// launch per step: (utterance, tile) workgroups.
//
// The utterance-wide scalars of the softmax / forward-recursion backward need no cross-tile
// pass over the values, because the forward context of step t is already a weighted sum of them:
//   DA[n] = dc1 . V1[n] + dalpha_next[n]              (gradient reaching alpha_t[n])
//   s1    = sum_n DA[n] alpha_t[n] = dc1 . c1_t + sum_n dalpha_next[n] alpha_t[n]
//   s3    = sum_n DS2[n] s2_t[n]   = dc2 . c2_t
//   s2sum = sum_n s_t[n] ds[n]     = sum_n s_t[n] DSN[n]   (the alpha path cancels: sum alpha = 1)
// where DSN[n] = sum_{j,f} df_next[n - j + padl][f] convW[j][f] is the transposed location
// convolution of the next reverse step's feature gradient (whole utterance, from LDS).  So each
// block needs only its own tile's V1/V2 rows, and the [B,N] alpha-gradient crosses steps as
//   Y[n] = s_t[n] (DA[n] - s1) / Sa,   dalpha_{t-1}[n] = (1-u) Y[n] + u Y[n+1].
// Then the tile's energies are recomputed from K1 (no [T',B,N,224] tensor is stored) and
// back-propagated through tanh: dK1/dK2 accumulated in place (each element owned by one thread),
// per-tile dq partials, location-feature gradients df (-> DSN of step t-1), and the small
// parameter grads accumulated per (utterance, tile) without atomics.
// Utterance b's tiles are blocks b, b+B, b+2B, ... (B % 8 == 0: one XCD, K1[b] stays in its L2).
namespace sat {
namespace {

constexpr int kMaxN = 1024, kMaxFb = 8;

struct AttnBwdP {
  int B, N, D1, M1, D2, M2, F, KW, NT, ntiles, att1_forward;
  float u;
  const float* dctx; int64_t dctx_sb;
  const float* ctx_t; int64_t ctx_sb;
  const float* y_next;
  const float* V1; const float* V2;
  const float* s_t; const float* a_t; const float* a_prev; const float* s_prev; const float* s2_t;
  const float* stats;
  const float* df_next;
  const float* q; int64_t q_sb;
  const float* K1; const float* K2;
  const float* v1; const float* b1; const float* convW; const float* convb; const float* locW;
  const float* v2;
  float* y_out;
  float* df_out;
  float* de1_out; float* de2_out;
  float* dqp;
};

// LDS: df_next of the whole utterance early, the per-wave dq partials late
constexpr int kBwdScratch = kMaxN * kMaxFb;
static_assert(kBwdScratch >= 16 * (kMaxD + 64), "dq flush must fit the scratch");

// WAVES waves per block (NT / WAVES tile positions per wave): the step is latency-bound, so
// more, shorter per-wave chains (8 waves = 2 per SIMD) hide the LDS / transcendental latencies.
template <int NT, int F, int WAVES>
__global__ void __launch_bounds__(64 * WAVES) attn_bwd_kernel(AttnBwdP p) {
  constexpr int NTH = 64 * WAVES;
  constexpr int PPW = NT / WAVES;
  constexpr int kPos = (kMaxN + NTH - 1) / NTH;   // utterance positions per thread
  constexpr int FL = F > 0 ? F : 1;
  constexpr bool FWD = F > 0;
  static_assert(NT % WAVES == 0 && NTH >= kMaxD, "tile / wave split");
  __shared__ float dc[2 * kMaxD];
  __shared__ float dsn_t[NT], dan_t[NT], stv[NT], s2v[NT], apv[NT + 1];
  __shared__ float qb[kMaxD], vv[kMaxD], q2s[64], v2s[64];
  __shared__ float locw[FL * kMaxD];
  __shared__ float cw[kMaxKW * FL + FL];
  __shared__ float fs[NT][FL], dfs[NT][FL];
  __shared__ float sp[NT + kMaxKW];
  __shared__ float de1[NT], de2[NT];
  __shared__ float red[3 * WAVES];
  __shared__ float scratch[kBwdScratch];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = blockIdx.x % p.B, tile = blockIdx.x / p.B;
  const int n0 = tile * NT, nt = min(NT, p.N - n0);
  const int64_t rb = (int64_t)b * p.N;
  const int padl = (p.KW - 1) / 2;
  const float u = p.u;
  const int D1 = p.D1, D2 = p.D2, N = p.N, M1 = p.M1, M2 = p.M2;
  const bool has_next = p.y_next != nullptr;     // false at the last decoder step

  // ---------------- burst: registers (indices clamped: no load behind a branch)
  float k1r[PPW][4], k2r[PPW], v1r[PPW][4], v2r[PPW];
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int n = min(n0 + wave + WAVES * i, N - 1);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int d = min(lane + 64 * s, D1 - 1);
      k1r[i][s] = p.K1[(rb + n) * D1 + d];
      v1r[i][s] = p.V1[(rb + n) * M1 + min(lane + 64 * s, M1 - 1)];
    }
    k2r[i] = p.K2[(rb + n) * D2 + min(lane, D2 - 1)];
    v2r[i] = p.V2[(rb + n) * M2 + min(lane, M2 - 1)];
  }
  float ry0[kPos], ry1[kPos], rat[kPos], rst[kPos];
#pragma unroll
  for (int i = 0; i < kPos; ++i) {
    const int n = tid + NTH * i;
    const int64_t o = rb + min(n, N - 1);
    ry0[i] = (has_next && n < N) ? p.y_next[o] : 0.f;
    ry1[i] = (has_next && n + 1 < N) ? p.y_next[o + 1] : 0.f;
    rat[i] = n < N ? p.a_t[o] : 0.f;
    rst[i] = n < N ? p.s_t[o] : 0.f;
  }
  // dc . c_t (the forward context of step t)
  float dcc1 = 0.f, dcc2 = 0.f;
  {
    const float* g = p.dctx + (int64_t)b * p.dctx_sb;
    const float* c = p.ctx_t + (int64_t)b * p.ctx_sb;
    for (int d = tid; d < M1 + M2; d += NTH) {
      const float gv = g[d];
      dc[d] = gv;
      if (d < M1) dcc1 = fmaf(gv, c[d], dcc1);
      else dcc2 = fmaf(gv, c[d], dcc2);
    }
  }
  // ---------------- burst: LDS (zero padded to 256 / 64)
  const float* q = p.q + (int64_t)b * p.q_sb;
  if (tid < kMaxD) {
    const int d = tid;
    const bool ok = d < D1;
    qb[d] = ok ? q[d] + (p.b1 ? p.b1[d] : 0.f) : 0.f;
    vv[d] = ok ? p.v1[d] : 0.f;
    if (d < 64) {
      q2s[d] = d < D2 ? q[D1 + d] : 0.f;
      v2s[d] = d < D2 ? p.v2[d] : 0.f;
    }
    if (FWD) {
#pragma unroll
      for (int f = 0; f < F; ++f) locw[f * kMaxD + d] = ok ? p.locW[f * D1 + d] : 0.f;
    }
  }
  float* dfall = scratch;   // [N][F] df_next of the whole utterance (free until the flush)
  if (tid < nt) {
    stv[tid] = p.s_t[rb + n0 + tid];
    s2v[tid] = p.s2_t[rb + n0 + tid];
  }
  if (FWD) {
    if (tid <= nt) apv[tid] = (n0 - 1 + tid >= 0 && n0 - 1 + tid < N) ? p.a_prev[rb + n0 - 1 + tid] : 0.f;
    for (int i = tid; i < p.KW * F; i += NTH) cw[i] = p.convW[i];
    if (tid < F) cw[p.KW * F + tid] = p.convb[tid];
    const int span = nt + p.KW - 1;
    for (int i = tid; i < span; i += NTH) {
      const int n = n0 - padl + i;
      sp[i] = (n >= 0 && n < N) ? p.s_prev[rb + n] : 0.f;
    }
    if (has_next)
      for (int i = tid; i < N * F; i += NTH) dfall[i] = p.df_next[rb * F + i];
  }
  __syncthreads();

  // ---------------- utterance-wide sums: s1 = dc1.c1 + sum dalpha_next alpha, s3 = dc2.c2,
  //                  s2sum = sum s DSN; the tile keeps its own DSN / dalpha_next
  float s1 = dcc1, s3 = dcc2, s2 = 0.f;
#pragma unroll
  for (int i = 0; i < kPos; ++i) {
    const int n = tid + NTH * i;
    if (n >= N) break;
    const float dan = (1.f - u) * ry0[i] + u * ry1[i];
    s1 = fmaf(dan, rat[i], s1);
    float dsn = 0.f;
    if (FWD && has_next) {
      for (int j = 0; j < p.KW; ++j) {
        const int m = n - j + padl;
        if (m < 0 || m >= N) continue;
#pragma unroll
        for (int f = 0; f < F; ++f) dsn = fmaf(dfall[m * F + f], cw[j * F + f], dsn);
      }
      s2 = fmaf(rst[i], dsn, s2);
    }
    const int r = n - n0;
    if (r >= 0 && r < nt) { dsn_t[r] = dsn; dan_t[r] = dan; }
  }
  if (FWD) {  // location features of the tile
    if (tid < NT * F) {
      const int nl = tid / F, f = tid - nl * F;
      float acc = cw[p.KW * F + f];
      for (int j = 0; j < p.KW; ++j) acc = fmaf(sp[nl + j], cw[j * F + f], acc);
      fs[nl][f] = acc;
    }
  }
  s1 = wave_sum_dpp(s1);
  s3 = wave_sum_dpp(s3);
  s2 = wave_sum_dpp(s2);
  if (lane == 0) { red[wave] = s1; red[WAVES + wave] = s3; red[2 * WAVES + wave] = s2; }
  __syncthreads();   // also publishes dsn_t / dan_t / fs
  s1 = 0.f; s3 = 0.f; s2 = 0.f;
#pragma unroll
  for (int w = 0; w < WAVES; ++w) {
    s1 += red[w]; s3 += red[WAVES + w]; s2 += red[2 * WAVES + w];
  }
  const float s2sum = FWD ? s2 : s1;
  const float Sa = FWD ? p.stats[b * 4 + 2] : 1.f;
  const float rSa = 1.f / Sa;

  // ---------------- tile: DA, DS2 (wave per position, lanes over the value dims) -> de, de2, Y
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int nl = wave + WAVES * i;
    if (nl >= nt) break;
    float a = 0.f;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int d = lane + 64 * s;
      if (d < M1) a = fmaf(dc[d], v1r[i][s], a);
    }
    float c = lane < M2 ? dc[M1 + lane] * v2r[i] : 0.f;
    a = wave_sum(a);
    c = wave_sum(c);
    if (lane == 0) {
      const int n = n0 + nl;
      const float DA = a + dan_t[nl];
      const float st = stv[nl];
      float ds;
      if (FWD) {
        const float da = (DA - s1) * rSa;
        const float prior = (1.f - u) * apv[nl + 1] + u * apv[nl] + 1e-7f;
        ds = dsn_t[nl] + da * prior;
        p.y_out[rb + n] = st * da;
      } else {
        ds = DA;
      }
      const float e1v = st * (ds - s2sum), e2v = s2v[nl] * (c - s3);
      de1[nl] = e1v;
      de2[nl] = e2v;
      p.de1_out[rb + n] = e1v;
      p.de2_out[rb + n] = e2v;
    }
  }
  __syncthreads();

  // ---------------- recompute the tile's energies, back-propagate through tanh: the query
  //                  gradient and the location-feature gradient (the critical path); the
  //                  parameter gradients are left to sat_attn_param_grads after the loop
  float aq[4] = {0, 0, 0, 0};
  float aq2 = 0.f;   // lane owns d2 = lane (D2 <= 64, checked on the host)
  const float q2 = q2s[lane], v2 = v2s[lane];
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int nl = wave + WAVES * i;
    if (nl >= nt) break;
    const float e = de1[nl];
    float fl[FL], dfp[FL];
#pragma unroll
    for (int f = 0; f < FL; ++f) { fl[f] = FWD ? fs[nl][f] : 0.f; dfp[f] = 0.f; }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int d = lane + 64 * k;
      float pre = k1r[i][k] + qb[d];
      float lw[FL];
#pragma unroll
      for (int f = 0; f < F; ++f) { lw[f] = locw[f * kMaxD + d]; pre = fmaf(fl[f], lw[f], pre); }
      const float z = tanh_fast(pre);
      const float dp = e * vv[d] * (1.f - z * z);
      aq[k] += dp;
#pragma unroll
      for (int f = 0; f < F; ++f) dfp[f] = fmaf(dp, lw[f], dfp[f]);
    }
#pragma unroll
    for (int f = 0; f < F; ++f) {
      const float sdf = wave_sum_dpp(dfp[f]);
      if (lane == 0) dfs[nl][f] = sdf;
    }
    {
      const float z = tanh_fast(k2r[i] + q2);
      aq2 = fmaf(de2[nl] * v2, 1.f - z * z, aq2);
    }
  }
  // ---------------- per-wave dq partials -> LDS ([dq D1 (256)][dq2 64] per wave; dfall is dead)
  constexpr int wstride = kMaxD + 64;
  float* r = scratch + wave * wstride;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 4; ++k) r[lane + 64 * k] = aq[k];
  r[kMaxD + lane] = aq2;
  __syncthreads();
  if (FWD && tid < nt * F) {
    const int nl = tid / F, f = tid - nl * F;
    p.df_out[(rb + n0 + nl) * F + f] = dfs[nl][f];
  }
  float* dqp = p.dqp + ((int64_t)b * p.ntiles + tile) * (D1 + D2);
  for (int d = tid; d < D1 + D2; d += NTH) {
    const int o = d < D1 ? d : kMaxD + (d - D1);
    float acc = 0.f;
#pragma unroll
    for (int w = 0; w < WAVES; ++w) acc += scratch[w * wstride + o];
    dqp[d] = acc;
  }
}

// ---------------------------------------------------------------- parameter gradients
// After the reverse loop, every per-step contribution to the attention parameters is summed in
// ONE pass over (t, b, n): the energy pre-activations are recomputed from K1/K2, the stored
// processed queries and location features, and the stored energy gradients de1/de2 (scalars per
// step and position):
//   dp[d] = de1 v1[d] (1 - z[d]^2),  z = tanh(K1[n] + q_t + b1 + f_t[n] W_loc)
//   dK1[n] = sum_t dp,  dv1 = sum z de1,  dW_loc[f] = sum f_t[n][f] dp,
//   dconvW[j][f] = sum s_{t-1}[n + j - padl] df_t[n][f],  dconvb[f] = sum df_t[n][f]
// (the same for source 2 without the location terms).  One wave per memory position, lanes
// over float4 slots of [D1 | D2]; the wave loops over the T' steps; the four positions of a
// workgroup are reduced through LDS into one partial row (summed by a column reduction).
template <int SLOTS, int F>
__device__ __forceinline__ void attn_pg_store(const SatAttnParamGrad& p, const float4* adk,
                                              const float4* adv,
                                              const float4 (*adw)[F > 0 ? F : 1], float acw);

template <int SLOTS, int F>
__device__ __forceinline__ void pg_recompute_body(const SatAttnParamGrad& p) {
  constexpr int FL = F > 0 ? F : 1;
  // wave-uniform (scalar) position: the per-step history addresses of de1 / de2 / loc are then
  // scalar and their loads go through the scalar cache instead of 64-bit VALU address math
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nq = (p.N + 3) / 4;
  // part `part` of the tsplit step ranges: workgroup index = part * (B * nq) + b * nq + n / 4
  const int rows = p.B * nq, part = blockIdx.x / rows, wgi = blockIdx.x - part * rows;
  const int ts = max(p.tsplit, 1);
  const int t_lo = (int)((int64_t)p.T * part / ts), t_hi = (int)((int64_t)p.T * (part + 1) / ts);
  const int b = wgi / nq, n = 4 * (wgi - b * nq) + wave;
  const int nn = min(n, p.N - 1);
  const int Q1 = p.D1 / 4, Q = Q1 + p.D2 / 4;
  const int padl = (p.KW - 1) / 2;
  const int64_t bn = (int64_t)b * p.N + nn;
  const int64_t TBN = (int64_t)p.B * p.N;

  // tanh(x) = 1 - 2 / (1 + 2^(kE x)), kE = 2 log2(e): K + b1 and W_loc are held pre-scaled by kE
  // and q is scaled once per step, so the exponent argument costs no extra multiply per element
  // (z agrees with tanh_fast to a few ulp; the forward's ZH is not read here)
  constexpr float kE = 2.8853900817779268f;
  // Factored step arithmetic: with r = 1 / (1 + 2^(kE x)), z = tanh(x) = 1 - 2 r and
  // 1 - z^2 = 4 r (1 - r) = 4 g, so per element and step only g, e g, e r and the F products
  // (f e) g are accumulated, in packed pairs; the step-independent factors 4 v (dK, dW_loc) and
  // sum_t e - 2 (.) (dv) are applied once after the loop.  (The per-element form spent ~25 % of
  // its VALU slots on register moves feeding the packed FMAs: 268 -> 227 VALU instructions per
  // 4 steps, 607 -> 471 us per launch, profiles/r05u_pg_factored_ab.txt.  Strength-reducing the
  // per-step history addresses as well moved 54 SALU instructions onto 16 more VALU ones: 510 us.)
  using f2 = __attribute__((ext_vector_type(2))) float;
  f2 kk[SLOTS][2], lw[SLOTS][FL][2];
  float4 vv[SLOTS];
  f2 aG[SLOTS][2], aR[SLOTS][2], aW[SLOTS][FL][2];
  float esum[SLOTS];
  bool m1[SLOTS];
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  const f2 z2 = {0.f, 0.f};
#pragma unroll
  for (int s = 0; s < SLOTS; ++s) {
    const int c = lane + 64 * s;
    m1[s] = c < Q1;
    const int c1 = min(c, Q1 - 1), c2 = min(max(c - Q1, 0), p.D2 / 4 - 1);
    // the step-independent part of tanh's exponent argument, pre-scaled: exp(2x) = 2^(kE x)
    const float4 k4 = m1[s] ? reinterpret_cast<const float4*>(p.K1 + bn * p.D1)[c1]
                            : reinterpret_cast<const float4*>(p.K2 + bn * p.D2)[c2];
    const float4 b4 = (m1[s] && p.b1) ? reinterpret_cast<const float4*>(p.b1)[c1] : z4;
    kk[s][0] = f2{kE * (k4.x + b4.x), kE * (k4.y + b4.y)};
    kk[s][1] = f2{kE * (k4.z + b4.z), kE * (k4.w + b4.w)};
    vv[s] = m1[s] ? reinterpret_cast<const float4*>(p.v1)[c1] : reinterpret_cast<const float4*>(p.v2)[c2];
#pragma unroll
    for (int f = 0; f < F; ++f) {
      const float4 w4 = m1[s] ? reinterpret_cast<const float4*>(p.locW + (int64_t)f * p.D1)[c1] : z4;
      lw[s][f][0] = f2{kE * w4.x, kE * w4.y};
      lw[s][f][1] = f2{kE * w4.z, kE * w4.w};
    }
    aG[s][0] = aG[s][1] = aR[s][0] = aR[s][1] = z2;
#pragma unroll
    for (int f = 0; f < FL; ++f) aW[s][f][0] = aW[s][f][1] = z2;
    esum[s] = 0.f;
  }
  // location-conv roles: lane < KW*F owns (j, f) of convW, the next F lanes own convb
  const int nconv = F > 0 ? p.KW * F : 0;
  const int cj = F > 0 ? lane / FL : 0, cf = F > 0 ? lane - cj * FL : 0;
  float acw = 0.f;
  // the step loop is latency-bound (a handful of dependent loads per step): issue the loads of
  // kU steps at once, then do their arithmetic
  constexpr int kU = 4;
  const f2 kE2 = {kE, kE};
  for (int t0 = t_lo; t0 < t_hi; t0 += kU) {
    float e1s[kU], e2s[kU], fls[kU][FL], sv[kU], dfv[kU];
    float4 qv[kU][SLOTS];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int t = min(t0 + u, t_hi - 1);
      const bool on = t0 + u < t_hi;
      const int64_t tb = (int64_t)t * TBN + bn;
      e1s[u] = on ? p.de1[tb] : 0.f;       // a step past T contributes exactly zero
      e2s[u] = on ? p.de2[tb] : 0.f;
#pragma unroll
      for (int f = 0; f < F; ++f) fls[u][f] = p.loc[tb * F + f];
      const float* qt = p.q + (int64_t)t * p.q_tstride + (int64_t)b * p.q_bstride;
#pragma unroll
      for (int s = 0; s < SLOTS; ++s)
        qv[u][s] = reinterpret_cast<const float4*>(qt)[min(lane + 64 * s, Q - 1)];
      sv[u] = 0.f; dfv[u] = 0.f;
      if (F > 0 && on && lane < nconv + F) {
        if (lane < nconv) {
          const int m = nn + cj - padl;
          sv[u] = (m >= 0 && m < p.N) ? p.s_prev[(int64_t)t * p.s_tstride + (int64_t)b * p.N + m] : 0.f;
          dfv[u] = p.df[tb * F + cf];
        } else {
          sv[u] = 1.f;
          dfv[u] = p.df[tb * F + (lane - nconv)];
        }
      }
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      acw = fmaf(sv[u], dfv[u], acw);
#pragma unroll
      for (int s = 0; s < SLOTS; ++s) {
        f2 pr[2] = {__builtin_elementwise_fma(kE2, f2{qv[u][s].x, qv[u][s].y}, kk[s][0]),
                    __builtin_elementwise_fma(kE2, f2{qv[u][s].z, qv[u][s].w}, kk[s][1])};
#pragma unroll
        for (int f = 0; f < F; ++f) {
          const f2 fl = {fls[u][f], fls[u][f]};
          pr[0] = __builtin_elementwise_fma(fl, lw[s][f][0], pr[0]);
          pr[1] = __builtin_elementwise_fma(fl, lw[s][f][1], pr[1]);
        }
        const float e = m1[s] ? e1s[u] : e2s[u];
        esum[s] += e;
        const f2 ee = {e, e};
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const f2 r = {__builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(pr[h].x)),
                        __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(pr[h].y))};
          const f2 g = __builtin_elementwise_fma(-r, r, r);          // r (1 - r)
          aG[s][h] = __builtin_elementwise_fma(ee, g, aG[s][h]);
          aR[s][h] = __builtin_elementwise_fma(ee, r, aR[s][h]);
#pragma unroll
          for (int f = 0; f < F; ++f) {
            const float fe = fls[u][f] * e;
            aW[s][f][h] = __builtin_elementwise_fma(f2{fe, fe}, g, aW[s][f][h]);
          }
        }
      }
    }
  }
  // the step-independent factors: dK = 4 v sum e g, dv = sum e - 2 sum e r, dW_loc = 4 v sum f e g
  float4 adk[SLOTS], adv[SLOTS], adw[SLOTS][FL];
#pragma unroll
  for (int s = 0; s < SLOTS; ++s) {
    const float4 v4 = make_float4(4.f * vv[s].x, 4.f * vv[s].y, 4.f * vv[s].z, 4.f * vv[s].w);
    adk[s] = make_float4(v4.x * aG[s][0].x, v4.y * aG[s][0].y, v4.z * aG[s][1].x, v4.w * aG[s][1].y);
    adv[s] = make_float4(fmaf(-2.f, aR[s][0].x, esum[s]), fmaf(-2.f, aR[s][0].y, esum[s]),
                         fmaf(-2.f, aR[s][1].x, esum[s]), fmaf(-2.f, aR[s][1].y, esum[s]));
#pragma unroll
    for (int f = 0; f < FL; ++f)
      adw[s][f] = make_float4(v4.x * aW[s][f][0].x, v4.y * aW[s][f][0].y, v4.z * aW[s][f][1].x,
                              v4.w * aW[s][f][1].y);
  }
  attn_pg_store<SLOTS, F>(p, adk, adv, adw, acw);
}

// outputs of the parameter-gradient passes: dK rows (overwrite); partial parameter row of the
// workgroup (its 4 positions, one per wave)
template <int SLOTS, int F>
__device__ __forceinline__ void attn_pg_store(const SatAttnParamGrad& p, const float4* adk,
                                              const float4* adv,
                                              const float4 (*adw)[F > 0 ? F : 1], float acw) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nq = (p.N + 3) / 4;
  const int rows = p.B * nq, part = blockIdx.x / rows, wgi = blockIdx.x - part * rows;
  const int b = wgi / nq, n = 4 * (wgi - b * nq) + wave;
  const bool live = n < p.N;
  // part k of a step-split launch writes its dK partial into slab k (summed by the entry point)
  const int64_t bn = (int64_t)b * p.N + min(n, p.N - 1) + (int64_t)part * p.B * p.N;
  const int Q1 = p.D1 / 4, Q = Q1 + p.D2 / 4;
  const int nconv = F > 0 ? p.KW * F : 0;
  bool ok[SLOTS], m1[SLOTS];
#pragma unroll
  for (int s = 0; s < SLOTS; ++s) { ok[s] = lane + 64 * s < Q; m1[s] = lane + 64 * s < Q1; }
  if (live) {
#pragma unroll
    for (int s = 0; s < SLOTS; ++s) {
      const int c = lane + 64 * s;
      if (!ok[s]) continue;
      if (m1[s]) reinterpret_cast<float4*>(p.dK1 + bn * p.D1)[c] = adk[s];
      else reinterpret_cast<float4*>(p.dK2 + bn * p.D2)[c - Q1] = adk[s];
    }
  }
  // pg layout: [dv1 D1][dWloc F*D1][dconvW KW*F][dconvb F][dv2 D2]
  extern __shared__ float red[];     // [4][pg_stride]
  float* r = red + wave * p.pg_stride;
  for (int i = lane; i < p.pg_stride; i += 64) r[i] = 0.f;
  __syncthreads();
  if (live) {
    const int D1 = p.D1;
    const int pconv = (1 + F) * D1, pv2 = pconv + nconv + F;
#pragma unroll
    for (int s = 0; s < SLOTS; ++s) {
      const int c = lane + 64 * s;
      if (!ok[s]) continue;
      if (m1[s]) {
        float* dv = r + 4 * c;
        dv[0] = adv[s].x; dv[1] = adv[s].y; dv[2] = adv[s].z; dv[3] = adv[s].w;
#pragma unroll
        for (int f = 0; f < F; ++f) {
          float* w = r + D1 + f * D1 + 4 * c;
          w[0] = adw[s][f].x; w[1] = adw[s][f].y; w[2] = adw[s][f].z; w[3] = adw[s][f].w;
        }
      } else {
        float* dv = r + pv2 + 4 * (c - Q1);
        dv[0] = adv[s].x; dv[1] = adv[s].y; dv[2] = adv[s].z; dv[3] = adv[s].w;
      }
    }
    if (F > 0 && lane < nconv + F) r[pconv + lane] = acw;
  }
  __syncthreads();
  float* out = p.pg + (int64_t)blockIdx.x * p.pg_stride;
  for (int i = threadIdx.x; i < p.pg_stride; i += 256) {
    const int ps = p.pg_stride;
    out[i] = (red[i] + red[ps + i]) + (red[2 * ps + i] + red[3 * ps + i]);
  }
}

// One launch over the (utterance, 4-position) workgroups.  (Round 3 also built a variant that
// streamed z from the forward's ZH history instead of recomputing it, alone and mixed per
// workgroup: no step gain at the same occupancy; removed.)
template <int SLOTS, int F>
__global__ void __launch_bounds__(256) attn_param_grad_kernel(SatAttnParamGrad p) {
  pg_recompute_body<SLOTS, F>(p);
}

template <int NT, int WAVES>
void launch_attn_bwd(const AttnBwdP& p, int F, int blocks, hipStream_t s) {
  const dim3 g(blocks), blk(64 * WAVES);
  switch (F) {
    case 0: hipLaunchKernelGGL((attn_bwd_kernel<NT, 0, WAVES>), g, blk, 0, s, p); break;
    case 1: hipLaunchKernelGGL((attn_bwd_kernel<NT, 1, WAVES>), g, blk, 0, s, p); break;
    case 2: hipLaunchKernelGGL((attn_bwd_kernel<NT, 2, WAVES>), g, blk, 0, s, p); break;
    case 3: hipLaunchKernelGGL((attn_bwd_kernel<NT, 3, WAVES>), g, blk, 0, s, p); break;
    case 4: hipLaunchKernelGGL((attn_bwd_kernel<NT, 4, WAVES>), g, blk, 0, s, p); break;
    case 5: hipLaunchKernelGGL((attn_bwd_kernel<NT, 5, WAVES>), g, blk, 0, s, p); break;
    case 6: hipLaunchKernelGGL((attn_bwd_kernel<NT, 6, WAVES>), g, blk, 0, s, p); break;
    case 7: hipLaunchKernelGGL((attn_bwd_kernel<NT, 7, WAVES>), g, blk, 0, s, p); break;
    default: hipLaunchKernelGGL((attn_bwd_kernel<NT, 8, WAVES>), g, blk, 0, s, p); break;
  }
}

}  // namespace
}  // namespace sat

using namespace sat;

extern "C" int sat_attn_pg_stride(int32_t D1, int32_t D2, int32_t F, int32_t KW) {
  return (D1 + F * D1 + KW * F + F + D2 + 3) / 4 * 4;
}

extern "C" int sat_attn_param_grad_rows(int32_t B, int32_t N) { return B * ((N + 3) / 4); }

namespace sat {
namespace {
// dK[0] = dK[0] + dK[1] + ... + dK[k-1] over the slabs of a step-split launch (fixed order)
__global__ void __launch_bounds__(256) pg_slab_sum_kernel(float4* dK, int64_t n4, int k) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x) {
    float4 a = dK[i];
    for (int s = 1; s < k; ++s) {
      const float4 v = dK[s * n4 + i];
      a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
    dK[i] = a;
  }
}
}  // namespace
}  // namespace sat

extern "C" int sat_attn_param_grads(const SatAttnParamGrad* a, void* stream) {
  SAT_CHECK_ARG(a && a->T > 0 && a->B > 0 && a->N > 0, "sat_attn_param_grads: bad sizes");
  SAT_CHECK_ARG(a->tsplit >= 0 && a->tsplit <= 8 && std::max(1, a->tsplit) <= a->T,
                "sat_attn_param_grads: tsplit in 0..8 and <= T");
  SAT_CHECK_ARG(a->D1 % 4 == 0 && a->D2 % 4 == 0 && a->D1 > 0 && a->D2 > 0 &&
                (a->D1 + a->D2) / 4 <= 128, "sat_attn_param_grads: D1, D2 multiples of 4, D1+D2 <= 512");
  const int F = a->att1_forward ? a->F : 0, KW = a->att1_forward ? a->KW : 0;
  // compiled variants: F = 0 (any width), F = 5 with D1 + D2 <= 256, F = 8 (the loc history's
  // row stride is the template's F, so any other F would be read with the wrong stride)
  SAT_CHECK_ARG(F == 0 || F == 8 || (F == 5 && (a->D1 + a->D2) <= 256),
                "sat_attn_param_grads: location features F must be 0, 8 or 5 (D1 + D2 <= 256)");
  SAT_CHECK_ARG(KW * F + F <= 64, "sat_attn_param_grads: location conv needs KW*F + F <= 64");
  SAT_CHECK_ARG(a->pg_stride >= sat_attn_pg_stride(a->D1, a->D2, F, KW) && a->pg_stride <= 8192,
                "sat_attn_param_grads: pg stride");
  SAT_CHECK_ARG(a->K1 && a->K2 && a->q && a->v1 && a->v2 && a->de1 && a->de2 && a->dK1 &&
                a->dK2 && a->pg, "sat_attn_param_grads: null pointer");
  SAT_CHECK_ARG(F == 0 || (a->locW && a->loc && a->s_prev && a->df),
                "sat_attn_param_grads: forward attention needs loc / s_prev / df histories");
  SAT_CHECK_ARG(aligned16(a->K1) && aligned16(a->K2) && aligned16(a->q) && aligned16(a->v1) &&
                aligned16(a->v2) && aligned16(a->dK1) && aligned16(a->dK2) &&
                (!a->b1 || aligned16(a->b1)) && (!a->locW || aligned16(a->locW)) &&
                a->q_tstride % 4 == 0 && a->q_bstride % 4 == 0,
                "sat_attn_param_grads: 16-byte aligned operands");
  SatAttnParamGrad p = *a;
  p.F = F; p.KW = KW;
  const int slots = ((a->D1 + a->D2) / 4 + 63) / 64;
  const int ts = std::max(1, a->tsplit);
  const dim3 grid(ts * sat_attn_param_grad_rows(a->B, a->N));
  const size_t shm = 4 * (size_t)a->pg_stride * sizeof(float);
  hipStream_t s = as_stream(stream);
  if (slots == 1 && F == 5) hipLaunchKernelGGL((attn_param_grad_kernel<1, 5>), grid, dim3(256), shm, s, p);
  else if (slots == 1 && F == 0) hipLaunchKernelGGL((attn_param_grad_kernel<1, 0>), grid, dim3(256), shm, s, p);
  else if (F == 0) hipLaunchKernelGGL((attn_param_grad_kernel<2, 0>), grid, dim3(256), shm, s, p);
  else hipLaunchKernelGGL((attn_param_grad_kernel<2, 8>), grid, dim3(256), shm, s, p);
  SAT_LAUNCH_CHECK("sat_attn_param_grads");
  if (ts > 1) {
    const int64_t n1 = (int64_t)a->B * a->N * a->D1 / 4, n2 = (int64_t)a->B * a->N * a->D2 / 4;
    hipLaunchKernelGGL(pg_slab_sum_kernel, dim3((unsigned)std::min<int64_t>((n1 + 255) / 256, 2048)),
                       dim3(256), 0, s, reinterpret_cast<float4*>(a->dK1), n1, ts);
    hipLaunchKernelGGL(pg_slab_sum_kernel, dim3((unsigned)std::min<int64_t>((n2 + 255) / 256, 2048)),
                       dim3(256), 0, s, reinterpret_cast<float4*>(a->dK2), n2, ts);
    SAT_LAUNCH_CHECK("sat_attn_param_grads (dK slabs)");
  }
  return SAT_OK;
}

extern "C" int sat_attn_step_bwd(const SatAttnStepBwd* a, void* stream) {
  SAT_CHECK_ARG(a && a->B > 0 && a->N > 0 && a->N <= kMaxN, "sat_attn_step_bwd: bad sizes (N <= 1024)");
  SAT_CHECK_ARG(a->D1 <= kMaxD && a->D2 <= 64 && a->M2 <= 64 && a->M1 + a->M2 <= 2 * kMaxD,
                "sat_attn_step_bwd: D1 <= 256, D2 <= 64");
  SAT_CHECK_ARG(a->M1 <= 256 && a->M1 > 0 && a->M2 > 0 && a->D1 > 0 && a->D2 > 0,
                "sat_attn_step_bwd: M1 <= 256");
  SAT_CHECK_ARG((a->NT == 8 || a->NT == 16 || a->NT == 32) && a->ntiles == ceil_div(a->N, a->NT),
                "sat_attn_step_bwd: tile size must be 8, 16 or 32");
  SAT_CHECK_ARG(!a->att1_forward || (a->F <= kMaxFb && a->KW <= kMaxKW),
                "sat_attn_step_bwd: location conv too large (F <= 8)");
  SAT_CHECK_ARG(a->dctx && a->ctx_t && a->V1 && a->V2 && a->s_t && a->a_t && a->s2_t && a->q &&
                a->K1 && a->K2 && a->v1 && a->v2 && a->de1_out && a->de2_out && a->dqp,
                "sat_attn_step_bwd: null pointer");
  SAT_CHECK_ARG(!a->att1_forward || (a->a_prev && a->s_prev && a->stats && a->convW &&
                                     a->convb && a->locW && a->y_out && a->df_out &&
                                     (a->y_next == nullptr) == (a->df_next == nullptr)),
                "sat_attn_step_bwd: forward attention state missing");
  AttnBwdP p;
  p.B = a->B; p.N = a->N; p.D1 = a->D1; p.M1 = a->M1; p.D2 = a->D2; p.M2 = a->M2; p.F = a->F;
  p.KW = a->KW; p.NT = a->NT; p.ntiles = a->ntiles; p.att1_forward = a->att1_forward; p.u = a->u;
  p.dctx = a->dctx; p.dctx_sb = a->dctx_sb; p.ctx_t = a->ctx_t; p.ctx_sb = a->ctx_sb;
  p.y_next = a->att1_forward ? a->y_next : nullptr;
  p.V1 = a->V1; p.V2 = a->V2;
  p.s_t = a->s_t; p.a_t = a->a_t; p.a_prev = a->a_prev; p.s_prev = a->s_prev; p.s2_t = a->s2_t;
  p.stats = a->stats; p.df_next = a->df_next; p.q = a->q; p.q_sb = a->q_sb;
  p.K1 = a->K1; p.K2 = a->K2; p.v1 = a->v1; p.b1 = a->b1; p.convW = a->convW; p.convb = a->convb;
  p.locW = a->locW; p.v2 = a->v2; p.y_out = a->y_out; p.df_out = a->df_out;
  p.de1_out = a->de1_out; p.de2_out = a->de2_out; p.dqp = a->dqp;

  hipStream_t s = as_stream(stream);
  const int blocks = a->B * a->ntiles;
  const int F = a->att1_forward ? a->F : 0;
  // waves per block: 0 = default (16: two positions per wave at NT = 32, measured fastest);
  // the tile size picks the per-wave position count
  const int waves = a->waves == 0 ? 16 : a->waves;
  SAT_CHECK_ARG(waves == 4 || waves == 8 || waves == 16, "sat_attn_step_bwd: waves in {4, 8, 16}");
  SAT_CHECK_ARG(a->NT >= waves || a->NT == 8, "sat_attn_step_bwd: NT >= waves");
  if (a->NT == 8) launch_attn_bwd<8, 4>(p, F, blocks, s);
  else if (a->NT == 16) {
    if (waves == 4) launch_attn_bwd<16, 4>(p, F, blocks, s);
    else if (waves == 8) launch_attn_bwd<16, 8>(p, F, blocks, s);
    else launch_attn_bwd<16, 16>(p, F, blocks, s);
  } else {
    if (waves == 4) launch_attn_bwd<32, 4>(p, F, blocks, s);
    else if (waves == 8) launch_attn_bwd<32, 8>(p, F, blocks, s);
    else launch_attn_bwd<32, 16>(p, F, blocks, s);
  }
  SAT_LAUNCH_CHECK("sat_attn_step_bwd");
  return SAT_OK;
}
