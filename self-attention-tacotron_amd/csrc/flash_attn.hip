// Fused causal scaled-dot-product attention for the decoder head's self-attention
// (RNNTransformer, modules/module.py:743-765, use_subsequent_mask=True; the mechanism is
// ScaledDotProductAttentionMechanism, modules/self_attention.py:45-65): per (utterance, head)
// P = softmax(Q K^T / sqrt(dh) + causal mask), Pd = P * probs_mask (dropout), O = Pd V --
// WITHOUT materialising the [L][L] scores / probabilities.  Head width dh = 128, fp32 MFMA
// (v_mfma_f32_16x16x4_f32: exact fp32 products, the fp32 vector rate).
//
// Layout of the work (all three kernels):
//  * one wave owns 16 rows of the [L][L] score matrix -- 16 queries (forward, dQ) or 16 keys
//    (dK / dV) -- and keeps its own operand rows (32 of the 128 head columns per lane) and its
//    accumulators in registers for the whole launch;
//  * a workgroup = 4 waves = 64 consecutive rows of one (utterance, head); the other operand's
//    rows stream through LDS in stages of 32 (double-buffered, rows padded to 132 floats so the
//    16 rows a lane group reads sit in distinct banks);
//  * every 16 x 16 score tile is formed TRANSPOSED relative to the rows the wave owns, so the
//    softmax statistics of a row live in one lane (plus a 4-lane-group reduction for the max),
//    and the tile's registers are directly the k-operand of the next MFMA (the tile's rows are
//    the lane's 4 registers x 4 lane groups = the MFMA's k index): no LDS round trip for P / dS;
//  * causal: tiles wholly above the diagonal are skipped; the longest rows are dispatched first
//    and the shortest last, so the two co-resident workgroups of a CU carry equal work.
//
// Forward stores O and the row statistic lse = max + log2(sum) (log2 domain of the scaled
// scores); the backward recomputes P from it: a small pass forms delta = rowsum(dO * O) (the
// softmax-backward row term), then ONE launch runs both roles -- dQ (query-owned rows) and
// dK / dV (key-owned rows).
// Numerics: fp32 throughout; the online softmax and the per-tile split of the 128-long dot
// products change the summation order against the materialised path (sat_softmax_fwd + GEMMs),
// not the precision.
#include "sat_common.h"

namespace sat {
namespace {

constexpr int FD = 128;      // head width
constexpr int ST = 32;       // streamed rows per LDS stage
constexpr int RS = FD + 4;   // LDS row stride (floats)
constexpr float kLog2e = 1.4426950408889634f;

using f32x4 = __attribute__((ext_vector_type(4))) float;

struct FlashP {
  int B, H, L, nblk;          // nblk = ceil(L / 64) row blocks per (utterance, head)
  int causal;                 // (the dh = 128 kernels are causal only)
  float c;                    // scale * log2(e): exponent factor of the raw scores
  float scale;                // 1 / sqrt(dh)
  int64_t ld;                 // row stride of q, k, v, o, dout, dq, dk, dv ([B][L][ld], head h at h*128)
  const float* q; const float* k; const float* v;
  const float* mask;          // [B][H][L][L] dropout mask values (0 or 1/keep), NULL = none
  float* o; float* lse;       // forward outputs; lse [B][H][L]
  const float* dout;          // dL/dO
  float* delta;               // [B][H][L]: rowsum(dO * O), written by the dQ kernel
  float* dq; float* dk; float* dv;
};

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// reductions over the 4 lane groups of 16 (lanes l, l^16, l^32, l^48): v_permlane16/32_swap
__device__ __forceinline__ float grp4_max(float x) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  x = fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
  const auto t = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(t[0]), __uint_as_float(t[1]));
}
__device__ __forceinline__ float grp4_sum(float x) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  x = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  const auto t = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(t[0]) + __uint_as_float(t[1]);
}

// row block of this workgroup, longest first then shortest: with 2 workgroups per CU the
// dispatcher's in-order placement pairs block j with block nblk-1-j
__device__ __forceinline__ int block_order(int blk, int nblk, bool heavy_high) {
  const int half = (nblk + 1) / 2;
  const int r = blk < half ? blk : nblk - 1 - (blk - half);   // 0, 1, .., then nblk-1, nblk-2, ..
  return heavy_high ? nblk - 1 - r : r;
}

// 32 consecutive floats of a row (head columns [32 g, 32 g + 32)) into registers
__device__ __forceinline__ void load_row32(float (&r)[32], const float* src, bool ok) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float4 x = ok ? *reinterpret_cast<const float4*>(src + 4 * j) : make_float4(0.f, 0.f, 0.f, 0.f);
    r[4 * j] = x.x; r[4 * j + 1] = x.y; r[4 * j + 2] = x.z; r[4 * j + 3] = x.w;
  }
}

// a stage of ST rows x 128 columns of two [B][L][ld] operands: 256 threads x 4 float4 each
struct Stage2 {
  float4 a[4], b[4];
  __device__ __forceinline__ void load(const float* pa, const float* pb, int64_t ld, int row0, int L,
                                       int tid) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int idx = tid + 256 * r, row = row0 + (idx >> 5), c4 = idx & 31;
      const bool ok = row < L;
      a[r] = ok ? *reinterpret_cast<const float4*>(pa + row * ld + 4 * c4) : make_float4(0.f, 0.f, 0.f, 0.f);
      b[r] = ok ? *reinterpret_cast<const float4*>(pb + row * ld + 4 * c4) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  __device__ __forceinline__ void store(float* sa, float* sb, int tid) const {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int idx = tid + 256 * r, row = idx >> 5, c4 = idx & 31;
      *reinterpret_cast<float4*>(sa + row * RS + 4 * c4) = a[r];
      *reinterpret_cast<float4*>(sb + row * RS + 4 * c4) = b[r];
    }
  }
};

// T[m][n] = sum_d A[row m][d] R[n][d] for the 16 x 16 tile whose A rows (16, stride RS) sit in
// LDS at `a` and whose R rows are the lanes' registers (lane (n, g) holds R[n][32 g + s]);
// the lane gets T[4 g + i][n], i = 0..3.  Two accumulators break the MFMA's 40-cycle
// dependent latency (32-cycle issue).
__device__ __forceinline__ f32x4 tile_dot(const float* a, const float (&r)[32], int n, int g) {
  f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = {0.f, 0.f, 0.f, 0.f};
  const float* ar = a + n * RS + 32 * g;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float4 x = *reinterpret_cast<const float4*>(ar + 4 * j);
    s0 = mfma4(x.x, r[4 * j], s0);
    s1 = mfma4(x.y, r[4 * j + 1], s1);
    s0 = mfma4(x.z, r[4 * j + 2], s0);
    s1 = mfma4(x.w, r[4 * j + 3], s1);
  }
  return s0 + s1;
}

// acc[t][i] += sum_s A[4 g + s][16 t + n] * w[s] over the 16 streamed rows at `a` (stride RS):
// the transposed product whose k index is the tile's row (the lane's registers w)
__device__ __forceinline__ void tile_acc(f32x4 (&acc)[8], const float* a, const float (&w)[4], int n,
                                         int g) {
  const float* ar = a + 4 * g * RS + n;
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int t = 0; t < 8; ++t) acc[t] = mfma4(ar[s * RS + 16 * t], w[s], acc[t]);
}

// ---------------------------------------------------------------- forward
__global__ void __launch_bounds__(256) flash_fwd_kernel(FlashP p) {
  __shared__ __attribute__((aligned(16))) float ks[2][ST * RS];
  __shared__ __attribute__((aligned(16))) float vs[2][ST * RS];
  const int nbh = p.B * p.H, bh = blockIdx.x % nbh;
  const int qb = block_order(blockIdx.x / nbh, p.nblk, true);
  const int b = bh / p.H, h = bh % p.H, L = p.L;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, n = lane & 15, g = lane >> 4;
  const int Q0 = qb * 64, q0 = Q0 + 16 * w, qi = q0 + n;
  const int64_t base = (int64_t)b * L * p.ld + h * FD;
  const float* kp = p.k + base;
  const float* vp = p.v + base;
  const float* mrow = p.mask ? p.mask + ((int64_t)bh * L + (qi < L ? qi : 0)) * L : nullptr;
  float qr[32];
  load_row32(qr, p.q + base + (int64_t)qi * p.ld + 32 * g, qi < L);
  f32x4 acc[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.f;
  const int nst = (min(L, Q0 + 64) - 1) / ST + 1;
  Stage2 stg;
  stg.load(kp, vp, p.ld, 0, L, tid);
  stg.store(ks[0], vs[0], tid);
  __syncthreads();
  for (int st = 0; st < nst; ++st) {
    const int buf = st & 1;
    if (st + 1 < nst) stg.load(kp, vp, p.ld, (st + 1) * ST, L, tid);
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      const int key0 = st * ST + sub * 16;
      if (key0 <= q0 + 15) {          // wave-uniform: key0 <= q0, every lane has a valid key
        const int kk = key0 + 4 * g;
        float4 mk = make_float4(1.f, 1.f, 1.f, 1.f);
        if (mrow) mk = kk < L ? *reinterpret_cast<const float4*>(mrow + kk) : make_float4(0.f, 0.f, 0.f, 0.f);
        const f32x4 sv = tile_dot(ks[buf] + sub * 16 * RS, qr, n, g);
        float sc[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) sc[i] = kk + i > qi ? -INFINITY : sv[i] * p.c;
        const float mt = grp4_max(fmaxf(fmaxf(sc[0], sc[1]), fmaxf(sc[2], sc[3])));
        const float mn = fmaxf(m, mt);
        const float alpha = __builtin_amdgcn_exp2f(m - mn);
        const float mkv[4] = {mk.x, mk.y, mk.z, mk.w};
        float pd[4], ps = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float e = __builtin_amdgcn_exp2f(sc[i] - mn);
          ps += e;
          pd[i] = e * mkv[i];
        }
        l = l * alpha + ps;
        m = mn;
#pragma unroll
        for (int t = 0; t < 8; ++t) acc[t] *= alpha;
        tile_acc(acc, vs[buf] + sub * 16 * RS, pd, n, g);
      }
    }
    if (st + 1 < nst) stg.store(ks[buf ^ 1], vs[buf ^ 1], tid);
    __syncthreads();
  }
  const float lt = grp4_sum(l);
  if (qi < L) {
    const float inv = 1.f / lt;
    float* orow = p.o + base + (int64_t)qi * p.ld + 4 * g;
#pragma unroll
    for (int t = 0; t < 8; ++t)
      *reinterpret_cast<float4*>(orow + 16 * t) =
          make_float4(acc[t][0] * inv, acc[t][1] * inv, acc[t][2] * inv, acc[t][3] * inv);
    if (g == 0) p.lse[(int64_t)bh * L + qi] = m + __log2f(lt);
  }
}

// ---------------------------------------------------------------- backward: delta
// delta_q = sum_j Pd_qj dPd_qj = dO_q . O_q per (utterance, head, query), the softmax-backward
// row term both backward roles read (same lane layout as the roles: lane (n, g) sums head
// columns [32 g, 32 g + 32) of row q0 + n, then the 4-group sum)
__global__ void __launch_bounds__(256) flash_delta_kernel(FlashP p) {
  const int nbh = p.B * p.H, bh = blockIdx.x % nbh, qb = blockIdx.x / nbh;
  const int b = bh / p.H, h = bh % p.H, L = p.L;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, n = lane & 15, g = lane >> 4;
  const int qi = qb * 64 + 16 * w + n;
  const bool qok = qi < L;
  const int64_t roff = (int64_t)b * L * p.ld + h * FD + (int64_t)qi * p.ld + 32 * g;
  float dor[32], orr[32];
  load_row32(dor, p.dout + roff, qok);
  load_row32(orr, p.o + roff, qok);
  float part = 0.f;
#pragma unroll
  for (int s = 0; s < 32; ++s) part = fmaf(dor[s], orr[s], part);
  const float dl = grp4_sum(part);
  if (qok && g == 0) p.delta[(int64_t)bh * L + qi] = dl;
}

// ---------------------------------------------------------------- backward: dQ
// dS = scale * P * (dPd * mask - delta)
__device__ __forceinline__ void flash_bwd_dq(const FlashP& p, int bh, int qb, float* smem) {
  float (*ks)[ST * RS] = reinterpret_cast<float (*)[ST * RS]>(smem);
  float (*vs)[ST * RS] = reinterpret_cast<float (*)[ST * RS]>(smem + 2 * ST * RS);
  const int b = bh / p.H, h = bh % p.H, L = p.L;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, n = lane & 15, g = lane >> 4;
  const int Q0 = qb * 64, q0 = Q0 + 16 * w, qi = q0 + n;
  const bool qok = qi < L;
  const int64_t base = (int64_t)b * L * p.ld + h * FD;
  const float* kp = p.k + base;
  const float* vp = p.v + base;
  const float* mrow = p.mask ? p.mask + ((int64_t)bh * L + (qok ? qi : 0)) * L : nullptr;
  const int64_t roff = base + (int64_t)qi * p.ld + 32 * g;
  float qr[32], dor[32];
  load_row32(qr, p.q + roff, qok);
  load_row32(dor, p.dout + roff, qok);
  const float dl = qok ? p.delta[(int64_t)bh * L + qi] : 0.f;
  const float ls = qok ? p.lse[(int64_t)bh * L + qi] : 0.f;
  f32x4 acc[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nst = (min(L, Q0 + 64) - 1) / ST + 1;
  Stage2 stg;
  stg.load(kp, vp, p.ld, 0, L, tid);
  stg.store(ks[0], vs[0], tid);
  __syncthreads();
  for (int st = 0; st < nst; ++st) {
    const int buf = st & 1;
    if (st + 1 < nst) stg.load(kp, vp, p.ld, (st + 1) * ST, L, tid);
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      const int key0 = st * ST + sub * 16;
      if (key0 <= q0 + 15) {
        const int kk = key0 + 4 * g;
        float4 mk = make_float4(1.f, 1.f, 1.f, 1.f);
        if (mrow) mk = kk < L ? *reinterpret_cast<const float4*>(mrow + kk) : make_float4(0.f, 0.f, 0.f, 0.f);
        const float mkv[4] = {mk.x, mk.y, mk.z, mk.w};
        const f32x4 sv = tile_dot(ks[buf] + sub * 16 * RS, qr, n, g);
        const f32x4 gv = tile_dot(vs[buf] + sub * 16 * RS, dor, n, g);   // dPd^T = V dO^T
        float ds[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float pv = kk + i > qi ? 0.f : __builtin_amdgcn_exp2f(sv[i] * p.c - ls);
          ds[i] = pv * (gv[i] * mkv[i] - dl) * p.scale;
        }
        tile_acc(acc, ks[buf] + sub * 16 * RS, ds, n, g);               // dQ^T += K^T dS^T
      }
    }
    if (st + 1 < nst) stg.store(ks[buf ^ 1], vs[buf ^ 1], tid);
    __syncthreads();
  }
  if (qok) {
    float* drow = p.dq + base + (int64_t)qi * p.ld + 4 * g;
#pragma unroll
    for (int t = 0; t < 8; ++t)
      *reinterpret_cast<float4*>(drow + 16 * t) = make_float4(acc[t][0], acc[t][1], acc[t][2], acc[t][3]);
  }
}

// ---------------------------------------------------------------- backward: dK, dV
__device__ __forceinline__ void flash_bwd_dkdv(const FlashP& p, int bh, int kb, float* smem) {
  float (*qs)[ST * RS] = reinterpret_cast<float (*)[ST * RS]>(smem);
  float (*gs)[ST * RS] = reinterpret_cast<float (*)[ST * RS]>(smem + 2 * ST * RS);
  float (*lss)[ST] = reinterpret_cast<float (*)[ST]>(smem + 4 * ST * RS);
  float (*dls)[ST] = reinterpret_cast<float (*)[ST]>(smem + 4 * ST * RS + 2 * ST);
  const int b = bh / p.H, h = bh % p.H, L = p.L;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, n = lane & 15, g = lane >> 4;
  const int K0 = kb * 64, k0 = K0 + 16 * w, kj = k0 + n;
  const bool kok = kj < L;
  const int64_t base = (int64_t)b * L * p.ld + h * FD;
  const float* qp = p.q + base;
  const float* gp = p.dout + base;
  const float* mcol = p.mask ? p.mask + (int64_t)bh * L * L + (kok ? kj : 0) : nullptr;
  const int64_t roff = base + (int64_t)kj * p.ld + 32 * g;
  float kr[32], vr[32];
  load_row32(kr, p.k + roff, kok);
  load_row32(vr, p.v + roff, kok);
  f32x4 ak[8], av[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    ak[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    av[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const int st0 = K0 / ST, nst = (L - 1) / ST + 1;
  const float* lsep = p.lse + (int64_t)bh * L;
  const float* delp = p.delta + (int64_t)bh * L;
  Stage2 stg;
  float sl = 0.f, sd = 0.f;
  auto load_rows = [&](int st) {
    stg.load(qp, gp, p.ld, st * ST, L, tid);
    if (tid < ST) {
      const int r = st * ST + tid;
      sl = r < L ? lsep[r] : INFINITY;
      sd = r < L ? delp[r] : 0.f;
    }
  };
  auto store_rows = [&](int buf) {
    stg.store(qs[buf], gs[buf], tid);
    if (tid < ST) {
      lss[buf][tid] = sl;
      dls[buf][tid] = sd;
    }
  };
  load_rows(st0);
  store_rows(0);
  __syncthreads();
  for (int st = st0; st < nst; ++st) {
    const int buf = (st - st0) & 1;
    if (st + 1 < nst) load_rows(st + 1);
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      const int qs0 = st * ST + sub * 16;
      if (qs0 + 15 >= k0 && qs0 < L) {    // wave-uniform: some query of the tile sees a key
        const int qq = qs0 + 4 * g;        // this lane's 4 queries qq .. qq+3
        float mkv[4] = {1.f, 1.f, 1.f, 1.f};
        if (mcol) {
#pragma unroll
          for (int i = 0; i < 4; ++i) mkv[i] = qq + i < L ? mcol[(int64_t)(qq + i) * L] : 0.f;
        }
        const float* qt = qs[buf] + sub * 16 * RS;
        const float* gt = gs[buf] + sub * 16 * RS;
        const f32x4 sv = tile_dot(qt, kr, n, g);    // S[q][kj]
        const f32x4 gv = tile_dot(gt, vr, n, g);    // dPd[q][kj]
        float pd[4], ds[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = sub * 16 + 4 * g + i;
          const float pv = (qq + i < kj || !kok) ? 0.f
                                                 : __builtin_amdgcn_exp2f(sv[i] * p.c - lss[buf][r]);
          pd[i] = pv * mkv[i];
          ds[i] = pv * (gv[i] * mkv[i] - dls[buf][r]) * p.scale;
        }
        tile_acc(av, gt, pd, n, g);                 // dV^T += dO^T Pd
        tile_acc(ak, qt, ds, n, g);                 // dK^T += Q^T dS
      }
    }
    if (st + 1 < nst) store_rows(buf ^ 1);
    __syncthreads();
  }
  if (kok) {
    float* krow = p.dk + base + (int64_t)kj * p.ld + 4 * g;
    float* vrow = p.dv + base + (int64_t)kj * p.ld + 4 * g;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      *reinterpret_cast<float4*>(krow + 16 * t) = make_float4(ak[t][0], ak[t][1], ak[t][2], ak[t][3]);
      *reinterpret_cast<float4*>(vrow + 16 * t) = make_float4(av[t][0], av[t][1], av[t][2], av[t][3]);
    }
  }
}

// Both backward roles in ONE launch (they are independent once delta is known): workgroup
// index -> (row-block rank, role, utterance x head), rank-major, so the longest blocks of both
// roles are dispatched first and the shortest fill the slots they leave
__global__ void __launch_bounds__(256, 2) flash_bwd_kernel(FlashP p) {
  __shared__ __attribute__((aligned(16))) float smem[4 * ST * RS + 4 * ST];
  const int nbh = p.B * p.H, rank = blockIdx.x / (2 * nbh), within = blockIdx.x - rank * 2 * nbh;
  const int bh = within % nbh;
  if (within < nbh) flash_bwd_dkdv(p, bh, block_order(rank, p.nblk, false), smem);
  else flash_bwd_dq(p, bh, block_order(rank, p.nblk, true), smem);
}

// ---------------------------------------------------------------- narrow heads
// The encoder's self-attention (SelfAttentionCBHGEncoder, modules/module.py:425-438: 2 heads of
// 16 over the L = N <= 256 source positions, no causal mask, dropout on the probabilities): the
// whole (utterance, head) fits one workgroup's LDS, and its 200 x 200 x 16 products are far too
// small for MFMA tiles (the materialised path spends a chain of ~12 launches and four [L][L]
// tensors on it).  A workgroup = 64 rows, 4 lanes per row, lane g4 of a row takes the keys (or
// queries) g4, g4 + 4, ...; the other operand's rows of the (utterance, head) sit in LDS.
//  * forward: pass 1 streams the scaled scores into a running (max, sum) per lane, the 4 lanes
//    combine them into lse; pass 2 recomputes each score, P = 2^(s - lse), and accumulates
//    O = sum_j P mask V_j -- no per-row score array, so the kernel holds ~3 DH registers;
//  * backward, two roles in one launch: dQ (query-owned rows: dQ_i = scale sum_j dS_ij K_j) and
//    dK / dV (key-owned rows: dV_j = sum_i Pd_ij dO_i, dK_j = scale sum_i dS_ij Q_i) with
//    dS = P (mask dPd - delta), delta_i = dO_i . O_i formed where it is needed (no extra pass).
// Same lse / delta conventions as the dh = 128 kernels above (log2 domain of the scaled scores).
constexpr int kNarrowMaxL = 256;

__device__ __forceinline__ float row4_max(float x) {
  x = fmaxf(x, __shfl_xor(x, 1, 64));
  return fmaxf(x, __shfl_xor(x, 2, 64));
}
__device__ __forceinline__ float row4_sum(float x) {
  x += __shfl_xor(x, 1, 64);
  return x + __shfl_xor(x, 2, 64);
}
// running (max, sum of 2^(s - max)) of two lanes merged; an empty lane has max = -inf
__device__ __forceinline__ void lse_merge(float& m, float& z, float m2, float z2) {
  const float mn = fmaxf(m, m2);
  if (mn == -INFINITY) return;
  z = (m == -INFINITY ? 0.f : z * exp2f(m - mn)) + (m2 == -INFINITY ? 0.f : z2 * exp2f(m2 - mn));
  m = mn;
}

template <int DH>
__device__ __forceinline__ void load_head_row(float (&r)[DH], const float* src, float mul) {
#pragma unroll
  for (int c = 0; c < DH / 4; ++c) {
    const float4 x = reinterpret_cast<const float4*>(src)[c];
    r[4 * c] = mul * x.x; r[4 * c + 1] = mul * x.y; r[4 * c + 2] = mul * x.z; r[4 * c + 3] = mul * x.w;
  }
}
template <int DH>
__device__ __forceinline__ float dot_lds(const float (&r)[DH], const float* row) {
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < DH / 4; ++c) {
    const float4 x = reinterpret_cast<const float4*>(row)[c];
    s = fmaf(r[4 * c], x.x, s); s = fmaf(r[4 * c + 1], x.y, s);
    s = fmaf(r[4 * c + 2], x.z, s); s = fmaf(r[4 * c + 3], x.w, s);
  }
  return s;
}
template <int DH>
__device__ __forceinline__ void axpy_lds(float (&acc)[DH], float w, const float* row) {
#pragma unroll
  for (int c = 0; c < DH / 4; ++c) {
    const float4 x = reinterpret_cast<const float4*>(row)[c];
    acc[4 * c] = fmaf(w, x.x, acc[4 * c]); acc[4 * c + 1] = fmaf(w, x.y, acc[4 * c + 1]);
    acc[4 * c + 2] = fmaf(w, x.z, acc[4 * c + 2]); acc[4 * c + 3] = fmaf(w, x.w, acc[4 * c + 3]);
  }
}
// the row's 4 lanes sum their partial vectors; lane g4 stores its quarter (DH / 4 columns)
template <int DH>
__device__ __forceinline__ void store_row4(float (&acc)[DH], float* dst, float mul, int g4, bool live) {
#pragma unroll
  for (int d = 0; d < DH; ++d) acc[d] = row4_sum(acc[d]);
  if (!live) return;
#pragma unroll
  for (int d = 0; d < DH; ++d)
    if (d / (DH / 4) == g4) dst[d] = mul * acc[d];
}
// the (utterance, head) rows of two [B][L][ld] operands into LDS [L][DH] each
template <int DH>
__device__ __forceinline__ void stage_head(float* sa, float* sb, const float* a, const float* b,
                                           int64_t ld, int L) {
  for (int idx = threadIdx.x; idx < L * (DH / 4); idx += blockDim.x) {
    const int r = idx / (DH / 4), c = idx - r * (DH / 4);
    reinterpret_cast<float4*>(sa)[idx] = *reinterpret_cast<const float4*>(a + r * ld + 4 * c);
    reinterpret_cast<float4*>(sb)[idx] = *reinterpret_cast<const float4*>(b + r * ld + 4 * c);
  }
}

template <int DH>
__global__ void __launch_bounds__(256) narrow_fwd_kernel(FlashP p) {
  extern __shared__ __attribute__((aligned(16))) float nsm[];
  const int L = p.L;
  float* Ks = nsm;
  float* Vs = nsm + L * DH;
  const int bh = blockIdx.x / p.nblk, blk = blockIdx.x - bh * p.nblk;
  const int b = bh / p.H, h = bh - b * p.H;
  const int64_t base = (int64_t)b * L * p.ld + h * DH;
  stage_head<DH>(Ks, Vs, p.k + base, p.v + base, p.ld, L);
  const int g4 = threadIdx.x & 3, i = blk * 64 + (threadIdx.x >> 2);
  const bool live = i < L;
  const int ii = live ? i : L - 1;
  float q[DH];
  load_head_row<DH>(q, p.q + base + ii * p.ld, p.c);
  __syncthreads();
  const int lim = p.causal ? ii + 1 : L;
  float m = -INFINITY, z = 0.f;
  for (int j = g4; j < lim; j += 4) {
    const float s = dot_lds<DH>(q, Ks + j * DH);
    if (s > m) { z = z * exp2f(m - s) + 1.f; m = s; }
    else z += exp2f(s - m);
  }
  lse_merge(m, z, __shfl_xor(m, 1, 64), __shfl_xor(z, 1, 64));
  lse_merge(m, z, __shfl_xor(m, 2, 64), __shfl_xor(z, 2, 64));
  const float lse = m + log2f(z);
  const float* mrow = p.mask ? p.mask + ((int64_t)bh * L + ii) * L : nullptr;
  float acc[DH];
#pragma unroll
  for (int d = 0; d < DH; ++d) acc[d] = 0.f;
  for (int j = g4; j < lim; j += 4) {
    float w = exp2f(dot_lds<DH>(q, Ks + j * DH) - lse);
    if (mrow) w *= mrow[j];
    axpy_lds<DH>(acc, w, Vs + j * DH);
  }
  store_row4<DH>(acc, p.o + base + ii * p.ld, 1.f, g4, live);
  if (live && g4 == 0) p.lse[(int64_t)bh * L + i] = lse;
}

// dQ role: 64 query rows; K, V of the (utterance, head) in LDS
template <int DH>
__device__ __forceinline__ void narrow_bwd_dq(const FlashP& p, int bh, int blk, float* sm) {
  const int L = p.L;
  float* Ks = sm;
  float* Vs = sm + L * DH;
  const int b = bh / p.H, h = bh - b * p.H;
  const int64_t base = (int64_t)b * L * p.ld + h * DH;
  stage_head<DH>(Ks, Vs, p.k + base, p.v + base, p.ld, L);
  const int g4 = threadIdx.x & 3, i = blk * 64 + (threadIdx.x >> 2);
  const bool live = i < L;
  const int ii = live ? i : L - 1;
  const int64_t row = base + ii * p.ld;
  float q[DH], dO[DH], o[DH];
  load_head_row<DH>(q, p.q + row, p.c);
  load_head_row<DH>(dO, p.dout + row, 1.f);
  load_head_row<DH>(o, p.o + row, 1.f);
  float delta = 0.f;
#pragma unroll
  for (int d = 0; d < DH; ++d) delta = fmaf(dO[d], o[d], delta);
  const float lse = p.lse[(int64_t)bh * L + ii];
  const float* mrow = p.mask ? p.mask + ((int64_t)bh * L + ii) * L : nullptr;
  __syncthreads();
  const int lim = p.causal ? ii + 1 : L;
  float acc[DH];
#pragma unroll
  for (int d = 0; d < DH; ++d) acc[d] = 0.f;
  for (int j = g4; j < lim; j += 4) {
    const float P = exp2f(dot_lds<DH>(q, Ks + j * DH) - lse);
    const float dpd = dot_lds<DH>(dO, Vs + j * DH);
    const float mk = mrow ? mrow[j] : 1.f;
    axpy_lds<DH>(acc, P * (mk * dpd - delta), Ks + j * DH);
  }
  store_row4<DH>(acc, p.dq + row, p.scale, g4, live);
}

// dK / dV role: 64 key rows; Q, dO, lse and delta of every query row in LDS
template <int DH>
__device__ __forceinline__ void narrow_bwd_dkdv(const FlashP& p, int bh, int blk, float* sm) {
  const int L = p.L;
  float* Qs = sm;
  float* Gs = sm + L * DH;
  float* ls = sm + 2 * L * DH;
  float* dl = ls + L;
  const int b = bh / p.H, h = bh - b * p.H;
  const int64_t base = (int64_t)b * L * p.ld + h * DH;
  stage_head<DH>(Qs, Gs, p.q + base, p.dout + base, p.ld, L);
  for (int r = threadIdx.x; r < L; r += blockDim.x) {
    const float* go = p.dout + base + r * p.ld;
    const float* oo = p.o + base + r * p.ld;
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < DH / 4; ++c) {
      const float4 x = reinterpret_cast<const float4*>(go)[c], y = reinterpret_cast<const float4*>(oo)[c];
      s = fmaf(x.x, y.x, s); s = fmaf(x.y, y.y, s); s = fmaf(x.z, y.z, s); s = fmaf(x.w, y.w, s);
    }
    dl[r] = s;
    ls[r] = p.lse[(int64_t)bh * L + r];
  }
  const int g4 = threadIdx.x & 3, j = blk * 64 + (threadIdx.x >> 2);
  const bool live = j < L;
  const int jj = live ? j : L - 1;
  const int64_t row = base + jj * p.ld;
  float k[DH], v[DH];
  load_head_row<DH>(k, p.k + row, p.c);
  load_head_row<DH>(v, p.v + row, 1.f);
  __syncthreads();
  const float* mcol = p.mask ? p.mask + (int64_t)bh * L * L + jj : nullptr;
  float dk[DH], dv[DH];
#pragma unroll
  for (int d = 0; d < DH; ++d) { dk[d] = 0.f; dv[d] = 0.f; }
  for (int i = (p.causal ? jj : 0) + g4; i < L; i += 4) {
    const float P = exp2f(dot_lds<DH>(k, Qs + i * DH) - ls[i]);
    const float mk = mcol ? mcol[(int64_t)i * L] : 1.f;
    const float dpd = dot_lds<DH>(v, Gs + i * DH);
    axpy_lds<DH>(dv, P * mk, Gs + i * DH);
    axpy_lds<DH>(dk, P * (mk * dpd - dl[i]), Qs + i * DH);
  }
  store_row4<DH>(dk, p.dk + row, p.scale, g4, live);
  store_row4<DH>(dv, p.dv + row, 1.f, g4, live);
}

template <int DH>
__global__ void __launch_bounds__(256) narrow_bwd_kernel(FlashP p) {
  extern __shared__ __attribute__((aligned(16))) float nsm[];
  const int nbh = p.B * p.H, role = blockIdx.x / (nbh * p.nblk);
  const int w = blockIdx.x - role * nbh * p.nblk, bh = w / p.nblk, blk = w - bh * p.nblk;
  if (role == 0) narrow_bwd_dkdv<DH>(p, bh, blk, nsm);
  else narrow_bwd_dq<DH>(p, bh, blk, nsm);
}

bool narrow(const SatFlashAttn* a) { return a->dh != FD; }
size_t narrow_lds(const SatFlashAttn* a) { return (2 * (size_t)a->L * a->dh + 2 * a->L) * sizeof(float); }

int check(const SatFlashAttn* a, bool bwd) {
  SAT_CHECK_ARG(a != nullptr, "sat_flash_attn: null descriptor");
  if (narrow(a)) {
    SAT_CHECK_ARG(a->B > 0 && a->H > 0 && a->L > 0 && a->L <= kNarrowMaxL &&
                      (a->dh == 8 || a->dh == 16 || a->dh == 32) && (a->causal == 0 || a->causal == 1) &&
                      a->ld >= (int64_t)a->H * a->dh && a->ld % 4 == 0 && narrow_lds(a) <= 65536,
                  "sat_flash_attn: narrow heads need dh in {8, 16, 32}, L <= 256, ld >= H * dh, "
                  "ld %% 4 == 0 and (2 L dh + 2 L) * 4 <= 64 KB");
    SAT_CHECK_ARG(a->q && a->k && a->v && a->o && a->lse, "sat_flash_attn: null q / k / v / o / lse");
    SAT_CHECK_ARG(aligned16(a->q) && aligned16(a->k) && aligned16(a->v) && aligned16(a->o),
                  "sat_flash_attn: operands must be 16-byte aligned");
    if (bwd)
      SAT_CHECK_ARG(a->dout && a->dq && a->dk && a->dv && aligned16(a->dout) && aligned16(a->dq) &&
                        aligned16(a->dk) && aligned16(a->dv),
                    "sat_flash_attn_bwd: null or unaligned dout / dq / dk / dv");
    return SAT_OK;
  }
  SAT_CHECK_ARG(a->B > 0 && a->H > 0 && a->L > 0 && a->dh == FD && a->causal == 1 && a->L % 4 == 0 &&
                    a->ld >= (int64_t)a->H * FD && a->ld % 4 == 0,
                "sat_flash_attn: needs dh == 128, causal, L %% 4 == 0, ld >= H * 128, ld %% 4 == 0");
  SAT_CHECK_ARG(a->q && a->k && a->v && a->o && a->lse, "sat_flash_attn: null q / k / v / o / lse");
  SAT_CHECK_ARG(aligned16(a->q) && aligned16(a->k) && aligned16(a->v) && aligned16(a->o) &&
                    (!a->mask || aligned16(a->mask)),
                "sat_flash_attn: operands must be 16-byte aligned");
  if (bwd)
    SAT_CHECK_ARG(a->dout && a->delta && a->dq && a->dk && a->dv && aligned16(a->dout) &&
                      aligned16(a->dq) && aligned16(a->dk) && aligned16(a->dv),
                  "sat_flash_attn_bwd: null or unaligned dout / delta / dq / dk / dv");
  return SAT_OK;
}

FlashP params(const SatFlashAttn* a) {
  FlashP p;
  p.B = a->B; p.H = a->H; p.L = a->L; p.nblk = (a->L + 63) / 64;
  p.causal = a->causal;
  p.scale = a->scale > 0.f ? a->scale : 1.f / std::sqrt((float)a->dh);
  p.c = p.scale * kLog2e;
  p.ld = a->ld;
  p.q = a->q; p.k = a->k; p.v = a->v; p.mask = a->mask;
  p.o = a->o; p.lse = a->lse;
  p.dout = a->dout; p.delta = a->delta; p.dq = a->dq; p.dk = a->dk; p.dv = a->dv;
  return p;
}

}  // namespace
}  // namespace sat

using namespace sat;

extern "C" int sat_flash_attn_fwd(const SatFlashAttn* a, void* stream) {
  if (const int rc = check(a, false)) return rc;
  const FlashP p = params(a);
  if (narrow(a)) {
    const dim3 g(p.B * p.H * p.nblk);
    const size_t shm = narrow_lds(a);
    hipStream_t s = as_stream(stream);
    if (a->dh == 8) hipLaunchKernelGGL(narrow_fwd_kernel<8>, g, dim3(256), shm, s, p);
    else if (a->dh == 16) hipLaunchKernelGGL(narrow_fwd_kernel<16>, g, dim3(256), shm, s, p);
    else hipLaunchKernelGGL(narrow_fwd_kernel<32>, g, dim3(256), shm, s, p);
    SAT_LAUNCH_CHECK("sat_flash_attn_fwd (narrow)");
    return SAT_OK;
  }
  hipLaunchKernelGGL(flash_fwd_kernel, dim3(p.B * p.H * p.nblk), dim3(256), 0, as_stream(stream), p);
  SAT_LAUNCH_CHECK("sat_flash_attn_fwd");
  return SAT_OK;
}

extern "C" int sat_flash_attn_bwd(const SatFlashAttn* a, void* stream) {
  if (const int rc = check(a, true)) return rc;
  const FlashP p = params(a);
  hipStream_t s = as_stream(stream);
  if (narrow(a)) {
    const dim3 g(2 * p.B * p.H * p.nblk);
    const size_t shm = narrow_lds(a);
    if (a->dh == 8) hipLaunchKernelGGL(narrow_bwd_kernel<8>, g, dim3(256), shm, s, p);
    else if (a->dh == 16) hipLaunchKernelGGL(narrow_bwd_kernel<16>, g, dim3(256), shm, s, p);
    else hipLaunchKernelGGL(narrow_bwd_kernel<32>, g, dim3(256), shm, s, p);
    SAT_LAUNCH_CHECK("sat_flash_attn_bwd (narrow)");
    return SAT_OK;
  }
  hipLaunchKernelGGL(flash_delta_kernel, dim3(p.B * p.H * p.nblk), dim3(256), 0, s, p);
  SAT_LAUNCH_CHECK("sat_flash_attn_bwd (delta)");
  hipLaunchKernelGGL(flash_bwd_kernel, dim3(2 * p.B * p.H * p.nblk), dim3(256), 0, s, p);
  SAT_LAUNCH_CHECK("sat_flash_attn_bwd (dQ, dK, dV)");
  return SAT_OK;
}
