// fp32 GEMM on CDNA4 matrix cores: v_mfma_f32_32x32x2_f32 (exact f32, = the f32 vector peak).
//
// One kernel template serves every dense product of the path: Dense layers, batched attention
// products, the Conv1D(SAME) of the CBHG (implicit im2col in the A loader -- no im2col buffer
// in HBM) and all their gradients (transposes are strides; conv dX / dW are A/B modes).
//
// Two kernels:
//  * gemm_lds_kernel (default whenever both operands are 16-byte loadable): LDS-DMA
//    (global_load_lds_dwordx4) into a 3-stage ring, counted waits, one raw barrier per K-tile,
//    fragments of tile k+1 read into a second register set while tile k's last MFMAs run; tile
//    64/128 x 64/128 and split-K chosen per launch by a cycle model (launch_lds);
//  * gemm_kernel (register-staged, any strides / modes): BM x BN x 32 tiles, GM x GN waves,
//    global -> registers -> double-buffered LDS, one barrier per K-tile.
// Weight-gradient products (K = T' * B = 16,000 rows, M x N <= 1024 x 1024) have too few output
// tiles to fill 256 CUs: they run split-K into an fp32 workspace slab [S][M][N] and a second
// launch sums the slabs in a fixed order and applies the epilogue (deterministic, no atomics).
#include "sat_common.h"

#include <cstdlib>

namespace sat {
namespace {

using f32x16 = __attribute__((ext_vector_type(16))) float;
using f4v = __attribute__((ext_vector_type(4))) float;
using f2v = __attribute__((ext_vector_type(2))) float;

// One operand's MFMA fragments of a K-tile (16 steps x S sub-tiles of 32) in the register shape
// its LDS reads produce, so the two sets carried around the K loop stay whole register tuples:
// K-major images are read 4 steps at a time (ds_read_b128), M/N-major ones one step at a time,
// and the compiler pairs the two sub-tiles of a step (ds_read2_b32) when S = 2 or two steps
// (ds_read2st64_b32) when S = 1.  (Scalar [16][S] arrays made it re-assemble the loop-carried
// set with up to 36 v_mov per K-tile, each behind a wait on the reads just issued.)
template <int S, bool KM>
struct Frag {
  f4v v[S][4];
  __device__ __forceinline__ float get(int i, int t) const { return v[i][t >> 2][t & 3]; }
  __device__ __forceinline__ void set(int i, int t, float x) { v[i][t >> 2][t & 3] = x; }
};
template <>
struct Frag<2, false> {
  f2v v[16];
  __device__ __forceinline__ float get(int i, int t) const { return v[t][i]; }
  __device__ __forceinline__ void set(int i, int t, float x) { v[t][i] = x; }
};

constexpr int BK = 32;

struct GemmP {
  int M, N, K;
  int a_mode, a_L, a_C, a_shift;
  const float* A;
  int64_t a_sm, a_sk, a_sbatch;
  int b_mode, b_taps, b_C, act;
  const float* B;
  int64_t b_sk, b_sn, b_sbatch;
  float* C;
  int64_t c_sm, c_sbatch;
  const float* bias;
  int64_t bias_sbatch;
  float alpha, beta;
  const float* mul;
  int64_t mul_sm, mul_sbatch;
  int batch2;
  int64_t a_sbatch2, b_sbatch2, c_sbatch2, mul_sbatch2;
  const float* add;
  int64_t add_sm, add_sbatch;
  int splits, kchunk;          // split-K: grid.z = nb x splits (LDS kernel; the register kernel
                               // splits batch-1 products only), partial slabs in ws
  int nb = 1;                  // batch x batch2 (the split-K reduce walks every batch's slabs)
  float* ws;
  int remap;                   // XCD-aware tile order over the xy plane
  int tri = 0;                 // SatGemmDesc.tri (causal structure hint, LDS kernel only)
  int probe;                   // sat_gemm_probe_mode: 1 skip DMA, 2 skip epilogue (probes only)
  // fused column sums of B (SatGemmDesc.colsum_out): the LDS kernel treats A as having one more
  // row of ones (index m_real = M - 1), whose output row goes to cs_out instead of C
  float* cs_out;
  int m_real;
  int64_t cs_sbatch = 0;       // batch stride of cs_out (SatGemmDesc.bias_sbatch; batch2 == 1);
                               // 0 with batch > 1: batch 0's sums only (a B shared by the batches)
  int grp_co;                  // conv-bank launches: output channels per conv (GRP > 0)
  // second A segment (SatGemmDesc.A2, dense K-contiguous A only): columns k >= k1 of A come
  // from A2 (row stride a2_sm), i.e. C = A[:, :k1] B[:k1] + A2 B[k1:] in one product
  const float* A2 = nullptr;
  int64_t a2_sm = 0;
  int k1 = 0;
  // second B segment (SatGemmDesc.B2): rows k >= k1 of B come from B2 (B_K: column stride b2_s,
  // B_N: row stride b2_s), i.e. C = A[:, :k1] B + A[:, k1:] B2 (with A2: A B + A2 B2)
  const float* B2 = nullptr;
  int64_t b2_s = 0;
  // second C segment (SatGemmDesc.C2): output columns n >= n1 go to C2 (row stride c2_sm) at
  // column n - n1 (n1 a multiple of the tile width: the choice is per tile)
  float* C2 = nullptr;
  int64_t c2_sm = 0;
  int n1 = 0;
};

// j -> g with g (g + 1) / 2 <= j < (g + 1) (g + 2) / 2: conv K_{g+1} of the bank owns the
// (tap, channel-block) pairs j = g (g + 1) / 2 + tap, tap < g + 1 (taps of K1..Kmax in order)
__device__ __forceinline__ int tri_inv(int j) {
  int g = (int)((sqrtf(8.f * j + 1.f) - 1.f) * 0.5f);
  if ((g + 1) * (g + 2) / 2 <= j) ++g;
  if (g * (g + 1) / 2 > j) --g;
  return g;
}

// Operand loader variants, chosen on the host so the main loop carries no mode branches.
enum AMode { A_K = 0, A_M = 1, A_IM2COL = 2, A_IM2COLT = 3, A_GEN = 4 };
enum BMode { B_N = 0, B_K = 1, B_FLIP = 2, B_GEN = 3 };

// generic (scalar) element access, any strides / modes
__device__ __forceinline__ float load_a(const GemmP& p, const float* A, int m, int k) {
  if (m >= p.M || k >= p.K) return 0.f;
  if (p.a_mode == 0) return A[m * p.a_sm + k * p.a_sk];
  if (p.a_mode == 1) {
    const int s = m / p.a_L, n = m - s * p.a_L;
    const int tap = k / p.a_C, c = k - tap * p.a_C;
    const int row = n + tap - p.a_shift;
    if (row < 0 || row >= p.a_L) return 0.f;
    return A[(int64_t)(s * p.a_L + row) * p.a_sm + c * p.a_sk];
  }
  const int s = k / p.a_L, n = k - s * p.a_L;
  const int tap = m / p.a_C, c = m - tap * p.a_C;
  const int row = n + tap - p.a_shift;
  if (row < 0 || row >= p.a_L) return 0.f;
  return A[(int64_t)(s * p.a_L + row) * p.a_sm + c * p.a_sk];
}

__device__ __forceinline__ float load_b(const GemmP& p, const float* B, int k, int n) {
  if (k >= p.K || n >= p.N) return 0.f;
  if (p.b_mode == 0) return B[k * p.b_sk + n * p.b_sn];
  const int tap = k / p.b_C, o = k - tap * p.b_C;
  return B[((int64_t)(p.b_taps - 1 - tap) * p.N + n) * p.b_C + o];
}

__device__ __forceinline__ float apply_act(float v, int act) {
  switch (act) {
    case 1: return fmaxf(v, 0.f);
    case 2: return tanhf(v);
    case 3: return 1.f / (1.f + expf(-v));
    case 4: return v / (1.f + fabsf(v));   // softsign (MultiSpeakerPreNet speaker_projection)
    default: return v;
  }
}

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

template <int BM, int BN, int AM, int BMD, int GM = 2, int GN = 2>
__global__ void __launch_bounds__(64 * GM * GN) gemm_kernel(GemmP p) {
  constexpr int NT = 64 * GM * GN;                               // GM x GN waves
  constexpr int WM = BM / GM, WN = BN / GN;
  constexpr int SM = WM / 32, SN = WN / 32;
  constexpr bool A_MC = (AM == A_M || AM == A_IM2COLT);        // loads run along m
  constexpr bool B_NC = (BMD == B_N);                          // loads run along n
  constexpr int PA = A_MC ? 4 : 1, PB = B_NC ? 4 : 1;          // LDS row padding
  constexpr int NA = (AM == A_GEN) ? BM * BK / NT : BM * BK / (4 * NT);   // per thread
  constexpr int NB = (BMD == B_GEN) ? BN * BK / NT : BN * BK / (4 * NT);
  __shared__ __attribute__((aligned(16))) float As[2][BK][BM + PA];
  __shared__ __attribute__((aligned(16))) float Bs[2][BK][BN + PB];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = (wave / GN) * WM, wn = (wave % GN) * WN;
  int tx = blockIdx.x, ty = blockIdx.y;
  if (p.remap) {   // bijective XCD swizzle: consecutive tiles (one A row panel) share an L2
    const int nwg = gridDim.x * gridDim.y, orig = blockIdx.y * gridDim.x + blockIdx.x;
    const int q = nwg >> 3, r = nwg & 7, xcd = orig & 7;
    const int t = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
    ty = t / gridDim.x;
    tx = t - ty * gridDim.x;
  }
  int bz, bz2, split;
  if (p.splits > 1) { bz = 0; bz2 = 0; split = blockIdx.z; }
  else { bz = blockIdx.z / p.batch2; bz2 = blockIdx.z - bz * p.batch2; split = 0; }
  const int m0 = ty * BM, n0 = tx * BN;
  const float* A = p.A + bz * p.a_sbatch + bz2 * p.a_sbatch2;
  const float* B = p.B + bz * p.b_sbatch + bz2 * p.b_sbatch2;
  const int kbeg = split * p.kchunk;
  const int kend = min(p.K, kbeg + p.kchunk);

  // ---- per-thread loader state hoisted out of the K loop
  const float* arow[NA > 0 ? NA : 1];      // im2col: row base of this thread's output rows
  int an[NA > 0 ? NA : 1];                 // im2col: position in utterance, -BIG if invalid
  int aps[NA > 0 ? NA : 1], apn[NA > 0 ? NA : 1];   // im2col-T: (s, n) of the current k
  if constexpr (AM == A_IM2COL) {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int gm = m0 + ((tid + i * NT) >> 3);
      const int s = gm / p.a_L, n = gm - s * p.a_L;
      arow[i] = A + (int64_t)s * p.a_L * p.a_sm;
      an[i] = gm < p.M ? n : -(1 << 28);
    }
  }
  if constexpr (AM == A_IM2COLT) {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int pos = kbeg + (tid + i * NT) / (BM / 4);
      aps[i] = pos / p.a_L;
      apn[i] = pos - aps[i] * p.a_L;
    }
  }
  int atap = 0, ac0 = 0;
  if constexpr (AM == A_IM2COLT) { atap = m0 / p.a_C; ac0 = m0 - atap * p.a_C; }

  float4 ra4[(AM == A_GEN) ? 1 : NA];
  float ras[(AM == A_GEN) ? NA : 1];
  float4 rb4[(BMD == B_GEN) ? 1 : NB];
  float rbs[(BMD == B_GEN) ? NB : 1];
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);

  auto fetch = [&](int k0) {
    if constexpr (AM == A_K) {
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int e = tid + i * NT, m = e >> 3, kq = (e & 7) * 4;
        const int gm = m0 + m, gk = k0 + kq;
        ra4[i] = (gm < p.M && gk < kend) ? ld4(A + (int64_t)gm * p.a_sm + gk) : z4;
      }
    } else if constexpr (AM == A_M) {
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int e = tid + i * NT, k = e / (BM / 4), mq = (e % (BM / 4)) * 4;
        const int gm = m0 + mq, gk = k0 + k;
        ra4[i] = (gm < p.M && gk < kend) ? ld4(A + (int64_t)gk * p.a_sk + gm) : z4;
      }
    } else if constexpr (AM == A_IM2COL) {
      const int tap = k0 / p.a_C, c0 = k0 - tap * p.a_C;
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int kq = ((tid + i * NT) & 7) * 4;
        const int row = an[i] + tap - p.a_shift;
        const bool ok = row >= 0 && row < p.a_L && k0 + kq < kend;
        ra4[i] = ok ? ld4(arow[i] + (int64_t)row * p.a_sm + c0 + kq) : z4;
      }
    } else if constexpr (AM == A_IM2COLT) {
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int e = tid + i * NT, k = e / (BM / 4), mq = (e % (BM / 4)) * 4;
        const int row = apn[i] + atap - p.a_shift;
        const bool ok = (k0 + k < kend) && row >= 0 && row < p.a_L && (m0 + mq < p.M);
        ra4[i] = ok ? ld4(A + (int64_t)(aps[i] * p.a_L + row) * p.a_sm + ac0 + mq) : z4;
        apn[i] += BK;                                  // next K-tile of this thread
        while (apn[i] >= p.a_L) { apn[i] -= p.a_L; ++aps[i]; }
      }
    } else {
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int e = tid + i * NT, m = e / BK, k = e % BK;
        ras[i] = (k0 + k < kend) ? load_a(p, A, m0 + m, k0 + k) : 0.f;
      }
    }
    if constexpr (BMD == B_N) {
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const int e = tid + i * NT, k = e / (BN / 4), nq = (e % (BN / 4)) * 4;
        const int gk = k0 + k, gn = n0 + nq;
        rb4[i] = (gk < kend && gn < p.N) ? ld4(B + (int64_t)gk * p.b_sk + gn) : z4;
      }
    } else if constexpr (BMD == B_K) {
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const int e = tid + i * NT, n = e >> 3, kq = (e & 7) * 4;
        const int gk = k0 + kq, gn = n0 + n;
        rb4[i] = (gk < kend && gn < p.N) ? ld4(B + (int64_t)gn * p.b_sn + gk) : z4;
      }
    } else if constexpr (BMD == B_FLIP) {
      const int tap = k0 / p.b_C, o0 = k0 - tap * p.b_C;
      const float* Wt = B + (int64_t)(p.b_taps - 1 - tap) * p.N * p.b_C + o0;
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const int e = tid + i * NT, n = e >> 3, kq = (e & 7) * 4;
        const int gn = n0 + n;
        rb4[i] = (gn < p.N && k0 + kq < kend) ? ld4(Wt + (int64_t)gn * p.b_C + kq) : z4;
      }
    } else {
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const int e = tid + i * NT, n = e / BK, k = e % BK;
        rbs[i] = (k0 + k < kend) ? load_b(p, B, k0 + k, n0 + n) : 0.f;
      }
    }
  };
  auto stash = [&](int buf) {
    if constexpr (AM == A_K || AM == A_IM2COL) {
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int e = tid + i * NT, m = e >> 3, kq = (e & 7) * 4;
        As[buf][kq + 0][m] = ra4[i].x; As[buf][kq + 1][m] = ra4[i].y;
        As[buf][kq + 2][m] = ra4[i].z; As[buf][kq + 3][m] = ra4[i].w;
      }
    } else if constexpr (AM == A_M || AM == A_IM2COLT) {
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int e = tid + i * NT, k = e / (BM / 4), mq = (e % (BM / 4)) * 4;
        *reinterpret_cast<float4*>(&As[buf][k][mq]) = ra4[i];
      }
    } else {
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int e = tid + i * NT, m = e / BK, k = e % BK;
        As[buf][k][m] = ras[i];
      }
    }
    if constexpr (BMD == B_N) {
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const int e = tid + i * NT, k = e / (BN / 4), nq = (e % (BN / 4)) * 4;
        *reinterpret_cast<float4*>(&Bs[buf][k][nq]) = rb4[i];
      }
    } else if constexpr (BMD == B_K || BMD == B_FLIP) {
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const int e = tid + i * NT, n = e >> 3, kq = (e & 7) * 4;
        Bs[buf][kq + 0][n] = rb4[i].x; Bs[buf][kq + 1][n] = rb4[i].y;
        Bs[buf][kq + 2][n] = rb4[i].z; Bs[buf][kq + 3][n] = rb4[i].w;
      }
    } else {
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const int e = tid + i * NT, n = e / BK, k = e % BK;
        Bs[buf][k][n] = rbs[i];
      }
    }
  };

  // NC independent accumulator chains per sub-tile (k-steps round-robin): a wave with a single
  // 32x32 sub-tile would otherwise issue a chain of dependent MFMAs (measured: MFMA pipe 44 %
  // busy, 69 % of wave cycles issue-stalled); the copies are summed before the epilogue
  constexpr int NC = (SM * SN >= 4) ? 1 : 4 / (SM * SN);
  f32x16 acc[SM][SN], accx[NC > 1 ? NC - 1 : 1][SM][SN];
#pragma unroll
  for (int i = 0; i < SM; ++i)
#pragma unroll
    for (int j = 0; j < SN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        acc[i][j][r] = 0.f;
#pragma unroll
        for (int c = 0; c < (NC > 1 ? NC - 1 : 1); ++c) accx[c][i][j][r] = 0.f;
      }

  const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;
  const int li = lane & 31, lk = lane >> 5;
  if (nk > 0) {
    fetch(kbeg);
    stash(0);
    __syncthreads();
  }
  int cur = 0;
  for (int kt = 0; kt < nk; ++kt) {
    const bool more = kt + 1 < nk;
    if (more) fetch(kbeg + (kt + 1) * BK);
    // every operand of the K-tile goes to registers first (distinct registers per k-step, so
    // the LDS round trip is paid once per tile, not once per MFMA group); the next tile's LDS
    // stash is issued halfway through the MFMA stream
    float a[BK / 2][SM], b[BK / 2][SN];
#pragma unroll
    for (int kk = 0; kk < BK; kk += 2) {
#pragma unroll
      for (int i = 0; i < SM; ++i) a[kk / 2][i] = As[cur][kk + lk][wm + i * 32 + li];
#pragma unroll
      for (int j = 0; j < SN; ++j) b[kk / 2][j] = Bs[cur][kk + lk][wn + j * 32 + li];
    }
    __builtin_amdgcn_sched_barrier(0);   // keep the reads ahead of the MFMA stream
#pragma unroll
    for (int kk = 0; kk < BK / 2; ++kk) {
#pragma unroll
      for (int i = 0; i < SM; ++i)
#pragma unroll
        for (int j = 0; j < SN; ++j) {
          if (NC == 1 || kk % NC == 0)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[kk][i], b[kk][j], acc[i][j], 0, 0, 0);
          else
            accx[kk % NC - 1][i][j] =
                __builtin_amdgcn_mfma_f32_32x32x2f32(a[kk][i], b[kk][j], accx[kk % NC - 1][i][j], 0, 0, 0);
        }
      if (kk == BK / 4 - 1 && more) stash(cur ^ 1);
    }
    __syncthreads();
    cur ^= 1;
  }

  if constexpr (NC > 1) {
#pragma unroll
    for (int i = 0; i < SM; ++i)
#pragma unroll
      for (int j = 0; j < SN; ++j)
#pragma unroll
        for (int c = 0; c < NC - 1; ++c) acc[i][j] += accx[c][i][j];
  }

  // epilogue: C/D map of 32x32 f32 MFMA: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
  if (p.splits > 1) {
    float* slab = p.ws + (int64_t)split * p.M * p.N;
#pragma unroll
    for (int i = 0; i < SM; ++i)
#pragma unroll
      for (int j = 0; j < SN; ++j) {
        const int col = n0 + wn + j * 32 + li;
        if (col >= p.N) continue;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = m0 + wm + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lk;
          if (row < p.M) slab[(int64_t)row * p.N + col] = acc[i][j][r];
        }
      }
    return;
  }
  float* C = p.C + bz * p.c_sbatch + bz2 * p.c_sbatch2;
  const float* bias = p.bias ? p.bias + bz * p.bias_sbatch : nullptr;
  const float* mul = p.mul ? p.mul + bz * p.mul_sbatch + bz2 * p.mul_sbatch2 : nullptr;
  const float* add = p.add ? p.add + bz * p.add_sbatch : nullptr;
#pragma unroll
  for (int i = 0; i < SM; ++i)
#pragma unroll
    for (int j = 0; j < SN; ++j) {
      const int col = n0 + wn + j * 32 + li;
      if (col >= p.N) continue;
      const float bv = bias ? bias[col] : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lk;
        if (row >= p.M) continue;
        float* dst = C + (int64_t)row * p.c_sm + col;
        float v = p.alpha * acc[i][j][r];
        if (p.beta != 0.f) v += p.beta * (*dst);
        v = apply_act(v + bv, p.act);
        if (mul) v *= mul[(int64_t)row * p.mul_sm + col];
        if (add) v += add[(int64_t)row * p.add_sm + col];
        *dst = v;
      }
    }
}

// split-K finish: sum each batch's S slabs in order, then the same epilogue as gemm_kernel.
// Four consecutive outputs per thread (16-byte slab loads when N % 4 == 0) and four slab loads
// in flight per trip: the pass is latency-bound, not bandwidth-bound, at these sizes.
// batch b's column-sum row (null: batch b > 0 of a shared-B product writes none)
__device__ __forceinline__ float* batch_cs(const GemmP& p, int b) {
  return (!p.cs_out || (b > 0 && p.cs_sbatch == 0)) ? nullptr : p.cs_out + b * p.cs_sbatch;
}
// null: the column-sum row of a batch that writes none
__device__ __forceinline__ float* out_ptr(const GemmP& p, float* C, float* cs, int row, int col) {
  if (p.cs_out && row == p.m_real) return cs ? cs + col : nullptr;
  return C + (int64_t)row * p.c_sm + col;
}
__device__ __forceinline__ float splitk_epilogue(const GemmP& p, const float* dst, int row,
                                                 int col, float s) {
  float v = p.alpha * s;
  if (p.beta != 0.f) v += p.beta * (*dst);
  v = apply_act(v + (p.bias ? p.bias[col] : 0.f), p.act);
  if (p.mul) v *= p.mul[(int64_t)row * p.mul_sm + col];
  if (p.add) v += p.add[(int64_t)row * p.add_sm + col];
  return v;
}
// batch b of a split-K launch: its output block (batched splits carry no bias / mul / add:
// launch_lds plans them only without)
__device__ __forceinline__ float* batch_c(const GemmP& p, int b) {
  const int bz = b / p.batch2, bz2 = b - bz * p.batch2;
  return p.C + bz * p.c_sbatch + bz2 * p.c_sbatch2;
}
__global__ void __launch_bounds__(256) gemm_splitk_reduce(GemmP p) {
  const int64_t total = (int64_t)p.M * p.N;
  if ((p.N & 3) == 0) {
    const int64_t total4 = total >> 2;
    const float4* ws4 = reinterpret_cast<const float4*>(p.ws);
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < p.nb * total4;
         e += (int64_t)gridDim.x * blockDim.x) {
      const int b = (int)(e / total4);
      const int64_t i = e - b * total4;
      const float4* src = ws4 + (int64_t)b * p.splits * total4 + i;
      float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
      int k = 0;
      for (; k + 4 <= p.splits; k += 4) {
        float4 v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = src[(int64_t)(k + q) * total4];
#pragma unroll
        for (int q = 0; q < 4; ++q) { a.x += v[q].x; a.y += v[q].y; a.z += v[q].z; a.w += v[q].w; }
      }
      for (; k < p.splits; ++k) {
        const float4 v = src[(int64_t)k * total4];
        a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
      }
      const int row = (int)((4 * i) / p.N), col = (int)(4 * i - (int64_t)row * p.N);
      float* dst = out_ptr(p, batch_c(p, b), batch_cs(p, b), row, col);
      if (!dst) continue;
      dst[0] = splitk_epilogue(p, dst, row, col, a.x);
      dst[1] = splitk_epilogue(p, dst + 1, row, col + 1, a.y);
      dst[2] = splitk_epilogue(p, dst + 2, row, col + 2, a.z);
      dst[3] = splitk_epilogue(p, dst + 3, row, col + 3, a.w);
    }
    return;
  }
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < p.nb * total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int b = (int)(e / total);
    const int64_t i = e - b * total;
    const int row = (int)(i / p.N), col = (int)(i - (int64_t)row * p.N);
    const float* src = p.ws + (int64_t)b * p.splits * total + i;
    float s = 0.f;
    for (int k = 0; k < p.splits; ++k) s += src[(int64_t)k * total];
    float* dst = out_ptr(p, batch_c(p, b), batch_cs(p, b), row, col);
    if (!dst) continue;
    *dst = splitk_epilogue(p, dst, row, col, s);
  }
}

// Skinny products (M <= 8 rows: the free-running decoder's per-step projections at batch 8,
// inference.py): the 64-row tile kernels run such a product on N / 64 workgroups that each
// stream K x 64 weights alone (8.7 us per launch measured).  Here a workgroup owns 16 columns
// for all M rows, 256 threads = 16 k-slices x 16 columns: each thread accumulates its slice for
// the M rows (A staged in LDS, W read as 64-byte row segments), then the 16 slices are summed
// in a fixed order (2 shuffles + an LDS pass over the 4 waves).  Same epilogue as the tiles.
constexpr int kSkinnyM = 8;
__global__ void __launch_bounds__(256) gemm_skinny_kernel(GemmP p) {
  extern __shared__ __attribute__((aligned(16))) float sk_smem[];
  float* As = sk_smem;                                  // [M][K]
  float* red = sk_smem + (size_t)p.M * p.K;             // [4 waves][8 rows][16 cols]
  const int tid = threadIdx.x, nl = tid & 15, ks = tid >> 4;
  const int n = blockIdx.x * 16 + nl;
  const int M = p.M, K = p.K;
  // A -> LDS, 8 loads per thread in flight per batch (a dependent load / store per element
  // serialises the round trips: 5 us at K = 256)
  for (int base = 0; base < M * K; base += 8 * 256) {
    float v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int i = base + q * 256 + tid;
      const int m = i / K, k = i - m * K;
      v[q] = i < M * K ? p.A[(int64_t)m * p.a_sm + (int64_t)k * p.a_sk] : 0.f;
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int i = base + q * 256 + tid;
      if (i < M * K) As[i] = v[q];
    }
  }
  __syncthreads();
  float acc[kSkinnyM];
#pragma unroll
  for (int m = 0; m < kSkinnyM; ++m) acc[m] = 0.f;
  if (n < p.N) {
    // the slice's weights in chunks of 16 loads issued before any use (one round trip per
    // chunk: the product is latency-bound at these sizes)
    const float* wc = p.B + (int64_t)n * p.b_sn;
    for (int k0 = ks; k0 < K; k0 += 256) {
      float w[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int k = k0 + 16 * q;
        w[q] = k < K ? wc[(int64_t)k * p.b_sk] : 0.f;
      }
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int k = k0 + 16 * q;
        if (k < K) {
#pragma unroll
          for (int m = 0; m < kSkinnyM; ++m)
            if (m < M) acc[m] = fmaf(As[m * K + k], w[q], acc[m]);
        }
      }
    }
  }
  // k-slices ks = 4 wave + (lane >> 4): lanes l, l ^ 16, l ^ 32, l ^ 48 share a column
#pragma unroll
  for (int m = 0; m < kSkinnyM; ++m) {
    acc[m] += __shfl_xor(acc[m], 16, 64);
    acc[m] += __shfl_xor(acc[m], 32, 64);
  }
  const int wave = tid >> 6, lane = tid & 63;
  if (lane < 16) {
#pragma unroll
    for (int m = 0; m < kSkinnyM; ++m) red[(wave * kSkinnyM + m) * 16 + lane] = acc[m];
  }
  __syncthreads();
  if (tid < M * 16) {
    const int m = tid >> 4, c = tid & 15, col = blockIdx.x * 16 + c;
    if (col < p.N) {
      const float sum = ((red[(0 * kSkinnyM + m) * 16 + c] + red[(1 * kSkinnyM + m) * 16 + c]) +
                         red[(2 * kSkinnyM + m) * 16 + c]) + red[(3 * kSkinnyM + m) * 16 + c];
      float* dst = p.C + (int64_t)m * p.c_sm + col;
      float v = p.alpha * sum;
      if (p.beta != 0.f) v += p.beta * (*dst);
      v = apply_act(v + (p.bias ? p.bias[col] : 0.f), p.act);
      if (p.add) v += p.add[(int64_t)m * p.add_sm + col];
      *dst = v;
    }
  }
}

// Degenerate plain products (the stop-token projection, `stop = x w + b` and its input
// gradient): tiles of 64 columns or 16-deep K slices would be almost all padding there.
// N == 1 with row-contiguous A: one wave per output row, lanes over K (float4 when aligned).
__global__ void __launch_bounds__(256) gemm_n1_kernel(GemmP p, int vec) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= p.M) return;
  const float* a = p.A + (int64_t)row * p.a_sm;
  float s = 0.f;
  if (vec) {
    for (int k = 4 * lane; k < p.K; k += 256) {
      const float4 av = *reinterpret_cast<const float4*>(a + k);
      s += av.x * p.B[(int64_t)k * p.b_sk] + av.y * p.B[(int64_t)(k + 1) * p.b_sk] +
           av.z * p.B[(int64_t)(k + 2) * p.b_sk] + av.w * p.B[(int64_t)(k + 3) * p.b_sk];
    }
  } else {
    for (int k = lane; k < p.K; k += 64) s += a[k] * p.B[(int64_t)k * p.b_sk];
  }
  s = wave_sum(s);
  if (lane == 0) {
    float* dst = p.C + (int64_t)row * p.c_sm;
    *dst = splitk_epilogue(p, dst, row, 0, s);
  }
}
// N == 1 with a column-contiguous A (a_sm == 1: A = X^T, the stop-token layer's weight
// gradient dw = X^T dstop, 256 x 1 x 16000): workgroup (column block, K slice) = 64 columns x
// 4 row groups, coalesced along m; the K slices' partials go to split-K slabs [split][M] and
// gemm_splitk_reduce applies the epilogue.  The fused column sum (cs_out) is row m_real of a
// virtual ones column of X.  Replaces a register-kernel tile launch (28 us + 25 us reduce).
__global__ void __launch_bounds__(256) gemm_tn1_kernel(GemmP p) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int m = blockIdx.x * 64 + lane, split = blockIdx.y;
  const int kbeg = split * p.kchunk, kend = min(p.K, kbeg + p.kchunk);
  float acc = 0.f;
  if (m < p.M) {
    const bool ones = p.cs_out && m == p.m_real;
    for (int k = kbeg + g; k < kend; k += 4) {
      const float x = ones ? 1.f : p.A[(int64_t)k * p.a_sk + m];
      acc += x * p.B[(int64_t)k * p.b_sk];
    }
  }
  red[g][lane] = acc;
  __syncthreads();
  if (g == 0 && m < p.M)
    p.ws[(int64_t)split * p.M + m] = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
}

// K == 1: the outer product C = epilogue(alpha a b^T), one thread per output element
__global__ void __launch_bounds__(256) gemm_k1_kernel(GemmP p) {
  const int total = p.M * p.N;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int row = i / p.N, col = i - row * p.N;
    const float s = p.A[(int64_t)row * p.a_sm] * p.B[(int64_t)col * p.b_sn];
    float* dst = p.C + (int64_t)row * p.c_sm + col;
    *dst = splitk_epilogue(p, dst, row, col, s);
  }
}

// ---------------------------------------------------------------------------------------------
// LDS-DMA pipelined variant// ---------------------------------------------------------------------------------------------
// LDS-DMA pipelined variant (the default for every vector-loadable operand mode).
//
// Operand tiles go global -> LDS with global_load_lds_dwordx4 (no VGPR staging, no ds_write
// pass) into a 3-stage ring, so two K-tiles are in flight while one is multiplied; waits are
// counted (vmcnt(LPT) leaves the newest tile in flight) and the per-K-tile barrier is a raw
// s_barrier (a __syncthreads would drain every outstanding DMA).  The LDS images are lane-linear
// copies of the global tile:
//   * K-major image [rows][32] (operand contiguous along k: A_K, A_IM2COL, B_K, B_FLIP), the
//     16-byte chunk q of row r stored at slot q ^ ((r >> 1) & 7) (swizzle applied on the SOURCE
//     address), read back with ds_read_b128: 4 k values per lane -- conflict-free over the four
//     16-lane groups of ds_read_b128;
//   * M/N-major image [32][rows] (contiguous along m / n: A_M, A_IM2COLT, B_N), read with
//     ds_read_b32, 32 consecutive floats per 32-lane group -- conflict-free without a swizzle.
// The reduction index is permuted inside a K-tile, identically for both operands: MFMA step
// t = 4 jj + i takes k = 8 jj + 4 h + i in lane half h (h = lane >> 5), so a ds_read_b128 of
// chunk 2 jj + h feeds four consecutive steps.  Out-of-range chunks (tile edges, conv padding)
// are read from a zero page, so the loads need no branches and no masks.
__device__ __attribute__((aligned(16))) float g_gemm_zero[64];
__device__ __attribute__((aligned(16))) float g_gemm_ones[64] = {
    1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f,
    1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f,
    1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f,
    1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f};

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void raw_barrier() { asm volatile("s_barrier" ::: "memory"); }
// s_waitcnt simm16 of gfx9 with only lgkmcnt(0): vmcnt 63 ([3:0] | [15:14]), expcnt 7 ([6:4])
constexpr int kLgkm0 = 0xC07F;

// One global_load_lds_dwordx4: 16 bytes per lane into LDS at lds_off + 16 * lane.  Issued from
// inline asm so the compiler does not track it: its own wait insertion would otherwise put a
// vmcnt(0) before every ds_read of the ring (it cannot tell the ring's stages apart) and drain
// the pipeline each K-tile.  Completion is ordered by the explicit counted waits below.
__device__ __forceinline__ void dma16(const float* src, uint32_t lds_off) {
  int keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(lds_off)
      : "memory");
}

// GRP selects the conv-bank launches of sat_cbhg_convbank_fwd/bwd (0 = plain product):
//   1 forward  : output column block g*Co.. = Conv1D K_{g+1}(x), reduction (g+1)*C per tile;
//   2 dX       : ONE product over K = sum_g (g+1)*Co, k -> (g, tap, o) of dY's column block g;
//   3 dW       : ONE product over M = sum_g (g+1)*C, rows (g, tap, ci) read dY's column block g.
// waves per workgroup: 4 (2 x 2) for every tile but 128 x 128, which runs 8 (2 x 4, each wave
// 64 x 32 as on the 128 x 64 tile) so its one workgroup per CU still has two waves per SIMD
// The large tiles 256 x 128 / 128 x 256 run 8 waves of 64 x 64 (4 x 2 / 2 x 4) over a 2-stage
// ring (96 KB, one workgroup per CU): half the tiles -- half the per-tile prologues and
// epilogues -- of 128 x 128 on the 16000-row products, and 4 MFMAs per 4 fragment values.
template <int BM, int BN>
constexpr int lds_waves() { return (BM * BN >= 128 * 128) ? 8 : 4; }
template <int BM, int BN>
constexpr int lds_wgm() { return BM == 256 ? 4 : 2; }       // waves along M
template <int BM, int BN>
constexpr int lds_stages() { return BM * BN > 128 * 128 ? 2 : 3; }

template <int BM, int BN, int AM, int BMD, int GRP = 0>
__global__ void __launch_bounds__((64 * lds_waves<BM, BN>())) gemm_lds_kernel(GemmP p) {
  constexpr int ST = lds_stages<BM, BN>();
  constexpr int NWV = lds_waves<BM, BN>(), WGM = lds_wgm<BM, BN>(), WGN = NWV / WGM;
  constexpr int WM = BM / WGM, WN = BN / WGN;         // WGM x WGN waves
  constexpr int SM = WM / 32, SN = WN / 32;           // 32x32 MFMA sub-tiles per wave
  constexpr bool AKM = (AM == A_K || AM == A_IM2COL); // A image K-major
  constexpr bool BKM = (BMD == B_K || BMD == B_FLIP); // B image K-major
  constexpr int A_SZ = BM * BK, B_SZ = BN * BK, ST_SZ = A_SZ + B_SZ;
  constexpr int NA = BM / (8 * NWV), NB = BN / (8 * NWV);   // 1-KB DMA instructions per wave per tile
  constexpr int LPT = NA + NB;
  static_assert(LPT <= 24, "vmcnt budget");
  __shared__ __attribute__((aligned(16))) float lds[ST * ST_SZ];
  const uint32_t lds_base = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) float*)lds);

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = (w / WGN) * WM, wn = (w % WGN) * WN;
  int tx = blockIdx.x, ty = blockIdx.y;
  if (p.remap) {   // bijective XCD swizzle: consecutive tiles (one A row panel) share an L2
    const int nwg = gridDim.x * gridDim.y, orig = blockIdx.y * gridDim.x + blockIdx.x;
    const int q = nwg >> 3, r = nwg & 7, xcd = orig & 7;
    const int t = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
    ty = t / gridDim.x;
    tx = t - ty * gridDim.x;
  }
  // grid.z = batch index x splits + split (split-K) or the batch index
  const int bb = p.splits > 1 ? (int)blockIdx.z / p.splits : (int)blockIdx.z;
  const int split = p.splits > 1 ? (int)blockIdx.z - bb * p.splits : 0;
  const int bz = bb / p.batch2, bz2 = bb - bz * p.batch2;
  // conv-bank forward: column blocks have different reductions ((g + 1) * C), so the tiles go
  // out longest-first (every row tile of the widest bank, then the next, ...): the greedy
  // dispatcher then ends the launch on the short tiles.  A row-major order with a per-row
  // rotation left long tiles among the last dispatched (a list-scheduling model of the C2 shape:
  // makespan 160 vs 121 units for a 116 lower bound).  Consecutive workgroups still land on
  // different XCDs (the dispatcher deals workgroup i to XCD i % 8).
  if constexpr (GRP == 1) {
    const int i = blockIdx.y * gridDim.x + blockIdx.x, c = i / gridDim.y;
    tx = gridDim.x - 1 - c;
    ty = i - c * gridDim.y;
  }
  const int m0 = ty * BM, n0 = tx * BN;
  const float* A = p.A + bz * p.a_sbatch + bz2 * p.a_sbatch2;
  const float* B = p.B + bz * p.b_sbatch + bz2 * p.b_sbatch2;
  // second reduction segments (A2 / B2) share their operand's batch strides
  const float* A2 = p.A2 ? p.A2 + bz * p.a_sbatch + bz2 * p.a_sbatch2 : nullptr;
  const float* B2 = p.B2 ? p.B2 + bz * p.b_sbatch + bz2 * p.b_sbatch2 : nullptr;
  int Kt = p.K, shift = p.a_shift, atap = 0, ac0 = 0;
  if constexpr (GRP == 1) {
    const int g = n0 / p.grp_co, t = g + 1;
    Kt = t * p.a_C;
    shift = (t - 1) / 2;
    B += (int64_t)p.grp_co * p.a_C * (t * (t - 1) / 2) - (int64_t)g * p.grp_co;
  }
  if constexpr (AM == A_IM2COLT) {
    if constexpr (GRP == 3) {
      const int j = m0 / p.a_C, g = tri_inv(j);
      atap = j - g * (g + 1) / 2;
      ac0 = m0 - j * p.a_C;
      shift = g / 2;
      B += (int64_t)g * p.grp_co;
    } else {
      atap = m0 / p.a_C;
      ac0 = m0 - atap * p.a_C;
    }
  }
  // causal structure (SatGemmDesc.tri): tiles wholly above the diagonal are not needed (1);
  // a triangular A's zero K-tiles are not loaded (2: lower, 3: upper) -- exact zeros either way
  if (p.tri == 1 && n0 >= m0 + BM) return;
  int kbeg = split * p.kchunk;
  int kend = min(Kt, kbeg + p.kchunk);
  if (p.tri == 2) kend = min(kend, m0 + BM);
  if (p.tri == 3) kbeg = max(kbeg, m0 / BK * BK);
  const float* zero = g_gemm_zero;
  const float* ones = g_gemm_ones;

  // ---- per-lane loader state, advanced by one K-tile per issue
  // K-major images: instruction i of wave w covers rows (NWV i + w) * 8 + (lane >> 3); the lane's
  // chunk (after the swizzle) is the same for every instruction
  const int kq = 4 * ((lane & 7) ^ ((4 * (w & 1) + (lane >> 4)) & 7));
  // M/N-major images: instruction i covers k rows (NWV i + w) * (256 / rows) + lane / (rows / 4)
  const float* aptr[NA];
  int ai[NA];
  int arow[NA];                                        // A_K: the lane's (clamped) row per DMA
  const int amq = AKM ? 0 : 4 * (lane % (BM / 4));
  bool aone[NA];                                       // the fused column-sum row of ones
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    aone[i] = false;
    if constexpr (AM == A_K) {
      const int gm = m0 + (NWV * i + w) * 8 + (lane >> 3);
      aone[i] = p.cs_out != nullptr && gm == p.m_real;
      ai[i] = gm < p.M && !aone[i];
      arow[i] = min(gm, (p.cs_out ? p.m_real : p.M) - 1);
      aptr[i] = (A2 && kbeg >= p.k1) ? A2 + (int64_t)arow[i] * p.a2_sm + (kbeg - p.k1) + kq
                                       : A + (int64_t)arow[i] * p.a_sm + kbeg + kq;
    } else if constexpr (AM == A_IM2COL) {   // (utterance, position) of the output row
      const int gm = m0 + (NWV * i + w) * 8 + (lane >> 3);
      const int s = gm / p.a_L, n = gm - s * p.a_L;
      aptr[i] = A + (int64_t)s * p.a_L * p.a_sm;
      ai[i] = gm < p.M ? n : -(1 << 28);
    } else if constexpr (AM == A_M) {
      ai[i] = kbeg + (NWV * i + w) * (256 / BM) + lane / (BM / 4);     // k row
      aptr[i] = A + (int64_t)ai[i] * p.a_sk + m0 + amq;
    } else {
      ai[i] = kbeg + (NWV * i + w) * (256 / BM) + lane / (BM / 4);     // k position
      aptr[i] = nullptr;
    }
  }
  const bool aones = !AKM && p.cs_out != nullptr && m0 + amq == p.m_real;   // m_real % 4 == 0
  const bool amok = AKM ? true : (m0 + amq < p.M && !aones);
  const float* bptr[NB];
  int bi[NB];
  int bcol[NB];                                        // B_K: the lane's (clamped) column per DMA
  const int bnq = BKM ? 0 : 4 * (lane % (BN / 4));
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    if constexpr (BKM) {
      const int gn = n0 + (NWV * i + w) * 8 + (lane >> 3);
      bi[i] = gn < p.N;
      const int gc = min(gn, p.N - 1);
      bcol[i] = gc;
      bptr[i] = (BMD == B_K) ? ((B2 && kbeg >= p.k1) ? B2 + (int64_t)gc * p.b2_s + (kbeg - p.k1) + kq
                                                       : B + (int64_t)gc * p.b_sn + kbeg + kq)
                             : B + (int64_t)gc * p.b_C + kq;
    } else {
      bcol[i] = 0;
      bi[i] = kbeg + (NWV * i + w) * (256 / BN) + lane / (BN / 4);
      bptr[i] = (B2 && kbeg >= p.k1) ? B2 + (int64_t)(bi[i] - p.k1) * p.b2_s + n0 + bnq
                                       : B + (int64_t)bi[i] * p.b_sk + n0 + bnq;
    }
  }
  const bool bnok = BKM ? true : (n0 + bnq < p.N);

  // DMA of K-tile k0 into ring stage `stage`; the running pointers advance by one K-tile
  auto issue = [&](int stage, int k0) {
    if (p.probe & 1) return;
    const uint32_t la = lds_base + (uint32_t)(stage * ST_SZ * 4);
    const uint32_t lb = la + A_SZ * 4;
    if constexpr (AM == A_K) {
      const bool kok = k0 + kq < kend;
      if (A2 && k0 == p.k1) {   // the reduction crosses into the second A segment
#pragma unroll
        for (int i = 0; i < NA; ++i) aptr[i] = A2 + (int64_t)arow[i] * p.a2_sm + kq;
      }
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        dma16(kok ? (ai[i] ? aptr[i] : (aone[i] ? ones : zero)) : zero, la + (NWV * i + w) * 1024);
        aptr[i] += BK;
      }
    } else if constexpr (AM == A_IM2COL) {
      int tap, c0, sh = shift;
      if constexpr (GRP == 2) {   // k -> (conv g, tap, channel) of dY's column block g
        const int j = k0 / p.grp_co, g = tri_inv(j);
        tap = j - g * (g + 1) / 2;
        c0 = k0 - j * p.grp_co + g * p.grp_co;
        sh = g - g / 2;
      } else {
        tap = k0 / p.a_C;
        c0 = k0 - tap * p.a_C;
      }
      const bool kok = k0 + kq < kend;
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int row = ai[i] + tap - sh;
        const bool ok = kok && row >= 0 && row < p.a_L;
        dma16(ok ? aptr[i] + (int64_t)row * p.a_sm + c0 + kq : zero, la + (NWV * i + w) * 1024);
      }
    } else if constexpr (AM == A_M) {
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        dma16(ai[i] < kend ? (amok ? aptr[i] : (aones ? ones : zero)) : zero,
              la + (NWV * i + w) * 1024);
        ai[i] += BK;
        aptr[i] += (int64_t)BK * p.a_sk;
      }
    } else {   // A_IM2COLT: m = tap * C + c (one tap per tile), k = (utterance, position)
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int pos = ai[i];
        const int s = pos / p.a_L, n = pos - s * p.a_L;
        const int row = n + atap - shift;
        const bool ok = amok && pos < kend && row >= 0 && row < p.a_L;
        dma16(ok ? A + (int64_t)(s * p.a_L + row) * p.a_sm + ac0 + amq : zero,
              la + (NWV * i + w) * 1024);
        ai[i] += BK;
      }
    }
    if constexpr (BMD == B_N) {
      if (B2 && k0 == p.k1) {   // the reduction crosses into the second B segment
#pragma unroll
        for (int i = 0; i < NB; ++i) bptr[i] = B2 + (int64_t)(bi[i] - p.k1) * p.b2_s + n0 + bnq;
      }
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        dma16((bnok && bi[i] < kend) ? bptr[i] : zero, lb + (NWV * i + w) * 1024);
        bi[i] += BK;
        bptr[i] += (int64_t)BK * p.b_sk;
      }
    } else if constexpr (BMD == B_K) {
      const bool kok = k0 + kq < kend;
      if (B2 && k0 == p.k1) {
#pragma unroll
        for (int i = 0; i < NB; ++i) bptr[i] = B2 + (int64_t)bcol[i] * p.b2_s + kq;
      }
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        dma16((bi[i] && kok) ? bptr[i] : zero, lb + (NWV * i + w) * 1024);
        bptr[i] += BK;
      }
    } else {   // B_FLIP: W[taps-1-tap][n][o], k = tap * C + o (one tap per tile)
      int64_t off;
      if constexpr (GRP == 2) {   // W_{g+1} of the bank at offset Co * C * g (g + 1) / 2
        const int j = k0 / p.b_C, g = tri_inv(j), tap = j - g * (g + 1) / 2;
        off = (int64_t)p.b_C * p.N * (g * (g + 1) / 2) + (int64_t)(g - tap) * p.N * p.b_C +
              (k0 - j * p.b_C);
      } else {
        const int tap = k0 / p.b_C, o0 = k0 - tap * p.b_C;
        off = (int64_t)(p.b_taps - 1 - tap) * p.N * p.b_C + o0;
      }
      const bool kok = k0 + kq < kend;
#pragma unroll
      for (int i = 0; i < NB; ++i)
        dma16((bi[i] && kok) ? bptr[i] + off : zero, lb + (NWV * i + w) * 1024);
    }
  };

  constexpr int NC = (SM * SN >= 4) ? 1 : 4 / (SM * SN);
  f32x16 acc[NC][SM][SN];
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int i = 0; i < SM; ++i)
#pragma unroll
      for (int j = 0; j < SN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[c][i][j][r] = 0.f;

  const int li = lane & 31, lh = lane >> 5;
  const int swz = (li >> 1) & 7;     // K-major read swizzle of this lane's rows
  // fragments of one K-tile: step t = 4 jj + i takes k = 8 jj + 4 h + i (both operands; Frag)
  using FA = Frag<SM, AKM>;
  using FB = Frag<SN, BKM>;
  auto read_frags = [&](int stage, FA& a, FB& b) {
    const float* la = lds + stage * ST_SZ;
    const float* lb = la + A_SZ;
    if constexpr (AKM) {
#pragma unroll
      for (int i = 0; i < SM; ++i)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          a.v[i][jj] = *reinterpret_cast<const f4v*>(la + (wm + i * 32 + li) * BK + 4 * ((2 * jj + lh) ^ swz));
        }
    } else {
#pragma unroll
      for (int t = 0; t < 16; ++t)
#pragma unroll
        for (int i = 0; i < SM; ++i)
          a.set(i, t, la[(8 * (t >> 2) + 4 * lh + (t & 3)) * BM + wm + i * 32 + li]);
    }
    if constexpr (BKM) {
#pragma unroll
      for (int j = 0; j < SN; ++j)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          b.v[j][jj] = *reinterpret_cast<const f4v*>(lb + (wn + j * 32 + li) * BK + 4 * ((2 * jj + lh) ^ swz));
        }
    } else {
#pragma unroll
      for (int t = 0; t < 16; ++t)
#pragma unroll
        for (int j = 0; j < SN; ++j)
          b.set(j, t, lb[(8 * (t >> 2) + 4 * lh + (t & 3)) * BN + wn + j * 32 + li]);
    }
  };
  auto mfma_steps = [&](int t0, int t1, const FA& a, const FB& b) {
#pragma unroll
    for (int t = t0; t < t1; ++t)
#pragma unroll
      for (int i = 0; i < SM; ++i)
#pragma unroll
        for (int j = 0; j < SN; ++j)
          acc[t % NC][i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(
              a.get(i, t), b.get(j, t), acc[t % NC][i][j], 0, 0, 0);
  };

  // Schedule per K-tile kt (fragments of kt already in registers): issue the DMA of kt+2 into
  // the stage read two tiles ago; MFMA steps 0-7; wait for this wave's DMA of kt+1 and barrier
  // (then every wave's kt+1 tile has landed, and every wave has finished reading the stage
  // the next issue overwrites); read kt+1's fragments into the other register set while
  // MFMA steps 8-15 of kt run.  Two register sets alternate, so the loop is unrolled by 2.
  const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;
  FA fa0, fa1;
  FB fb0, fb1;
  if (nk > 0) {
    issue(0, kbeg);
    if (nk > 1) issue(1, kbeg + BK);
    if (nk > 1) wait_vmcnt<LPT>(); else wait_vmcnt<0>();
    raw_barrier();
    read_frags(0, fa0, fb0);
  }
  // Two stages (the large tiles): the DMA of kt+2 goes into kt's own stage right after the
  // barrier that follows every wave's last read of it; it has the rest of kt and the first half
  // of kt+1 -- one K-tile of 64 MFMAs per wave -- to land.
  auto tile = [&](int kt, int stage, const FA& ca, const FB& cb, FA& na, FB& nb) {
    const bool more2 = kt + 2 < nk;
    if constexpr (ST == 3) {
      if (more2) issue(stage == 0 ? 2 : stage - 1, kbeg + (kt + 2) * BK);
    }
    mfma_steps(0, 8, ca, cb);
    // every fragment read of this K-tile has landed by now (issued a half K-tile ago); saying so
    // with the compiler-visible form of s_waitcnt lgkmcnt(0), on both paths, stops it from
    // making MFMA steps 8-15 wait behind the next tile's 16 reads (the in-order lgkmcnt cannot
    // single out the older reads those steps use)
    __builtin_amdgcn_s_waitcnt(kLgkm0);
    if (kt + 1 < nk) {
      if constexpr (ST == 3) {
        if (more2) wait_vmcnt<LPT>(); else wait_vmcnt<0>();
        raw_barrier();
        read_frags(stage == 2 ? 0 : stage + 1, na, nb);
      } else {
        wait_vmcnt<0>();
        raw_barrier();
        if (more2) issue(stage, kbeg + (kt + 2) * BK);
        read_frags(stage ^ 1, na, nb);
      }
    }
    mfma_steps(8, 16, ca, cb);
  };
  constexpr int STL = ST - 1;
  int stage = 0, kt = 0;
  for (; kt + 1 < nk; kt += 2) {
    tile(kt, stage, fa0, fb0, fa1, fb1);
    stage = stage == STL ? 0 : stage + 1;
    tile(kt + 1, stage, fa1, fb1, fa0, fb0);
    stage = stage == STL ? 0 : stage + 1;
  }
  if (kt < nk) tile(kt, stage, fa0, fb0, fa1, fb1);

  if constexpr (NC > 1) {
#pragma unroll
    for (int c = 1; c < NC; ++c)
#pragma unroll
      for (int i = 0; i < SM; ++i)
#pragma unroll
        for (int j = 0; j < SN; ++j) acc[0][i][j] += acc[c][i][j];
  }

  if (p.probe & 2) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < SM; ++i)
#pragma unroll
      for (int j = 0; j < SN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) s += acc[0][i][j][r];
    if (s == 1234.5f) p.C[0] = s;
    return;
  }
  // epilogue: C/D map of 32x32 f32 MFMA: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5).
  // Whole tiles with a plain epilogue (the common case) take a branch-free store loop.
  const bool full = (m0 + BM <= p.M) && (n0 + BN <= p.N);
  if (p.splits > 1) {
    float* slab = p.ws + (int64_t)blockIdx.z * p.M * p.N;    // slab (batch, split)
#pragma unroll
    for (int i = 0; i < SM; ++i)
#pragma unroll
      for (int j = 0; j < SN; ++j) {
        const int col = n0 + wn + j * 32 + li;
        const int row0 = m0 + wm + i * 32 + 4 * lh;
        float* dst = slab + (int64_t)row0 * p.N + col;
        if (full) {
#pragma unroll
          for (int r = 0; r < 16; ++r) dst[((r & 3) + 8 * (r >> 2)) * p.N] = acc[0][i][j][r];
        } else if (col < p.N) {
#pragma unroll
          for (int r = 0; r < 16; ++r)
            if (row0 + (r & 3) + 8 * (r >> 2) < p.M)
              dst[((r & 3) + 8 * (r >> 2)) * p.N] = acc[0][i][j][r];
        }
      }
    return;
  }
  float* C = p.C + bz * p.c_sbatch + bz2 * p.c_sbatch2;
  int64_t cs = p.c_sm;
  if (p.C2 && n0 >= p.n1) {   // this tile's columns live in the second output (batch 1 only)
    C = p.C2 - p.n1;
    cs = p.c2_sm;
  }
  const float* bias = p.bias ? p.bias + bz * p.bias_sbatch : nullptr;
  const float* mul = p.mul ? p.mul + bz * p.mul_sbatch + bz2 * p.mul_sbatch2 : nullptr;
  const float* add = p.add ? p.add + bz * p.add_sbatch : nullptr;
  if (full && !mul && !add && p.beta == 0.f && p.act == 0 && !p.cs_out) {
#pragma unroll
    for (int i = 0; i < SM; ++i)
#pragma unroll
      for (int j = 0; j < SN; ++j) {
        const int col = n0 + wn + j * 32 + li;
        const float bv = bias ? bias[col] : 0.f;
        float* dst = C + (int64_t)(m0 + wm + i * 32 + 4 * lh) * cs + col;
#pragma unroll
        for (int r = 0; r < 16; ++r) dst[((r & 3) + 8 * (r >> 2)) * cs] = p.alpha * acc[0][i][j][r] + bv;
      }
    return;
  }
#pragma unroll
  for (int i = 0; i < SM; ++i)
#pragma unroll
    for (int j = 0; j < SN; ++j) {
      const int col = n0 + wn + j * 32 + li;
      if (col >= p.N) continue;
      const float bv = bias ? bias[col] : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (row >= p.M) continue;
        float* dst;
        if (p.cs_out && row == p.m_real) {
          float* cso = batch_cs(p, bb);
          if (!cso) continue;
          dst = cso + col;
        } else {
          dst = C + (int64_t)row * cs + col;
        }
        float v = p.alpha * acc[0][i][j][r];
        if (p.beta != 0.f) v += p.beta * (*dst);
        v = apply_act(v + bv, p.act);
        if (mul) v *= mul[(int64_t)row * p.mul_sm + col];
        if (add) v += add[(int64_t)row * p.add_sm + col];
        *dst = v;
      }
    }
}

// Skinny product C[M][N] = alpha * A[M][K] . Bt[N][K]^T + beta * C with both operands' rows
// contiguous in K (a per-decoder-step [B=32] x [4U=1024] x [288] gradient product): 8 lanes
// per output element, 16-byte loads, 3 xor-shuffles -- no LDS, no barrier, 288 workgroups.
__global__ void __launch_bounds__(256) rowdot_kernel(int M, int N, int K, const float* __restrict__ A,
                                                     int64_t lda, const float* __restrict__ Bt,
                                                     int64_t ldb, float* __restrict__ C, int64_t ldc,
                                                     float alpha, float beta) {
  const int ks = threadIdx.x & 7;
  const int64_t pairg = (int64_t)blockIdx.x * 32 + (threadIdx.x >> 3);
  const int m = (int)(pairg / N), n = (int)(pairg - (int64_t)(pairg / N) * N);
  float acc = 0.f;
  if (m < M) {
    const float4* a = reinterpret_cast<const float4*>(A + m * lda);
    const float4* bt = reinterpret_cast<const float4*>(Bt + n * ldb);
#pragma unroll 8
    for (int c = ks; c < (K >> 2); c += 8) {
      const float4 x = a[c], w = bt[c];
      acc += x.x * w.x + x.y * w.y + x.z * w.z + x.w * w.w;
    }
  }
  acc += __shfl_xor(acc, 1, 64);
  acc += __shfl_xor(acc, 2, 64);
  acc += __shfl_xor(acc, 4, 64);
  if (m < M && ks == 0) {
    float* dst = C + m * ldc + n;
    *dst = beta != 0.f ? alpha * acc + beta * (*dst) : alpha * acc;
  }
}

}  // namespace
}  // namespace sat

extern "C" int sat_gemm_rowdot(int32_t M, int32_t N, int32_t K, const float* A, int64_t lda,
                               const float* Bt, int64_t ldb, float* C, int64_t ldc, float alpha,
                               float beta, void* stream) {
  using namespace sat;
  SAT_CHECK_ARG(M >= 0 && N > 0 && K >= 0 && A && Bt && C, "sat_gemm_rowdot: bad args");
  SAT_CHECK_ARG(K % 4 == 0 && lda % 4 == 0 && ldb % 4 == 0 && aligned16(A) && aligned16(Bt),
                "sat_gemm_rowdot: rows must be 16-byte aligned with K % 4 == 0");
  if (M == 0) return SAT_OK;
  const int64_t pairs = (int64_t)M * N;
  hipLaunchKernelGGL(rowdot_kernel, dim3((unsigned)((pairs + 31) / 32)), dim3(256), 0,
                     as_stream(stream), M, N, K, A, lda, Bt, ldb, C, ldc, alpha, beta);
  SAT_LAUNCH_CHECK("sat_gemm_rowdot");
  return SAT_OK;
}

using namespace sat;

template <int BM, int BN, int GM = 2, int GN = 2>
static hipError_t launch_tiles(int am, int bm, dim3 grid, hipStream_t s, const GemmP& p) {
#define SAT_GEMM_CASE(A_, B_)                                                               \
  if (am == A_ && bm == B_) {                                                               \
    hipLaunchKernelGGL((gemm_kernel<BM, BN, A_, B_, GM, GN>), grid, dim3(64 * GM * GN), 0, s, p);            \
    return hipGetLastError();                                                               \
  }
  SAT_GEMM_CASE(A_K, B_N)
  SAT_GEMM_CASE(A_K, B_K)
  SAT_GEMM_CASE(A_M, B_N)
  SAT_GEMM_CASE(A_M, B_K)
  SAT_GEMM_CASE(A_IM2COL, B_N)
  SAT_GEMM_CASE(A_IM2COL, B_FLIP)
  SAT_GEMM_CASE(A_IM2COLT, B_N)
#undef SAT_GEMM_CASE
  hipLaunchKernelGGL((gemm_kernel<BM, BN, A_GEN, B_GEN, GM, GN>), grid, dim3(64 * GM * GN), 0, s, p);
  return hipGetLastError();
}

// Tuning hook for probes (tools/probes/gemm_sweep.py): a forced tile / split-K plan for the
// calling thread's next launches on the LDS kernel (bm = 0 restores the cost model).
static thread_local int t_force_bm = 0, t_force_bn = 0, t_force_s = 0, t_probe = 0;
extern "C" int sat_gemm_probe_mode(int32_t m) {
  SAT_CHECK_ARG(m >= 0 && m <= 3, "sat_gemm_probe_mode: bad mode");
  t_probe = m;
  return SAT_OK;
}
extern "C" int sat_gemm_force_plan(int32_t bm, int32_t bn, int32_t splits) {
  SAT_CHECK_ARG(bm == 0 || ((((bm == 64 || bm == 128) && (bn == 64 || bn == 128)) ||
                              (bm == 256 && bn == 128) || (bm == 128 && bn == 256)) && splits >= 1),
                "sat_gemm_force_plan: bad plan");
  t_force_bm = bm; t_force_bn = bn; t_force_s = splits;
  return SAT_OK;
}

// SAT_GEMM_LDS=0 selects the register-staged kernel for every product (A/B switch).
static bool gemm_lds_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("SAT_GEMM_LDS");
    return !(e && e[0] == '0');
  }();
  return on;
}

// SAT_GEMM_SKINNY=0 sends M <= 8 products to the tile kernels (A/B switch).
static bool gemm_skinny_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("SAT_GEMM_SKINNY");
    return !(e && e[0] == '0');
  }();
  return on;
}

static void launch_splitk_reduce(const GemmP& p, hipStream_t s) {
  const int64_t total = (int64_t)p.M * p.N * p.nb;
  const int64_t work = (p.N % 4 == 0) ? total / 4 : total;
  const int blocks = (int)std::min<int64_t>((work + 255) / 256, 2048);
  hipLaunchKernelGGL(gemm_splitk_reduce, dim3(blocks), dim3(256), 0, s, p);
}

template <int BM, int BN>
static hipError_t launch_lds_tiles(int am, int bm, dim3 grid, hipStream_t s, const GemmP& p) {
#define SAT_GEMM_CASE(A_, B_)                                                               \
  if (am == A_ && bm == B_) {                                                               \
    hipLaunchKernelGGL((gemm_lds_kernel<BM, BN, A_, B_>), grid, dim3(64 * lds_waves<BM, BN>()), 0, s, p); \
    return hipGetLastError();                                                               \
  }
  SAT_GEMM_CASE(A_K, B_N)
  SAT_GEMM_CASE(A_K, B_K)
  SAT_GEMM_CASE(A_M, B_N)
  SAT_GEMM_CASE(A_M, B_K)
  SAT_GEMM_CASE(A_IM2COL, B_N)
  SAT_GEMM_CASE(A_IM2COL, B_FLIP)
  SAT_GEMM_CASE(A_IM2COLT, B_N)
#undef SAT_GEMM_CASE
  return hipErrorInvalidValue;
}

struct LdsPlan { int bm, bn, splits, kchunk; };

// Tile shape and split-K factor minimising a cycle model of the launch: MFMA cycles per CU
// (tiles spread over 256 CUs, BM*BN*kchunk/128 cycles per tile at an efficiency set by the
// resident waves x sub-tiles per wave) + an unhidden pipeline fill/drain per residency round
// (occupancy set by the 3-stage LDS ring) + the split-K reduce (launch + slab traffic).
// c_div: BM must divide it (im2col-T: one tap per tile); n_div: BN must divide it (conv bank).
static LdsPlan plan_lds(int M, int N, int K, int nb, bool can_split, int64_t ws_bytes, int c_div,
                        int n_div) {
  struct Cand { int bm, bn, occ; };
  // (ties go to the first: two 128x64 workgroups per CU overlap each other's epilogue)
  static const Cand cands[4] = {{128, 64, 2}, {64, 128, 2}, {128, 128, 1}, {64, 64, 3}};
  can_split = can_split && K >= 512;
  double best = 1e30;
  LdsPlan pl{0, 0, 1, K};
  for (int c = 0; c < 4; ++c) {
    const Cand& cd = cands[c];
    if ((c_div && c_div % cd.bm != 0) || (n_div && n_div % cd.bn != 0)) continue;
    const int gx = ceil_div(N, cd.bn), gy = ceil_div(M, cd.bm);
    const int64_t base = (int64_t)gx * gy * nb;
    const int smax = can_split ? std::min(64, std::max(1, K / 256)) : 1;
    for (int S = 1; S <= smax; S = (S < 4 ? S + 1 : S * 2)) {
      const int kc = (ceil_div(K, S) + BK - 1) / BK * BK;
      const int Se = ceil_div(K, kc);
      if (Se > 1 && (int64_t)Se * nb * M * N * 4 > ws_bytes) break;
      const int64_t tiles = base * Se;
      const int64_t per_cu = (tiles + 255) / 256;
      // MFMA efficiency vs resident waves x 32x32 sub-tiles per wave (probe: gemm_sweep.py)
      const int conc = (int)std::min<int64_t>(cd.occ, per_cu);
      const double eta = std::min(0.85, 0.35 + 0.2 * conc * (cd.bm / 64) * (cd.bn / 64));
      const double mfma = (double)per_cu * cd.bm * cd.bn * std::max(kc, BK) / 128.0 / eta;
      const double fill = (double)((per_cu + cd.occ - 1) / cd.occ) * 4000.0;
      // reduce launch: ~5 us measured per launch in the step (rocprof) + its slab traffic
      const double red = Se > 1 ? 2400.0 * (4.5 + (double)M * N * Se * 4 / 3.0e6) : 0.0;
      const double cost = mfma + fill + red;
      if (cost < best * 0.97) { best = cost; pl = {cd.bm, cd.bn, Se, Se > 1 ? kc : K}; }
    }
  }
  if (t_force_bm > 0) {
    if ((c_div && c_div % t_force_bm != 0) || (n_div && n_div % t_force_bn != 0)) return pl;
    int bs = can_split ? t_force_s : 1;
    const int kc = (ceil_div(K, bs) + BK - 1) / BK * BK;
    bs = ceil_div(K, kc);
    if (bs > 1 && (int64_t)bs * nb * M * N * 4 > ws_bytes) return LdsPlan{0, 0, 1, K};
    pl = {t_force_bm, t_force_bn, bs, bs > 1 ? kc : K};
  }
  return pl;
}

// Measured plans for the training step's own products (tools/gemm_census.py --sweep on one
// MI355X, profiles/r06q_gemm_census_sweep.txt: every forced tile / split-K plan of the LDS kernel
// timed on the step's descriptors): used where the best measured plan beat the cycle model's
// choice by >= 4 % (the first matching entry; a large-tile entry is followed by the plan it
// replaced, taken under SAT_GEMM_BIG=0).  Keyed on the descriptor's (M, N, K, batches, operand modes); any other
// product, a forced plan (sat_gemm_force_plan) or SAT_GEMM_PLAN_TABLE=0 takes the model.
struct PlanEntry { int M, N, K, nb, am, bm, tbm, tbn, splits; };
static const PlanEntry kMeasuredPlans[] = {
    // decoder: LSTM-stack input projection / its input gradient, the attention-LSTM weight
    // gradient over [prenet | contexts | h] rows
    {16000, 1024, 544, 1, A_K, B_N, 128, 256, 1},    // 160.3 -> 150.4 (profiles/r06ze_*)
    {16000, 1024, 544, 1, A_K, B_N, 128, 128, 1},    // 173.9 -> 160.3 us
    {16000, 544, 1024, 1, A_K, B_K, 64, 64, 2},      // 187.4 -> 176.9
    {544, 1024, 16000, 1, A_M, B_N, 64, 64, 12},     // 204.1 -> 194.5
    // weight gradients of the 128- / 256-wide dense layers (x^T dy over B T' or B N rows)
    {128, 128, 6400, 1, A_M, B_N, 64, 64, 32},       // 18.3 -> 15.6 (x 8 per step)
    {256, 256, 6400, 1, A_M, B_N, 64, 64, 12},       // 26.6 -> 23.4
    {256, 32, 6400, 1, A_M, B_N, 64, 64, 32},        // 18.5 -> 15.4
    {32, 32, 6400, 1, A_M, B_N, 64, 64, 32},         // 18.0 -> 15.1 (x 2)
    {256, 128, 16000, 1, A_M, B_N, 64, 64, 24},      // 32.0 -> 27.3
    {256, 256, 16000, 1, A_M, B_N, 64, 64, 24},      // 42.1 -> 39.8
    {256, 224, 16000, 1, A_M, B_N, 64, 64, 24},      // 41.7 -> 39.8
    {200, 256, 500, 32, A_M, B_N, 64, 64, 1},        // 33.1 -> 29.0 (memory values, batched)
    // encoder / head forward and input gradients at 6400 / 16000 rows
    {6400, 128, 128, 2, A_K, B_N, 64, 64, 1},        // 11.4 -> 10.2 (x 4)
    {6400, 256, 256, 1, A_K, B_N, 64, 64, 1},        // 25.8 -> 20.7
    {6400, 224, 256, 1, A_K, B_N, 64, 64, 1},        // 22.5 -> 18.7
    {6400, 256, 224, 1, A_K, B_K, 64, 64, 1},        // 22.9 -> 18.4
    {16000, 128, 256, 1, A_K, B_N, 64, 64, 1},       // 28.1 -> 23.0
    {16000, 1024, 128, 1, A_K, B_N, 128, 256, 1},    // 52.3 -> 48.2
    // CBHG projections (Conv1D K = 3 as im2col products)
    {6400, 128, 6144, 1, A_IM2COL, B_N, 64, 64, 6},  // 125.2 -> 116.5
    {6400, 2048, 384, 1, A_IM2COL, B_FLIP, 128, 256, 1},  // 111.5 -> 108.0
    {6400, 2048, 384, 1, A_IM2COL, B_FLIP, 64, 128, 1},   // 116.3 -> 111.5
    {6144, 128, 6400, 1, A_IM2COLT, B_N, 64, 128, 8},     // 115.7 -> 111.1
};
// SAT_GEMM_BIG=0: no 256 x 128 / 128 x 256 tile from the table or the conv bank (A/B switch)
static bool gemm_big_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("SAT_GEMM_BIG");
    return !(e && e[0] == '0');
  }();
  return on;
}
static bool gemm_plan_table_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("SAT_GEMM_PLAN_TABLE");
    return !(e && e[0] == '0');
  }();
  return on;
}
// the measured plan of a product, or {0} (then the cycle model plans it)
static LdsPlan measured_plan(int M, int N, int K, int nb, int am, int bm, bool can_split,
                             int64_t ws_bytes, int Mp, int c_div) {
  if (!gemm_plan_table_enabled() || t_force_bm > 0) return LdsPlan{0, 0, 1, K};
  for (const PlanEntry& e : kMeasuredPlans) {
    if (e.M != M || e.N != N || e.K != K || e.nb != nb || e.am != am || e.bm != bm) continue;
    if (c_div && c_div % e.tbm != 0) break;
    if ((e.tbm > 128 || e.tbn > 128) && !gemm_big_enabled()) continue;   // the next entry
    if (e.splits == 1) return LdsPlan{e.tbm, e.tbn, 1, K};
    if (!can_split) break;
    const int kc = (ceil_div(K, e.splits) + BK - 1) / BK * BK;
    const int se = ceil_div(K, kc);
    if (se > 1 && (int64_t)se * nb * Mp * N * 4 > ws_bytes) break;
    return LdsPlan{e.tbm, e.tbn, se, se > 1 ? kc : K};
  }
  return LdsPlan{0, 0, 1, K};
}

template <int BM, int BN, int GRP>
static hipError_t launch_lds_grp(int am, int bm, dim3 grid, hipStream_t s, const GemmP& p) {
  if constexpr (GRP == 0) return launch_lds_tiles<BM, BN>(am, bm, grid, s, p);
  if constexpr (GRP == 1)
    hipLaunchKernelGGL((gemm_lds_kernel<BM, BN, A_IM2COL, B_N, 1>), grid, dim3(64 * lds_waves<BM, BN>()), 0, s, p);
  if constexpr (GRP == 2)
    hipLaunchKernelGGL((gemm_lds_kernel<BM, BN, A_IM2COL, B_FLIP, 2>), grid, dim3(64 * lds_waves<BM, BN>()), 0, s, p);
  if constexpr (GRP == 3)
    hipLaunchKernelGGL((gemm_lds_kernel<BM, BN, A_IM2COLT, B_N, 3>), grid, dim3(64 * lds_waves<BM, BN>()), 0, s, p);
  return hipGetLastError();
}

template <int GRP>
static int launch_lds_plan(const LdsPlan& pl, int am, int bm, int nb, GemmP& p, hipStream_t s,
                           const char* what) {
  if (pl.bm == 0) {   // only a forced plan (sat_gemm_force_plan) can be infeasible
    set_error("%s: forced plan does not fit the split-K scratch", what);
    return SAT_ERR_ARGUMENT;
  }
  const int gx = ceil_div(p.N, pl.bn), gy = ceil_div(p.M, pl.bm);
  p.splits = pl.splits;
  p.kchunk = pl.kchunk;
  p.remap = (GRP == 0 && gx * gy >= 16) ? 1 : 0;
  p.nb = nb;
  const dim3 grid(gx, gy, pl.splits > 1 ? pl.splits * nb : nb);
  hipError_t e;
  if constexpr (GRP == 0 || GRP == 2) {
    if (pl.bm == 256 && pl.bn == 128) {
      e = launch_lds_grp<256, 128, GRP>(am, bm, grid, s, p);
      goto launched;
    }
  }
  if constexpr (GRP == 0) {
    if (pl.bm == 128 && pl.bn == 256) {
      e = launch_lds_grp<128, 256, GRP>(am, bm, grid, s, p);
      goto launched;
    }
  }
  if (pl.bm > 128 || pl.bn > 128) {
    set_error("%s: no %d x %d tile for this product", what, pl.bm, pl.bn);
    return SAT_ERR_ARGUMENT;
  }
  if (pl.bm == 128 && pl.bn == 128) e = launch_lds_grp<128, 128, GRP>(am, bm, grid, s, p);
  else if (pl.bm == 128) e = launch_lds_grp<128, 64, GRP>(am, bm, grid, s, p);
  else if (pl.bn == 128) e = launch_lds_grp<64, 128, GRP>(am, bm, grid, s, p);
  else e = launch_lds_grp<64, 64, GRP>(am, bm, grid, s, p);
launched:
  if (e != hipSuccess) {
    set_error("%s: launch failed: %s", what, hipGetErrorString(e));
    return SAT_ERR_HIP;
  }
  if (pl.splits > 1) {
    launch_splitk_reduce(p, s);
    SAT_LAUNCH_CHECK("split-k reduce");
  }
  return SAT_OK;
}

// Plan + launch on the LDS-DMA kernel.  Returns 1 (nothing launched) when an operand is not
// vector-loadable.
static int launch_lds(const SatGemmDesc* d, GemmP& p, int nb, hipStream_t s) {
  const bool astr = (p.a_sbatch % 4 == 0) && (p.a_sbatch2 % 4 == 0) && aligned16(d->A);
  const bool bstr = (p.b_sbatch % 4 == 0) && (p.b_sbatch2 % 4 == 0) && aligned16(d->B);
  int am = -1, bm = -1;
  if (d->a_mode == 0) {
    if (astr && d->a_sk == 1 && d->a_sm % 4 == 0 && d->K % 4 == 0) am = A_K;
    else if (astr && d->a_sm == 1 && d->a_sk % 4 == 0 && d->M % 4 == 0) am = A_M;
  } else if (d->a_mode == 1) {
    if (astr && d->a_sk == 1 && d->a_sm % 4 == 0 && d->a_C % BK == 0) am = A_IM2COL;
  } else {
    if (astr && d->a_sk == 1 && d->a_sm % 4 == 0 && d->a_C % 64 == 0) am = A_IM2COLT;
  }
  if (d->b_mode == 0) {
    if (bstr && d->b_sn == 1 && d->b_sk % 4 == 0 && d->N % 4 == 0) bm = B_N;
    else if (bstr && d->b_sk == 1 && d->b_sn % 4 == 0 && d->K % 4 == 0) bm = B_K;
  } else {
    if (bstr && d->b_C % BK == 0) bm = B_FLIP;
  }
  if (am < 0 || bm < 0) return 1;
  if ((am == A_IM2COL && bm != B_N && bm != B_FLIP) || (am == A_IM2COLT && bm != B_N) ||
      (bm == B_FLIP && am != A_IM2COL))
    return 1;
  if (p.cs_out && am == A_M && p.m_real % 4 != 0) return 1;   // the ones chunk must start at m_real
  // no split-K under a causal hint: the skipped tiles would leave their slab partials stale and
  // the reduce would write them into C above the diagonal
  // (a batched split-K: the reduce's epilogue has no per-batch bias / mul / add)
  const bool split_ok = (nb == 1 || (!p.bias && !p.mul && !p.add)) && d->ws != nullptr &&
                        !p.C2 && p.tri == 0;
  LdsPlan pl = measured_plan(d->M, d->N, d->K, nb, am, bm, split_ok, d->ws_bytes, p.M,
                             am == A_IM2COLT ? d->a_C : 0);
  if (pl.bm == 0)
    pl = plan_lds(p.M, d->N, d->K, nb, split_ok, d->ws_bytes, am == A_IM2COLT ? d->a_C : 0, 0);
  if (pl.bm == 0) return 1;
  return launch_lds_plan<0>(pl, am, bm, nb, p, s, "sat_gemm");
}

// Can the two reduction segments (A2 / B2) run as ONE LDS-kernel reduction?  Otherwise
// sat_gemm splits the descriptor into two accumulating launches (gemm_split_segments).
static bool segments_fused_ok(const SatGemmDesc* d) {
  return d->a_mode == 0 && d->b_mode == 0 && !d->colsum_out && d->k1 > 0 && d->k1 < d->K &&
         d->k1 % BK == 0 && gemm_lds_enabled() && !t_probe &&
         (!d->A2 || (d->a_sk == 1 && aligned16(d->A2) && d->a2_sm % 4 == 0)) &&
         (!d->B2 || (aligned16(d->B2) && d->b2_s % 4 == 0 && (d->b_sn == 1 || d->b_sk == 1)));
}

extern "C" int sat_gemm(const SatGemmDesc* d, void* stream);

// A segmented product the fused path cannot take (k1 not a multiple of the K-tile, the LDS
// kernel switched off by SAT_GEMM_LDS=0, operands not vector-loadable): C = [A | A2] [B ; B2]
// as  C = alpha A[:, :k1] B[:k1] + beta C + bias + add,  then  C += alpha A[:, k1:] B[k1:]
// (the epilogue must be linear: no activation / mul, no C2 / colsum_out).  Same result up to
// the summation order of the two partial products.
static int gemm_split_segments(const SatGemmDesc* d, void* stream) {
  SAT_CHECK_ARG(d->a_mode == 0 && d->b_mode == 0 && d->k1 > 0 && d->k1 < d->K && !d->C2 &&
                    !d->colsum_out && d->act == 0 && !d->mul,
                "sat_gemm: segmented operands outside the fused path need a dense product "
                "with 0 < k1 < K and a linear epilogue (no act / mul / C2 / colsum_out)");
  SatGemmDesc d1 = *d;
  d1.A2 = nullptr; d1.B2 = nullptr; d1.k1 = 0;
  d1.K = d->k1;
  int rc = sat_gemm(&d1, stream);
  if (rc != SAT_OK) return rc;
  SatGemmDesc d2 = *d;
  d2.A2 = nullptr; d2.B2 = nullptr; d2.k1 = 0;
  d2.K = d->K - d->k1;
  if (d->A2) { d2.A = d->A2; d2.a_sm = d->a2_sm; d2.a_sk = 1; }
  else d2.A = d->A + (int64_t)d->k1 * d->a_sk;
  if (d->B2) {
    d2.B = d->B2;
    if (d->b_sn == 1) { d2.b_sk = d->b2_s; d2.b_sn = 1; } else { d2.b_sk = 1; d2.b_sn = d->b2_s; }
  } else {
    d2.B = d->B + (int64_t)d->k1 * d->b_sk;
  }
  d2.beta = 1.f; d2.bias = nullptr; d2.bias_sbatch = 0; d2.add = nullptr;
  return sat_gemm(&d2, stream);
}

extern "C" int sat_gemm(const SatGemmDesc* d, void* stream) {
  using namespace sat;
  SAT_CHECK_ARG(d != nullptr, "sat_gemm: null descriptor");
  SAT_CHECK_ARG(d->M >= 0 && d->N >= 0 && d->K >= 0 && d->batch >= 1, "sat_gemm: bad sizes");
  SAT_CHECK_ARG(d->a_mode >= 0 && d->a_mode <= 2 && d->b_mode >= 0 && d->b_mode <= 1,
                "sat_gemm: bad operand mode");
  SAT_CHECK_ARG(d->a_mode == 0 || d->a_L > 0, "sat_gemm: conv mode needs a_L > 0");
  SAT_CHECK_ARG(d->a_mode == 0 || d->a_C > 0, "sat_gemm: im2col mode needs a_C > 0");
  SAT_CHECK_ARG(d->b_mode != 1 || (d->b_C > 0 && d->b_taps > 0), "sat_gemm: bad conv kernel");
  SAT_CHECK_ARG(d->act >= 0 && d->act <= 4, "sat_gemm: bad activation");
  if (d->M == 0 || d->N == 0) return SAT_OK;
  SAT_CHECK_ARG(d->A && d->B && d->C, "sat_gemm: null operand");
  GemmP p;
  p.M = d->M; p.N = d->N; p.K = d->K;
  p.a_mode = d->a_mode; p.a_L = d->a_L; p.a_C = d->a_C; p.a_shift = d->a_shift;
  p.A = d->A; p.a_sm = d->a_sm; p.a_sk = d->a_sk; p.a_sbatch = d->a_sbatch;
  p.b_mode = d->b_mode; p.b_taps = d->b_taps; p.b_C = d->b_C; p.act = d->act;
  p.B = d->B; p.b_sk = d->b_sk; p.b_sn = d->b_sn; p.b_sbatch = d->b_sbatch;
  p.C = d->C; p.c_sm = d->c_sm; p.c_sbatch = d->c_sbatch;
  p.bias = d->bias; p.bias_sbatch = d->bias_sbatch;
  p.alpha = d->alpha; p.beta = d->beta;
  p.mul = d->mul; p.mul_sm = d->mul_sm; p.mul_sbatch = d->mul_sbatch;
  p.batch2 = d->batch2 > 0 ? d->batch2 : 1;
  p.a_sbatch2 = d->a_sbatch2; p.b_sbatch2 = d->b_sbatch2; p.c_sbatch2 = d->c_sbatch2;
  p.mul_sbatch2 = d->mul_sbatch2;
  p.add = d->add; p.add_sm = d->add_sm; p.add_sbatch = d->add_sbatch;
  p.probe = t_probe;
  p.cs_out = nullptr;
  p.m_real = d->M;
  p.tri = (d->tri >= 1 && d->tri <= 3) ? d->tri : 0;
  // the causal hint is a plain-product option: the fused bias-gradient row, the segmented
  // operands and the second output block would each see skipped tiles / K-ranges
  SAT_CHECK_ARG(p.tri == 0 || (!d->colsum_out && !d->A2 && !d->B2 && !d->C2),
                "sat_gemm: tri cannot be combined with colsum_out, A2 / B2 or C2");
  hipStream_t s = as_stream(stream);
  const int nb = d->batch * p.batch2;
  p.ws = reinterpret_cast<float*>(d->ws);
  if (d->C2) {
    // two output column blocks: only the LDS kernel's unsplit epilogue takes them
    SAT_CHECK_ARG(nb == 1 && !d->colsum_out && !d->mul && !d->add && d->n1 > 0 && d->n1 < d->N &&
                      d->n1 % 128 == 0 && gemm_lds_enabled() && !t_probe,
                  "sat_gemm: C2 needs a batch-1 product without colsum_out / mul / add and "
                  "n1 %% 128 == 0");
    p.C2 = d->C2; p.c2_sm = d->c2_sm; p.n1 = d->n1;
  }
  if ((d->A2 || d->B2) && !segments_fused_ok(d)) return gemm_split_segments(d, stream);
  if (d->A2 || d->B2 || d->C2) {
    if (d->A2 || d->B2) {
      // two reduction segments: A2 (dense K-contiguous A) and / or B2 (dense B, B's layout)
      SAT_CHECK_ARG(d->a_mode == 0 && d->b_mode == 0 && !d->colsum_out && d->k1 > 0 &&
                        d->k1 < d->K && d->k1 % BK == 0 && gemm_lds_enabled() && !t_probe,
                    "sat_gemm: A2 / B2 need a dense product, 0 < k1 < K, k1 %% 32 == 0, "
                    "no colsum_out");
      SAT_CHECK_ARG(!d->A2 || (d->a_sk == 1 && aligned16(d->A2) && d->a2_sm % 4 == 0),
                    "sat_gemm: A2 needs K-contiguous A and 16-byte aligned A2 rows");
      SAT_CHECK_ARG(!d->B2 || (aligned16(d->B2) && d->b2_s % 4 == 0 &&
                               (d->b_sn == 1 || d->b_sk == 1)),
                    "sat_gemm: B2 needs 16-byte aligned rows / columns");
      p.A2 = d->A2; p.a2_sm = d->a2_sm; p.k1 = d->k1;
      p.B2 = d->B2; p.b2_s = d->b2_s;
    }
    const int r = launch_lds(d, p, nb, s);
    if (r == 1 && (d->A2 || d->B2) && !d->C2) return gemm_split_segments(d, stream);
    SAT_CHECK_ARG(r != 1, "sat_gemm: segmented operands are not vector-loadable");
    return r;
  }
  if (nb == 1 && d->a_mode == 0 && d->b_mode == 0 && !t_probe && d->N == 1 && d->a_sm == 1 &&
      d->M >= 64 && d->K >= 1024 && !d->bias && d->act == 0 && !d->mul && !d->add && d->ws) {
    // N == 1 weight gradient (gemm_tn1_kernel): K slices of >= 256 rows, partials reduced by
    // gemm_splitk_reduce with the usual epilogue (and the fused column sum as row m_real)
    const int Mx = d->M + (d->colsum_out ? 1 : 0);
    int S = std::min(64, d->K / 256);
    while (S > 1 && (int64_t)S * Mx * 4 > d->ws_bytes) --S;
    if (S > 1) {
      p.cs_out = d->colsum_out;
      p.cs_sbatch = 0;
      p.M = Mx;
      p.kchunk = ceil_div(d->K, S);
      p.splits = ceil_div(d->K, p.kchunk);
      hipLaunchKernelGGL(gemm_tn1_kernel, dim3(ceil_div(Mx, 64), p.splits), dim3(256), 0, s, p);
      SAT_LAUNCH_CHECK("sat_gemm (N == 1, transposed A)");
      launch_splitk_reduce(p, s);
      SAT_LAUNCH_CHECK("sat_gemm (N == 1 reduce)");
      return SAT_OK;
    }
  }
  if (d->colsum_out) {
    // C = alpha A B + beta C and colsum_out = alpha 1^T B + beta colsum_out (the bias gradient of
    // a weight-gradient product) in ONE launch: A gets a row of ones
    SAT_CHECK_ARG(p.batch2 == 1 && d->a_mode == 0 && d->b_mode == 0 && !d->bias && d->act == 0 &&
                      !d->mul && !d->add,
                  "sat_gemm: colsum_out needs a plain product with batch2 == 1 (no bias/act/mul/add)");
    // bias_sbatch == 0 means "batch 0's sums only", which is right only when every batch reads
    // the same B; with a batch-strided B the other batches' sums would be dropped silently
    SAT_CHECK_ARG(nb <= 1 || d->bias_sbatch != 0 || d->b_sbatch == 0,
                  "sat_gemm: colsum_out of a batched product with a batch-strided B needs "
                  "bias_sbatch (one [N] row per batch)");
    if (gemm_lds_enabled()) {
      p.cs_out = d->colsum_out;
      p.cs_sbatch = d->bias_sbatch;     // batch b's sums at colsum_out + b * bias_sbatch
      p.bias_sbatch = 0;
      p.M = d->M + 1;
      const int r = launch_lds(d, p, nb, s);
      if (r != 1) return r;
      p.cs_out = nullptr;
      p.M = d->M;
    }
    if (nb > 1) {   // not vector-loadable: one batch-1 product per batch
      for (int b = 0; b < nb; ++b) {
        SatGemmDesc d1 = *d;
        d1.batch = 1;
        d1.A = d->A + b * d->a_sbatch; d1.B = d->B + b * d->b_sbatch; d1.C = d->C + b * d->c_sbatch;
        d1.colsum_out = (b > 0 && d->bias_sbatch == 0) ? nullptr : d->colsum_out + b * d->bias_sbatch;
        d1.a_sbatch = d1.b_sbatch = d1.c_sbatch = d1.bias_sbatch = 0;
        const int rc = sat_gemm(&d1, stream);
        if (rc != SAT_OK) return rc;
      }
      return SAT_OK;
    }
    // operands not vector-loadable: the product, then the column sums as a separate reduction
    SatGemmDesc d2 = *d;
    d2.colsum_out = nullptr;
    const int rc = sat_gemm(&d2, stream);
    if (rc != SAT_OK) return rc;
    const int64_t need = sat_workspace_colreduce(d->K, d->N);
    SAT_CHECK_ARG(d->ws && d->ws_bytes >= need,
                  "sat_gemm: colsum_out fallback needs ws_bytes >= sat_workspace_colreduce(K, N)");
    SAT_CHECK_ARG(d->b_sn == 1, "sat_gemm: colsum_out fallback needs B rows contiguous");
    return colsum_alpha(d->B, d->b_sk, d->K, d->N, d->colsum_out, d->alpha, d->beta, d->ws, s);
  }
  if (nb == 1 && d->a_mode == 0 && d->b_mode == 0 && !t_probe && d->M <= kSkinnyM && d->N > 1 &&
      d->K > 1 && !d->mul && (int64_t)d->M * d->K * 4 + 4 * kSkinnyM * 16 * 4 <= 64 * 1024 &&
      gemm_skinny_enabled()) {
    const size_t shm = ((size_t)d->M * d->K + 4 * kSkinnyM * 16) * sizeof(float);
    hipLaunchKernelGGL(gemm_skinny_kernel, dim3(ceil_div(d->N, 16)), dim3(256), shm, s, p);
    SAT_LAUNCH_CHECK("sat_gemm (skinny)");
    return SAT_OK;
  }
  if (nb == 1 && d->a_mode == 0 && d->b_mode == 0 && !t_probe &&
      ((d->N == 1 && d->a_sk == 1) || (d->K == 1 && (int64_t)d->M * d->N < (1LL << 31)))) {
    if (d->N == 1) {
      const int vec = (d->K % 4 == 0 && d->a_sm % 4 == 0 && aligned16(d->A)) ? 1 : 0;
      hipLaunchKernelGGL(gemm_n1_kernel, dim3(ceil_div(d->M, 4)), dim3(256), 0, s, p, vec);
    } else {
      const int64_t total = (int64_t)d->M * d->N;
      hipLaunchKernelGGL(gemm_k1_kernel, dim3((int)std::min<int64_t>((total + 255) / 256, 4096)),
                         dim3(256), 0, s, p);
    }
    SAT_LAUNCH_CHECK("sat_gemm (degenerate shape)");
    return SAT_OK;
  }
  if (gemm_lds_enabled()) {
    const int r = launch_lds(d, p, nb, s);
    if (r != 1) return r;   // 1: operand layout not vector-loadable, use the register path
  }
  // 128x128 tiles when the output is large, and for long-K weight-gradient products whose
  // output is wide enough (split-K then supplies the workgroups; measured per shape with
  // tools/gemm_census.py: 544x1024x16000 354 -> 262 us, 6144x128x6400 191 -> 136 us, while
  // 256x256 / 128x512 outputs are faster on 64x64 tiles)
  const bool wide_dw = nb == 1 && d->K >= 4096 && d->ws != nullptr &&
                       ((d->M >= 256 && d->N >= 512) || d->M >= 2048);
  const bool big = ((int64_t)d->M * d->N * nb >= (int64_t)256 * 128 * 128 || wide_dw) &&
                   d->N >= 96 && d->M >= 96;
  const int BMs = big ? 128 : 64;
  // ---- operand loader variants (vector paths need 16-B aligned rows / batch strides)
  const bool astr = (p.a_sbatch % 4 == 0) && (p.a_sbatch2 % 4 == 0) && aligned16(d->A);
  const bool bstr = (p.b_sbatch % 4 == 0) && (p.b_sbatch2 % 4 == 0) && aligned16(d->B);
  int am = A_GEN, bm = B_GEN;
  if (d->a_mode == 0) {
    if (astr && d->a_sk == 1 && d->a_sm % 4 == 0 && d->K % 4 == 0) am = A_K;
    else if (astr && d->a_sm == 1 && d->a_sk % 4 == 0 && d->M % 4 == 0) am = A_M;
  } else if (d->a_mode == 1) {
    if (astr && d->a_sk == 1 && d->a_sm % 4 == 0 && d->a_C % BK == 0) am = A_IM2COL;
  } else {
    if (astr && d->a_sk == 1 && d->a_sm % 4 == 0 && d->a_C % BMs == 0) am = A_IM2COLT;
  }
  if (d->b_mode == 0) {
    if (bstr && d->b_sn == 1 && d->b_sk % 4 == 0 && d->N % 4 == 0) bm = B_N;
    else if (bstr && d->b_sk == 1 && d->b_sn % 4 == 0 && d->K % 4 == 0) bm = B_K;
  } else {
    if (bstr && d->b_C % BK == 0) bm = B_FLIP;
  }
  if (am == A_GEN || bm == B_GEN) { am = A_GEN; bm = B_GEN; }   // instantiated combinations
  const int gx = ceil_div(d->N, BMs), gy = ceil_div(d->M, BMs);
  const int tiles = gx * gy * nb;
  // split-K for weight-gradient-shaped products (few output tiles, long reduction)
  p.splits = 1;
  p.kchunk = d->K;
  p.ws = reinterpret_cast<float*>(d->ws);
  if (nb == 1 && tiles < 160 && d->K >= 512 && d->ws != nullptr) {
    int S = std::min<int>(std::max(1, 384 / tiles), std::max(1, d->K / 256));
    S = std::min(S, 64);
    while (S > 1 && (int64_t)S * d->M * d->N * 4 > d->ws_bytes) --S;
    if (S > 1) {
      p.kchunk = (ceil_div(d->K, S) + BK - 1) / BK * BK;
      S = ceil_div(d->K, p.kchunk);
      p.splits = S;
    }
  }
  p.remap = (gx * gy >= 16) ? 1 : 0;
  const int gz = p.splits > 1 ? p.splits : nb;
  const dim3 grid(gx, gy, gz);
  // (a 4x2-wave 128x128 variant, gemm_kernel<128, 128, ., ., 4, 2>, measured 2-15 % slower on
  // the step's shapes: tile and wave shape are not what limits this kernel)
  const hipError_t e = big ? launch_tiles<128, 128>(am, bm, grid, s, p)
                           : launch_tiles<64, 64>(am, bm, grid, s, p);
  if (e != hipSuccess) {
    set_error("sat_gemm: launch failed: %s", hipGetErrorString(e));
    return SAT_ERR_HIP;
  }
  if (p.splits > 1) {
    const int64_t total = (int64_t)d->M * d->N;
    const int64_t work = (d->N % 4 == 0) ? total / 4 : total;
    const int blocks = (int)std::min<int64_t>((work + 255) / 256, 2048);
    hipLaunchKernelGGL(gemm_splitk_reduce, dim3(blocks), dim3(256), 0, s, p);
    SAT_LAUNCH_CHECK("sat_gemm(split-k reduce)");
  }
  return SAT_OK;
}

// ---------------------------------------------------------------- CBHG conv bank (one launch
// per direction instead of max_k; see include/sat_abi.h)
static int convbank_check(const SatConvBank* d) {
  SAT_CHECK_ARG(d != nullptr, "sat_cbhg_convbank: null descriptor");
  SAT_CHECK_ARG(d->S > 0 && d->L > 0 && d->max_k >= 1 && d->max_k <= 64,
                "sat_cbhg_convbank: bad sizes");
  SAT_CHECK_ARG(d->C > 0 && d->C % 64 == 0 && d->Co > 0 && d->Co % 64 == 0,
                "sat_cbhg_convbank: C and Co must be multiples of 64");
  SAT_CHECK_ARG(d->x && d->W && d->y && aligned16(d->x) && aligned16(d->W) && aligned16(d->y) &&
                    d->x_sm % 4 == 0 && d->y_sm % 4 == 0 && d->x_sm >= d->C &&
                    d->y_sm >= (int64_t)d->max_k * d->Co,
                "sat_cbhg_convbank: operands must be 16-byte aligned rows");
  return SAT_OK;
}

static GemmP convbank_base(const SatConvBank* d) {
  GemmP p;
  std::memset(&p, 0, sizeof(p));
  p.batch2 = 1;
  p.alpha = 1.f;
  p.a_L = d->L;
  p.grp_co = d->Co;
  p.ws = reinterpret_cast<float*>(d->ws);
  p.probe = t_probe;
  return p;
}

extern "C" int sat_cbhg_convbank_fwd(const SatConvBank* d, void* stream) {
  const int r = convbank_check(d);
  if (r != SAT_OK) return r;
  GemmP p = convbank_base(d);
  p.M = d->S * d->L;
  p.N = d->max_k * d->Co;
  p.K = d->max_k * d->C;                    // longest reduction (K_max); per tile (k) * C
  p.a_mode = 1; p.a_C = d->C;
  p.A = d->x; p.a_sm = d->x_sm; p.a_sk = 1;
  p.B = d->W; p.b_sk = d->Co; p.b_sn = 1;
  p.C = d->y; p.c_sm = d->y_sm;
  p.bias = d->bias;
  // plan on the mean reduction; no split (3,200 tiles at the C2 shape already fill the chip)
  LdsPlan pl = plan_lds(p.M, p.N, (d->max_k + 1) * d->C / 2, 1, false, 0, 0, d->Co);
  // measured at the C2 shape (tools/probes/conv_sol.py): 64x128 352 us, 64x64 384, 128x* 405
  // (row-major dispatch; longest-first dispatch, gemm_lds_kernel, takes 64x128 to 282 us)
  if ((t_force_bm == 0 || pl.bm > 128 || pl.bn > 128) && d->Co % 128 == 0) pl = {64, 128, 1, p.K};
  else if (pl.bm > 128 || pl.bn > 128) pl = {64, 64, 1, p.K};   // no large tile for this launch
  LdsPlan fixed = pl;
  fixed.splits = 1;
  fixed.kchunk = p.K;
  return launch_lds_plan<1>(fixed, A_IM2COL, B_N, 1, p, as_stream(stream),
                            "sat_cbhg_convbank_fwd");
}

extern "C" int sat_cbhg_convbank_bwd(const SatConvBank* d, void* stream) {
  const int r = convbank_check(d);
  if (r != SAT_OK) return r;
  hipStream_t s = as_stream(stream);
  const int pairs = d->max_k * (d->max_k + 1) / 2;     // (k, tap) pairs of the bank
  if (d->dW) {
    SAT_CHECK_ARG(aligned16(d->dW), "sat_cbhg_convbank_bwd: dW must be 16-byte aligned");
    GemmP p = convbank_base(d);
    p.M = pairs * d->C; p.N = d->Co; p.K = d->S * d->L;
    p.a_mode = 2; p.a_C = d->C;
    p.A = d->x; p.a_sm = d->x_sm; p.a_sk = 1;
    p.B = d->y; p.b_sk = d->y_sm; p.b_sn = 1;
    p.C = d->dW; p.c_sm = d->Co;
    p.beta = d->beta_dw;
    LdsPlan pl = plan_lds(p.M, p.N, p.K, 1, d->ws != nullptr, d->ws_bytes, d->C, 0);
    // a dW-only call is the caller running it beside the dX product on another stream (the
    // training step): measured as that pair at the C2 shape (tools/probes/bank_dw_plans.py),
    // 128 x 128 tiles split 2 take 640 us with dX against 728 for the cost model's choice, whose
    // larger grid crowds the dX product out (alone they are 494 / 368 us, so a call doing both
    // products serially keeps the cost model); the step 13.99 -> 13.91 ms (profiles/r05q_tail_ab.txt)
    const int kc2 = (ceil_div(p.K, 2) + BK - 1) / BK * BK;
    if (t_force_bm == 0 && !d->dx && d->C % 128 == 0 && p.K >= 4096 && d->ws != nullptr &&
        (int64_t)ceil_div(p.K, kc2) * p.M * p.N * 4 <= d->ws_bytes)
      pl = {128, 128, ceil_div(p.K, kc2), kc2};
    const int e = launch_lds_plan<3>(pl, A_IM2COLT, B_N, 1, p, s, "sat_cbhg_convbank_bwd(dW)");
    if (e != SAT_OK) return e;
  }
  if (d->dx) {
    SAT_CHECK_ARG(aligned16(d->dx) && d->dx_sm % 4 == 0 && d->dx_sm >= d->C,
                  "sat_cbhg_convbank_bwd: dx must be 16-byte aligned rows");
    GemmP p = convbank_base(d);
    p.M = d->S * d->L; p.N = d->C; p.K = pairs * d->Co;
    p.a_mode = 1; p.a_C = d->Co;
    p.A = d->y; p.a_sm = d->y_sm; p.a_sk = 1;
    p.b_mode = 1; p.b_C = d->Co; p.b_taps = d->max_k;
    p.B = d->W;
    p.C = d->dx; p.c_sm = d->dx_sm;
    p.beta = d->beta_dx;
    LdsPlan pl = plan_lds(p.M, p.N, p.K, 1, d->ws != nullptr, d->ws_bytes, 0, 0);
    // measured at the C2 shape (tools/probes/convbank_bwd_probe.py): 128 x 128 tiles split 4
    // ways 373 us, the cost model's choice 414 (odd splits 490+: their chunks straddle banks);
    // 256 x 128 tiles split 8 ways (200 workgroups, 56 CUs left to the weight gradient beside
    // it): 366 -> 315 us alone, 642 -> 590 us with the weight gradient on a second stream
    // (tools/probes/big_tile_probe.py, profiles/r06ze_big_tile_probe.txt)
    const bool big = gemm_big_enabled() && d->C % 128 == 0;
    const int ns = big ? 8 : 4;
    const int kcs = (ceil_div(p.K, ns) + BK - 1) / BK * BK;
    if (t_force_bm == 0 && d->C % 128 == 0 && p.M >= 4096 && d->ws != nullptr &&
        (int64_t)ceil_div(p.K, kcs) * p.M * p.N * 4 <= d->ws_bytes)
      pl = {big ? 256 : 128, 128, ceil_div(p.K, kcs), kcs};
    const int e = launch_lds_plan<2>(pl, A_IM2COL, B_FLIP, 1, p, s, "sat_cbhg_convbank_bwd(dX)");
    if (e != SAT_OK) return e;
  }
  return SAT_OK;
}
