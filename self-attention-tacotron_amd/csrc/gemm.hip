// fp32 GEMM on CDNA4 matrix cores: v_mfma_f32_32x32x2_f32 (exact f32, = the f32 vector peak).
//
// One kernel template serves every dense product of the path: Dense layers, batched attention
// products, the Conv1D(SAME) of the CBHG (implicit im2col in the A loader -- no im2col buffer
// in HBM) and all their gradients (transposes are strides; conv dX / dW are A/B modes).
//
// Tile: BM x BN x 16, 256 threads = 4 waves in a 2x2 grid, each wave (BM/2)x(BN/2) made of
// 32x32 MFMA sub-tiles.  Global -> registers (next tile prefetched while the current one is
// multiplied) -> LDS ([k][m] / [k][n] images, +1 padding so the transposing stores are
// conflict-free) -> one f32 per lane per MFMA operand (ds_read_b32, contiguous per 32 lanes).
#include "sat_common.h"

namespace sat {
namespace {

using f32x16 = __attribute__((ext_vector_type(16))) float;

constexpr int BK = 16;

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
  int a_kcontig, b_ncontig;
};

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
  // mode 2: transposed im2col, (i, k) -> im2col(k, i)
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
    default: return v;
  }
}

template <int BM, int BN>
__global__ void __launch_bounds__(256) gemm_kernel(GemmP p) {
  constexpr int WM = BM / 2, WN = BN / 2;         // per-wave tile
  constexpr int SM = WM / 32, SN = WN / 32;       // 32x32 sub-tiles per wave
  constexpr int EA = BM * BK / 256, EB = BN * BK / 256;
  __shared__ float As[BK][BM + 1];
  __shared__ float Bs[BK][BN + 1];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = (wave >> 1) * WM, wn = (wave & 1) * WN;
  const int bz = blockIdx.z / p.batch2, bz2 = blockIdx.z - bz * p.batch2;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const float* A = p.A + bz * p.a_sbatch + bz2 * p.a_sbatch2;
  const float* B = p.B + bz * p.b_sbatch + bz2 * p.b_sbatch2;

  float ra[EA], rb[EB];
  auto fetch = [&](int k0) {
#pragma unroll
    for (int i = 0; i < EA; ++i) {
      const int e = tid + i * 256;
      int m, k;
      if (p.a_kcontig) { m = e / BK; k = e % BK; } else { k = e / BM; m = e % BM; }
      ra[i] = load_a(p, A, m0 + m, k0 + k);
    }
#pragma unroll
    for (int i = 0; i < EB; ++i) {
      const int e = tid + i * 256;
      int k, n;
      if (p.b_ncontig) { k = e / BN; n = e % BN; } else { n = e / BK; k = e % BK; }
      rb[i] = load_b(p, B, k0 + k, n0 + n);
    }
  };
  auto stash = [&]() {
#pragma unroll
    for (int i = 0; i < EA; ++i) {
      const int e = tid + i * 256;
      int m, k;
      if (p.a_kcontig) { m = e / BK; k = e % BK; } else { k = e / BM; m = e % BM; }
      As[k][m] = ra[i];
    }
#pragma unroll
    for (int i = 0; i < EB; ++i) {
      const int e = tid + i * 256;
      int k, n;
      if (p.b_ncontig) { k = e / BN; n = e % BN; } else { n = e / BK; k = e % BK; }
      Bs[k][n] = rb[i];
    }
  };

  f32x16 acc[SM][SN];
#pragma unroll
  for (int i = 0; i < SM; ++i)
#pragma unroll
    for (int j = 0; j < SN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int nk = (p.K + BK - 1) / BK;
  fetch(0);
  stash();
  __syncthreads();
  const int li = lane & 31, lk = lane >> 5;
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) fetch((kt + 1) * BK);
#pragma unroll
    for (int kk = 0; kk < BK; kk += 2) {
      float a[SM], b[SN];
#pragma unroll
      for (int i = 0; i < SM; ++i) a[i] = As[kk + lk][wm + i * 32 + li];
#pragma unroll
      for (int j = 0; j < SN; ++j) b[j] = Bs[kk + lk][wn + j * 32 + li];
#pragma unroll
      for (int i = 0; i < SM; ++i)
#pragma unroll
        for (int j = 0; j < SN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
    if (kt + 1 < nk) {
      stash();
      __syncthreads();
    }
  }

  // epilogue: C/D map of 32x32 f32 MFMA: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
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

}  // namespace
}  // namespace sat

extern "C" int sat_gemm(const SatGemmDesc* d, void* stream) {
  using namespace sat;
  SAT_CHECK_ARG(d != nullptr, "sat_gemm: null descriptor");
  SAT_CHECK_ARG(d->M >= 0 && d->N >= 0 && d->K >= 0 && d->batch >= 1, "sat_gemm: bad sizes");
  SAT_CHECK_ARG(d->a_mode >= 0 && d->a_mode <= 2 && d->b_mode >= 0 && d->b_mode <= 1,
                "sat_gemm: bad operand mode");
  SAT_CHECK_ARG(d->a_mode == 0 || d->a_L > 0, "sat_gemm: conv mode needs a_L > 0");
  SAT_CHECK_ARG(d->a_mode == 0 || d->a_C > 0, "sat_gemm: im2col mode needs a_C > 0");
  SAT_CHECK_ARG(d->b_mode != 1 || (d->b_C > 0 && d->b_taps > 0), "sat_gemm: bad conv kernel");
  SAT_CHECK_ARG(d->act >= 0 && d->act <= 3, "sat_gemm: bad activation");
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
  // coalescing order of the tile loaders
  p.a_kcontig = (d->a_mode == 1) ? 1 : (d->a_mode == 2 ? 0 : (d->a_sk == 1 ? 1 : 0));
  p.b_ncontig = (d->b_mode == 1) ? 0 : (d->b_sn == 1 ? 1 : 0);
  hipStream_t s = as_stream(stream);
  const bool big = (int64_t)d->M * d->N >= (int64_t)256 * 128 * 128 && d->N >= 96 && d->M >= 96;
  if (big) {
    dim3 grid(ceil_div(d->N, 128), ceil_div(d->M, 128), d->batch * p.batch2);
    hipLaunchKernelGGL((gemm_kernel<128, 128>), grid, dim3(256), 0, s, p);
  } else {
    dim3 grid(ceil_div(d->N, 64), ceil_div(d->M, 64), d->batch * p.batch2);
    hipLaunchKernelGGL((gemm_kernel<64, 64>), grid, dim3(256), 0, s, p);
  }
  SAT_LAUNCH_CHECK("sat_gemm");
  return SAT_OK;
}
