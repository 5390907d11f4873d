// Bandwidth-bound kernels of the path: memory masking, embedding, BatchNormalization, max-pool,
// highway combine, row softmax (self-attention), activation backward, the fused loss.
// All reductions are deterministic (fixed per-thread order + fixed-shape tree), except the
// embedding backward scatter-add (deterministic: one workgroup per table row, ids scanned in order).
#include "sat_common.h"

namespace sat {
namespace {

inline int grid_for(int64_t n, int block = 256, int cap = 4096) {
  return (int)std::max<int64_t>(1, std::min<int64_t>((n + block - 1) / block, cap));
}

#define GRID_STRIDE(i, n) \
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < (n); i += (int64_t)gridDim.x * blockDim.x)

// ---------------------------------------------------------------- memory masking
__global__ void seq_mask_kernel(const float* __restrict__ x, float* __restrict__ out, int B, int N,
                                int C, const int64_t* __restrict__ lengths) {
  const int64_t total = (int64_t)B * N * C;
  GRID_STRIDE(i, total) {
    const int64_t row = i / C;
    const int b = (int)(row / N), n = (int)(row - (int64_t)b * N);
    out[i] = n < lengths[b] ? x[i] : 0.f;
  }
}

// ---------------------------------------------------------------- embedding (ext tacotron2)
__global__ void embed_fwd_kernel(const float* __restrict__ table, const int64_t* __restrict__ ids,
                                 float* __restrict__ out, int64_t R, int D, int V, int64_t offset,
                                 int* err) {
  GRID_STRIDE(i, R * D) {
    const int64_t r = i / D;
    const int c = (int)(i - r * D);
    const int64_t id = ids[r] - offset;
    if (id < 0 || id >= V) {
      out[i] = 0.f;
      if (err) *err = 1;
    } else {
      out[i] = table[id * D + c];
    }
  }
}

// Deterministic scatter-add: one workgroup per (table row v, 256-column block) scans the ids in
// chunks of 256 and adds the rows that hit v in ascending r -- a fixed summation order, so the
// gradient is bit-reproducible run to run (fp32 atomics are not: their order follows timing).
// Per chunk each wave ballots its 64 ids against v; the matches are then walked lowest bit first.
__global__ void __launch_bounds__(256) embed_bwd_kernel(const float* __restrict__ dout,
                                                        const int64_t* __restrict__ ids,
                                                        float* __restrict__ dtable, int64_t R,
                                                        int D, int V, int64_t offset) {
  __shared__ unsigned long long hit[4];
  const int v = blockIdx.x, c = blockIdx.y * 256 + threadIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float acc = 0.f;
  bool any = false;
  for (int64_t r0 = 0; r0 < R; r0 += 256) {
    const int64_t r = r0 + threadIdx.x;
    const bool m = r < R && ids[r] - offset == v;
    const unsigned long long b = __builtin_amdgcn_ballot_w64(m);
    if (lane == 0) hit[wave] = b;
    __syncthreads();
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      unsigned long long bits = hit[w];
      while (bits) {
        const int k = __builtin_ctzll(bits);
        bits &= bits - 1;
        any = true;
        if (c < D) acc += dout[(r0 + 64 * w + k) * D + c];
      }
    }
    __syncthreads();
  }
  if (any && c < D) dtable[(int64_t)v * D + c] += acc;
}

// Two-phase variant for R <= kEmbRows: (1) the workgroup lists the rows that hit v in
// ascending order in LDS (every thread's ids loaded up front, then per 256-row chunk a ballot and
// a popcount prefix place each match); (2) each column thread sums its list entries in list order
// with kEmbG loads in flight -- the same row-ordered sum as embed_bwd_kernel, without one
// dependent load latency per hit.
constexpr int kEmbRows = 8192, kEmbG = 8;
__global__ void __launch_bounds__(256) embed_bwd_list_kernel(const float* __restrict__ dout,
                                                             const int64_t* __restrict__ ids,
                                                             float* __restrict__ dtable, int R,
                                                             int D, int64_t offset) {
  __shared__ int list[kEmbRows];
  __shared__ int wcount[2][4];
  const int v = blockIdx.x, c = blockIdx.y * 256 + threadIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  constexpr int kPer = kEmbRows / 256;
  bool hit[kPer];
#pragma unroll
  for (int i = 0; i < kPer; ++i) {
    const int r = i * 256 + threadIdx.x;
    hit[i] = r < R && ids[r] - offset == v;
  }
  int n = 0;
  const unsigned long long below = (1ull << lane) - 1ull;
#pragma unroll
  for (int i = 0; i < kPer; ++i) {
    if (i * 256 >= R) break;
    const unsigned long long b = __builtin_amdgcn_ballot_w64(hit[i]);
    if (lane == 0) wcount[i & 1][wave] = __builtin_popcountll(b);
    __syncthreads();
    int base = n;
    for (int w = 0; w < wave; ++w) base += wcount[i & 1][w];
    if (hit[i]) list[base + __builtin_popcountll(b & below)] = i * 256 + threadIdx.x;
    n += wcount[i & 1][0] + wcount[i & 1][1] + wcount[i & 1][2] + wcount[i & 1][3];
  }
  __syncthreads();
  if (n == 0 || c >= D) return;
  float acc = 0.f;
  for (int j0 = 0; j0 < n; j0 += kEmbG) {
    float x[kEmbG];
#pragma unroll
    for (int k = 0; k < kEmbG; ++k) {
      const int j = min(j0 + k, n - 1);
      x[k] = dout[(int64_t)list[j] * D + c];
    }
#pragma unroll
    for (int k = 0; k < kEmbG; ++k)
      if (j0 + k < n) acc += x[k];
  }
  dtable[(int64_t)v * D + c] += acc;
}

// ---------------------------------------------------------------- column reductions
// out1[c] = sum_m x[m, c]  (and out2[c] = sum_m x[m,c]*y[m,c] when y != null), fp64 accumulation.
// Block = 256 threads = 64 columns x 4 row groups; grid = ceil(C/64) x RB row blocks (partials
// combined by a second pass in colreduce_finish).
__global__ void colreduce_kernel(const float* __restrict__ x, int64_t ldx, const float* __restrict__ y,
                                 int64_t ldy, int M, int C, double* __restrict__ part1,
                                 double* __restrict__ part2, int mode, const float* __restrict__ mean,
                                 const float* __restrict__ var, float eps, const float* __restrict__ gate,
                                 int64_t ldg) {
  // mode 0: sum(x), sum(x*x)         (BN statistics; part2 = sum of squares)
  // mode 1: sum(dy), sum(dy * xhat)  (BN backward; x = dy, y = pre-BN input, mean/var given,
  //                                   gate = post-BN ReLU output or null)
  // mode 2: sum(x), sum(x * y)       (bias grads / generic)
  __shared__ double s1[4][64], s2[4][64];
  const int lane = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const int rows_per = (M + gridDim.y - 1) / gridDim.y;
  const int r0 = blockIdx.y * rows_per, r1 = min(M, r0 + rows_per);
  double a1 = 0.0, a2 = 0.0;
  if (c < C) {
    float mu = 0.f, rs = 0.f;
    if (mode == 1) { mu = mean[c]; rs = rsqrtf(var[c] + eps); }
    // 4 rows per trip, their loads issued together (the trip is latency-bound otherwise)
    int m = r0 + grp;
    for (; m + 12 < r1; m += 16) {
      float v[4], w[4], gv[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int64_t mm = m + 4 * q;
        v[q] = x[mm * ldx + c];
        w[q] = (mode == 1 || (mode == 2 && y)) ? y[mm * ldy + c] : 0.f;
        gv[q] = (mode == 1 && gate) ? gate[mm * ldg + c] : 1.f;
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (mode == 0) { a1 += v[q]; a2 += (double)v[q] * v[q]; }
        else if (mode == 1) {
          const float g = gv[q] <= 0.f ? 0.f : v[q];
          a1 += g; a2 += (double)g * ((w[q] - mu) * rs);
        } else {
          a1 += v[q];
          if (y) a2 += (double)v[q] * w[q];
        }
      }
    }
    for (; m < r1; m += 4) {
      float v = x[(int64_t)m * ldx + c];
      if (mode == 0) { a1 += v; a2 += (double)v * v; }
      else if (mode == 1) {
        if (gate && gate[(int64_t)m * ldg + c] <= 0.f) v = 0.f;
        const float xh = (y[(int64_t)m * ldy + c] - mu) * rs;
        a1 += v; a2 += (double)v * xh;
      } else {
        a1 += v;
        if (y) a2 += (double)v * y[(int64_t)m * ldy + c];
      }
    }
  }
  s1[grp][lane] = a1;
  s2[grp][lane] = a2;
  __syncthreads();
  if (grp == 0 && c < C) {
    part1[(int64_t)blockIdx.y * C + c] = s1[0][lane] + s1[1][lane] + s1[2][lane] + s1[3][lane];
    part2[(int64_t)blockIdx.y * C + c] = s2[0][lane] + s2[1][lane] + s2[2][lane] + s2[3][lane];
  }
}

// sum of the RB row-block partials of column c: block = 64 columns x 4 row slices, every
// thread's loads issued together, the 4 slices combined in a fixed order (deterministic)
__device__ __forceinline__ void sum_partials(const double* part1, const double* part2, int RB, int C,
                                             int c, double& s, double& q) {
  __shared__ double r1[4][64], r2[4][64];
  const int lane = threadIdx.x & 63, sl = threadIdx.x >> 6;
  double a = 0.0, b = 0.0;
  if (c < C) {
#pragma unroll 16
    for (int r = sl; r < RB; r += 4) { a += part1[(int64_t)r * C + c]; b += part2[(int64_t)r * C + c]; }
  }
  r1[sl][lane] = a;
  r2[sl][lane] = b;
  __syncthreads();
  s = (r1[0][lane] + r1[1][lane]) + (r1[2][lane] + r1[3][lane]);
  q = (r2[0][lane] + r2[1][lane]) + (r2[2][lane] + r2[3][lane]);
}

// BN statistics finish: mean, biased var; moving averages (momentum, Bessel-corrected var).
__global__ void bn_stats_finish_kernel(const double* part1, const double* part2, int RB, int M, int C,
                                       float* mean, float* var, float* mov_mean, float* mov_var,
                                       float momentum) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  double s, q;
  sum_partials(part1, part2, RB, C, c, s, q);
  if (threadIdx.x < 64 && c < C) {
    const double mu = s / M;
    const double v = fmax(q / M - mu * mu, 0.0);
    mean[c] = (float)mu;
    var[c] = (float)v;
    if (mov_mean) {
      const double unb = M > 1 ? v * M / (M - 1) : v;
      mov_mean[c] = (float)(momentum * mov_mean[c] + (1.0 - momentum) * mu);
      mov_var[c] = (float)(momentum * mov_var[c] + (1.0 - momentum) * unb);
    }
  }
}

// generic finish: out1[c] = beta*out1[c] + sum1 ; out2 likewise (either may be null)
// and, when given, acc1[c] += sum1, acc2[c] += sum2 (gradient accumulation)
__global__ void colreduce_finish_kernel(const double* part1, const double* part2, int RB, int C,
                                        float* out1, float* out2, float beta, float* acc1,
                                        float* acc2) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  double s, q;
  sum_partials(part1, part2, RB, C, c, s, q);
  if (threadIdx.x < 64 && c < C) {
    if (out1) out1[c] = beta != 0.f ? (float)(beta * out1[c] + s) : (float)s;
    if (out2) out2[c] = beta != 0.f ? (float)(beta * out2[c] + q) : (float)q;
    if (acc1) acc1[c] += (float)s;
    if (acc2) acc2[c] += (float)q;
  }
}

// ---------------------------------------------------------------- BatchNormalization apply / bwd
__global__ void bn_apply_kernel(const float* __restrict__ x, int64_t ldx, float* __restrict__ y,
                                int64_t ldy, int M, int C, const float* __restrict__ mean,
                                const float* __restrict__ var, float eps, const float* __restrict__ gamma,
                                const float* __restrict__ beta, int relu, const float* __restrict__ res,
                                int64_t ldr) {
  GRID_STRIDE(i, (int64_t)M * C) {
    const int64_t m = i / C;
    const int c = (int)(i - m * C);
    float v = gamma[c] * (x[m * ldx + c] - mean[c]) * rsqrtf(var[c] + eps) + beta[c];
    if (relu) v = fmaxf(v, 0.f);
    if (res) v += res[m * ldr + c];
    y[m * ldy + c] = v;
  }
}

// float4 variants of the two BN element passes (C and every leading dimension % 4 == 0,
// 16-byte aligned, M*C < 2^31): 32-bit row arithmetic once per four channels and 16-byte
// accesses; per element the same expressions as the scalar kernels (bit-identical)
// one BN(+ReLU) output element (shared by bn_apply4_kernel and bn_apply_pool4c_kernel so the two
// produce the same bits)
__device__ __forceinline__ float bn_val(float x, float g, float m, float v, float b, float eps,
                                        int relu) {
  float o = g * (x - m) * rsqrtf(v + eps) + b;
  if (relu) o = fmaxf(o, 0.f);
  return o;
}

__global__ void bn_apply4_kernel(const float* __restrict__ x, int ldx, float* __restrict__ y,
                                 int ldy, int M, int C, const float* __restrict__ mean,
                                 const float* __restrict__ var, float eps,
                                 const float* __restrict__ gamma, const float* __restrict__ beta,
                                 int relu, const float* __restrict__ res, int ldr) {
  const int C4 = C >> 2, n4 = M * C4;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < n4; e += gridDim.x * blockDim.x) {
    const int m = e / C4, c = 4 * (e - m * C4);
    const float4 xv = *reinterpret_cast<const float4*>(x + m * ldx + c);
    const float4 mu = *reinterpret_cast<const float4*>(mean + c);
    const float4 va = *reinterpret_cast<const float4*>(var + c);
    const float4 ga = *reinterpret_cast<const float4*>(gamma + c);
    const float4 be = *reinterpret_cast<const float4*>(beta + c);
    float4 rv = make_float4(0.f, 0.f, 0.f, 0.f);
    if (res) rv = *reinterpret_cast<const float4*>(res + m * ldr + c);
    const float xs[4] = {xv.x, xv.y, xv.z, xv.w}, ms[4] = {mu.x, mu.y, mu.z, mu.w};
    const float vs[4] = {va.x, va.y, va.z, va.w}, gs[4] = {ga.x, ga.y, ga.z, ga.w};
    const float bs[4] = {be.x, be.y, be.z, be.w}, rs[4] = {rv.x, rv.y, rv.z, rv.w};
    float o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float v = bn_val(xs[k], gs[k], ms[k], vs[k], bs[k], eps, relu);
      if (res) v += rs[k];
      o[k] = v;
    }
    *reinterpret_cast<float4*>(y + m * ldy + c) = make_float4(o[0], o[1], o[2], o[3]);
  }
}

__global__ void bn_bwd_apply4_kernel(const float* __restrict__ dy, int lddy,
                                     const float* __restrict__ x, int ldx,
                                     const float* __restrict__ gate, int ldg,
                                     float* __restrict__ dx, int lddx, int M, int C,
                                     const float* __restrict__ mean, const float* __restrict__ var,
                                     float eps, const float* __restrict__ gamma,
                                     const float* __restrict__ sum_dy,
                                     const float* __restrict__ sum_dyx, int training,
                                     float beta_out) {
  const int C4 = C >> 2, n4 = M * C4;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < n4; e += gridDim.x * blockDim.x) {
    const int m = e / C4, c = 4 * (e - m * C4);
    const float4 gv = *reinterpret_cast<const float4*>(dy + m * lddy + c);
    float4 gt = make_float4(1.f, 1.f, 1.f, 1.f), xv = gt, ov = make_float4(0.f, 0.f, 0.f, 0.f);
    if (gate) gt = *reinterpret_cast<const float4*>(gate + m * ldg + c);
    if (training) xv = *reinterpret_cast<const float4*>(x + m * ldx + c);
    if (beta_out != 0.f) ov = *reinterpret_cast<const float4*>(dx + m * lddx + c);
    const float4 va = *reinterpret_cast<const float4*>(var + c);
    const float4 ga = *reinterpret_cast<const float4*>(gamma + c);
    float4 mu = make_float4(0.f, 0.f, 0.f, 0.f), s1 = mu, s2 = mu;
    if (training) {
      mu = *reinterpret_cast<const float4*>(mean + c);
      s1 = *reinterpret_cast<const float4*>(sum_dy + c);
      s2 = *reinterpret_cast<const float4*>(sum_dyx + c);
    }
    const float gs[4] = {gv.x, gv.y, gv.z, gv.w}, ts[4] = {gt.x, gt.y, gt.z, gt.w};
    const float xs[4] = {xv.x, xv.y, xv.z, xv.w}, os[4] = {ov.x, ov.y, ov.z, ov.w};
    const float vs[4] = {va.x, va.y, va.z, va.w}, gms[4] = {ga.x, ga.y, ga.z, ga.w};
    const float ms[4] = {mu.x, mu.y, mu.z, mu.w}, s1s[4] = {s1.x, s1.y, s1.z, s1.w};
    const float s2s[4] = {s2.x, s2.y, s2.z, s2.w};
    float o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float g = gs[k];
      if (gate && ts[k] <= 0.f) g = 0.f;
      const float rs = rsqrtf(vs[k] + eps);
      float v;
      if (training) {
        const float xh = (xs[k] - ms[k]) * rs;
        v = gms[k] * rs * (g - s1s[k] / M - xh * s2s[k] / M);
      } else {
        v = gms[k] * rs * g;
      }
      o[k] = beta_out != 0.f ? beta_out * os[k] + v : v;
    }
    *reinterpret_cast<float4*>(dx + m * lddx + c) = make_float4(o[0], o[1], o[2], o[3]);
  }
}

// dx = gamma*rstd*(g - s1/M - xhat*s2/M)   (training) ; gamma*rstd*g (eval), g = gated dy
__global__ void bn_bwd_apply_kernel(const float* __restrict__ dy, int64_t lddy, const float* __restrict__ x,
                                    int64_t ldx, const float* __restrict__ gate, int64_t ldg,
                                    float* __restrict__ dx, int64_t lddx, int M, int C,
                                    const float* __restrict__ mean, const float* __restrict__ var,
                                    float eps, const float* __restrict__ gamma,
                                    const float* __restrict__ sum_dy, const float* __restrict__ sum_dyx,
                                    int training, float beta_out) {
  GRID_STRIDE(i, (int64_t)M * C) {
    const int64_t m = i / C;
    const int c = (int)(i - m * C);
    float g = dy[m * lddy + c];
    if (gate && gate[m * ldg + c] <= 0.f) g = 0.f;
    const float rs = rsqrtf(var[c] + eps);
    float v;
    if (training) {
      const float xh = (x[m * ldx + c] - mean[c]) * rs;
      v = gamma[c] * rs * (g - sum_dy[c] / M - xh * sum_dyx[c] / M);
    } else {
      v = gamma[c] * rs * g;
    }
    float* o = dx + m * lddx + c;
    *o = beta_out != 0.f ? beta_out * (*o) + v : v;
  }
}

// ---------------------------------------------------------------- MaxPooling1D(2, 1, SAME)
__global__ void maxpool_fwd_kernel(const float* __restrict__ x, float* __restrict__ y, int B, int N,
                                   int C) {
  GRID_STRIDE(i, (int64_t)B * N * C) {
    const int64_t row = i / C;
    const int n = (int)(row % N);
    const float a = x[i];
    y[i] = (n + 1 < N) ? fmaxf(a, x[i + C]) : a;
  }
}

// routes dy[n] to argmax of window {n, n+1} (first index on ties, as TF MaxPoolGrad)
__global__ void maxpool_bwd_kernel(const float* __restrict__ x, const float* __restrict__ dy,
                                   float* __restrict__ dx, int B, int N, int C) {
  GRID_STRIDE(i, (int64_t)B * N * C) {
    const int64_t row = i / C;
    const int n = (int)(row % N);
    float g = 0.f;
    // own window n: goes to n if x[n] >= x[n+1] (or n is last)
    if (n + 1 >= N || x[i] >= x[i + C]) g += dy[i];
    // window n-1 picks n when x[n-1] < x[n]
    if (n > 0 && x[i - C] < x[i]) g += dy[i - C];
    dx[i] = g;
  }
}

// float4 variants (C % 4 == 0, 16-byte aligned, < 2^31 elements): 32-bit row / position
// arithmetic once per four channels -- the 64-bit divisions above dominated these passes
// (54 us for the CBHG bank output).  Same comparisons and sums: bit-identical.
__device__ __forceinline__ float maxpool_grad1(float a, float nx, float px, float d, float pd,
                                               bool last, bool first) {
  float g = 0.f;
  if (last || a >= nx) g += d;
  if (!first && px < a) g += pd;
  return g;
}
__global__ void maxpool_fwd4_kernel(const float4* __restrict__ x, float4* __restrict__ y,
                                    unsigned N, unsigned C4, unsigned total4) {
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < total4; i += gridDim.x * blockDim.x) {
    const unsigned n = (i / C4) % N;
    const float4 a = x[i];
    if (n + 1 < N) {
      const float4 b = x[i + C4];
      y[i] = make_float4(fmaxf(a.x, b.x), fmaxf(a.y, b.y), fmaxf(a.z, b.z), fmaxf(a.w, b.w));
    } else {
      y[i] = a;
    }
  }
}
// chunked variant: a thread owns kMpL consecutive positions of one (utterance, float4 column),
// loads its x / dy window (positions n0-1 .. n0+kMpL) once, all loads in flight together,
// instead of every position re-reading both neighbours (≈ 2.5x the bytes through L2)
constexpr int kMpL = 8;
__global__ void maxpool_bwd4c_kernel(const float4* __restrict__ x, const float4* __restrict__ dy,
                                     float4* __restrict__ dx, int N, int C4, int nchunk,
                                     int total) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= total) return;
  const int c = tid % C4;
  const int rest = tid / C4;
  const int ch = rest % nchunk, b = rest / nchunk;
  const int n0 = ch * kMpL;
  const int64_t base = (int64_t)b * N * C4 + c;
  float4 xv[kMpL + 2], dv[kMpL + 1];
#pragma unroll
  for (int k = 0; k < kMpL + 2; ++k) {        // xv[k] = x at position n0 - 1 + k (clamped)
    const int n = min(max(n0 - 1 + k, 0), N - 1);
    xv[k] = x[base + (int64_t)n * C4];
  }
#pragma unroll
  for (int k = 0; k < kMpL + 1; ++k) {        // dv[k] = dy at position n0 - 1 + k (clamped)
    const int n = min(max(n0 - 1 + k, 0), N - 1);
    dv[k] = dy[base + (int64_t)n * C4];
  }
#pragma unroll
  for (int k = 1; k <= kMpL; ++k) {
    const int n = n0 - 1 + k;
    if (n >= N) break;
    const bool last = n + 1 >= N, first = n == 0;
    const float4 a = xv[k], nx = xv[k + 1], px = xv[k - 1], d = dv[k], pd = dv[k - 1];
    dx[base + (int64_t)n * C4] =
        make_float4(maxpool_grad1(a.x, nx.x, px.x, d.x, pd.x, last, first),
                    maxpool_grad1(a.y, nx.y, px.y, d.y, pd.y, last, first),
                    maxpool_grad1(a.z, nx.z, px.z, d.z, pd.z, last, first),
                    maxpool_grad1(a.w, nx.w, px.w, d.w, pd.w, last, first));
  }
}
__global__ void maxpool_fwd4c_kernel(const float4* __restrict__ x, float4* __restrict__ y, int N,
                                     int C4, int nchunk, int total) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= total) return;
  const int c = tid % C4;
  const int rest = tid / C4;
  const int ch = rest % nchunk, b = rest / nchunk;
  const int n0 = ch * kMpL;
  const int64_t base = (int64_t)b * N * C4 + c;
  float4 xv[kMpL + 1];
#pragma unroll
  for (int k = 0; k < kMpL + 1; ++k) {        // xv[k] = x at position n0 + k (clamped)
    const int n = min(n0 + k, N - 1);
    xv[k] = x[base + (int64_t)n * C4];
  }
#pragma unroll
  for (int k = 0; k < kMpL; ++k) {
    const int n = n0 + k;
    if (n >= N) break;
    const float4 a = xv[k], b2 = xv[k + 1];
    y[base + (int64_t)n * C4] = n + 1 < N ? make_float4(fmaxf(a.x, b2.x), fmaxf(a.y, b2.y),
                                                        fmaxf(a.z, b2.z), fmaxf(a.w, b2.w))
                                          : a;
  }
}
// BN(+ReLU) apply and the stride-1 width-2 max-pool over time in one pass (the CBHG conv bank,
// modules/module.py:79-80): a thread owns kMpL consecutive positions of one (utterance, float4
// column) as in maxpool_fwd4c_kernel, forms the BN outputs of positions n0 .. n0 + kMpL once
// (the next chunk's first one again), writes y (kept for the backward) and the pooled output.
__global__ void bn_apply_pool4c_kernel(const float4* __restrict__ x, float4* __restrict__ y,
                                       float4* __restrict__ mp, int N, int C4, int nchunk,
                                       int total, const float4* __restrict__ mean,
                                       const float4* __restrict__ var, float eps,
                                       const float4* __restrict__ gamma,
                                       const float4* __restrict__ beta, int relu) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= total) return;
  const int c = tid % C4;
  const int rest = tid / C4;
  const int ch = rest % nchunk, b = rest / nchunk;
  const int n0 = ch * kMpL;
  const int64_t base = (int64_t)b * N * C4 + c;
  const float4 mu = mean[c], va = var[c], ga = gamma[c], be = beta[c];
  float4 xv[kMpL + 1];
#pragma unroll
  for (int k = 0; k < kMpL + 1; ++k) {        // positions n0 + k (clamped)
    const int n = min(n0 + k, N - 1);
    xv[k] = x[base + (int64_t)n * C4];
  }
  float4 yv[kMpL + 1];
#pragma unroll
  for (int k = 0; k < kMpL + 1; ++k)
    yv[k] = make_float4(bn_val(xv[k].x, ga.x, mu.x, va.x, be.x, eps, relu),
                        bn_val(xv[k].y, ga.y, mu.y, va.y, be.y, eps, relu),
                        bn_val(xv[k].z, ga.z, mu.z, va.z, be.z, eps, relu),
                        bn_val(xv[k].w, ga.w, mu.w, va.w, be.w, eps, relu));
#pragma unroll
  for (int k = 0; k < kMpL; ++k) {
    const int n = n0 + k;
    if (n >= N) break;
    const float4 a = yv[k], b2 = yv[k + 1];
    y[base + (int64_t)n * C4] = a;
    mp[base + (int64_t)n * C4] = n + 1 < N ? make_float4(fmaxf(a.x, b2.x), fmaxf(a.y, b2.y),
                                                         fmaxf(a.z, b2.z), fmaxf(a.w, b2.w))
                                           : a;
  }
}

__global__ void maxpool_bwd4_kernel(const float4* __restrict__ x, const float4* __restrict__ dy,
                                    float4* __restrict__ dx, unsigned N, unsigned C4,
                                    unsigned total4) {
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < total4; i += gridDim.x * blockDim.x) {
    const unsigned n = (i / C4) % N;
    const bool last = n + 1 >= N, first = n == 0;
    const float4 a = x[i], d = dy[i];
    const float4 nx = last ? a : x[i + C4];
    const float4 px = first ? a : x[i - C4];
    const float4 pd = first ? d : dy[i - C4];
    dx[i] = make_float4(maxpool_grad1(a.x, nx.x, px.x, d.x, pd.x, last, first),
                        maxpool_grad1(a.y, nx.y, px.y, d.y, pd.y, last, first),
                        maxpool_grad1(a.z, nx.z, px.z, d.z, pd.z, last, first),
                        maxpool_grad1(a.w, nx.w, px.w, d.w, pd.w, last, first));
  }
}

// ---------------------------------------------------------------- HighwayNet (ext tacotron2)
__global__ void highway_fwd_kernel(const float* __restrict__ h, const float* __restrict__ t,
                                   const float* __restrict__ x, float* __restrict__ y, int64_t n) {
  GRID_STRIDE(i, n) { y[i] = h[i] * t[i] + x[i] * (1.f - t[i]); }
}

// the highway layer after ONE batched product of its H and T pre-activations (x [W_H | W_T] +
// [b_H | b_T] as a batch of two): h = relu(h_pre), t = sigmoid(t_pre) written back in place (the
// backward's operands; the same arithmetic as the GEMM epilogue's activations), y = h t + x (1 - t)
__global__ void highway_act_fwd_kernel(float* __restrict__ h, float* __restrict__ t,
                                       const float* __restrict__ x, float* __restrict__ y,
                                       int64_t n) {
  GRID_STRIDE(i, n) {
    const float hv = fmaxf(h[i], 0.f), tv = 1.f / (1.f + expf(-t[i]));
    h[i] = hv;
    t[i] = tv;
    y[i] = hv * tv + x[i] * (1.f - tv);
  }
}

__global__ void highway_bwd_kernel(const float* __restrict__ h, const float* __restrict__ t,
                                   const float* __restrict__ x, const float* __restrict__ dy,
                                   float* __restrict__ dh_pre, float* __restrict__ dt_pre,
                                   float* __restrict__ dx, int64_t n) {
  GRID_STRIDE(i, n) {
    const float g = dy[i], tv = t[i], hv = h[i];
    dh_pre[i] = hv > 0.f ? g * tv : 0.f;
    dt_pre[i] = g * (hv - x[i]) * tv * (1.f - tv);
    dx[i] = g * (1.f - tv);
  }
}

// ---------------------------------------------------------------- activation backward
// dx = dy * act'(y) [* mask], act: 1 relu (y>0), 2 tanh (1-y^2), 3 sigmoid y(1-y),
// 4 softsign (1-|y|)^2, 0 identity
__global__ void act_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ y,
                               const float* __restrict__ mask, float* __restrict__ dx, int64_t n,
                               int act, float beta) {
  GRID_STRIDE(i, n) {
    float g = dy[i];
    if (mask) g *= mask[i];
    const float yv = y ? y[i] : 0.f;
    if (act == 1) g = yv > 0.f ? g : 0.f;
    else if (act == 2) g *= 1.f - yv * yv;
    else if (act == 3) g *= yv * (1.f - yv);
    else if (act == 4) { const float a = 1.f - fabsf(yv); g *= a * a; }
    dx[i] = beta != 0.f ? beta * dx[i] + g : g;
  }
}

__global__ void axpby_kernel(const float* __restrict__ x, float* __restrict__ y, int64_t n, float a,
                             float b) {
  GRID_STRIDE(i, n) { y[i] = a * x[i] + (b != 0.f ? b * y[i] : 0.f); }
}

// z = x + y on float4 (the self-attention transformer's residual, modules/module.py:363-371)
__global__ void add3_kernel(const float4* __restrict__ x, const float4* __restrict__ y,
                            float4* __restrict__ z, int64_t n4) {
  GRID_STRIDE(i, n4) {
    const float4 a = x[i], b = y[i];
    z[i] = make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
  }
}

// ---------------------------------------------------------------- row softmax (self-attention)
// P = softmax(scale * S) over the last dim, optional causal mask (col > row-in-sequence -> -inf),
// Pd = P * mask (dropout on probabilities).  One wave per row.
__global__ void softmax_fwd_kernel(const float* __restrict__ S, float* __restrict__ P,
                                   float* __restrict__ Pd, const float* __restrict__ mask, int64_t R,
                                   int L, int Lq, int causal, float scale) {
  const int lane = threadIdx.x & 63;
  const int64_t r = blockIdx.x * (int64_t)(blockDim.x >> 6) + (threadIdx.x >> 6);
  if (r >= R) return;
  const int qi = (int)(r % Lq);
  const int lim = causal ? min(L, qi + 1) : L;
  const float* s = S + r * L;
  float mx = -INFINITY;
  for (int j = lane; j < lim; j += 64) mx = fmaxf(mx, s[j] * scale);
  mx = wave_max(mx);
  float z = 0.f;
  for (int j = lane; j < lim; j += 64) z += expf(s[j] * scale - mx);
  z = wave_sum(z);
  const float inv = 1.f / z;
  for (int j = lane; j < L; j += 64) {
    const float pv = j < lim ? expf(s[j] * scale - mx) * inv : 0.f;
    P[r * L + j] = pv;
    if (Pd) Pd[r * L + j] = mask ? pv * mask[r * L + j] : pv;
  }
}

// dS = scale * P * (dP - sum_j dP_j P_j), dP = dPd * mask.  Causal rows read P / dPd only up to
// the diagonal (beyond it P is zero and dPd may be unwritten: the score products skip the tiles
// above it, SatGemmDesc.tri) and write dS = 0 there -- the same bits as the full row's terms.
__global__ void softmax_bwd_kernel(const float* __restrict__ P, const float* __restrict__ dPd,
                                   const float* __restrict__ mask, float* __restrict__ dS, int64_t R,
                                   int L, int Lq, int causal, float scale) {
  const int lane = threadIdx.x & 63;
  const int64_t r = blockIdx.x * (int64_t)(blockDim.x >> 6) + (threadIdx.x >> 6);
  if (r >= R) return;
  const int lim = causal ? min(L, (int)(r % Lq) + 1) : L;
  const float* p = P + r * L;
  const float* g = dPd + r * L;
  const float* m = mask ? mask + r * L : nullptr;
  float acc = 0.f;
  for (int j = lane; j < lim; j += 64) acc += (m ? g[j] * m[j] : g[j]) * p[j];
  acc = wave_sum(acc);
  for (int j = lane; j < L; j += 64) {
    const float dp = j < lim ? (m ? g[j] * m[j] : g[j]) : 0.f;
    dS[r * L + j] = j < lim ? scale * p[j] * (dp - acc) : 0.f;
  }
}

// Register-resident variants for rows of at most 64*NC columns: each row is read once (every
// load of the row issued before the first reduction) instead of two / three dependent passes.
// Same operations in the same per-lane order as the kernels above: bit-identical results.
template <int NC>
__global__ void softmax_fwd_reg_kernel(const float* __restrict__ S, float* __restrict__ P,
                                       float* __restrict__ Pd, const float* __restrict__ mask,
                                       int64_t R, int L, int Lq, int causal, float scale) {
  const int lane = threadIdx.x & 63;
  const int64_t r = blockIdx.x * (int64_t)(blockDim.x >> 6) + (threadIdx.x >> 6);
  if (r >= R) return;
  const int qi = (int)(r % Lq);
  const int lim = causal ? min(L, qi + 1) : L;
  const float* s = S + r * L;
  float v[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int j = lane + 64 * c;
    v[c] = j < lim ? s[j] * scale : -INFINITY;
  }
  float mx = -INFINITY;
#pragma unroll
  for (int c = 0; c < NC; ++c) mx = fmaxf(mx, v[c]);
  mx = wave_max(mx);
  float z = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    v[c] = lane + 64 * c < lim ? expf(v[c] - mx) : 0.f;
    z += v[c];
  }
  z = wave_sum(z);
  const float inv = 1.f / z;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int j = lane + 64 * c;
    if (j >= L) break;
    const float pv = j < lim ? v[c] * inv : 0.f;
    P[r * L + j] = pv;
    if (Pd) Pd[r * L + j] = mask ? pv * mask[r * L + j] : pv;
  }
}

template <int NC>
__global__ void softmax_bwd_reg_kernel(const float* __restrict__ P, const float* __restrict__ dPd,
                                       const float* __restrict__ mask, float* __restrict__ dS,
                                       int64_t R, int L, int Lq, int causal, float scale) {
  const int lane = threadIdx.x & 63;
  const int64_t r = blockIdx.x * (int64_t)(blockDim.x >> 6) + (threadIdx.x >> 6);
  if (r >= R) return;
  const int lim = causal ? min(L, (int)(r % Lq) + 1) : L;
  const float* p = P + r * L;
  const float* g = dPd + r * L;
  const float* m = mask ? mask + r * L : nullptr;
  float pv[NC], dp[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int j = lane + 64 * c;
    pv[c] = j < lim ? p[j] : 0.f;
    dp[c] = j < lim ? (m ? g[j] * m[j] : g[j]) : 0.f;
  }
  float acc = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c)
    if (lane + 64 * c < lim) acc += dp[c] * pv[c];
  acc = wave_sum(acc);
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int j = lane + 64 * c;
    if (j >= L) break;
    dS[r * L + j] = j < lim ? scale * pv[c] * (dp[c] - acc) : 0.f;
  }
}

// ---------------------------------------------------------------- loss (models/models.py:159-173)
// pass 1 (one workgroup): sums and non-zero-weight counts
// Loss pass 1: kLossBlocks workgroups, flat over float4s when M % 4 == 0 (else one wave per row),
// fp64 partials {sum w|mel-tgt|, #weighted elements, sum w*xent, #weighted stop entries} per
// workgroup; pass 1b sums them in a fixed order (deterministic) and writes
// out = {loss, L1, BCE, count1, count2}.
constexpr int kLossBlocks = 256;

__global__ void __launch_bounds__(256) loss_partial_kernel(
    const float* __restrict__ mel, const float* __restrict__ tgt, const float* __restrict__ tmask,
    const float* __restrict__ stop, const float* __restrict__ done, const float* __restrict__ dmask,
    int B, int T, int M, int Tp, double* __restrict__ part) {
  __shared__ double sh[4][4];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  double l1 = 0.0, c1 = 0.0, bce = 0.0, c2 = 0.0;
  const int rows = B * T;
  const bool vec = (M & 3) == 0;
  if (vec) {
    // flat over the float4s of all rows (a wave per row left 44 of 64 lanes idle at M = 80 and
    // walked 31 dependent row loads per wave); loads are unconditional, the weight selects
    const int M4 = M >> 2;
    const int64_t n4 = (int64_t)rows * M4;
    const float4* m4 = reinterpret_cast<const float4*>(mel);
    const float4* t4 = reinterpret_cast<const float4*>(tgt);
#pragma unroll 4
    for (int64_t e = blockIdx.x * 256 + threadIdx.x; e < n4; e += (int64_t)gridDim.x * 256) {
      const int64_t r = e / M4;
      const float w = tmask[r];
      const float4 x = m4[e], y = t4[e];
      const float acc = fabsf(x.x - y.x) + fabsf(x.y - y.y) + fabsf(x.z - y.z) + fabsf(x.w - y.w);
      l1 += w != 0.f ? (double)w * acc : 0.0;
      c1 += (w != 0.f && e == r * M4) ? (double)M : 0.0;
    }
  }
  for (int r = blockIdx.x * 4 + wv; !vec && r < rows; r += gridDim.x * 4) {
    const float w = tmask[r];
    if (w == 0.f) continue;                       // wave-uniform
    const float* mr = mel + (int64_t)r * M;
    const float* tr = tgt + (int64_t)r * M;
    float acc = 0.f;
    for (int c = lane; c < M; c += 64) acc += fabsf(mr[c] - tr[c]);
    l1 += (double)w * acc;
    if (lane == 0) c1 += (double)M;
  }
  const int n2 = B * Tp;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n2; i += gridDim.x * 256) {
    const float w = dmask[i];
    if (w != 0.f) {
      const float x = stop[i], z = done[i];
      bce += (double)w * (fmaxf(x, 0.f) - x * z + log1pf(expf(-fabsf(x))));
      c2 += 1.0;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    l1 += __shfl_xor(l1, o, 64); c1 += __shfl_xor(c1, o, 64);
    bce += __shfl_xor(bce, o, 64); c2 += __shfl_xor(c2, o, 64);
  }
  if (lane == 0) { sh[0][wv] = l1; sh[1][wv] = c1; sh[2][wv] = bce; sh[3][wv] = c2; }
  __syncthreads();
  if (threadIdx.x < 4) {
    const int k = threadIdx.x;
    part[blockIdx.x * 4 + k] = (sh[k][0] + sh[k][1]) + (sh[k][2] + sh[k][3]);
  }
}

__global__ void __launch_bounds__(256) loss_finish_kernel(const double* __restrict__ part,
                                                          int nblocks, float l1w,
                                                          float* __restrict__ out) {
  __shared__ double sh[4][4];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  double a[4] = {0, 0, 0, 0};
  for (int i = threadIdx.x; i < nblocks; i += 256)
#pragma unroll
    for (int k = 0; k < 4; ++k) a[k] += part[i * 4 + k];
#pragma unroll
  for (int k = 0; k < 4; ++k)
    for (int o = 32; o > 0; o >>= 1) a[k] += __shfl_xor(a[k], o, 64);
  if (lane == 0)
#pragma unroll
    for (int k = 0; k < 4; ++k) sh[k][wv] = a[k];
  __syncthreads();
  if (threadIdx.x == 0) {
    double t[4];
    for (int k = 0; k < 4; ++k) t[k] = (sh[k][0] + sh[k][1]) + (sh[k][2] + sh[k][3]);
    const double cl1 = fmax(t[1], 1.0), cb = fmax(t[3], 1.0);
    const double L1 = t[0] / cl1, BCE = t[2] / cb;
    out[0] = (float)(l1w * L1 + BCE);   // loss
    out[1] = (float)L1;
    out[2] = (float)BCE;
    out[3] = (float)cl1;                // counts, used by the gradient pass
    out[4] = (float)cb;
  }
}

// pass 2: dmel = l1w * sign(mel - tgt) * w / count ; dstop = (sigmoid(x) - z) * w / count
__global__ void loss_grad_kernel(const float* __restrict__ mel, const float* __restrict__ tgt,
                                 const float* __restrict__ tmask, const float* __restrict__ stop,
                                 const float* __restrict__ done, const float* __restrict__ dmask,
                                 int B, int T, int M, int Tp, const float* __restrict__ red,
                                 float l1w, float* __restrict__ dmel, float* __restrict__ dstop) {
  const int64_t n1 = (int64_t)B * T * M, n2 = (int64_t)B * Tp;
  const float s1 = l1w / red[3], s2 = 1.f / red[4];
  GRID_STRIDE(i, n1 + n2) {
    if (i < n1) {
      const float w = tmask[i / M];
      const float dlt = mel[i] - tgt[i];
      const float sg = dlt > 0.f ? 1.f : (dlt < 0.f ? -1.f : 0.f);
      dmel[i] = w * sg * s1;
    } else {
      const int64_t j = i - n1;
      const float w = dmask[j];
      dstop[j] = w * (1.f / (1.f + expf(-stop[j])) - done[j]) * s2;
    }
  }
}

// out[c][r] = in[r][c]  (32x32 tiles through LDS)
__global__ void transpose_kernel(const float* __restrict__ in, int64_t ldi, float* __restrict__ out,
                                 int64_t ldo, int R, int C) {
  __shared__ float t[32][33];
  const int r0 = blockIdx.y * 32, c0 = blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;   // 256 threads: 8 rows per pass
  for (int i = ty; i < 32; i += 8) {
    const int r = r0 + i, c = c0 + tx;
    t[i][tx] = (r < R && c < C) ? in[(int64_t)r * ldi + c] : 0.f;
  }
  __syncthreads();
  for (int i = ty; i < 32; i += 8) {
    const int c = c0 + i, r = r0 + tx;
    if (c < C && r < R) out[(int64_t)c * ldo + r] = t[tx][i];
  }
}

// dword fill of a buffer (zero-initialised step buffers, error words): dwordx4 stores where the
// pointer allows, the head / tail one dword at a time
__global__ void fill32_kernel(unsigned* __restrict__ p, int64_t n, unsigned bits) {
  const int64_t head = std::min<int64_t>(n, (int64_t)((16 - (reinterpret_cast<uintptr_t>(p) & 15)) & 15) / 4);
  const int64_t n4 = (n - head) / 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint4* q = reinterpret_cast<uint4*>(p + head);
  const uint4 v = make_uint4(bits, bits, bits, bits);
  for (int64_t i = i0; i < n4; i += stride) q[i] = v;
  if (i0 < head) p[i0] = bits;
  const int64_t t0 = head + 4 * n4;
  if (i0 < n - t0) p[t0 + i0] = bits;
}

// dst[i][j][k] = src[i][j][k] over an [n0][n1][n2] box, both with unit innermost stride and any
// outer strides (a transpose(0, 1) made contiguous, a strided slice copied into a step buffer):
// one thread per float4 of a row when every row start is 16-byte aligned, else per float
template <bool V4>
__global__ void copy3d_kernel(const float* __restrict__ src, int64_t s0, int64_t s1,
                              float* __restrict__ dst, int64_t d0, int64_t d1, int n0, int n1,
                              int n2) {
  const int w = V4 ? n2 / 4 : n2;
  const int64_t total = (int64_t)n0 * n1 * w;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int k = (int)(e % w);
    const int64_t r = e / w;
    const int j = (int)(r % n1), i = (int)(r / n1);
    if (V4) {
      *reinterpret_cast<float4*>(dst + i * d0 + j * d1 + 4 * k) =
          *reinterpret_cast<const float4*>(src + i * s0 + j * s1 + 4 * k);
    } else {
      dst[i * d0 + j * d1 + k] = src[i * s0 + j * s1 + k];
    }
  }
}

}  // namespace
}  // namespace sat

using namespace sat;

extern "C" int sat_transpose(const float* in, int64_t ldi, float* out, int64_t ldo, int32_t R,
                             int32_t C, void* stream) {
  SAT_CHECK_ARG(in && out && R >= 0 && C >= 0, "sat_transpose: bad args");
  if (R == 0 || C == 0) return SAT_OK;
  hipLaunchKernelGGL(transpose_kernel, dim3(ceil_div(C, 32), ceil_div(R, 32)), dim3(256), 0,
                     as_stream(stream), in, ldi, out, ldo, R, C);
  SAT_LAUNCH_CHECK("sat_transpose");
  return SAT_OK;
}

extern "C" int sat_fill32(void* p, int64_t n, uint32_t bits, void* stream) {
  SAT_CHECK_ARG(n >= 0 && (p || n == 0) && (reinterpret_cast<uintptr_t>(p) & 3) == 0,
                "sat_fill32: bad args (4-byte aligned pointer, n >= 0)");
  if (n == 0) return SAT_OK;
  const int64_t blocks = std::min<int64_t>(std::max<int64_t>((n / 4 + 255) / 256, 1), 4096);
  hipLaunchKernelGGL(fill32_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream),
                     static_cast<unsigned*>(p), n, bits);
  SAT_LAUNCH_CHECK("sat_fill32");
  return SAT_OK;
}

extern "C" int sat_copy3d(const float* src, int64_t s0, int64_t s1, float* dst, int64_t d0,
                          int64_t d1, int32_t n0, int32_t n1, int32_t n2, void* stream) {
  SAT_CHECK_ARG(src && dst && n0 >= 0 && n1 >= 0 && n2 >= 0, "sat_copy3d: bad args");
  const int64_t total = (int64_t)n0 * n1 * n2;
  if (total == 0) return SAT_OK;
  const bool v4 = n2 % 4 == 0 && s0 % 4 == 0 && s1 % 4 == 0 && d0 % 4 == 0 && d1 % 4 == 0 &&
                  aligned16(src) && aligned16(dst);
  const int64_t items = v4 ? total / 4 : total;
  const int64_t blocks = std::min<int64_t>((items + 255) / 256, 8192);
  if (v4)
    hipLaunchKernelGGL(copy3d_kernel<true>, dim3((unsigned)blocks), dim3(256), 0,
                       as_stream(stream), src, s0, s1, dst, d0, d1, n0, n1, n2);
  else
    hipLaunchKernelGGL(copy3d_kernel<false>, dim3((unsigned)blocks), dim3(256), 0,
                       as_stream(stream), src, s0, s1, dst, d0, d1, n0, n1, n2);
  SAT_LAUNCH_CHECK("sat_copy3d");
  return SAT_OK;
}

extern "C" int sat_seq_mask(const float* x, float* out, int32_t B, int32_t N, int32_t C,
                            const int64_t* lengths, void* stream) {
  SAT_CHECK_ARG(x && out && lengths && B > 0 && N > 0 && C > 0, "sat_seq_mask: bad args");
  const int64_t total = (int64_t)B * N * C;
  hipLaunchKernelGGL(seq_mask_kernel, dim3(grid_for(total)), dim3(256), 0, as_stream(stream), x,
                     out, B, N, C, lengths);
  SAT_LAUNCH_CHECK("sat_seq_mask");
  return SAT_OK;
}

extern "C" int sat_embedding_fwd(const float* table, const int64_t* ids, float* out, int64_t R,
                                 int32_t D, int32_t V, int64_t offset, int32_t* err, void* stream) {
  SAT_CHECK_ARG(table && ids && out && R >= 0 && D > 0 && V > 0, "sat_embedding_fwd: bad args");
  if (R == 0) return SAT_OK;
  hipLaunchKernelGGL(embed_fwd_kernel, dim3(grid_for(R * D)), dim3(256), 0, as_stream(stream),
                     table, ids, out, R, D, V, offset, err);
  SAT_LAUNCH_CHECK("sat_embedding_fwd");
  return SAT_OK;
}

extern "C" int sat_embedding_bwd(const float* dout, const int64_t* ids, float* dtable, int64_t R,
                                 int32_t D, int32_t V, int64_t offset, void* stream) {
  SAT_CHECK_ARG(dout && ids && dtable && R >= 0 && D > 0 && V > 0, "sat_embedding_bwd: bad args");
  if (R == 0) return SAT_OK;
  if (R <= kEmbRows)
    hipLaunchKernelGGL(embed_bwd_list_kernel, dim3(V, ceil_div(D, 256)), dim3(256), 0,
                       as_stream(stream), dout, ids, dtable, (int)R, D, offset);
  else
    hipLaunchKernelGGL(embed_bwd_kernel, dim3(V, ceil_div(D, 256)), dim3(256), 0,
                       as_stream(stream), dout, ids, dtable, R, D, V, offset);
  SAT_LAUNCH_CHECK("sat_embedding_bwd");
  return SAT_OK;
}

// 64 rows per workgroup (one unrolled trip of 16 rows per row group), up to 256 row blocks
static int row_blocks(int M) { return std::max(1, std::min(256, (M + 63) / 64)); }

extern "C" int64_t sat_workspace_colreduce(int32_t M, int32_t C) {
  // bytes: fp64 partials [2][RB][C] + two fp32 sums [C] used by the column reductions below
  return (int64_t)2 * row_blocks(M) * C * (int64_t)sizeof(double) + (int64_t)2 * C * 4;
}

extern "C" int sat_bn_stats(const float* x, int64_t ldx, int32_t M, int32_t C, float* mean,
                            float* var, float* mov_mean, float* mov_var, float momentum,
                            void* workspace, void* stream) {
  SAT_CHECK_ARG(x && mean && var && workspace && M > 0 && C > 0, "sat_bn_stats: bad args");
  const int RB = row_blocks(M);
  double* p1 = reinterpret_cast<double*>(workspace);
  double* p2 = p1 + (int64_t)RB * C;
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL(colreduce_kernel, dim3(ceil_div(C, 64), RB), dim3(256), 0, s, x, ldx,
                     (const float*)nullptr, (int64_t)0, M, C, p1, p2, 0, (const float*)nullptr,
                     (const float*)nullptr, 0.f, (const float*)nullptr, (int64_t)0);
  hipLaunchKernelGGL(bn_stats_finish_kernel, dim3(ceil_div(C, 64)), dim3(256), 0, s, p1, p2, RB, M, C,
                     mean, var, mov_mean, mov_var, momentum);
  SAT_LAUNCH_CHECK("sat_bn_stats");
  return SAT_OK;
}

extern "C" int sat_bn_apply(const float* x, int64_t ldx, float* y, int64_t ldy, int32_t M,
                            int32_t C, const float* mean, const float* var, float eps,
                            const float* gamma, const float* beta, int32_t relu, const float* res,
                            int64_t ldr, void* stream) {
  SAT_CHECK_ARG(x && y && mean && var && gamma && beta && M > 0 && C > 0, "sat_bn_apply: bad args");
  const bool v4 = C % 4 == 0 && ldx % 4 == 0 && ldy % 4 == 0 && (!res || ldr % 4 == 0) &&
                  aligned16(x) && aligned16(y) && (!res || aligned16(res)) && aligned16(mean) &&
                  aligned16(var) && aligned16(gamma) && aligned16(beta) &&
                  (int64_t)M * std::max<int64_t>({ldx, ldy, ldr, C}) < (1LL << 31);
  if (v4)
    hipLaunchKernelGGL(bn_apply4_kernel, dim3(grid_for((int64_t)M * C / 4)), dim3(256), 0,
                       as_stream(stream), x, (int)ldx, y, (int)ldy, M, C, mean, var, eps, gamma,
                       beta, relu, res, (int)ldr);
  else
    hipLaunchKernelGGL(bn_apply_kernel, dim3(grid_for((int64_t)M * C)), dim3(256), 0,
                       as_stream(stream), x, ldx, y, ldy, M, C, mean, var, eps, gamma, beta, relu,
                       res, ldr);
  SAT_LAUNCH_CHECK("sat_bn_apply");
  return SAT_OK;
}

extern "C" int sat_bn_bwd(const float* dy, int64_t lddy, const float* x, int64_t ldx,
                          const float* gate, int64_t ldg, float* dx, int64_t lddx, int32_t M,
                          int32_t C, const float* mean, const float* var, float eps,
                          const float* gamma, float* dgamma, float* dbeta, int32_t training,
                          float beta_out, void* workspace, void* stream) {
  SAT_CHECK_ARG(dy && x && dx && mean && var && gamma && dgamma && dbeta && workspace,
                "sat_bn_bwd: bad args");
  const int RB = row_blocks(M);
  double* p1 = reinterpret_cast<double*>(workspace);
  double* p2 = p1 + (int64_t)RB * C;
  hipStream_t s = as_stream(stream);
  float* sum1 = reinterpret_cast<float*>(p2 + (int64_t)RB * C);
  float* sum2 = sum1 + C;
  hipLaunchKernelGGL(colreduce_kernel, dim3(ceil_div(C, 64), RB), dim3(256), 0, s, dy, lddy, x,
                     ldx, M, C, p1, p2, 1, mean, var, eps, gate, ldg);
  // dbeta += sum(g), dgamma += sum(g * xhat)  (gradients accumulate into the grad arena)
  hipLaunchKernelGGL(colreduce_finish_kernel, dim3(ceil_div(C, 64)), dim3(256), 0, s, p1, p2, RB, C,
                     sum1, sum2, 0.f, dbeta, dgamma);
  const bool v4 = C % 4 == 0 && lddy % 4 == 0 && ldx % 4 == 0 && lddx % 4 == 0 &&
                  (!gate || ldg % 4 == 0) && aligned16(dy) && aligned16(x) && aligned16(dx) &&
                  (!gate || aligned16(gate)) && aligned16(mean) && aligned16(var) &&
                  aligned16(gamma) && aligned16(sum1) && aligned16(sum2) &&
                  (int64_t)M * std::max<int64_t>({lddy, ldx, lddx, ldg, C}) < (1LL << 31);
  if (v4)
    hipLaunchKernelGGL(bn_bwd_apply4_kernel, dim3(grid_for((int64_t)M * C / 4)), dim3(256), 0, s,
                       dy, (int)lddy, x, (int)ldx, gate, (int)ldg, dx, (int)lddx, M, C, mean, var,
                       eps, gamma, sum1, sum2, training, beta_out);
  else
    hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(grid_for((int64_t)M * C)), dim3(256), 0, s, dy,
                       lddy, x, ldx, gate, ldg, dx, lddx, M, C, mean, var, eps, gamma, sum1, sum2,
                       training, beta_out);
  SAT_LAUNCH_CHECK("sat_bn_bwd");
  return SAT_OK;
}

// column sums scattered to up to kColSegs destinations: out_k[c - col_k] = beta * out_k[..] + sum
constexpr int kColSegs = 8;
struct ColSegs {
  float* dst[kColSegs];
  int col[kColSegs];
  int n[kColSegs];
  int nseg;
};
__global__ void colreduce_scatter_finish_kernel(const double* part1, int RB, int C, ColSegs g,
                                                float beta) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  double s, q;
  sum_partials(part1, part1, RB, C, c, s, q);
  if (threadIdx.x < 64 && c < C) {
    for (int k = 0; k < g.nseg; ++k) {
      const int j = c - g.col[k];
      if (j >= 0 && j < g.n[k]) {
        float* o = g.dst[k] + j;
        *o = beta != 0.f ? (float)(beta * *o + s) : (float)s;
      }
    }
  }
}

extern "C" int sat_colsum_scatter(const float* x, int64_t ldx, int32_t M, int32_t C,
                                  const SatColSegment* segs, int32_t nseg, float beta,
                                  void* workspace, void* stream) {
  SAT_CHECK_ARG(x && segs && workspace && M >= 0 && C > 0 && nseg > 0 && nseg <= kColSegs,
                "sat_colsum_scatter: bad args (nseg 1..%d)", kColSegs);
  ColSegs g{};
  g.nseg = nseg;
  for (int k = 0; k < nseg; ++k) {
    SAT_CHECK_ARG(segs[k].dst && segs[k].col >= 0 && segs[k].n > 0 && segs[k].col + segs[k].n <= C,
                  "sat_colsum_scatter: segment %d out of range", k);
    g.dst[k] = segs[k].dst;
    g.col[k] = segs[k].col;
    g.n[k] = segs[k].n;
  }
  if (M == 0) return SAT_OK;
  const int RB = row_blocks(M);
  double* p1 = reinterpret_cast<double*>(workspace);
  double* p2 = p1 + (int64_t)RB * C;
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL(colreduce_kernel, dim3(ceil_div(C, 64), RB), dim3(256), 0, s, x, ldx,
                     (const float*)nullptr, (int64_t)0, M, C, p1, p2, 2, (const float*)nullptr,
                     (const float*)nullptr, 0.f, (const float*)nullptr, (int64_t)0);
  hipLaunchKernelGGL(colreduce_scatter_finish_kernel, dim3(ceil_div(C, 64)), dim3(256), 0, s, p1,
                     RB, C, g, beta);
  SAT_LAUNCH_CHECK("sat_colsum_scatter");
  return SAT_OK;
}

// out = alpha * colsum(x) + beta * out (the GEMM's colsum_out fallback, sat_gemm: alpha applies
// to the column sums exactly as the fused LDS path applies it)
__global__ void colreduce_finish_alpha_kernel(const double* part1, int RB, int C, float* out,
                                              float alpha, float beta) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  double s, q;
  sum_partials(part1, part1, RB, C, c, s, q);
  if (threadIdx.x < 64 && c < C)
    out[c] = beta != 0.f ? (float)(beta * out[c] + (double)alpha * s) : (float)((double)alpha * s);
}

int sat::colsum_alpha(const float* x, int64_t ldx, int32_t M, int32_t C, float* out, float alpha,
                 float beta, void* workspace, hipStream_t s) {
  SAT_CHECK_ARG(x && out && workspace && M >= 0 && C > 0, "sat_gemm colsum_out: bad args");
  if (M == 0 && beta == 1.f) return SAT_OK;
  const int RB = row_blocks(std::max(M, 1));
  double* p1 = reinterpret_cast<double*>(workspace);
  double* p2 = p1 + (int64_t)RB * C;
  if (M > 0)
    hipLaunchKernelGGL(colreduce_kernel, dim3(ceil_div(C, 64), RB), dim3(256), 0, s, x, ldx,
                       (const float*)nullptr, (int64_t)0, M, C, p1, p2, 2, (const float*)nullptr,
                       (const float*)nullptr, 0.f, (const float*)nullptr, (int64_t)0);
  else
    (void)zero_dwords(p1, 2 * (int64_t)RB * C, s);
  hipLaunchKernelGGL(colreduce_finish_alpha_kernel, dim3(ceil_div(C, 64)), dim3(256), 0, s, p1,
                     RB, C, out, alpha, beta);
  SAT_LAUNCH_CHECK("sat_gemm colsum_out");
  return SAT_OK;
}

extern "C" int sat_colsum(const float* x, int64_t ldx, int32_t M, int32_t C, float* out,
                          float beta, void* workspace, void* stream) {
  SAT_CHECK_ARG(x && out && workspace && M >= 0 && C > 0, "sat_colsum: bad args");
  if (M == 0) return SAT_OK;
  const int RB = row_blocks(M);
  double* p1 = reinterpret_cast<double*>(workspace);
  double* p2 = p1 + (int64_t)RB * C;
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL(colreduce_kernel, dim3(ceil_div(C, 64), RB), dim3(256), 0, s, x, ldx,
                     (const float*)nullptr, (int64_t)0, M, C, p1, p2, 2, (const float*)nullptr,
                     (const float*)nullptr, 0.f, (const float*)nullptr, (int64_t)0);
  hipLaunchKernelGGL(colreduce_finish_kernel, dim3(ceil_div(C, 64)), dim3(256), 0, s, p1, p2, RB, C,
                     out, (float*)nullptr, beta, (float*)nullptr, (float*)nullptr);
  SAT_LAUNCH_CHECK("sat_colsum");
  return SAT_OK;
}

extern "C" int sat_maxpool2(const float* x, float* y, int32_t B, int32_t N, int32_t C,
                            void* stream) {
  SAT_CHECK_ARG(x && y && B > 0 && N > 0 && C > 0, "sat_maxpool2: bad args");
  const int64_t total = (int64_t)B * N * C;
  const int64_t nthreads = (int64_t)B * ((N + kMpL - 1) / kMpL) * (C / 4);
  if (C % 4 == 0 && total < (1LL << 31) && aligned16(x) && aligned16(y) && nthreads >= 65536)
    hipLaunchKernelGGL(maxpool_fwd4c_kernel, dim3(ceil_div(nthreads, 256)), dim3(256), 0,
                       as_stream(stream), reinterpret_cast<const float4*>(x),
                       reinterpret_cast<float4*>(y), N, C / 4, (N + kMpL - 1) / kMpL,
                       (int)nthreads);
  else if (C % 4 == 0 && total < (1LL << 31) && aligned16(x) && aligned16(y))
    hipLaunchKernelGGL(maxpool_fwd4_kernel, dim3(grid_for(total / 4)), dim3(256), 0,
                       as_stream(stream), reinterpret_cast<const float4*>(x),
                       reinterpret_cast<float4*>(y), (unsigned)N, (unsigned)(C / 4),
                       (unsigned)(total / 4));
  else
    hipLaunchKernelGGL(maxpool_fwd_kernel, dim3(grid_for(total)), dim3(256), 0,
                       as_stream(stream), x, y, B, N, C);
  SAT_LAUNCH_CHECK("sat_maxpool2");
  return SAT_OK;
}

extern "C" int sat_bn_apply_maxpool2(const float* x, float* y, float* mp, int32_t B, int32_t N,
                                     int32_t C, const float* mean, const float* var, float eps,
                                     const float* gamma, const float* beta, int32_t relu,
                                     void* stream) {
  SAT_CHECK_ARG(x && y && mp && mean && var && gamma && beta && B > 0 && N > 0 && C > 0,
                "sat_bn_apply_maxpool2: bad args");
  const int64_t total = (int64_t)B * N * C;
  if (C % 4 == 0 && total < (1LL << 31) && aligned16(x) && aligned16(y) && aligned16(mp) &&
      aligned16(mean) && aligned16(var) && aligned16(gamma) && aligned16(beta)) {
    const int64_t nthreads = (int64_t)B * ((N + kMpL - 1) / kMpL) * (C / 4);
    hipLaunchKernelGGL(bn_apply_pool4c_kernel, dim3(ceil_div(nthreads, 256)), dim3(256), 0,
                       as_stream(stream), reinterpret_cast<const float4*>(x),
                       reinterpret_cast<float4*>(y), reinterpret_cast<float4*>(mp), N, C / 4,
                       (N + kMpL - 1) / kMpL, (int)nthreads,
                       reinterpret_cast<const float4*>(mean), reinterpret_cast<const float4*>(var),
                       eps, reinterpret_cast<const float4*>(gamma),
                       reinterpret_cast<const float4*>(beta), relu);
    SAT_LAUNCH_CHECK("sat_bn_apply_maxpool2");
    return SAT_OK;
  }
  const int r = sat_bn_apply(x, C, y, C, B * N, C, mean, var, eps, gamma, beta, relu, nullptr, 0,
                             stream);
  return r != SAT_OK ? r : sat_maxpool2(y, mp, B, N, C, stream);
}

extern "C" int sat_maxpool2_bwd(const float* x, const float* dy, float* dx, int32_t B, int32_t N,
                                int32_t C, void* stream) {
  SAT_CHECK_ARG(x && dy && dx && B > 0 && N > 0 && C > 0, "sat_maxpool2_bwd: bad args");
  const int64_t total = (int64_t)B * N * C;
  const int64_t nthreads = (int64_t)B * ((N + kMpL - 1) / kMpL) * (C / 4);
  if (C % 4 == 0 && total < (1LL << 31) && aligned16(x) && aligned16(dy) && aligned16(dx) &&
      nthreads >= 65536)
    hipLaunchKernelGGL(maxpool_bwd4c_kernel, dim3(ceil_div(nthreads, 256)), dim3(256), 0,
                       as_stream(stream), reinterpret_cast<const float4*>(x),
                       reinterpret_cast<const float4*>(dy), reinterpret_cast<float4*>(dx), N,
                       C / 4, (N + kMpL - 1) / kMpL, (int)nthreads);
  else if (C % 4 == 0 && total < (1LL << 31) && aligned16(x) && aligned16(dy) && aligned16(dx))
    hipLaunchKernelGGL(maxpool_bwd4_kernel, dim3(grid_for(total / 4)), dim3(256), 0,
                       as_stream(stream), reinterpret_cast<const float4*>(x),
                       reinterpret_cast<const float4*>(dy), reinterpret_cast<float4*>(dx),
                       (unsigned)N, (unsigned)(C / 4), (unsigned)(total / 4));
  else
    hipLaunchKernelGGL(maxpool_bwd_kernel, dim3(grid_for(total)), dim3(256), 0,
                       as_stream(stream), x, dy, dx, B, N, C);
  SAT_LAUNCH_CHECK("sat_maxpool2_bwd");
  return SAT_OK;
}

extern "C" int sat_highway_fwd(const float* h, const float* t, const float* x, float* y, int64_t n,
                               void* stream) {
  SAT_CHECK_ARG(h && t && x && y && n >= 0, "sat_highway_fwd: bad args");
  hipLaunchKernelGGL(highway_fwd_kernel, dim3(grid_for(n)), dim3(256), 0, as_stream(stream), h, t,
                     x, y, n);
  SAT_LAUNCH_CHECK("sat_highway_fwd");
  return SAT_OK;
}

extern "C" int sat_highway_act_fwd(float* h, float* t, const float* x, float* y, int64_t n,
                                   void* stream) {
  SAT_CHECK_ARG(h && t && x && y && n >= 0, "sat_highway_act_fwd: bad args");
  hipLaunchKernelGGL(highway_act_fwd_kernel, dim3(grid_for(n)), dim3(256), 0, as_stream(stream), h,
                     t, x, y, n);
  SAT_LAUNCH_CHECK("sat_highway_act_fwd");
  return SAT_OK;
}

extern "C" int sat_highway_bwd(const float* h, const float* t, const float* x, const float* dy,
                               float* dh_pre, float* dt_pre, float* dx, int64_t n, void* stream) {
  SAT_CHECK_ARG(h && t && x && dy && dh_pre && dt_pre && dx, "sat_highway_bwd: bad args");
  hipLaunchKernelGGL(highway_bwd_kernel, dim3(grid_for(n)), dim3(256), 0, as_stream(stream), h, t,
                     x, dy, dh_pre, dt_pre, dx, n);
  SAT_LAUNCH_CHECK("sat_highway_bwd");
  return SAT_OK;
}

extern "C" int sat_act_bwd(const float* dy, const float* y, const float* mask, float* dx, int64_t n,
                           int32_t act, float beta, void* stream) {
  SAT_CHECK_ARG(dy && dx && n >= 0 && act >= 0 && act <= 4, "sat_act_bwd: bad args");
  SAT_CHECK_ARG(act == 0 || y, "sat_act_bwd: activation output needed");
  hipLaunchKernelGGL(act_bwd_kernel, dim3(grid_for(n)), dim3(256), 0, as_stream(stream), dy, y,
                     mask, dx, n, act, beta);
  SAT_LAUNCH_CHECK("sat_act_bwd");
  return SAT_OK;
}

extern "C" int sat_axpby(const float* x, float* y, int64_t n, float a, float b, void* stream) {
  SAT_CHECK_ARG(x && y && n >= 0, "sat_axpby: bad args");
  hipLaunchKernelGGL(axpby_kernel, dim3(grid_for(n)), dim3(256), 0, as_stream(stream), x, y, n, a,
                     b);
  SAT_LAUNCH_CHECK("sat_axpby");
  return SAT_OK;
}

extern "C" int sat_add(const float* x, const float* y, float* z, int64_t n, void* stream) {
  SAT_CHECK_ARG(x && y && z && n >= 0 && n % 4 == 0 && aligned16(x) && aligned16(y) &&
                    aligned16(z), "sat_add: 16-byte aligned operands, n % 4 == 0");
  if (n == 0) return SAT_OK;
  hipLaunchKernelGGL(add3_kernel, dim3(grid_for(n / 4)), dim3(256), 0, as_stream(stream),
                     reinterpret_cast<const float4*>(x), reinterpret_cast<const float4*>(y),
                     reinterpret_cast<float4*>(z), n / 4);
  SAT_LAUNCH_CHECK("sat_add");
  return SAT_OK;
}

extern "C" int sat_softmax_fwd(const float* S, float* P, float* Pd, const float* mask, int64_t R,
                               int32_t L, int32_t Lq, int32_t causal, float scale, void* stream) {
  SAT_CHECK_ARG(S && P && R >= 0 && L > 0 && Lq > 0, "sat_softmax_fwd: bad args");
  const dim3 g(ceil_div(R, 4)), b(256);
  hipStream_t s = as_stream(stream);
  if (L <= 256) hipLaunchKernelGGL(softmax_fwd_reg_kernel<4>, g, b, 0, s, S, P, Pd, mask, R, L, Lq, causal, scale);
  else if (L <= 512) hipLaunchKernelGGL(softmax_fwd_reg_kernel<8>, g, b, 0, s, S, P, Pd, mask, R, L, Lq, causal, scale);
  else if (L <= 1024) hipLaunchKernelGGL(softmax_fwd_reg_kernel<16>, g, b, 0, s, S, P, Pd, mask, R, L, Lq, causal, scale);
  else hipLaunchKernelGGL(softmax_fwd_kernel, g, b, 0, s, S, P, Pd, mask, R, L, Lq, causal, scale);
  SAT_LAUNCH_CHECK("sat_softmax_fwd");
  return SAT_OK;
}

extern "C" int sat_softmax_bwd(const float* P, const float* dPd, const float* mask, float* dS,
                               int64_t R, int32_t L, int32_t Lq, int32_t causal, float scale,
                               void* stream) {
  SAT_CHECK_ARG(P && dPd && dS && R >= 0 && L > 0 && (!causal || Lq > 0),
                "sat_softmax_bwd: bad args");
  const dim3 g(ceil_div(R, 4)), b(256);
  hipStream_t s = as_stream(stream);
  const int lq = Lq > 0 ? Lq : 1;
  if (L <= 256) hipLaunchKernelGGL(softmax_bwd_reg_kernel<4>, g, b, 0, s, P, dPd, mask, dS, R, L, lq, causal, scale);
  else if (L <= 512) hipLaunchKernelGGL(softmax_bwd_reg_kernel<8>, g, b, 0, s, P, dPd, mask, dS, R, L, lq, causal, scale);
  else if (L <= 1024) hipLaunchKernelGGL(softmax_bwd_reg_kernel<16>, g, b, 0, s, P, dPd, mask, dS, R, L, lq, causal, scale);
  else hipLaunchKernelGGL(softmax_bwd_kernel, g, b, 0, s, P, dPd, mask, dS, R, L, lq, causal, scale);
  SAT_LAUNCH_CHECK("sat_softmax_bwd");
  return SAT_OK;
}

extern "C" int64_t sat_workspace_loss(void) { return (int64_t)kLossBlocks * 4 * sizeof(double); }

extern "C" int sat_loss_fwd_bwd(const float* mel, const float* tgt, const float* tmask,
                                const float* stop, const float* done, const float* dmask,
                                int32_t B, int32_t T, int32_t M, int32_t Tp, float l1_weight,
                                float* out, float* dmel, float* dstop, void* workspace,
                                void* stream) {
  SAT_CHECK_ARG(mel && tgt && tmask && stop && done && dmask && out && workspace,
                "sat_loss_fwd_bwd: bad args");
  SAT_CHECK_ARG(((M & 3) != 0) || (((uintptr_t)mel | (uintptr_t)tgt) & 15) == 0,
                "sat_loss_fwd_bwd: mel/targets must be 16-byte aligned");
  hipStream_t s = as_stream(stream);
  double* part = reinterpret_cast<double*>(workspace);
  hipLaunchKernelGGL(loss_partial_kernel, dim3(kLossBlocks), dim3(256), 0, s, mel, tgt, tmask,
                     stop, done, dmask, B, T, M, Tp, part);
  hipLaunchKernelGGL(loss_finish_kernel, dim3(1), dim3(256), 0, s, part, kLossBlocks, l1_weight,
                     out);
  if (dmel && dstop) {
    const int64_t n = (int64_t)B * T * M + (int64_t)B * Tp;
    hipLaunchKernelGGL(loss_grad_kernel, dim3(grid_for(n)), dim3(256), 0, s, mel, tgt, tmask, stop,
                       done, dmask, B, T, M, Tp, out, l1_weight, dmel, dstop);
  }
  SAT_LAUNCH_CHECK("sat_loss_fwd_bwd");
  return SAT_OK;
}
