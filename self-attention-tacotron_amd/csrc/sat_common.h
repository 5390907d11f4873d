// Internal helpers shared by the libsat_hip kernels (gfx950 / CDNA4 only).
#pragma once
#include <algorithm>

#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <cmath>

#include "sat_abi.h"

namespace sat {

constexpr int kWave = 64;

// thread-local last error (sat_last_error_string)
void set_error(const char* fmt, ...);

// Segment clocks of the persistent kernels (the `prof` descriptors' buffers): compiled in only
// for instrumented builds (make EXTRA=-DSAT_SEGMENT_CLOCKS=1 BUILD=build_clk OUT=...); the
// production build carries neither the clock reads nor the per-phase flag tests
#ifndef SAT_SEGMENT_CLOCKS
#define SAT_SEGMENT_CLOCKS 0
#endif
#define SAT_CHECK_ARG(cond, ...)                                                            \
  do {                                                                                      \
    if (!(cond)) {                                                                          \
      ::sat::set_error(__VA_ARGS__);                                                        \
      return SAT_ERR_ARGUMENT;                                                              \
    }                                                                                       \
  } while (0)

#define SAT_LAUNCH_CHECK(name)                                                              \
  do {                                                                                      \
    hipError_t e_ = hipGetLastError();                                                      \
    if (e_ != hipSuccess) {                                                                 \
      ::sat::set_error("%s: launch failed: %s", name, hipGetErrorString(e_));               \
      return SAT_ERR_HIP;                                                                   \
    }                                                                                       \
  } while (0)

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + __expf(-x)); }

// accurate tanh (the parity bar is 1e-4 mean-L1 over 500 recurrent steps: no fast approximations)
__device__ __forceinline__ float tanhf_(float x) { return tanhf(x); }
__device__ __forceinline__ float sigmf(float x) { return 1.0f / (1.0f + expf(-x)); }

static inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// block-wide reductions; `scratch` needs blockDim.x/64 floats; result broadcast to all threads
__device__ __forceinline__ float block_sum(float v, float* scratch) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) scratch[w] = v;
  __syncthreads();
  float r = 0.f;
  for (int i = 0; i < nw; ++i) r += scratch[i];
  return r;
}
__device__ __forceinline__ float block_max(float v, float* scratch) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_max(v);
  __syncthreads();
  if (lane == 0) scratch[w] = v;
  __syncthreads();
  float r = -INFINITY;
  for (int i = 0; i < nw; ++i) r = fmaxf(r, scratch[i]);
  return r;
}

// DPP lane permutes (VALU, no LDS crossbar): quad_perm xor1 / xor2, row_half_mirror, row_mirror
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
// sum over each aligned group of 8 lanes (result in every lane of the group)
__device__ __forceinline__ float group8_sum(float v) {
  v += dpp<0xB1>(v);
  v += dpp<0x4E>(v);
  v += dpp<0x141>(v);
  return v;
}
__device__ __forceinline__ float group8_max(float v) {
  v = fmaxf(v, dpp<0xB1>(v));
  v = fmaxf(v, dpp<0x4E>(v));
  v = fmaxf(v, dpp<0x141>(v));
  return v;
}
// sum over each aligned group of 16 / 32 lanes (result in every lane of the group)
__device__ __forceinline__ float group16_sum(float v) {
  v = group8_sum(v);
  return v + dpp<0x140>(v);
}
__device__ __forceinline__ float group32_sum(float v) {
  v = group16_sum(v);
  return v + __shfl_xor(v, 16, 64);
}
// full-wave sum: DPP within rows of 16, then 4 readlanes (uniform result)
__device__ __forceinline__ float wave_sum_dpp(float v) {
  v = group8_sum(v);
  v += dpp<0x140>(v);
  const float a = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
  const float b = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
  const float c = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
  const float d = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
  return (a + b) + (c + d);
}

// full-wave max: DPP within rows of 16, then 4 readlanes (uniform result)
__device__ __forceinline__ float wave_max_dpp(float v) {
  v = group8_max(v);
  v = fmaxf(v, dpp<0x140>(v));
  const float a = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
  const float b = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
  const float c = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
  const float d = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
  return fmaxf(fmaxf(a, b), fmaxf(c, d));
}
// reductions over lanes 0..7 only (DPP, no LDS crossbar), broadcast as a uniform value
__device__ __forceinline__ float lanes8_sum(float v) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(group8_sum(v)), 0));
}
__device__ __forceinline__ float lanes8_max(float v) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(group8_max(v)), 0));
}

// tanh via one v_exp_f32 and one reciprocal: |error| ~2e-7 absolute, saturates correctly
// (exp overflow -> +1, underflow -> -1).  Used for the attention energies (1.4 M per step).
__device__ __forceinline__ float tanh_fast(float x) {
  const float e = __expf(2.f * x);
  return 1.f - 2.f * __builtin_amdgcn_rcpf(1.f + e);
}
// logistic with one v_exp_f32 and one reciprocal (no IEEE division sequence); saturates to 0 / 1
__device__ __forceinline__ float sigmoid_fast(float x) {
  return __builtin_amdgcn_rcpf(1.f + __expf(-x));
}
// the ZoneoutLSTM cells' tanh, formed as 2 sigmoid(2x) - 1 in EVERY LSTM kernel (persistent and
// per-step, forward and BPTT), so the training and incremental paths agree on the cell bit for bit
__device__ __forceinline__ float tanh_lstm(float x) {
  return fmaf(2.f, sigmoid_fast(2.f * x), -1.f);
}

// Workgroup barrier for LDS hand-offs only: waits for the wave's own LDS (and scalar) accesses,
// not for its outstanding global stores.  __syncthreads() also drains vmcnt (its workgroup
// release fence), which in the persistent kernels stalls every barrier behind the step's
// history / hand-off stores (0.2-0.7 us per barrier measured, decoder_persistent8.hip).  Use
// only where no other wave of the workgroup reads the stored global data.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// out = alpha * (column sums of x [M, C]) + beta * out, fp64 partials (elementwise.hip)
int colsum_alpha(const float* x, int64_t ldx, int32_t M, int32_t C, float* out, float alpha,
                 float beta, void* workspace, hipStream_t s);

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

inline int ceil_div(int64_t a, int64_t b) { return static_cast<int>((a + b - 1) / b); }

// Scratch, counters and error words of the persistent launches are cleared by a kernel rather
// than hipMemsetAsync: under hipGraph replay an 8-byte memset node was seen to write 0x16161616
// instead of 0 into an error word (tools/probes/graph_vs_eager.py), which made polls give up and
// the guarded optimiser skip the step.  A kernel node has no such path.
__global__ static void zero_dwords_kernel(unsigned* __restrict__ p, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    p[i] = 0u;
}
inline hipError_t zero_dwords(void* p, int64_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 1024);
  hipLaunchKernelGGL(zero_dwords_kernel, dim3(blocks), dim3(256), 0, s,
                     reinterpret_cast<unsigned*>(p), n);
  return hipGetLastError();
}
inline hipError_t zero_words(int* p, int n, hipStream_t s) { return zero_dwords(p, n, s); }

// Up to four disjoint dword ranges cleared by ONE launch (grid row y = range): a persistent
// launcher's scratch + error words used to cost two to four ~5 us kernel nodes per call.
struct ZeroRanges {
  unsigned* p[4];
  int64_t n[4];
};
__global__ static void zero_ranges_kernel(ZeroRanges r) {
  unsigned* __restrict__ p = r.p[blockIdx.y];
  const int64_t n = r.n[blockIdx.y];
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    p[i] = 0u;
}
inline hipError_t zero_ranges(hipStream_t s, void* p0, int64_t n0, void* p1, int64_t n1,
                              void* p2 = nullptr, int64_t n2 = 0, void* p3 = nullptr,
                              int64_t n3 = 0) {
  ZeroRanges r{};
  void* ps[4] = {p0, p1, p2, p3};
  const int64_t ns[4] = {n0, n1, n2, n3};
  int k = 0;
  int64_t nmax = 0;
  for (int i = 0; i < 4; ++i)
    if (ps[i] && ns[i] > 0) {
      r.p[k] = reinterpret_cast<unsigned*>(ps[i]);
      r.n[k] = ns[i];
      nmax = std::max(nmax, ns[i]);
      ++k;
    }
  if (k == 0) return hipSuccess;
  const int blocks = (int)std::min<int64_t>((nmax + 255) / 256, 1024);
  hipLaunchKernelGGL(zero_ranges_kernel, dim3(blocks, k), dim3(256), 0, s, r);
  return hipGetLastError();
}

}  // namespace sat
