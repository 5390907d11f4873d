// Hand-off latency probe (tools only): two workgroups on one XCD ping-pong a 1-KB tagged record
// (64 lanes x 16 B, the persistent kernels' record shape) with the persistent kernels' store /
// load forms (persistent.h), for three poll styles:
//   0  load, wait, s_sleep 1, repeat        (the kernels' loop)
//   1  load, wait, repeat                   (no sleep)
//   2  two loads in flight, staggered       (check the older while the newer travels)
// Prints ns per one-way hand-off (half a round trip).  Measured (two boxes): style 0 263-276 ns;
// style 2 117 ns on one box and 388 ns on another -- not adopted (rejected).
#include "../../self-attention-tacotron_amd/csrc/persistent.h"

using namespace sat;

template <int STYLE>
__device__ float4 poll(__amdgpu_buffer_rsrc_t r, int idx4, unsigned want) {
  if constexpr (STYLE == 2) {
    // raw asm: the compiler's wait insertion drains both loads before the first check
    v4u a, b;
    const int off = idx4 * 16;
    asm volatile(
        "buffer_load_dwordx4 %0, %2, %3, 0 offen sc1\n\t"
        "s_sleep 2\n\t"
        "buffer_load_dwordx4 %1, %2, %3, 0 offen sc1\n\t"
        "s_waitcnt vmcnt(1)"
        : "=&v"(a), "=&v"(b) : "v"(off), "s"(r) : "memory");
    for (unsigned spins = 0; spins < (1u << 22); ++spins) {
      float4 fa = make_float4(__uint_as_float(a[0]), __uint_as_float(a[1]), __uint_as_float(a[2]), __uint_as_float(a[3]));
      if (__builtin_amdgcn_ballot_w64(!tag_ok4(fa, want)) == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        return fa;
      }
      asm volatile(
          "buffer_load_dwordx4 %0, %1, %2, 0 offen sc1\n\t"
          "s_waitcnt vmcnt(1)"
          : "=&v"(a) : "v"(off), "s"(r) : "memory");
      float4 fb = make_float4(__uint_as_float(b[0]), __uint_as_float(b[1]), __uint_as_float(b[2]), __uint_as_float(b[3]));
      if (__builtin_amdgcn_ballot_w64(!tag_ok4(fb, want)) == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        return fb;
      }
      asm volatile(
          "buffer_load_dwordx4 %0, %1, %2, 0 offen sc1\n\t"
          "s_waitcnt vmcnt(1)"
          : "=&v"(b) : "v"(off), "s"(r) : "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    return make_float4(0.f, 0.f, 0.f, 0.f);
  } else {
    for (unsigned spins = 0; spins < (1u << 22); ++spins) {
      asm volatile("" ::: "memory");
      const float4 a = ldc4(r, idx4);
      if (__builtin_amdgcn_ballot_w64(!tag_ok4(a, want)) == 0) return a;
      if (STYLE == 0) __builtin_amdgcn_s_sleep(1);
    }
    return make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

template <int STYLE>
__global__ void __launch_bounds__(64) pingpong_kernel(float* buf, int rounds, long long* out,
                                                      unsigned* xcc) {
  const int me = blockIdx.x == 0 ? 0 : 1;
  if (blockIdx.x != 0 && blockIdx.x != 8) return;
  const auto r = rsrc(buf);
  const int lane = threadIdx.x;
  if (lane == 0) xcc[me] = xcc_id();
  float acc = 0.f;
  const long long t0 = wall_clock64();
  for (int k = 0; k < rounds; ++k) {
    const unsigned bit = lsb_tag(k);
    const int slot = k & 1;
    if (me == 0) {
      stc4x(true, r, (slot * 2 + 0) * 64 + lane, tagf4(make_float4(acc, 1.f, 2.f, 3.f), bit));
      const float4 v = poll<STYLE>(r, (slot * 2 + 1) * 64 + lane, bit);
      acc += v.x;
    } else {
      const float4 v = poll<STYLE>(r, (slot * 2 + 0) * 64 + lane, bit);
      acc += v.y;
      stc4x(true, r, (slot * 2 + 1) * 64 + lane, tagf4(make_float4(acc, 1.f, 2.f, 3.f), bit));
    }
  }
  const long long t1 = wall_clock64();
  if (lane == 0) out[me] = t1 - t0;
  if (acc == 12345.f) buf[0] = acc;
}

extern "C" int pingpong(int style, float* buf, int rounds, long long* out, unsigned* xcc,
                        void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (style == 0) hipLaunchKernelGGL(pingpong_kernel<0>, dim3(16), dim3(64), 0, s, buf, rounds, out, xcc);
  if (style == 1) hipLaunchKernelGGL(pingpong_kernel<1>, dim3(16), dim3(64), 0, s, buf, rounds, out, xcc);
  if (style == 2) hipLaunchKernelGGL(pingpong_kernel<2>, dim3(16), dim3(64), 0, s, buf, rounds, out, xcc);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

