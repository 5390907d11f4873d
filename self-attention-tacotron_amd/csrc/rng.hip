// Library plumbing (version, errors) and the counter-based mask generator.
#include <cstdarg>
#include "sat_common.h"

namespace sat {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

namespace {

// Philox-4x32-10 (Salmon et al., SC'11): 4 x 32-bit outputs per (counter, key).
__device__ __forceinline__ uint4 philox(uint4 ctr, uint2 key) {
  constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = __umulhi(M0, ctr.x), lo0 = M0 * ctr.x;
    const uint32_t hi1 = __umulhi(M1, ctr.z), lo1 = M1 * ctr.z;
    ctr = make_uint4(hi1 ^ ctr.y ^ key.x, lo1, hi0 ^ ctr.w ^ key.y, lo0);
    key.x += W0;
    key.y += W1;
  }
  return ctr;
}

__global__ void rng_fill_kernel(float* __restrict__ out, int64_t n, const uint64_t* seed_ptr,
                                uint64_t stream_id, float keep, float on) {
  const uint64_t seed = seed_ptr[0];
  const uint2 key = make_uint2((uint32_t)seed, (uint32_t)(seed >> 32));
  const int64_t groups = (n + 3) / 4;
  for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g < groups;
       g += (int64_t)gridDim.x * blockDim.x) {
    const uint4 r = philox(make_uint4((uint32_t)g, (uint32_t)(g >> 32), (uint32_t)stream_id,
                                      (uint32_t)(stream_id >> 32)), key);
    const uint32_t v[4] = {r.x, r.y, r.z, r.w};
    const float inv = 2.3283064365386963e-10f;  // 2^-32
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t i = g * 4 + j;
      if (i < n) out[i] = ((float)v[j] * inv < keep) ? on : 0.f;
    }
  }
}

// sat_rng_fill_segments: the masks of a training step in one launch.  Group gl of segment s
// draws exactly what rng_fill_kernel draws for group gl of its own launch (same Philox counter
// and key), so every mask is bit-identical to its own launch.
constexpr int kMaxRngSeg = 32;
struct RngSegs {
  int nseg;
  int64_t gstart[kMaxRngSeg + 1];
  SatRngSegment seg[kMaxRngSeg];
};
__global__ void rng_fill_segments_kernel(float* __restrict__ out, const uint64_t* seed_ptr,
                                         RngSegs ss) {
  // segment = blockIdx.y (uniform: its fields stay in scalar registers), grid-stride over its
  // groups along x
  const uint64_t seed = seed_ptr[0];
  const uint2 key = make_uint2((uint32_t)seed, (uint32_t)(seed >> 32));
  const SatRngSegment sg = ss.seg[blockIdx.y];
  const int64_t groups = (sg.n + 3) / 4;
  for (int64_t gl = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; gl < groups;
       gl += (int64_t)gridDim.x * blockDim.x) {
    const uint4 r = philox(make_uint4((uint32_t)gl, (uint32_t)(gl >> 32), (uint32_t)sg.stream_id,
                                      (uint32_t)(sg.stream_id >> 32)), key);
    const uint32_t v[4] = {r.x, r.y, r.z, r.w};
    const float inv = 2.3283064365386963e-10f;  // 2^-32
    float o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = ((float)v[j] * inv < sg.keep) ? sg.on_value : 0.f;
    const int64_t i0 = sg.offset + gl * 4;
    if ((reinterpret_cast<uintptr_t>(out + i0) & 15) == 0 && gl * 4 + 3 < sg.n) {   // one 16-B store
      *reinterpret_cast<float4*>(out + i0) = make_float4(o[0], o[1], o[2], o[3]);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (gl * 4 + j < sg.n) out[i0 + j] = o[j];
    }
  }
}

__global__ void counter_add_kernel(uint64_t* c, uint64_t inc) { c[0] += inc; }

}  // namespace
}  // namespace sat

extern "C" int sat_version(void) { return 10; }

extern "C" int sat_abi_version(void) { return SAT_ABI_VERSION; }

extern "C" const char* sat_last_error_string(void) { return sat::g_err; }

extern "C" int sat_device_arch(char* buf, int len) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) {
    sat::set_error("hipGetDevice failed");
    return SAT_ERR_HIP;
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) {
    sat::set_error("hipGetDeviceProperties failed");
    return SAT_ERR_HIP;
  }
  snprintf(buf, len, "%s", prop.gcnArchName);
  return SAT_OK;
}

extern "C" int sat_rng_fill(float* out, int64_t n, const uint64_t* seed_ptr, uint64_t stream_id,
                            float keep, float on_value, void* stream) {
  using namespace sat;
  SAT_CHECK_ARG(n >= 0, "sat_rng_fill: n < 0");
  if (n == 0) return SAT_OK;
  SAT_CHECK_ARG(out && seed_ptr, "sat_rng_fill: null pointer");
  const int64_t groups = (n + 3) / 4;
  const int blocks = (int)std::min<int64_t>((groups + 255) / 256, 4096);
  hipLaunchKernelGGL(rng_fill_kernel, dim3(blocks), dim3(256), 0, as_stream(stream), out, n,
                     seed_ptr, stream_id, keep, on_value);
  SAT_LAUNCH_CHECK("sat_rng_fill");
  return SAT_OK;
}

extern "C" int sat_rng_fill_segments(float* out, const SatRngSegment* segs, int32_t nseg,
                                     const uint64_t* seed_ptr, void* stream) {
  using namespace sat;
  SAT_CHECK_ARG(nseg >= 0 && nseg <= kMaxRngSeg, "sat_rng_fill_segments: 0 <= nseg <= 32");
  if (nseg == 0) return SAT_OK;
  SAT_CHECK_ARG(out && segs && seed_ptr, "sat_rng_fill_segments: null pointer");
  RngSegs ss;
  ss.nseg = nseg;
  ss.gstart[0] = 0;
  for (int s = 0; s < nseg; ++s) {
    SAT_CHECK_ARG(segs[s].n >= 0 && segs[s].offset >= 0, "sat_rng_fill_segments: bad segment");
    ss.seg[s] = segs[s];
    ss.gstart[s + 1] = ss.gstart[s] + (segs[s].n + 3) / 4;
  }
  int64_t gmax = 0;
  for (int s = 0; s < nseg; ++s) gmax = std::max<int64_t>(gmax, (segs[s].n + 3) / 4);
  if (gmax == 0) return SAT_OK;
  const int blocks = (int)std::min<int64_t>((gmax + 255) / 256, 1024);
  hipLaunchKernelGGL(rng_fill_segments_kernel, dim3(blocks, nseg), dim3(256), 0, as_stream(stream),
                     out, seed_ptr, ss);
  SAT_LAUNCH_CHECK("sat_rng_fill_segments");
  return SAT_OK;
}

extern "C" int sat_counter_add(uint64_t* counter, uint64_t inc, void* stream) {
  using namespace sat;
  SAT_CHECK_ARG(counter, "sat_counter_add: null pointer");
  hipLaunchKernelGGL(counter_add_kernel, dim3(1), dim3(1), 0, as_stream(stream), counter, inc);
  SAT_LAUNCH_CHECK("sat_counter_add");
  return SAT_OK;
}
