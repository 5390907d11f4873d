// Micro-benchmark (tools only, not shipped): cost of a group barrier + payload hand-off inside a
// persistent kernel on MI355X, with the guide's sc1-store / sc1-load form (no L2 fences).
// Grid of G*W workgroups; workgroup w belongs to group w % G (blocks b and b+8 share an XCD
// under round-robin placement).  Each round: every workgroup publishes a 16-B record (sc1
// stores), arrives on its group counter (agent-scope atomic), polls it (sc1 loads, bounded),
// then reads all records of its group (sc1 loads) and checks they carry this round's tag.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

typedef float v4f __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st_sc1(float4* p, float4 x) {
  v4f v = {x.x, x.y, x.z, x.w};
  asm volatile("global_store_dwordx4 %0, %1, off sc1" :: "v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ float4 ld_sc1(const float4* p) {
  v4f v;
  asm volatile("global_load_dwordx4 %0, %1, off sc1\n s_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
  return make_float4(v.x, v.y, v.z, v.w);
}

extern "C" __global__ void __launch_bounds__(256) probe_kernel(int G, int rounds, unsigned* ctr,
                                                               float4* rec, int* err,
                                                               long long* clk) {
  const int w = blockIdx.x, g = w % G, nper = gridDim.x / G, idx = w / G;
  __shared__ int ok;
  long long t0 = wall_clock64();
  for (int r = 1; r <= rounds; ++r) {
    if (threadIdx.x == 0) st_sc1(rec + w, make_float4((float)r, (float)w, 0.f, 0.f));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      __hip_atomic_fetch_add(ctr + 32 * g, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned target = (unsigned)(r * nper);
      long spins = 0;
      while (__hip_atomic_load(ctr + 32 * g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > (1l << 24)) { atomicAdd(err + 1, 1); break; }
      }
      ok = 1;
    }
    __syncthreads();
    if (threadIdx.x < nper) {
      const int src = g + G * threadIdx.x;
      const float4 v = ld_sc1(rec + src);
      if (v.x != (float)r || v.y != (float)src) atomicAdd(err, 1);
    }
    (void)idx;
  }
  if (threadIdx.x == 0) clk[w] = wall_clock64() - t0;
}

extern "C" int launch_probe(int G, int W, int rounds, unsigned* ctr, float4* rec, int* err,
                            long long* clk, void* stream) {
  hipLaunchKernelGGL(probe_kernel, dim3(W), dim3(256), 0, (hipStream_t)stream, G, rounds, ctr,
                     rec, err, clk);
  return (int)hipGetLastError();
}
