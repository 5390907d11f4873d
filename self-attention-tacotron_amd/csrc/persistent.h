// In-kernel hand-off primitives of the persistent decoder kernels (decoder_persistent.hip,
// decoder_persistent_bwd.hip): device-coherent sc1 buffer accesses and a bounded group barrier.
// Form: MI355X_MICROARCH.md, inter-workgroup visibility, "sc1 loads in place of the acquire"
// table row 1 -- producers store sc1 and drain (s_waitcnt vmcnt(0)) before the workgroup
// barrier; one lane arrives on the group counter (agent-scope atomic) and polls it; every load
// of another workgroup's bytes is an sc1 load.
#pragma once
#include "sat_common.h"

namespace sat {
namespace {

typedef unsigned v4u __attribute__((ext_vector_type(4)));

// ---- device-coherent (sc1: L1-bypassing, write-through) accesses for the hand-offs; buffer
//      forms so the compiler batches them like plain loads
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ float ldc(__amdgpu_buffer_rsrc_t r, int idx) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, idx * 4, 0, 16));
}
__device__ __forceinline__ float4 ldc4(__amdgpu_buffer_rsrc_t r, int idx4) {
  const v4u v = __builtin_amdgcn_raw_buffer_load_b128(r, idx4 * 16, 0, 16);
  return make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]),
                     __uint_as_float(v[3]));
}
__device__ __forceinline__ void stc(__amdgpu_buffer_rsrc_t r, int idx, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, idx * 4, 0, 16);
}
__device__ __forceinline__ void stc4(__amdgpu_buffer_rsrc_t r, int idx4, float4 v) {
  const v4u w = {__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z),
                 __float_as_uint(v.w)};
  __builtin_amdgcn_raw_buffer_store_b128(w, r, idx4 * 16, 0, 16);
}

__device__ __forceinline__ void group_barrier(unsigned* ctr, unsigned target, int* err) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every wave drains its sc1 stores
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned spins = 0;
    while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if ((++spins & 1023u) == 0) {
        if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) break;
        if (spins > (1u << 22)) {   // ~0.2 s: a workgroup never arrived (not co-resident?)
          __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
    }
  }
  __syncthreads();
}


}  // namespace
}  // namespace sat
