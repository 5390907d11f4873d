// In-kernel hand-off primitives of the persistent decoder kernels (decoder_persistent.hip,
// decoder_persistent_bwd.hip): device-coherent sc1 buffer accesses and a bounded group barrier.
// Form: MI355X_MICROARCH.md, inter-workgroup visibility, "sc1 loads in place of the acquire"
// table row 1 -- producers store sc1 and drain (s_waitcnt vmcnt(0)) before the workgroup
// barrier; one lane arrives on the group counter (agent-scope atomic) and polls it; every load
// of another workgroup's bytes is an sc1 load.
#pragma once
#include "sat_common.h"
#include <cstdlib>

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

// ---- data-tagged hand-offs (MI355X_MICROARCH.md "handoff-1to1": the data IS the flag)
// (1) 8-byte granules {value, tag}: one sc1 dwordx2 store, untorn; used where a value may be
//     non-finite (raw energies: -inf at padded positions).
typedef unsigned v2u __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void stg(__amdgpu_buffer_rsrc_t r, int granule, float v, unsigned tag) {
  const v2u w = {__float_as_uint(v), tag};
  __builtin_amdgcn_raw_buffer_store_b64(w, r, granule * 8, 0, 16);
}
__device__ __forceinline__ v2u ldg(__amdgpu_buffer_rsrc_t r, int granule) {
  return __builtin_amdgcn_raw_buffer_load_b64(r, granule * 8, 0, 16);
}
// (2) step parity in the mantissa LSB of every handed-off float (bulk payloads: contexts,
//     query partials, states).  A 4-byte word is never torn, so each word carries its own
//     validity and a 16-byte sc1 store needs no flag, no drain and no barrier.  Slots alternate
//     by step parity (slot s & 1); the bit for step s is ((s >> 1) + 1) & 1, so a slot's
//     previous occupant (step s - 2) always carries the other bit and zeroed scratch (LSB 0)
//     never matches steps 0 and 1 -- provided every slot's first occupant is written at sequence
//     number 0 or 1 (a slot first written at 2 would match its zeroes).  Cost: <= 1 ulp (6e-8 relative) on the tagged values, which
//     every consumer reads identically.  Only finite values are tagged.
__device__ __forceinline__ unsigned lsb_tag(int s) { return (unsigned)(((s >> 1) + 1) & 1); }
__device__ __forceinline__ float tagf(float x, unsigned bit) {
  return __uint_as_float((__float_as_uint(x) & ~1u) | bit);
}
__device__ __forceinline__ float4 tagf4(float4 v, unsigned bit) {
  return make_float4(tagf(v.x, bit), tagf(v.y, bit), tagf(v.z, bit), tagf(v.w, bit));
}
__device__ __forceinline__ bool tag_ok(float x, unsigned bit) {
  return ((__float_as_uint(x) ^ bit) & 1u) == 0;
}
__device__ __forceinline__ bool tag_ok4(float4 v, unsigned bit) {
  return (((__float_as_uint(v.x) ^ bit) | (__float_as_uint(v.y) ^ bit) |
           (__float_as_uint(v.z) ^ bit) | (__float_as_uint(v.w) ^ bit)) & 1u) == 0;
}
// ---- XCD-local store policy of a hand-off group.  A plain (aux 0) buffer store is written
//      through the CU's L1 into its XCD's L2 and the line STAYS there, where an sc1 load from
//      any CU of the same XCD finds it; an sc1 store drops the line (MI355X_MICROARCH.md,
//      stores row), so a same-XCD consumer then reads at the cross-XCD rate.  The plain form is
//      used only when the group has CHECKED at run time (xcd_local_group) that every producer
//      and consumer of its hand-offs sits on one XCD; otherwise every store stays sc1.
__device__ __forceinline__ void stc4x(bool xl, __amdgpu_buffer_rsrc_t r, int idx4, float4 v) {
  const v4u w = {__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z),
                 __float_as_uint(v.w)};
  if (xl) __builtin_amdgcn_raw_buffer_store_b128(w, r, idx4 * 16, 0, 0);
  else __builtin_amdgcn_raw_buffer_store_b128(w, r, idx4 * 16, 0, 16);
}
__device__ __forceinline__ void stgx(bool xl, __amdgpu_buffer_rsrc_t r, int granule, float v,
                                     unsigned tag) {
  const v2u w = {__float_as_uint(v), tag};
  if (xl) __builtin_amdgcn_raw_buffer_store_b64(w, r, granule * 8, 0, 0);
  else __builtin_amdgcn_raw_buffer_store_b64(w, r, granule * 8, 0, 16);
}
__device__ __forceinline__ void stcx(bool xl, __amdgpu_buffer_rsrc_t r, int idx, float v) {
  if (xl) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, idx * 4, 0, 0);
  else __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, idx * 4, 0, 16);
}
// host: SAT_XCD_LOCAL=0 forces sc1 stores everywhere (A/B switch of the store policy)
static inline int xcd_local_env() {
  const char* e = getenv("SAT_XCD_LOCAL");
  return (e && e[0] == '0') ? 0 : 1;
}
__device__ __forceinline__ unsigned xcc_id() {
  unsigned x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
  return x;
}
// Placement check of one hand-off group (members blockIdx = g + stride * i, i < n <= 64): every
// member publishes XCC_ID + 1 (sc1) into its word of `ids` (zeroed scratch), wave 0 polls the
// group's words (sc1, bounded) and the group is XCD-local iff all ids agree.  Every member reads
// the same words, so every member reaches the same verdict.  A timeout raises err and returns
// false (sc1 everywhere).  Call from all threads of the workgroup (it ends in a barrier).
__device__ __forceinline__ bool xcd_local_group(unsigned* ids, int g, int stride, int n,
                                                int* err) {
  __shared__ int verdict;
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(ids, 0, 0x7fffffff, 0x00020000);
  if (threadIdx.x == 0) {
    __builtin_amdgcn_raw_buffer_store_b32(xcc_id() + 1u, r, blockIdx.x * 4, 0, 16);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    unsigned v = 0, spins = 0;
    bool ok = true;
    for (;;) {
      v = lane < n ? __builtin_amdgcn_raw_buffer_load_b32(r, (g + stride * lane) * 4, 0, 16) : 1u;
      if (__builtin_amdgcn_ballot_w64(v == 0u) == 0) break;
      __builtin_amdgcn_s_sleep(1);
      if ((++spins & 255u) == 255u) {
        if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0 ||
            spins > (1u << 20)) {
          if (spins > (1u << 20)) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ok = false;
          break;
        }
      }
    }
    const unsigned first = __builtin_amdgcn_readfirstlane(v);
    const bool same = __builtin_amdgcn_ballot_w64(lane < n && v != first) == 0;
    if (lane == 0) verdict = (ok && same) ? 1 : 0;
  }
  __syncthreads();
  return verdict != 0;
}

// bounded-spin bookkeeping of a poll loop: every 256 spins look at the error word; after
// ~2^20 spins (a producer never published: grid not co-resident) raise it.  Returns true when
// the loop must give up (the grid then drains with garbage and the host reports err).
__device__ __forceinline__ bool poll_give_up(unsigned spins, int* err) {
  if ((spins & 255u) != 255u) return false;
  if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return true;
  if (spins > (1u << 20)) {
    __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return true;
  }
  return false;
}

// s_waitcnt vmcnt(0) in the compiler-visible form (gfx9 simm16: vmcnt 0, expcnt 7, lgkmcnt 15):
// the waitcnt pass sees it and drops the loads it covers from its pending state.  Inline asm
// is opaque to that pass, so an asm drain before a step loop still leaves the prologue's loads
// "pending" at the loop header and their waits land inside the loop.
__device__ __forceinline__ void vm_drain() { __builtin_amdgcn_s_waitcnt(0x0F70); }

// One global_load_lds_dwordx4: 16 bytes per active lane from src into LDS at lds_addr + 16 *
// lane (lds_addr wave-uniform).  Issued from inline asm, so the waitcnt pass does not track it:
// the caller orders it with its own s_waitcnt vmcnt (the counter retires in issue order) and a
// barrier before other waves read the bytes.
__device__ __forceinline__ void lds_dma16(const void* src, uint32_t lds_addr) {
  int keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(__builtin_amdgcn_readfirstlane(lds_addr))
      : "memory");
}
__device__ __forceinline__ uint32_t lds_addr_of(const void* p) {
  return (uint32_t)(uintptr_t)((__attribute__((address_space(3))) const char*)p);
}

// ---- wave-level dot helpers shared by the persistent kernels
__device__ __forceinline__ float dot4(float4 a, float4 b, float acc) {
  acc = fmaf(a.x, b.x, acc);
  acc = fmaf(a.y, b.y, acc);
  acc = fmaf(a.z, b.z, acc);
  return fmaf(a.w, b.w, acc);
}

// Transpose-reduce across the 64 lanes of a wave: v[0..N-1] are per-lane partial sums of N
// different outputs; each halving exchange pairs (v[i], v[i + n/2]) over one lane bit, after
// which every lane keeps the half its bit selects, summed with its partner's.  All VALU, no
// LDS: the 32- and 16-lane exchanges are gfx950 v_permlane32_swap / v_permlane16_swap (after
// the swap x' + y' is already the kept half's sum), the 8/4-lane ones DPP row shifts (lane l
// adds lane l+H where bit H of l is clear, lane l-H where it is set).  Lane bits left over when
// the values run out are plain butterflies, so every lane of a 64/N block ends with the total.
__device__ __forceinline__ float fsum_swap32(float x, float y) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(y), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float fsum_swap16(float x, float y) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(y), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xF, 0xF, true));
}
template <int H, int HALF>
__device__ __forceinline__ void tr_dpp(float* v, int lane) {
  const bool hi = (lane & H) != 0;
#pragma unroll
  for (int i = 0; i < HALF; ++i) {
    const float sa = v[i] + dpp_mov<0x100 + H>(v[i]);                // row_shl:H (lane l+H)
    const float sb = v[i + HALF] + dpp_mov<0x110 + H>(v[i + HALF]);  // row_shr:H (lane l-H)
    v[i] = hi ? sb : sa;
  }
}
// 32 outputs: lanes 2m, 2m+1 hold output m
__device__ __forceinline__ void transpose_reduce32(float* v, int lane) {
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = fsum_swap32(v[i], v[i + 16]);
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = fsum_swap16(v[i], v[i + 8]);
  tr_dpp<8, 4>(v, lane);
  tr_dpp<4, 2>(v, lane);
  tr_dpp<2, 1>(v, lane);
  v[0] += dpp_mov<0xB1>(v[0]);   // quad_perm [1,0,3,2]: lane l ^ 1
}
// 8 outputs: lanes 8m..8m+7 hold output m
__device__ __forceinline__ void transpose_reduce8(float* v, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = fsum_swap32(v[i], v[i + 4]);
#pragma unroll
  for (int i = 0; i < 2; ++i) v[i] = fsum_swap16(v[i], v[i + 2]);
  tr_dpp<8, 1>(v, lane);
  {   // lane bit 2: partner l ^ 4 via row shifts
    const float up = dpp_mov<0x104>(v[0]), dn = dpp_mov<0x114>(v[0]);
    v[0] += (lane & 4) ? dn : up;
  }
  v[0] += dpp_mov<0x4E>(v[0]);   // lane l ^ 2
  v[0] += dpp_mov<0xB1>(v[0]);   // lane l ^ 1
}
// 16 outputs: lanes 4m..4m+3 hold output m
__device__ __forceinline__ void transpose_reduce16(float* v, int lane) {
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = fsum_swap32(v[i], v[i + 8]);
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = fsum_swap16(v[i], v[i + 4]);
  tr_dpp<8, 2>(v, lane);
  tr_dpp<4, 1>(v, lane);
  v[0] += dpp_mov<0xB1>(v[0]);   // lane l ^ 1
  v[0] += dpp_mov<0x4E>(v[0]);   // quad_perm [2,3,0,1]: lane l ^ 2
}

}  // namespace
}  // namespace sat

namespace sat {
// one-utterance-per-8-workgroups layout of the attention-chain forward (decoder_persistent8.hip)
bool dec_attn_fwd8_eligible(const SatDecAttnFwd* a);
int dec_attn_fwd8_launch(const SatDecAttnFwd* a, hipStream_t s);
bool dec_attn_bwd8_eligible(const SatDecAttnBwd* a);   // decoder_persistent8_bwd.hip
int dec_attn_bwd8_launch(const SatDecAttnBwd* a, hipStream_t s);
}  // namespace sat
