// Hand-off skeleton of the attention-chain forward (tools only): the grid, groups and record
// shapes of dec_attn_fwd8_kernel (256 workgroups x 512 threads, group = 8 workgroups
// blockIdx = g + 32 j, per step two 8-producer hand-offs of 1-KB LSB-tagged records, every wave
// staging one producer's record), with a configurable dummy dependent-FMA chain before each
// publish (critical compute) and between publish and poll (shadow compute).  Measures what the
// two hand-offs cost per step at the kernel's geometry with no real work.
#include "../../self-attention-tacotron_amd/csrc/persistent.h"

using namespace sat;

__device__ __forceinline__ float spin(float x, int n) {
  for (int i = 0; i < n; ++i) x = fmaf(x, 0.999f, 0.001f);
  return x;
}

// pre: 0 = poll after the shadow compute; 1 = first poll load issued before the shadow (checked
// after it); 2 = issued halfway through the shadow
// nbar: further LDS-synchronised phases per hand-off (each: one LDS write, barrier, dependent
// LDS read of another wave's word) -- the empty-phase floor of the real kernel's schedule
__global__ void __launch_bounds__(512) ring8_kernel(float* RA, float* RB, int T, int crit,
                                                    int shadow, int xl_on, int pre, int nbar,
                                                    int* err, long long* clk) {
  __shared__ float ph_w[8][64];
  __shared__ float4 st[8][64];
  const int g = blockIdx.x % 32, j = blockIdx.x / 32;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const auto rA = rsrc(RA), rB = rsrc(RB);
  const bool xl = xl_on != 0;
  float acc = (float)threadIdx.x * 1e-3f;
  bool gave_up = false;
  const long long t0 = wall_clock64();
  for (int t = 0; t < T; ++t) {
    const unsigned bit = lsb_tag(t);
    for (int ph = 0; ph < 2; ++ph) {
      const auto r = ph ? rB : rA;
      acc = spin(acc, crit);
      // publish: wave w writes float4 chunks 8w .. 8w+7 of its workgroup's record (lanes 0..7)
      const int rec = (((t & 1) * 32 + g) * 8 + j) * 64;
      if (lane < 8) stc4x(xl, r, rec + 8 * wave + lane, tagf4(make_float4(acc, 1.f, 2.f, 3.f), bit));
      const long long tpub = wall_clock64();
      // poll: wave w stages producer w's whole record (64 float4)
      const int src = (((t & 1) * 32 + g) * 8 + wave) * 64 + lane;
      float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
      bool ok = false;
      if (pre == 1) {
        x = ldc4(r, src);
        acc = spin(acc, shadow);
      } else if (pre == 2) {
        acc = spin(acc, shadow / 2);
        x = ldc4(r, src);
        acc = spin(acc, shadow - shadow / 2);
      } else {
        acc = spin(acc, shadow);
      }
      const long long tp = wall_clock64();
      unsigned spins = 0;
      for (;; ++spins) {
        if (!ok && (spins > 0 || pre == 0)) x = ldc4(r, src);
        ok = tag_ok4(x, bit);
        if (__builtin_amdgcn_ballot_w64(!ok) == 0 || gave_up) break;
        if (poll_give_up(spins, err)) { gave_up = true; break; }
        __builtin_amdgcn_s_sleep(1);
      }
      const long long tq = wall_clock64();
      st[wave][lane] = x;
      lds_barrier();
      acc += st[(wave + 1) & 7][lane].x * 1e-6f;
      for (int k = 0; k < nbar; ++k) {
        ph_w[wave][lane] = acc;
        lds_barrier();
        acc += ph_w[(wave + 1 + k) & 7][lane ^ 1] * 1e-6f;
      }
      const long long tr = wall_clock64();
      // event record of block 0, wave 0, steps 100..163: {poll start, poll done, after barrier,
      // spins} relative to the step's publish
      if (blockIdx.x == 0 && t >= 100 && t < 164 && threadIdx.x == 0) {
        long long* e = clk + 256 + ((t - 100) * 2 + ph) * 4;
        e[0] = tp - tpub; e[1] = tq - tpub; e[2] = tr - tpub; e[3] = spins;
      }
    }
  }
  const long long t1 = wall_clock64();
  if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
  if (acc == 12345.f) RA[0] = acc;
}

extern "C" int ring8(float* RA, float* RB, int T, int crit, int shadow, int xl, int pre,
                     int nbar, int* err, long long* clk, void* stream) {
  hipLaunchKernelGGL(ring8_kernel, dim3(256), dim3(512), 0, static_cast<hipStream_t>(stream), RA,
                     RB, T, crit, shadow, xl, pre, nbar, err, clk);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
