// Optimiser step over the flat parameter / gradient arenas (models/models.py:175-189, 283-287):
//   lr   = lr0 * 4000^0.5 * min(s * 4000^-1.5, s^-0.5),  s = global_step * step_factor + 1
//   g   *= clip / max(global_norm(g), clip)                       (tf.clip_by_global_norm)
//   tf.train.AdamOptimizer:  m = b1 m + (1-b1) g ; v = b2 v + (1-b2) g^2 ;
//                            p -= lr * sqrt(1-b2^t)/(1-b1^t) * m / (sqrt(v) + eps),  t = step+1
// Everything that changes per step (global_step, the norm, lr_t) lives in device memory, so the
// whole training step can be captured once in a hipGraph and replayed.
// Health guard: the step's error words (the persistent kernels' hand-off timeouts, the embedding
// id-range flag) are read on the device; if any is set the update is skipped entirely (params,
// moments and global_step untouched) and status = {skipped steps, first error code seen} records
// it, so a replayed graph never applies garbage and the host can raise without a sync.
#include "sat_common.h"

namespace sat {
namespace {

constexpr int kNormBlocks = 1024;

__global__ void __launch_bounds__(256) sumsq_kernel(const float* __restrict__ g, int64_t n,
                                                    double* __restrict__ part) {
  __shared__ double sh[4];
  double acc = 0.0;
  const int64_t n4 = n >> 2;
  const float4* g4 = reinterpret_cast<const float4*>(g);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float4 v = g4[i];
    acc += (double)v.x * v.x + (double)v.y * v.y + (double)v.z * v.z + (double)v.w * v.w;
  }
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
    const float v = g[(n4 << 2) + threadIdx.x];
    acc += (double)v * v;
  }
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = sh[0] + sh[1] + sh[2] + sh[3];
}

// scalars: [0] global norm (of grad_scale * g), [1] total scale applied to g, [2] lr (decayed), [3] lr_t (bias corrected)
__global__ void adam_prepare_kernel(const double* __restrict__ part, int nparts,
                                    int64_t* __restrict__ global_step, float* __restrict__ scalars,
                                    double lr0, int decay, int step_factor, double b1, double b2,
                                    double clip, int do_clip, double gscale,
                                    const int* __restrict__ health, int n_health,
                                    int* __restrict__ status, int* __restrict__ skip) {
  __shared__ double sh[256];
  __shared__ int bad;
  if (threadIdx.x == 0) bad = 0;
  __syncthreads();
  if ((int)threadIdx.x < n_health && health[threadIdx.x] != 0) atomicCAS(&bad, 0, health[threadIdx.x]);
  double acc = 0.0;
  for (int i = threadIdx.x; i < nparts; i += blockDim.x) acc += part[i];
  sh[threadIdx.x] = acc;
  __syncthreads();
  for (int s = blockDim.x / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) sh[threadIdx.x] += sh[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    *skip = bad != 0 ? 1 : 0;
    if (bad != 0) {                       // unhealthy step: no update, no step increment
      if (status) {
        status[0] += 1;
        if (status[1] == 0) status[1] = bad;
      }
      return;
    }
    const double norm = gscale * sqrt(sh[0]);
    const double scale = gscale * (do_clip ? clip / fmax(norm, clip) : 1.0);
    const int64_t gs = *global_step;
    double lr = lr0;
    if (decay) {
      const double warm = 4000.0;
      const double s = (double)(gs * step_factor + 1);
      lr = lr0 * sqrt(warm) * fmin(s * pow(warm, -1.5), 1.0 / sqrt(s));
    }
    const double t = (double)(gs + 1);
    const double lr_t = lr * sqrt(1.0 - pow(b2, t)) / (1.0 - pow(b1, t));
    scalars[0] = (float)norm;
    scalars[1] = (float)scale;
    scalars[2] = (float)lr;
    scalars[3] = (float)lr_t;
    *global_step = gs + 1;
  }
}

__global__ void __launch_bounds__(256) adam_update_kernel(float* __restrict__ p,
                                                          const float* __restrict__ g,
                                                          float* __restrict__ m, float* __restrict__ v,
                                                          int64_t n, const float* __restrict__ scalars,
                                                          float b1, float b2, float eps,
                                                          const int* __restrict__ skip) {
  if (*skip) return;
  const float scale = scalars[1], lr_t = scalars[3];
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float gg = g[i] * scale;
    const float mm = b1 * m[i] + (1.f - b1) * gg;
    const float vv = b2 * v[i] + (1.f - b2) * gg * gg;
    m[i] = mm;
    v[i] = vv;
    p[i] -= lr_t * mm / (sqrtf(vv) + eps);
  }
}

// data-parallel exchange tail (dp.py): health words as floats (|code|: a SUM over ranks is
// non-zero iff some rank's word was, and exact when one rank failed), BN moving statistics
// pre-scaled by 1/world (the SUM then leaves their mean)
__global__ void __launch_bounds__(256) exchange_pack_kernel(const int* __restrict__ health,
                                                            int n_health, float* __restrict__ bn,
                                                            int64_t n_bn, float* __restrict__ tail,
                                                            float bn_scale) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < n_health) tail[i] = fabsf((float)health[i]);
  for (int64_t k = i; k < n_bn; k += (int64_t)gridDim.x * blockDim.x) bn[k] *= bn_scale;
}

__global__ void exchange_unpack_kernel(const float* __restrict__ tail, int n_health,
                                       int* __restrict__ health) {
  const int i = threadIdx.x;
  if (i < n_health) health[i] = (int)fminf(tail[i], 2147483520.f);
}

}  // namespace
}  // namespace sat

using namespace sat;

extern "C" int sat_exchange_pack(const int32_t* health, int32_t n_health, float* bn, int64_t n_bn,
                                 float* tail, float bn_scale, void* stream) {
  SAT_CHECK_ARG(n_health >= 0 && n_health <= 256 && n_bn >= 0 && (n_health == 0 || (health && tail)) &&
                    (n_bn == 0 || bn),
                "sat_exchange_pack: health 0..256 words (+ tail), bn >= 0 floats");
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>((n_bn + 255) / 256, 64));
  hipLaunchKernelGGL(exchange_pack_kernel, dim3(blocks), dim3(256), 0, as_stream(stream), health,
                     n_health, bn, n_bn, tail, bn_scale);
  SAT_LAUNCH_CHECK("sat_exchange_pack");
  return SAT_OK;
}

extern "C" int sat_exchange_unpack(const float* tail, int32_t n_health, int32_t* health,
                                   void* stream) {
  SAT_CHECK_ARG(n_health >= 0 && n_health <= 256 && (n_health == 0 || (health && tail)),
                "sat_exchange_unpack: health 0..256 words");
  hipLaunchKernelGGL(exchange_unpack_kernel, dim3(1), dim3(256), 0, as_stream(stream), tail,
                     n_health, health);
  SAT_LAUNCH_CHECK("sat_exchange_unpack");
  return SAT_OK;
}

// workspace: fp64 norm partials, then the skip word of the health guard
extern "C" int64_t sat_workspace_adam(void) { return (int64_t)kNormBlocks * sizeof(double) + 16; }

extern "C" int sat_global_norm_sq(const float* g, int64_t n, double* part, void* stream) {
  SAT_CHECK_ARG(g && part && n >= 0, "sat_global_norm_sq: bad args");
  hipLaunchKernelGGL(sumsq_kernel, dim3(kNormBlocks), dim3(256), 0, as_stream(stream), g, n, part);
  SAT_LAUNCH_CHECK("sat_global_norm_sq");
  return SAT_OK;
}

extern "C" int sat_adam_step(float* params, const float* grads, float* m, float* v, int64_t n,
                             int64_t* global_step, float* scalars, void* workspace,
                             const SatAdamConfig* cfg, const int32_t* health, int32_t n_health,
                             int32_t* status, void* stream) {
  SAT_CHECK_ARG(params && grads && m && v && global_step && scalars && workspace && cfg && n >= 0,
                "sat_adam_step: bad args");
  SAT_CHECK_ARG(n_health >= 0 && n_health <= 256 && (n_health == 0 || health),
                "sat_adam_step: health words: 0..256 int32 (pointer needed when n_health > 0)");
  SAT_CHECK_ARG(cfg->grad_scale > 0.f, "sat_adam_step: grad_scale must be > 0");
  hipStream_t s = as_stream(stream);
  double* part = reinterpret_cast<double*>(workspace);
  int* skip = reinterpret_cast<int*>(part + kNormBlocks);
  hipLaunchKernelGGL(sumsq_kernel, dim3(kNormBlocks), dim3(256), 0, s, grads, n, part);
  hipLaunchKernelGGL(adam_prepare_kernel, dim3(1), dim3(256), 0, s, part, kNormBlocks, global_step,
                     scalars, (double)cfg->lr0, cfg->decay, cfg->step_factor, (double)cfg->beta1,
                     (double)cfg->beta2, (double)cfg->clip_norm, cfg->clip_norm > 0.f ? 1 : 0,
                     (double)cfg->grad_scale, health, n_health, status, skip);
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 8192);
  hipLaunchKernelGGL(adam_update_kernel, dim3(blocks), dim3(256), 0, s, params, grads, m, v, n,
                     scalars, cfg->beta1, cfg->beta2, cfg->eps, skip);
  SAT_LAUNCH_CHECK("sat_adam_step");
  return SAT_OK;
}
