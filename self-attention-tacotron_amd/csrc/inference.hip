// Free-running (PREDICT) decoding support: the stop-token termination test of the tacotron2
// StopTokenBasedInferenceHelper (analog in the reference: modules/helpers.py:154-158) evaluated
// on the device, so a captured chunk of decoder steps needs no host round trip per step.
#include "sat_common.h"

namespace sat {
namespace {

// After step t: finished iff t > min_iters and sigmoid(stop[b]) > 0.5 for every utterance b
// (tf.reduce_all); the first such t is latched into state[0] (initialised to -1 by the caller).
__global__ void __launch_bounds__(256) stop_check_kernel(const float* __restrict__ stop,
                                                         int64_t stride, int B, int t,
                                                         int min_iters, int* __restrict__ state) {
  __shared__ int all_done;
  if (threadIdx.x == 0) all_done = 1;
  __syncthreads();
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    const float s = 1.f / (1.f + expf(-stop[(int64_t)b * stride]));
    if (!(s > 0.5f)) atomicAnd(&all_done, 0);
  }
  __syncthreads();
  if (threadIdx.x == 0 && t > min_iters && all_done && state[0] < 0) state[0] = t;
}

}  // namespace
}  // namespace sat

using namespace sat;

extern "C" int sat_stop_check(const float* stop, int64_t stride, int32_t B, int32_t t,
                              int32_t min_iters, int32_t* state, void* stream) {
  SAT_CHECK_ARG(stop && state && B > 0 && t >= 0, "sat_stop_check: bad args");
  hipLaunchKernelGGL(stop_check_kernel, dim3(1), dim3(256), 0, as_stream(stream), stop, stride,
                     B, t, min_iters, state);
  SAT_LAUNCH_CHECK("sat_stop_check");
  return SAT_OK;
}
