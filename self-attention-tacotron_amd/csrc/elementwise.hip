// Small bandwidth-bound kernels of the path (vectorised where the shapes allow).
#include "sat_common.h"

namespace sat {
namespace {

// out[b, n, :] = x[b, n, :] * (n < len[b])      (TF _prepare_memory / sequence_mask)
__global__ void seq_mask_kernel(const float* __restrict__ x, float* __restrict__ out, int B, int N,
                                int C, const int64_t* __restrict__ lengths) {
  const int64_t total = (int64_t)B * N * C;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = i / C;
    const int b = (int)(row / N), n = (int)(row - (int64_t)b * N);
    out[i] = n < lengths[b] ? x[i] : 0.f;
  }
}

}  // namespace
}  // namespace sat

using namespace sat;

extern "C" int sat_seq_mask(const float* x, float* out, int32_t B, int32_t N, int32_t C,
                            const int64_t* lengths, void* stream) {
  SAT_CHECK_ARG(x && out && lengths && B > 0 && N > 0 && C > 0, "sat_seq_mask: bad args");
  const int64_t total = (int64_t)B * N * C;
  const int blocks = (int)std::min<int64_t>((total + 255) / 256, 2048);
  hipLaunchKernelGGL(seq_mask_kernel, dim3(blocks), dim3(256), 0, as_stream(stream), x, out, B, N,
                     C, lengths);
  SAT_LAUNCH_CHECK("sat_seq_mask");
  return SAT_OK;
}
