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

// One step of the decoder head's causal self-attention against its key/value cache
// (TransformerWrapper, modules/rnn_wrappers.py:87-124: the causal SelfAttentionTransformer re-run
// over the whole history keeps only its last row, i.e. one query row against the cached keys and
// values of steps 0..t -- ScaledDotProductAttentionMechanism, modules/self_attention.py:45-65,
// no dropout at inference).  One workgroup per (utterance, head): scores of the t + 1 cached
// rows (lane = row, float4 dot over the head dims), softmax(scale * s), the probability row into
// P (the decoder self-alignments the PREDICT spec returns), then o = p . V with the rows split
// over thread groups and summed in a fixed order.  Replaces the per-step gemm + softmax + copy +
// gemm (4 launches) of the launch path.
__global__ void __launch_bounds__(256) decode_attention_kernel(
    const float* __restrict__ qkv, int64_t qkv_sb, int64_t qkv_st, int H, int D, int t,
    float scale, float* __restrict__ P, int Tm, float* __restrict__ O, int64_t o_sb) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int b = blockIdx.x / H, h = blockIdx.x - b * H;
  const int dh = D / H, n = t + 1, tid = threadIdx.x;
  float* qs = sm;                    // [dh]
  float* ps = sm + dh;               // [n] scores, then probabilities
  float* red = ps + ((n + 3) & ~3);  // [256] reduction scratch
  const float* base = qkv + (int64_t)b * qkv_sb;
  for (int d = tid; d < dh; d += 256) qs[d] = base[(int64_t)t * qkv_st + h * dh + d];
  __syncthreads();
  float mx = -INFINITY;
  for (int j = tid; j < n; j += 256) {
    const float4* k4 = reinterpret_cast<const float4*>(base + (int64_t)j * qkv_st + D + h * dh);
    float a = 0.f;
    for (int d4 = 0; d4 < dh / 4; ++d4) {
      const float4 kv = k4[d4];
      const float4 qv = *reinterpret_cast<const float4*>(qs + 4 * d4);
      a = fmaf(qv.x, kv.x, a); a = fmaf(qv.y, kv.y, a);
      a = fmaf(qv.z, kv.z, a); a = fmaf(qv.w, kv.w, a);
    }
    a *= scale;
    ps[j] = a;
    mx = fmaxf(mx, a);
  }
  mx = block_max(mx, red);
  float sum = 0.f;
  for (int j = tid; j < n; j += 256) {
    const float e = __expf(ps[j] - mx);
    ps[j] = e;
    sum += e;
  }
  sum = block_sum(sum, red);
  const float rs = 1.f / sum;
  float* prow = P ? P + ((int64_t)(b * H + h) * Tm + t) * Tm : nullptr;
  for (int j = tid; j < n; j += 256) {
    const float pv = ps[j] * rs;
    ps[j] = pv;
    if (prow) prow[j] = pv;
  }
  __syncthreads();
  // o[d] = sum_j p_j v_j[d]: thread (g, d), G = 256 / dh row groups, rows j = g, g + G, ...
  const int G = 256 / dh, g = tid / dh, d = tid - g * dh;
  float a = 0.f;
  if (g < G) {
    const float* vcol = base + D + D + h * dh + d;
    for (int j = g; j < n; j += G) a = fmaf(ps[j], vcol[(int64_t)j * qkv_st], a);
  }
  __syncthreads();
  red[tid] = a;
  __syncthreads();
  if (tid < dh) {
    float o = 0.f;
    for (int k = 0; k < G; ++k) o += red[k * dh + tid];
    O[(int64_t)b * o_sb + h * dh + tid] = o;
  }
}

}  // namespace
}  // namespace sat

using namespace sat;

extern "C" int sat_decode_attention_step(const float* qkv, int64_t qkv_sb, int64_t qkv_st,
                                         int32_t B, int32_t H, int32_t D, int32_t t, float scale,
                                         float* P, int32_t Tm, float* O, int64_t o_sb,
                                         void* stream) {
  SAT_CHECK_ARG(qkv && O && B > 0 && H > 0 && D % H == 0 && t >= 0 && (!P || t < Tm),
                "sat_decode_attention_step: bad args");
  const int dh = D / H;
  SAT_CHECK_ARG(dh % 4 == 0 && dh <= 256 && 256 % dh == 0 && qkv_st % 4 == 0 && qkv_sb % 4 == 0 &&
                aligned16(qkv), "sat_decode_attention_step: head width must divide 256, % 4; "
                "16-byte aligned rows");
  const size_t shm = ((size_t)dh + (size_t)((t + 4) & ~3) + 256) * sizeof(float);
  SAT_CHECK_ARG(shm <= 64 * 1024, "sat_decode_attention_step: history too long");
  hipLaunchKernelGGL(decode_attention_kernel, dim3(B * H), dim3(256), shm, as_stream(stream), qkv,
                     qkv_sb, qkv_st, H, D, t, scale, P, Tm, O, o_sb);
  SAT_LAUNCH_CHECK("sat_decode_attention_step");
  return SAT_OK;
}

extern "C" int sat_stop_check(const float* stop, int64_t stride, int32_t B, int32_t t,
                              int32_t min_iters, int32_t* state, void* stream) {
  SAT_CHECK_ARG(stop && state && B > 0 && t >= 0, "sat_stop_check: bad args");
  hipLaunchKernelGGL(stop_check_kernel, dim3(1), dim3(256), 0, as_stream(stream), stop, stride,
                     B, t, min_iters, state);
  SAT_LAUNCH_CHECK("sat_stop_check");
  return SAT_OK;
}
