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
constexpr int kDecAttnThreads = 512;
template <int DH>
__global__ void __launch_bounds__(kDecAttnThreads) decode_attention_kernel(
    const float* __restrict__ qkv, int64_t qkv_sb, int64_t qkv_st, int H, int D, int t,
    float scale, float* __restrict__ P, int Tm, float* __restrict__ O, int64_t o_sb) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  constexpr int DQ = DH / 4;         // float4 per head row
  constexpr int NT = kDecAttnThreads;
  constexpr int G = NT / DQ;         // row groups of the p . V pass
  const int b = blockIdx.x / H, h = blockIdx.x - b * H;
  const int n = t + 1, tid = threadIdx.x;
  float* qs = sm;                    // [DH]
  float* ps = sm + DH;               // [n] scores, then probabilities
  float* red = ps + ((n + 3) & ~3);  // [NT * 4] reduction scratch
  const float* base = qkv + (int64_t)b * qkv_sb;
  for (int d = tid; d < DH; d += NT) qs[d] = base[(int64_t)t * qkv_st + h * DH + d];
  __syncthreads();
  // scores: lane = cached row; the row's DQ float4 loads are independent (unrolled: all in
  // flight), the query comes from LDS as broadcast float4 reads
  float mx = -INFINITY;
  for (int j = tid; j < n; j += NT) {
    const float4* k4 = reinterpret_cast<const float4*>(base + (int64_t)j * qkv_st + D + h * DH);
    float4 kv[DQ];
#pragma unroll
    for (int d4 = 0; d4 < DQ; ++d4) kv[d4] = k4[d4];
    float a0 = 0.f, a1 = 0.f;
#pragma unroll
    for (int d4 = 0; d4 < DQ; d4 += 2) {
      const float4 q0 = *reinterpret_cast<const float4*>(qs + 4 * d4);
      const float4 q1 = *reinterpret_cast<const float4*>(qs + 4 * d4 + 4);
      a0 = fmaf(q0.x, kv[d4].x, a0); a0 = fmaf(q0.y, kv[d4].y, a0);
      a0 = fmaf(q0.z, kv[d4].z, a0); a0 = fmaf(q0.w, kv[d4].w, a0);
      a1 = fmaf(q1.x, kv[d4 + 1].x, a1); a1 = fmaf(q1.y, kv[d4 + 1].y, a1);
      a1 = fmaf(q1.z, kv[d4 + 1].z, a1); a1 = fmaf(q1.w, kv[d4 + 1].w, a1);
    }
    const float a = (a0 + a1) * scale;
    ps[j] = a;
    mx = fmaxf(mx, a);
  }
  mx = block_max(mx, red);
  float sum = 0.f;
  for (int j = tid; j < n; j += NT) {
    const float e = __expf(ps[j] - mx);
    ps[j] = e;
    sum += e;
  }
  sum = block_sum(sum, red);
  const float rs = 1.f / sum;
  float* prow = P ? P + ((int64_t)(b * H + h) * Tm + t) * Tm : nullptr;
  for (int j = tid; j < n; j += NT) {
    const float pv = ps[j] * rs;
    ps[j] = pv;
    if (prow) prow[j] = pv;
  }
  __syncthreads();
  // o = sum_j p_j v_j: thread (g, d4) accumulates float4 column chunk d4 over rows g, g + G,
  // ... four rows in flight per trip; the G partial rows are summed in a fixed order
  const int g = tid / DQ, d4 = tid - g * DQ;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  const float* vbase = base + 2 * D + h * DH + 4 * d4;
  int j = g;
  for (; j + 7 * G < n; j += 8 * G) {
    float4 v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = *reinterpret_cast<const float4*>(vbase + (int64_t)(j + q * G) * qkv_st);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float pv = ps[j + q * G];
      acc.x = fmaf(pv, v[q].x, acc.x); acc.y = fmaf(pv, v[q].y, acc.y);
      acc.z = fmaf(pv, v[q].z, acc.z); acc.w = fmaf(pv, v[q].w, acc.w);
    }
  }
  for (; j < n; j += G) {
    const float4 v = *reinterpret_cast<const float4*>(vbase + (int64_t)j * qkv_st);
    const float pv = ps[j];
    acc.x = fmaf(pv, v.x, acc.x); acc.y = fmaf(pv, v.y, acc.y);
    acc.z = fmaf(pv, v.z, acc.z); acc.w = fmaf(pv, v.w, acc.w);
  }
  __syncthreads();
  reinterpret_cast<float4*>(red)[tid] = acc;
  __syncthreads();
  if (tid < DQ) {
    float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int k = 0; k < G; ++k) {
      const float4 r = reinterpret_cast<const float4*>(red)[k * DQ + tid];
      o.x += r.x; o.y += r.y; o.z += r.z; o.w += r.w;
    }
    reinterpret_cast<float4*>(O + (int64_t)b * o_sb + h * DH)[tid] = o;
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
  SAT_CHECK_ARG((dh == 32 || dh == 64 || dh == 128) && qkv_st % 4 == 0 && qkv_sb % 4 == 0 &&
                o_sb % 4 == 0 && aligned16(qkv) && aligned16(O),
                "sat_decode_attention_step: head width 32, 64 or 128; 16-byte aligned rows");
  const size_t shm = ((size_t)dh + (size_t)((t + 4) & ~3) + 4 * kDecAttnThreads) * sizeof(float);
  SAT_CHECK_ARG(shm <= 64 * 1024, "sat_decode_attention_step: history too long");
  hipStream_t s = as_stream(stream);
  if (dh == 128)
    hipLaunchKernelGGL(decode_attention_kernel<128>, dim3(B * H), dim3(kDecAttnThreads), shm, s, qkv, qkv_sb,
                       qkv_st, H, D, t, scale, P, Tm, O, o_sb);
  else if (dh == 64)
    hipLaunchKernelGGL(decode_attention_kernel<64>, dim3(B * H), dim3(kDecAttnThreads), shm, s, qkv, qkv_sb,
                       qkv_st, H, D, t, scale, P, Tm, O, o_sb);
  else
    hipLaunchKernelGGL(decode_attention_kernel<32>, dim3(B * H), dim3(kDecAttnThreads), shm, s, qkv, qkv_sb,
                       qkv_st, H, D, t, scale, P, Tm, O, o_sb);
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
