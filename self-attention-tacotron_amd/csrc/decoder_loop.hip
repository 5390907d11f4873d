// The teacher-forced decoder loop as ONE C entry each way (sat_decoder_loop_fwd /
// sat_decoder_loop_bwd), plus SURVEY.md's names for one ZoneoutLSTM step.
//
// DecoderRNNV2 = MultiRNNCell([DualSourceAttentionRNN, ZoneoutLSTM(256), ZoneoutLSTM(256)])
// (ext tacotron2, built at modules/module.py:1531-1540) under TransformerTrainingHelper
// (modules/helpers.py:13-58).  Teacher forcing makes the dependency one-way: the attention chain
// never reads the LSTM stack, so the loop is the attention chain's persistent launch, LSTM1's
// input projection for all steps (one two-segment GEMM), then the LSTM stack's persistent launch -- the
// sequence decoder.py decoder_forward issues, here behind one call so a C caller does not
// re-implement it.  The backward mirrors backward.py decoder_bwd's persistent path.
#include "sat_common.h"

namespace {

// C[M][N] (row stride ldc) = alpha A B + beta C (+ bias), plain dense operands
int dense(int M, int N, int K, const float* A, int64_t a_sm, int64_t a_sk, const float* B,
          int64_t b_sk, int64_t b_sn, float* C, int64_t c_sm, const float* bias, float beta,
          void* ws, int64_t ws_bytes, void* stream) {
  SatGemmDesc d;
  std::memset(&d, 0, sizeof(d));
  d.M = M; d.N = N; d.K = K; d.batch = 1; d.batch2 = 1;
  d.A = A; d.a_sm = a_sm; d.a_sk = a_sk;
  d.B = B; d.b_sk = b_sk; d.b_sn = b_sn;
  d.C = C; d.c_sm = c_sm;
  d.bias = bias;
  d.alpha = 1.f; d.beta = beta;
  d.ws = ws; d.ws_bytes = ws_bytes;
  return sat_gemm(&d, stream);
}

}  // namespace

using namespace sat;

extern "C" int sat_zlstm_step_fwd(const SatLstmFwd* a, void* stream) {
  return sat_lstm_step_fwd(a, stream);
}
extern "C" int sat_zlstm_step_bwd(const SatLstmBwd* a, void* stream) {
  return sat_lstm_step_bwd(a, stream);
}

extern "C" int sat_decoder_loop_fwd(const SatDecoderLoopFwd* a, void* stream) {
  SAT_CHECK_ARG(a && a->W1x && a->b1 && a->lstm.X1, "sat_decoder_loop_fwd: null argument");
  const SatDecAttnFwd& at = a->attn;
  const SatDecLstmFwd& ls = a->lstm;
  SAT_CHECK_ARG(at.B == ls.B && at.T == ls.T && ls.U > 0 && at.REC0 && at.H0RAW,
                "sat_decoder_loop_fwd: attention chain (B=%d, T=%d) and LSTM stack (B=%d, T=%d) "
                "disagree", at.B, at.T, ls.B, ls.T);
  int rc = sat_decoder_attention_fwd(&at, stream);
  if (rc != SAT_OK) return rc;
  const int U = at.U, R0 = at.M1 + at.M2 + at.U, G = 4 * ls.U, MB = at.T * at.B;
  float* X1 = const_cast<float*>(ls.X1);
  // X1 = [h0'_t | c1_t | c2_t] W1x + b1 as ONE reduction: the attention RNN's raw output and the
  // contexts (REC0 row t+1 holds step t's) are the two A segments (SatGemmDesc.A2)
  {
    SatGemmDesc d;
    std::memset(&d, 0, sizeof(d));
    d.M = MB; d.N = G; d.K = U + at.M1 + at.M2; d.batch = 1; d.batch2 = 1;
    d.A = at.H0RAW; d.a_sm = U; d.a_sk = 1;
    d.A2 = at.REC0 + (int64_t)at.B * R0; d.a2_sm = R0; d.k1 = U;
    d.B = a->W1x; d.b_sk = G; d.b_sn = 1;
    d.C = X1; d.c_sm = G;
    d.bias = a->b1;
    d.alpha = 1.f; d.beta = 0.f;
    d.ws = a->ws; d.ws_bytes = a->ws_bytes;
    rc = sat_gemm(&d, stream);
    if (rc != SAT_OK) return rc;
  }
  return sat_decoder_lstms_fwd(&ls, stream);
}

extern "C" int sat_decoder_loop_bwd(const SatDecoderLoopBwd* a, void* stream) {
  SAT_CHECK_ARG(a && a->W1x && a->DH0, "sat_decoder_loop_bwd: null argument");
  const SatDecLstmBwd& ls = a->lstm;
  const SatDecAttnBwd& at = a->attn;
  SAT_CHECK_ARG(at.B == ls.B && at.T == ls.T && at.DH0 == a->DH0 && at.RD && ls.DG1,
                "sat_decoder_loop_bwd: attention chain and LSTM stack disagree (B, T, DH0)");
  const int U = at.U, R0 = at.M1 + at.M2 + at.U, G = 4 * ls.U, MB = at.T * at.B;
  hipStream_t s = as_stream(stream);
  if (zero_dwords(at.RD, (int64_t)MB * R0, s) != hipSuccess) {
    set_error("sat_decoder_loop_bwd: RD clear failed");
    return SAT_ERR_HIP;
  }
  int rc = sat_decoder_lstms_bwd(&ls, stream);
  if (rc != SAT_OK) return rc;
  // dL/dh0'_t = DG1_t W1x[0:U]^T ;  dL/dctx_t = DG1_t W1x[U:U+M1+M2]^T  (into RD's ctx half):
  // the two output blocks of ONE product (SatGemmDesc.C2) when U is a whole number of tiles
  if (U % 128 == 0) {
    SatGemmDesc d;
    std::memset(&d, 0, sizeof(d));
    d.M = MB; d.N = R0; d.K = G; d.batch = 1; d.batch2 = 1;
    d.A = ls.DG1; d.a_sm = G; d.a_sk = 1;
    d.B = a->W1x; d.b_sk = 1; d.b_sn = G;
    d.C = a->DH0; d.c_sm = U;
    d.C2 = at.RD; d.c2_sm = R0; d.n1 = U;
    d.alpha = 1.f; d.beta = 0.f;
    d.ws = a->ws; d.ws_bytes = a->ws_bytes;
    rc = sat_gemm(&d, stream);
    if (rc != SAT_OK) return rc;
  } else {
    rc = dense(MB, U, G, ls.DG1, G, 1, a->W1x, 1, G, a->DH0, U, nullptr, 0.f, a->ws, a->ws_bytes,
               stream);
    if (rc != SAT_OK) return rc;
    rc = dense(MB, at.M1 + at.M2, G, ls.DG1, G, 1, a->W1x + (int64_t)U * G, 1, G, at.RD, R0,
               nullptr, 0.f, a->ws, a->ws_bytes, stream);
    if (rc != SAT_OK) return rc;
  }
  return sat_decoder_attention_bwd(&at, stream);
}
