// MultiHeadAttention of the self-attention blocks (modules/self_attention.py:108-128, with the
// ScaledDotProductAttentionMechanism of :45-65) as two C-ABI entries, sat_mha_fwd / sat_mha_bwd.
//
// Both are host-side schedules over the library's own kernels -- no new device code: the four
// projections and the per-(utterance, head) score / context products are sat_gemm launches
// (fp32 MFMA, heads addressed through the descriptor's two batch strides, so no head
// split/merge copies), the masked softmax and its gradient are sat_softmax_fwd/bwd, the bias
// gradients sat_colsum.  Launch-for-launch the same work the Python composition
// (model.mha_fwd / backward.mha_bwd) issued, reachable from C.
#include "sat_common.h"

namespace sat {
namespace {

constexpr int64_t kAlign = 256;
inline int64_t align_up(int64_t n) { return (n + kAlign - 1) / kAlign * kAlign; }

SatGemmDesc dense_desc() {
  SatGemmDesc g;
  std::memset(&g, 0, sizeof(g));
  g.batch = 1;
  g.batch2 = 1;
  g.alpha = 1.f;
  return g;
}

// C[R][N] (=| +=) X[R][K] @ W[K][N] + bias    (tf.layers.Dense over the last dim)
int dense(const float* X, const float* W, const float* bias, float* C, int R, int K, int N,
          float beta, const SatMha* d, hipStream_t s) {
  SatGemmDesc g = dense_desc();
  g.M = R; g.N = N; g.K = K;
  g.A = X; g.a_sm = K; g.a_sk = 1;
  g.B = W; g.b_sk = N; g.b_sn = 1;
  g.C = C; g.c_sm = N;
  g.bias = bias;
  g.beta = beta;
  g.ws = d->gemm_ws; g.ws_bytes = d->gemm_ws_bytes;
  return sat_gemm(&g, s);
}

// per (utterance b, head h) product on [B][L][D] activations viewed as [B][H][L][dh]:
// op(A)[L x K] @ op(B)[K x N]; strides given per operand as (row, col) inside one head block
struct HeadOp {
  const float* p;
  int64_t sr, sc;          // row / column stride inside one (b, h) block
  int64_t sb, sh;          // batch (utterance) and head strides
};

// tri: SatGemmDesc.tri when the attention is causal (triangular scores / probabilities)
int head_gemm(int M, int N, int K, HeadOp a, HeadOp b, float* C, int64_t c_sm, int64_t c_sb,
              int64_t c_sh, float alpha, const SatMha* d, hipStream_t s, int tri = 0) {
  SatGemmDesc g = dense_desc();
  g.M = M; g.N = N; g.K = K;
  g.tri = d->causal ? tri : 0;
  g.batch = d->B; g.batch2 = d->H;
  g.A = a.p; g.a_sm = a.sr; g.a_sk = a.sc; g.a_sbatch = a.sb; g.a_sbatch2 = a.sh;
  g.B = b.p; g.b_sk = b.sr; g.b_sn = b.sc; g.b_sbatch = b.sb; g.b_sbatch2 = b.sh;
  g.C = C; g.c_sm = c_sm; g.c_sbatch = c_sb; g.c_sbatch2 = c_sh;
  g.alpha = alpha;
  return sat_gemm(&g, s);
}

// the fused attention takes its two shapes when lse is given: the decoder head's (causal,
// dh = 128) and the encoder's narrow heads (dh <= 32, L <= 256; sat_flash_attn_fwd)
bool flash_ok(const SatMha* d) {
  const int dh = d->D / d->H;
  const bool wide = d->causal && dh == 128 && d->L % 4 == 0;
  const bool narrow = (dh == 8 || dh == 16 || dh == 32) && d->L <= 256 && d->D % 4 == 0 &&
                      (2LL * d->L * dh + 2LL * d->L) * 4 <= 65536;
  return d->lse && (wide || narrow) && aligned16(d->q) && aligned16(d->k) && aligned16(d->v) &&
         aligned16(d->o) && (!d->probs_mask || aligned16(d->probs_mask));
}

// scratch the descriptor's path needs: the fused path keeps only dO, dQ, dK, dV and the
// [B][H][L] row term delta (in the first score slab's place); the materialised path the two
// [B][H][L][L] score slabs as well
int64_t scratch_need(const SatMha* d) {
  return flash_ok(d) ? sat_mha_scratch_bytes_fused(d->B, d->L, d->D, d->H, d->out_dim)
                     : sat_mha_scratch_bytes(d->B, d->L, d->D, d->H, d->out_dim);
}

SatFlashAttn flash_desc(const SatMha* d) {
  SatFlashAttn fa;
  std::memset(&fa, 0, sizeof(fa));
  fa.B = d->B; fa.H = d->H; fa.L = d->L; fa.dh = d->D / d->H; fa.causal = d->causal ? 1 : 0;
  fa.scale = 1.f / std::sqrt((float)fa.dh);
  fa.ld = d->D;
  fa.q = d->q; fa.k = d->k; fa.v = d->v;
  fa.mask = d->probs_mask;
  fa.lse = d->lse;
  return fa;
}

int check(const SatMha* d, bool bwd) {
  SAT_CHECK_ARG(d != nullptr, "sat_mha: null descriptor");
  SAT_CHECK_ARG(d->B > 0 && d->L > 0 && d->W > 0 && d->D > 0 && d->H > 0 && d->D % d->H == 0 &&
                    d->out_dim > 0,
                "sat_mha: bad sizes (D must be a multiple of H)");
  SAT_CHECK_ARG(d->x && d->Wq && d->Wk && d->Wv && d->Wo && d->q && d->k && d->v &&
                    (d->P || flash_ok(d)) && d->o,
                "sat_mha: null tensor (P may be NULL only on the fused causal path)");
  SAT_CHECK_ARG(!d->probs_mask || d->Pd || flash_ok(d), "sat_mha: a probability mask needs Pd");
  if (bwd) {
    const bool all = d->dWq && d->dWk && d->dWv && d->dWo;
    const bool none = !d->dWq && !d->dWk && !d->dWv && !d->dWo;
    SAT_CHECK_ARG(d->dy && d->dx && (all || none),
                  "sat_mha_bwd: null gradient tensor (the four weight gradients: all or none)");
    SAT_CHECK_ARG(d->scratch && d->scratch_bytes >= scratch_need(d),
                  "sat_mha_bwd: scratch smaller than sat_mha_scratch_bytes() "
                  "(sat_mha_scratch_bytes_fused() on the fused path)");
  } else {
    SAT_CHECK_ARG(d->y && d->scratch && d->scratch_bytes >= scratch_need(d),
                  "sat_mha_fwd: needs y and scratch of sat_mha_scratch_bytes() "
                  "(sat_mha_scratch_bytes_fused() on the fused path)");
  }
  return SAT_OK;
}

#define SAT_TRY(expr)            \
  do {                           \
    const int rc_ = (expr);      \
    if (rc_ != SAT_OK) return rc_; \
  } while (0)

}  // namespace
}  // namespace sat

using namespace sat;

extern "C" int64_t sat_mha_scratch_bytes(int32_t B, int32_t L, int32_t D, int32_t H,
                                         int32_t out_dim) {
  const int64_t act = (int64_t)B * L * D * 4, score = (int64_t)B * H * L * L * 4;
  const int64_t cs = sat_workspace_colreduce(B * L, std::max(D, out_dim));
  // backward: dO, dQ, dK, dV [B L D], dPd, dS [B H L L], column-sum scratch; the forward uses
  // the first score slab for the raw scores
  return 4 * align_up(act) + 2 * align_up(score) + align_up(cs);
}

// the fused attention's (flash_ok) share of that: dO, dQ, dK, dV and delta [B][H][L] -- no
// O(L^2) slab in either direction
extern "C" int64_t sat_mha_scratch_bytes_fused(int32_t B, int32_t L, int32_t D, int32_t H,
                                               int32_t out_dim) {
  (void)out_dim;
  const int64_t act = (int64_t)B * L * D * 4, delta = (int64_t)B * H * L * 4;
  return 4 * align_up(act) + align_up(delta);
}

// y = Wo . concat_h(softmax(Q_h K_h^T / sqrt(dh)) [* mask] V_h) + bo,  Q/K/V = x W + b
extern "C" int sat_mha_fwd(const SatMha* d, void* stream) {
  SAT_TRY(check(d, false));
  hipStream_t s = as_stream(stream);
  const int B = d->B, L = d->L, D = d->D, H = d->H, dh = D / H, R = B * L;
  const int64_t LD = (int64_t)L * D, LL = (int64_t)L * L, HLL = H * LL;
  char* sc = static_cast<char*>(d->scratch) + 4 * align_up((int64_t)B * L * D * 4);
  float* S = reinterpret_cast<float*>(sc);
  // Q/K/V: ONE batched product when the three weights, biases and outputs are equally spaced
  // (the parameter arena stores query / key / value kernel + bias back to back; model.mha_fwd
  // allocates q, k, v as one [3][B][L][D] buffer) -- three times the tiles in one launch
  const int64_t sw = d->Wk - d->Wq, sb = d->bk - d->bq, so = d->k - d->q;
  if (d->bq && sw == d->Wv - d->Wk && sb == d->bv - d->bk && so == d->v - d->k) {
    SatGemmDesc g = dense_desc();
    g.M = R; g.N = D; g.K = d->W;
    g.batch = 3;
    g.A = d->x; g.a_sm = d->W; g.a_sk = 1; g.a_sbatch = 0;
    g.B = d->Wq; g.b_sk = D; g.b_sn = 1; g.b_sbatch = sw;
    g.C = d->q; g.c_sm = D; g.c_sbatch = so;
    g.bias = d->bq; g.bias_sbatch = sb;
    g.ws = d->gemm_ws; g.ws_bytes = d->gemm_ws_bytes;
    SAT_TRY(sat_gemm(&g, s));
  } else {
    SAT_TRY(dense(d->x, d->Wq, d->bq, d->q, R, d->W, D, 0.f, d, s));
    SAT_TRY(dense(d->x, d->Wk, d->bk, d->k, R, d->W, D, 0.f, d, s));
    SAT_TRY(dense(d->x, d->Wv, d->bv, d->v, R, d->W, D, 0.f, d, s));
  }
  if (flash_ok(d)) {
    // scores, causal softmax, dropout and contexts fused per (utterance, head); nothing
    // [L][L] is written (sat_flash_attn_fwd)
    SatFlashAttn fa = flash_desc(d);
    fa.o = d->o;
    SAT_TRY(sat_flash_attn_fwd(&fa, s));
    SAT_TRY(dense(d->o, d->Wo, d->bo, d->y, R, D, d->out_dim, 0.f, d, s));
    return SAT_OK;
  }
  // S[b,h] = Q_h K_h^T                                               (self_attention.py:55)
  // (causal: only the tiles on / below the diagonal; the softmax reads no further)
  SAT_TRY(head_gemm(L, L, dh, {d->q, D, 1, LD, dh}, {d->k, 1, D, LD, dh}, S, L, HLL, LL, 1.f, d,
                    s, 1));
  float* Pd = d->probs_mask ? d->Pd : d->P;
  SAT_TRY(sat_softmax_fwd(S, d->P, d->probs_mask ? d->Pd : nullptr, d->probs_mask,
                          (int64_t)B * H * L, L, L, d->causal, 1.f / std::sqrt((float)dh), s));
  // O[b, :, h] = Pd[b,h] V_h  (heads written in place of the [B][L][D] concat)
  // (causal: Pd is lower-triangular, each row tile's reduction stops at its last row)
  SAT_TRY(head_gemm(L, dh, L, {Pd, L, 1, HLL, LL}, {d->v, D, 1, LD, dh}, d->o, D, LD, dh, 1.f, d,
                    s, 2));
  SAT_TRY(dense(d->o, d->Wo, d->bo, d->y, R, D, d->out_dim, 0.f, d, s));
  return SAT_OK;
}

namespace sat {
namespace {
// the backward's scratch: dO, dQ, dK, dV [B L D], then dPd, dS [B H L L] (score slabs)
struct MhaBwdScratch {
  float *dO, *dQ, *dK, *dV, *dPd, *dS;
};
MhaBwdScratch bwd_scratch(const SatMha* d) {
  char* p = static_cast<char*>(d->scratch);
  const int64_t act = align_up((int64_t)d->B * d->L * d->D * 4);
  const int64_t score = align_up((int64_t)d->H * d->L * d->L * d->B * 4);
  return {reinterpret_cast<float*>(p), reinterpret_cast<float*>(p + act),
          reinterpret_cast<float*>(p + 2 * act), reinterpret_cast<float*>(p + 3 * act),
          reinterpret_cast<float*>(p + 4 * act), reinterpret_cast<float*>(p + 4 * act + score)};
}
// dW += X^T dY with db += colsum(dY) in the same launch
int mha_wgrad(const SatMha* d, const float* X, int K, const float* dY, int N, float* dW, float* db,
              hipStream_t s) {
  SatGemmDesc g = dense_desc();
  g.M = K; g.N = N; g.K = d->B * d->L;
  g.A = X; g.a_sm = 1; g.a_sk = K;
  g.B = dY; g.b_sk = N; g.b_sn = 1;
  g.C = dW; g.c_sm = N; g.beta = 1.f;
  g.ws = d->gemm_ws; g.ws_bytes = d->gemm_ws_bytes;
  g.colsum_out = db;
  return sat_gemm(&g, s);
}
// the three input projections' dW += x^T dQ|dK|dV, db += colsum: ONE batched product (A = x
// shared, batch stride 0; split-K over the three batches' slabs) when the gradients, their
// biases and dQ / dK / dV are equally spaced (the gradient arena mirrors the parameter arena:
// query / key / value kernel + bias back to back; dQ, dK, dV are consecutive scratch slabs)
int mha_wgrad_qkv(const SatMha* d, const float* dQ, const float* dK, const float* dV,
                  hipStream_t s) {
  const int64_t sw = d->dWk - d->dWq, so = dK - dQ;
  const bool nob = !d->dbq && !d->dbk && !d->dbv;
  const bool eqb = d->dbq && d->dbk && d->dbv && d->dbk - d->dbq == d->dbv - d->dbk;
  if (sw == d->dWv - d->dWk && so == dV - dK && (nob || eqb)) {
    SatGemmDesc g = dense_desc();
    g.M = d->W; g.N = d->D; g.K = d->B * d->L;
    g.batch = 3;
    g.A = d->x; g.a_sm = 1; g.a_sk = d->W; g.a_sbatch = 0;
    g.B = dQ; g.b_sk = d->D; g.b_sn = 1; g.b_sbatch = so;
    g.C = d->dWq; g.c_sm = d->D; g.c_sbatch = sw; g.beta = 1.f;
    g.colsum_out = d->dbq;
    g.bias_sbatch = eqb ? d->dbk - d->dbq : 0;   // the batches' column sums, bias_sbatch apart
    g.ws = d->gemm_ws; g.ws_bytes = d->gemm_ws_bytes;
    return sat_gemm(&g, s);
  }
  SAT_TRY(mha_wgrad(d, d->x, d->W, dQ, d->D, d->dWq, d->dbq, s));
  SAT_TRY(mha_wgrad(d, d->x, d->W, dK, d->D, d->dWk, d->dbk, s));
  return mha_wgrad(d, d->x, d->W, dV, d->D, d->dWv, d->dbv, s);
}
}  // namespace
}  // namespace sat

// The four projections' weight / bias gradients (ACCUMULATE) from the dO, dQ, dK, dV a
// weight-deferred sat_mha_bwd left in the scratch.
extern "C" int sat_mha_bwd_wgrad(const SatMha* d, void* stream) {
  SAT_TRY(check(d, true));
  SAT_CHECK_ARG(d->dWq && d->dWk && d->dWv && d->dWo, "sat_mha_bwd_wgrad: null weight gradient");
  hipStream_t s = as_stream(stream);
  const MhaBwdScratch sc = bwd_scratch(d);
  SAT_TRY(mha_wgrad(d, d->o, d->D, d->dy, d->out_dim, d->dWo, d->dbo, s));
  return mha_wgrad_qkv(d, sc.dQ, sc.dK, sc.dV, s);
}

// Gradients of sat_mha_fwd: parameter gradients ACCUMULATE (+=), dx is written.  With all four
// weight gradients NULL the weight / bias gradients are deferred to sat_mha_bwd_wgrad (same
// descriptor and scratch, e.g. on a stream of the caller's that runs beside the dx chain).
extern "C" int sat_mha_bwd(const SatMha* d, void* stream) {
  SAT_TRY(check(d, true));
  hipStream_t s = as_stream(stream);
  const int B = d->B, L = d->L, D = d->D, H = d->H, dh = D / H, R = B * L, Wi = d->W;
  const int64_t LD = (int64_t)L * D, LL = (int64_t)L * L, HLL = H * LL;
  const MhaBwdScratch sc = bwd_scratch(d);
  float* dO = sc.dO;
  float* dQ = sc.dQ;
  float* dK = sc.dK;
  float* dV = sc.dV;
  float* dPd = sc.dPd;
  float* dS = sc.dS;
  const float* Pd = d->probs_mask ? d->Pd : d->P;
  const bool wg = d->dWq != nullptr;    // weight gradients here (else deferred)
  auto dgrad = [&](const float* dY, int N, const float* W, int K, float* dX, float beta) {
    SatGemmDesc g = dense_desc();   // dX (=|+=) dY W^T
    g.M = R; g.N = K; g.K = N;
    g.A = dY; g.a_sm = N; g.a_sk = 1;
    g.B = W; g.b_sk = 1; g.b_sn = N;
    g.C = dX; g.c_sm = K; g.beta = beta;
    g.ws = d->gemm_ws; g.ws_bytes = d->gemm_ws_bytes;
    return sat_gemm(&g, s);
  };
  // output projection
  if (wg) SAT_TRY(mha_wgrad(d, d->o, D, d->dy, d->out_dim, d->dWo, d->dbo, s));
  SAT_TRY(dgrad(d->dy, d->out_dim, d->Wo, D, dO, 0.f));
  if (flash_ok(d)) {
    // dQ, dK, dV of the fused causal attention, probabilities recomputed from lse
    // (sat_flash_attn_bwd; delta in the unused score slab)
    SatFlashAttn fa = flash_desc(d);
    fa.o = d->o;
    fa.dout = dO;
    fa.delta = dPd;
    fa.dq = dQ; fa.dk = dK; fa.dv = dV;
    SAT_TRY(sat_flash_attn_bwd(&fa, s));
  } else {
  // dPd = dO_h V_h^T ;  dV_h = Pd^T dO_h
  // (causal: dPd only on / below the diagonal; Pd^T upper-triangular)
  SAT_TRY(head_gemm(L, L, dh, {dO, D, 1, LD, dh}, {d->v, 1, D, LD, dh}, dPd, L, HLL, LL, 1.f, d,
                    s, 1));
  SAT_TRY(head_gemm(L, dh, L, {Pd, 1, L, HLL, LL}, {dO, D, 1, LD, dh}, dV, D, LD, dh, 1.f, d, s,
                    3));
  SAT_TRY(sat_softmax_bwd(d->P, dPd, d->probs_mask, dS, (int64_t)B * H * L, L, L, d->causal,
                          1.f / std::sqrt((float)dh), s));
  // dQ_h = dS K_h ;  dK_h = dS^T Q_h
  SAT_TRY(head_gemm(L, dh, L, {dS, L, 1, HLL, LL}, {d->k, D, 1, LD, dh}, dQ, D, LD, dh, 1.f, d,
                    s, 2));
  SAT_TRY(head_gemm(L, dh, L, {dS, 1, L, HLL, LL}, {d->q, D, 1, LD, dh}, dK, D, LD, dh, 1.f, d,
                    s, 3));
  }
  // input projections
  if (wg) SAT_TRY(mha_wgrad_qkv(d, dQ, dK, dV, s));
  if (D % 32 == 0 && aligned16(d->Wq) && aligned16(d->Wk) && aligned16(dQ) && aligned16(dK)) {
    // dx = dQ Wq^T + dK Wk^T as ONE reduction (two-segment operands), then += dV Wv^T
    SatGemmDesc g = dense_desc();
    g.M = R; g.N = Wi; g.K = 2 * D;
    g.A = dQ; g.a_sm = D; g.a_sk = 1;
    g.A2 = dK; g.a2_sm = D; g.k1 = D;
    g.B = d->Wq; g.b_sk = 1; g.b_sn = D;
    g.B2 = d->Wk; g.b2_s = D;
    g.C = d->dx; g.c_sm = Wi; g.beta = 0.f;
    g.ws = d->gemm_ws; g.ws_bytes = d->gemm_ws_bytes;
    SAT_TRY(sat_gemm(&g, s));
  } else {
    SAT_TRY(dgrad(dQ, D, d->Wq, Wi, d->dx, 0.f));
    SAT_TRY(dgrad(dK, D, d->Wk, Wi, d->dx, 1.f));
  }
  SAT_TRY(dgrad(dV, D, d->Wv, Wi, d->dx, 1.f));
  return SAT_OK;
}
