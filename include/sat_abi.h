/*
 * libsat_hip -- C ABI of the MI355X-native Self-attention Tacotron hot path.
 *
 * The reference (rhoposit/self-attention-tacotron) is Python/TF1 with no FFI of its own; its
 * plugin surface for this path is Python:
 *   attention_mechanism_factory(AttentionOptions) -> mechanism(query, state)
 *       modules/attentions.py:25-62, modules/forward_attention.py:88-136
 *   ZoneoutLSTMCell / DecoderRNNV2 / DualSourceAttentionRNN step
 *       modules/module.py:1017-1048, 1522-1540 (ext tacotron2)
 *   RNNTransformer training branch (dynamic_decode + causal self-attention + projections)
 *       modules/module.py:726-765, modules/self_attention.py:13-144
 *   ZoneoutCBHG / SelfAttentionCBHGEncoder  modules/module.py:30-113, 374-441
 * Each entry point below replaces the TF ops of one of those functions; the Python host side
 * (package sat_amd) binds this header with ctypes and mirrors the Python surface.
 *
 * Conventions
 *  - fp32 row-major contiguous tensors unless a stride argument says otherwise; batch-major.
 *  - Every pointer is caller-owned DEVICE memory.  Nothing here allocates or synchronises, so
 *    every call can be captured into a hipGraph.  `stream` is a hipStream_t passed as void*.
 *  - Return 0 on success, a negative SAT_ERR_* code otherwise; sat_last_error_string() gives
 *    the message (thread-local).  No global mutable state: calls are re-entrant across
 *    streams and devices.
 */
#ifndef SAT_ABI_H
#define SAT_ABI_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SAT_OK 0
#define SAT_ERR_ARGUMENT -1
#define SAT_ERR_HIP -2
#define SAT_ERR_UNSUPPORTED -3

/* Layout version of every struct / signature below: bumped whenever one changes, so a binding
 * (or an A/B run loading an older build through SAT_LIB_OVERRIDE) can refuse a library whose
 * structs it would misread.  5: round-5 layout (SatAttnParamGrad without zh, sat_softmax_bwd
 * with Lq / causal, SatMha.lse); 6: SatMha.wgrad_stream / wgrad_ws; 7: SatAttnParamGrad.tsplit; 8: SatMha without
 * wgrad_stream / wgrad_ws (deferred weight gradients: sat_mha_bwd_wgrad). */
#define SAT_ABI_VERSION 8

/* ---------------------------------------------------------------- library */
int sat_version(void);                         /* 100*major + minor */
int sat_abi_version(void);                     /* SAT_ABI_VERSION the library was built with */
const char* sat_last_error_string(void);
int sat_device_arch(char* buf, int len);       /* gcnArchName of the current device */

/* ---------------------------------------------------------------- GEMM (fp32 MFMA 32x32x2)
 * C[b] = act(alpha * opA[b] @ opB[b] + beta * C[b] + bias[b])      (M x N, reduction K)
 * Replaces tf.layers.Dense / tf.tensordot (Projection, modules/module.py:626-643), the
 * Conv1D(SAME) of ext tacotron2 Conv1d (module.py:46-68) and their gradients.
 * A modes: 0 dense  A(m,k) = A[m*a_sm + k*a_sk]
 *          1 im2col A(m,k): m = s*L + n, k = tap*a_C + c, row = n + tap - a_shift,
 *                   A = A[(s*L+row)*a_sm + c*a_sk] if 0 <= row < L else 0   (Conv1D SAME)
 *          2 im2col-transposed A(i,k) = im2col(m=k, kk=i) with the mode-1 addressing
 *                   (conv dW = im2col(x)^T @ dY in one product)
 * B modes: 0 dense  B(k,n) = B[k*b_sk + n*b_sn]
 *          1 flipped conv kernel W[taps][N][b_C]: k = tap*b_C + o,
 *                   B = W[((taps-1-tap)*N + n)*b_C + o]                     (conv dX)
 * act: 0 none, 1 relu, 2 tanh, 3 sigmoid, 4 softsign.  bias may be NULL.
 * mul (optional, [M][N] row stride mul_sm): C = act(...) * mul  (fused dropout masks).
 * add (optional, row stride add_sm, 0 = broadcast one row): C = act(...) * mul + add
 *     (fused residual connections, e.g. SelfAttentionTransformer x + tanh(Dense(.))).
 * Batching: blockIdx.z = z1 * batch2 + z2 (batch = z1 count, batch2 >= 1 inner count); every
 * operand is offset by z1 * s?batch + z2 * s?batch2 (e.g. z1 = utterance, z2 = head).
 * ws/ws_bytes (optional caller scratch): enables deterministic split-K for products with few
 * output tiles and a long reduction (weight gradients); NULL disables it.
 */
typedef struct SatGemmDesc {
  int32_t M, N, K, batch;
  int32_t a_mode, a_L, a_C, a_shift;
  const float* A;
  int64_t a_sm, a_sk, a_sbatch;
  int32_t b_mode, b_taps, b_C, act;
  const float* B;
  int64_t b_sk, b_sn, b_sbatch;
  float* C;
  int64_t c_sm, c_sbatch;
  const float* bias;
  int64_t bias_sbatch;
  float alpha, beta;
  const float* mul;
  int64_t mul_sm, mul_sbatch;
  /* tri (a hint; 0 = off): the causal self-attention's triangular structure, per batch matrix
   * (row m = query position, column / reduction index = key position):
   *   1: only the lower triangle of C is needed (column n <= row m): output tiles wholly above
   *      the diagonal are skipped (C there is left unwritten);
   *   2: A is lower-triangular (A[m][k] == 0 for k > m): each tile's reduction stops at its
   *      last row;  3: A is upper-triangular (A[m][k] == 0 for k < m): it starts at its first.
   * The skipped terms are exact zeros, so 2 / 3 give the same bits as the full product.
   * Honoured by the LDS kernel; every other path computes the full product (also correct). */
  int32_t batch2, tri;
  int64_t a_sbatch2, b_sbatch2, c_sbatch2, mul_sbatch2;
  const float* add;
  int64_t add_sm, add_sbatch;
  void* ws;
  int64_t ws_bytes;
  /* optional: also colsum_out[n] = alpha * sum_k B[k][n] + beta * colsum_out[n] in the same
   * launch (the bias gradient of a weight-gradient product dW = X^T dY, db = 1^T dY); needs a
   * product without bias / act / mul / add and batch2 == 1; with batch > 1, batch b's sums go
   * to colsum_out + b * bias_sbatch (bias_sbatch is otherwise unused here; 0: batch 0's sums
   * only -- the batches of a shared B, b_sbatch == 0, have the same sums).  NULL = off. */
  float* colsum_out;
  /* optional second A segment: A's columns k >= k1 come from A2 (row stride a2_sm), i.e.
   * C = A[:, :k1] B[:k1] + A2 B[k1:] as ONE reduction (two inputs of one layer that live in
   * different buffers); dense product with K-contiguous A, k1 % 32 == 0, 16-byte aligned rows,
   * no colsum_out; a batched product offsets A2 by A's batch strides.  NULL = off. */
  const float* A2;
  int64_t a2_sm;
  int32_t k1, pad1;
  /* optional second output: columns n >= n1 of the product go to C2[m][n - n1] (row stride
   * c2_sm), i.e. two outputs of one A over the column blocks of one B (bias, when given, is
   * indexed by n); batch-1, no colsum_out / mul / add, n1 % 128 == 0.  NULL = off. */
  float* C2;
  int64_t c2_sm;
  int32_t n1, pad2;
  /* optional second B segment: B's rows k >= k1 come from B2 (B's layout, stride b2_s along its
   * non-contiguous dimension), i.e. C = A[:, :k1] B + A[:, k1:] B2 -- with A2 set too, A B + A2 B2:
   * a sum of two products of different operands as ONE reduction.  Same constraints as A2 (B2
   * offset by B's batch strides).  NULL = off.
   * A2 / B2 outside those constraints (k1 % 32 != 0, SAT_GEMM_LDS=0, operands not vector-
   * loadable): two accumulating launches instead (C = A[:, :k1] B[:k1] + beta C + bias + add,
   * then C += the k >= k1 part), which needs a linear epilogue (no act / mul / C2). */
  const float* B2;
  int64_t b2_s;
} SatGemmDesc;

int sat_gemm(const SatGemmDesc* desc, void* stream);
/* ---------------------------------------------------------------- step workspace
 * Bytes of caller-owned device scratch one teacher-forced training step uses besides the
 * parameter / gradient arenas and the activations: the sum of every entry's scratch query
 * (persistent decoder kernels fwd + BPTT, column reductions over the widest bias/BN span,
 * loss, Adam, both self-attention sites) plus the GEMM split-K budget, each 256-B aligned. */
typedef struct SatDims {
  int32_t B, N, Tp;               /* utterances, encoder positions, decoder steps (T / r) */
  int32_t enc_heads, dec_heads;   /* self-attention heads: encoder, decoder head */
  int32_t enc_D, dec_D;           /* self-attention model widths */
  int32_t max_cols;               /* widest column reduction (the 2048-channel conv bank) */
} SatDims;
int64_t sat_workspace_size(const SatDims* d);

/* ---------------------------------------------------------------- multi-head self-attention
 * MultiHeadAttention.call (modules/self_attention.py:108-128) with the
 * ScaledDotProductAttentionMechanism (:45-65): Q/K/V = x W + b ([B][L][W] -> [B][L][D]), per
 * (utterance, head) P = softmax(Q_h K_h^T / sqrt(D/H)) [causal: use_subsequent_mask],
 * Pd = P * probs_mask (dropout on the probabilities; NULL = none, then Pd may be NULL),
 * o = concat_h(Pd V_h), y = o Wo + bo ([B][L][out_dim]).  Used by the encoder's
 * SelfAttentionTransformer (module.py:363-371, 425-438) and the decoder head (:743-765).
 * fwd writes q, k, v, P, Pd, o (kept for the backward) and y.
 * bwd reads those plus dy, writes dx and ACCUMULATES dWq..dbo (bias gradients may be NULL).
 * scratch: sat_mha_scratch_bytes(B, L, D, H, out_dim) bytes of device memory (both
 * directions); gemm_ws: split-K scratch for the projections' weight gradients (may be NULL). */
typedef struct SatMha {
  int32_t B, L, W, D, H, causal;
  int32_t out_dim, pad0;
  const float* x;
  const float* Wq;
  const float* bq;
  const float* Wk;
  const float* bk;
  const float* Wv;
  const float* bv;
  const float* Wo;
  const float* bo;
  const float* probs_mask;
  float* q;
  float* k;
  float* v;
  float* P;
  float* Pd;
  float* o;
  float* y;
  const float* dy;
  float* dx;
  float* dWq;
  float* dbq;
  float* dWk;
  float* dbk;
  float* dWv;
  float* dbv;
  float* dWo;
  float* dbo;
  void* scratch;
  int64_t scratch_bytes;
  void* gemm_ws;
  int64_t gemm_ws_bytes;
  /* lse [B][H][L] (nullable): selects the fused attention (sat_flash_attn_fwd/bwd) for the
   * score / softmax / context stage on its two shapes -- causal with D / H == 128 and
   * L % 4 == 0 (the decoder head), or D / H in {8, 16, 32} with L <= 256, causal or not (the
   * encoder's self-attention).  The forward then writes lse instead of P / Pd (both may be
   * NULL, nothing [L][L] is materialised) and the backward recomputes the probabilities. */
  float* lse;
} SatMha;
int64_t sat_mha_scratch_bytes(int32_t B, int32_t L, int32_t D, int32_t H, int32_t out_dim);
/* the same for a descriptor that takes the fused attention (sat_flash_attn_*: lse set, the
 * head shapes of sat_flash_attn_fwd, 16-byte-aligned q / k / v / o / probs_mask): dO, dQ, dK,
 * dV [B][L][D] and the row term [B][H][L], no [B][H][L][L] slab */
int64_t sat_mha_scratch_bytes_fused(int32_t B, int32_t L, int32_t D, int32_t H, int32_t out_dim);
int sat_mha_fwd(const SatMha* d, void* stream);
/* dWq / dWk / dWv / dWo all NULL: the weight and bias gradients are deferred -- sat_mha_bwd
 * writes dx only and leaves dO, dQ, dK, dV in the scratch; sat_mha_bwd_wgrad (same descriptor
 * with the gradient pointers, same scratch, after sat_mha_bwd on any stream ordered after it)
 * accumulates them.  Nothing downstream of the input gradient reads them, so a caller can run
 * them beside the dx chain. */
int sat_mha_bwd(const SatMha* d, void* stream);
int sat_mha_bwd_wgrad(const SatMha* d, void* stream);

/* Fused scaled-dot-product attention (flash-style; ScaledDotProductAttentionMechanism,
 * modules/self_attention.py:45-65): per (utterance b, head h)
 * O_h = (softmax(Q_h K_h^T * scale [+ causal mask]) * mask_h) V_h without materialising the
 * [L][L] scores.  q, k, v, o, dout, dq, dk, dv are [B][L][ld] with head h in columns
 * [h*dh, h*dh+dh); mask [B][H][L][L] (dropout values, NULL = none); lse [B][H][L] the
 * log2-domain row statistic the forward writes and the backward reads; delta [B][H][L]
 * backward scratch (dh = 128 only).  Two shapes:
 *   dh = 128, causal = 1, L % 4 == 0 -- the decoder head (use_subsequent_mask=True,
 *     modules/module.py:743-765), MFMA tiles streaming the other operand through LDS;
 *   dh in {8, 16, 32}, causal 0 or 1, L <= 256, (2 L dh + 2 L) * 4 <= 64 KB -- the encoder's
 *     self-attention (modules/module.py:425-438), one (utterance, head) per workgroup's LDS.
 * 16-byte aligned operands, ld % 4 == 0.  scale <= 0 means 1/sqrt(dh).  bwd WRITES dq, dk, dv. */
typedef struct SatFlashAttn {
  int32_t B, H, L, dh, causal;
  float scale;
  int64_t ld;
  const float* q; const float* k; const float* v;
  const float* mask;
  float* o; float* lse;
  const float* dout; float* delta;
  float* dq; float* dk; float* dv;
} SatFlashAttn;
int sat_flash_attn_fwd(const SatFlashAttn* a, void* stream);
int sat_flash_attn_bwd(const SatFlashAttn* a, void* stream);

/* ---------------------------------------------------------------- CBHG conv bank
 * The K1..Kmax Conv1D(SAME) bank of ZoneoutCBHG (modules/module.py:77-80 over ext tacotron2
 * Conv1d, module.py:46-52): max_k convolutions of one input, outputs concatenated on channels.
 * W holds K1..Kmax back to back, Kk = [k][C][Co] at float offset Co*C*k(k-1)/2 (the parameter
 * arena order of params.py); bias [max_k*Co] may be NULL.  x rows [S*L][C] (stride x_sm).
 * fwd: y[:, (k-1)Co : kCo] = x (*) Kk + b_k for every k -- ONE launch over the output column
 *      blocks (longest reductions dispatched first).
 * bwd: dX = beta_dx*dX + sum_k conv_dx_k(dY[:, (k-1)Co : kCo]) -- ONE product over all
 *      (k, tap, channel) reduction indices; dW_k = beta_dw*dW_k + im2col(x)^T dY_k for every k
 *      -- ONE product over all (k, tap, c) rows.  y is dY here; dx or dW may be NULL.
 *      ws/ws_bytes: split-K scratch (NULL: no split).  Bias and BatchNorm gradients are column
 *      sums (sat_colsum / sat_bn_bwd).
 * Needs C % 64 == 0, Co % 64 == 0, 16-byte aligned rows.  Replaces the 3 x max_k per-conv
 * launches of the same products (sat_gemm a_mode 1 / 2, b_mode 1). */
typedef struct SatConvBank {
  int32_t S, L, C, max_k, Co, pad0;
  const float* x;
  int64_t x_sm;
  const float* W;
  const float* bias;
  float* y;
  int64_t y_sm;
  float* dx;
  int64_t dx_sm;
  float* dW;
  float beta_dx, beta_dw;
  void* ws;
  int64_t ws_bytes;
} SatConvBank;
int sat_cbhg_convbank_fwd(const SatConvBank* d, void* stream);
int sat_cbhg_convbank_bwd(const SatConvBank* d, void* stream);

/* Tuning hook (probes): force the tile (64/128 x 64/128) and split-K factor of the calling
 * thread's subsequent sat_gemm launches on the LDS-staged kernel; bm = 0 restores the planner. */
int sat_gemm_force_plan(int32_t bm, int32_t bn, int32_t splits);
/* Speed-of-light probe (tools/probes/gemm_sol.py): mode bit 0 skips the LDS kernel's operand
 * DMA, bit 1 its epilogue stores (results are then garbage); 0 = normal.  Calling thread only. */
int sat_gemm_probe_mode(int32_t mode);
/* Skinny product C = alpha * A . Bt^T + beta * C, A [M][K], Bt [N][K] rows contiguous in K
 * (16-B aligned, K % 4 == 0): the per-step gradient of the attention contexts through the
 * attention RNN's input weights (M = batch). */
int sat_gemm_rowdot(int32_t M, int32_t N, int32_t K, const float* A, int64_t lda, const float* Bt,
                    int64_t ldb, float* C, int64_t ldc, float alpha, float beta, void* stream);

/* ---------------------------------------------------------------- RNG masks
 * Counter-based (Philox-4x32-10) Bernoulli masks: out[i] = (u_i < keep) ? on_value : 0.
 * The per-step seed is read from DEVICE memory (seed_ptr[0]) so a captured graph draws fresh
 * masks on every replay.  Replaces the dropout draws of tf.layers.dropout / tf.nn.dropout
 * (PreNet, ZoneoutLSTMCell, modules/self_attention.py:60). */
int sat_rng_fill(float* out, int64_t n, const uint64_t* seed_ptr, uint64_t stream_id,
                 float keep, float on_value, void* stream);
/* Several masks laid out back to back in one buffer (the training step's mask arena), ONE
 * launch: segment s covers out[offset, offset + n) and draws exactly what
 * sat_rng_fill(out + offset, n, seed_ptr, stream_id, keep, on_value) draws.  nseg <= 32. */
typedef struct SatRngSegment {
  int64_t offset, n;
  uint64_t stream_id;
  float keep, on_value;
} SatRngSegment;
int sat_rng_fill_segments(float* out, const SatRngSegment* segs, int32_t nseg,
                          const uint64_t* seed_ptr, void* stream);
int sat_counter_add(uint64_t* counter, uint64_t inc, void* stream);

/* Free-running decoding: the termination test of the tacotron2 StopTokenBasedInferenceHelper
 * (analog modules/helpers.py:154-158) after decoder step t -- finished iff t > min_iters and
 * sigmoid(stop[b * stride]) > 0.5 for every b; the first finished t is latched into state[0]
 * (the caller initialises it to -1). */
int sat_stop_check(const float* stop, int64_t stride, int32_t B, int32_t t, int32_t min_iters,
                   int32_t* state, void* stream);

/* One step of the decoder head's causal self-attention against its key/value cache during
 * free-running decoding (TransformerWrapper, modules/rnn_wrappers.py:87-124, with
 * ScaledDotProductAttentionMechanism, modules/self_attention.py:45-65; eval: no dropout):
 * per utterance b and head h, s_j = scale * q_t . k_j (j = 0..t), p = softmax(s),
 * o = sum_j p_j v_j.  qkv row (b, j) = qkv + b*qkv_sb + j*qkv_st holds [q (D) | k (D) | v (D)]
 * of step j (the caller's projection writes row t first); P (nullable) receives p at
 * ((b*H + h)*Tm + t)*Tm + j; O row b (stride o_sb) receives the heads concatenated. */
int sat_decode_attention_step(const float* qkv, int64_t qkv_sb, int64_t qkv_st, int32_t B,
                              int32_t H, int32_t D, int32_t t, float scale, float* P, int32_t Tm,
                              float* O, int64_t o_sb, void* stream);

/* Free-running decoding as ONE persistent launch (C5; the PREDICT branch of RNNTransformer,
 * modules/module.py:766-784, under StopTokenBasedInferenceHelper, analog
 * modules/helpers.py:111-160): every decoder step -- prenets on the fed frame, attention RNN,
 * forward + additive attention, the two ZoneoutLSTMs, the KV-cached causal self-attention head,
 * the mel / stop projections and the stop test -- inside one launch of 256 workgroups (one
 * utterance per 32 workgroups).  Replaces the per-step launch sequence of
 * sat_lstm_step_fwd / sat_attn_step_fwd / sat_gemm / sat_decode_attention_step / sat_stop_check.
 * Shapes: the LJSpeech decoder (prenet 256/128, attention RNN 256, memories 256 + 32, attention
 * 224 + 32 with 5 x 10 location filters, LSTMs 256, self-attention 256 x 2 heads, 80 mels x r=2,
 * one fed frame), B <= 8, N <= 256, T <= 512.  Weights are packed by the caller
 * (inference.py FreeRunningDecoder._pack_persistent):
 *   Wzp = W_out[:, 80:160] W_p0, bzp = b_out[80:160] W_p0 + b_p0   (the fed frame folded into
 *         the first prenet layer; bp0 alone feeds step 0's go frame);
 *   Wqku = [W_q | W_k | W_v,h W_o,h W_t (h = 0, 1)], bqku = [b_q | b_k | 0],
 *   bz = (b_v W_o + b_o) W_t + b_t   (value, output projection and transform folded into the
 *         cached rows: z = h2' + tanh(sum_h softmax_h . u_h + bz));
 *   Wq = [W_q1 | W_q2] (query layers), Wms = [W_out | w_stop | 0] (row stride 164).
 * Outputs: MS[t][b] = [mel | stop | pad], AL1[t+1][b][n] (alignments), S2[t][b][n] (second
 * attention), SA_P[b][h][t][j] (nullable, self-alignment rows); state[0] := first finished step
 * (stop_mode 1: t > min_iters and sigmoid(stop) > 0.5 for every utterance), left at the caller's
 * -1 otherwise.  scratch: sat_decode_persistent_scratch_bytes(), 16-byte aligned; err: one word,
 * cleared by the call, non-zero after a hand-off timeout. */
typedef struct SatDecodePersistent {
  int32_t B, N, T, min_iters, stop_mode;
  float zc, zh, u, scale;
  const int64_t* lengths;                                  /* [B] */
  const float* K1; const float* V1;                        /* [B][N][224], [B][N][256] */
  const float* K2; const float* V2;                        /* [B][N][32], [B][N][32] */
  const float* Wzp; const float* bzp; const float* bp0;    /* [256][256], [256], [256] */
  const float* Wp1; const float* bp1;                      /* [256][128], [128] */
  const float* W0; const float* b0;                        /* [672][256][4], [256][4] */
  const float* Wq;                                         /* [256][256] */
  const float* b1; const float* v1;                        /* [224] attention bias, v_a */
  const float* convW; const float* convb; const float* locW;   /* [10][5], [5], [5][224] */
  const float* v2;                                         /* [32] */
  const float* W1; const float* bl1;                       /* [800][256][4], [256][4] */
  const float* W2; const float* bl2;                       /* [512][256][4], [256][4] */
  const float* Wqku; const float* bqku; const float* bz;   /* [256][1024], [1024], [256] */
  const float* Wms; const float* bms;                      /* [256][164], [164] */
  float* MS; float* AL1; float* S2; float* SA_P;
  int32_t* state;
  void* scratch; int64_t scratch_bytes;
  int32_t* err;
  int64_t* prof;   /* nullable: per-workgroup phase clocks of the -DSAT_DP_TRACE build */
} SatDecodePersistent;
int64_t sat_decode_persistent_scratch_bytes(void);
int sat_decode_persistent(const SatDecodePersistent* a, void* stream);

/* ---------------------------------------------------------------- (Zoneout)LSTM step
 * One time step of TF LSTMCell wrapped in ext tacotron2 ZoneoutLSTMCell,
 * as used by ZoneoutCBHG's BiLSTM (modules/module.py:93-108) and DecoderRNNV2 /
 * DualSourceAttentionRNN (module.py:1522-1540).  The input projection x@W_x+b is hoisted
 * (xproj, one GEMM over all steps); the kernel computes the recurrent product rin@W_r, the
 * gates (i, j, f, o; forget_bias 1), zoneout and the sequence-length copy-through of
 * bidirectional_dynamic_rnn.  Weights and gates are gate-interleaved: [K][U][4].
 * Output h_raw = h' (the cell output); state (c_out, h_out) = zoned state.
 * Training: mask_c/mask_h (1 = take new) ; eval: NULL masks -> (1-z)*new + z*old. */
typedef struct SatLstmFwd {
  int32_t B, U, K, t;
  const float* xproj; int64_t xproj_sb;   /* [B][U][4] row stride xproj_sb (includes bias) */
  const float* bias;                      /* [U][4], used when xproj == NULL */
  const float* rin; int64_t rin_sb;       /* recurrent input [B][K] */
  const float* W;                         /* [K][U][4] */
  const float* c_prev;                    /* [B][U] (NULL = zeros) */
  const float* h_prev; int64_t h_prev_sb; /* [B][U] (NULL = zeros) */
  const float* mask_c; const float* mask_h;
  float zc, zh;
  const int64_t* lengths;                 /* optional: step t valid iff t < lengths[b] */
  float* h_raw; int64_t h_raw_sb;
  float* c_out;
  float* h_out; int64_t h_out_sb;
  float* gates;                           /* [B][U][4] activated gates for the backward */
  /* optional further input segments (0 = none): the recurrent input row is
   * [rin (K - K1 - K2) | rin1 (K1) | rin2 (K2)] against W's K rows in that order, so a layer
   * whose inputs live in separate buffers (e.g. DecoderRNNV2's LSTM1: [h0' | contexts | h1])
   * runs its whole product -- input projection included, with xproj = NULL and `bias` -- in
   * one step launch (free-running decode, inference.py). */
  const float* rin1; int64_t rin1_sb;
  const float* rin2; int64_t rin2_sb;
  int32_t K1, K2;
} SatLstmFwd;

/* Backward of one step (reverse time).  dL/dh_t = dh_carry + dgates_{t+1} . W[hoff+u, :]
 * (the recurrent product is done here unless the caller passes it precomputed in `rec`),
 * dL/dh'_t = dy + sum(dq_i . wq_i[u]) + m_h dL/dh_t. */
typedef struct SatLstmBwd {
  int32_t B, U, K, hoff, t;
  const float* W;
  const float* dgates_next;
  const float* gates;
  const float* c_prev;
  const float* dy; int64_t dy_sb;
  const float* dq0; const float* wq0; int32_t dq0_n;
  const float* dq1; const float* wq1; int32_t dq1_n;
  int32_t dq_parts; int64_t dq_pstride, dq_bstride;   /* dq rows: sum over dq_parts partials */
  const float* dh_carry;
  const float* dc_carry;
  const float* mask_c; const float* mask_h;
  float zc, zh;
  const int64_t* lengths;
  float* dgates;
  float* dh_carry_out;
  float* dc_carry_out;
  const float* rec; int64_t rec_sb;   /* optional [B][U]: the recurrent product
                                         dgates_next . W[hoff + u] precomputed by the caller
                                         (then dgates_next is not read) */
} SatLstmBwd;

int sat_lstm_step_fwd(const SatLstmFwd* args, void* stream);
/* 1..4 independent steps (e.g. the attention RNN at t, decoder LSTM1 at t-C, LSTM2 at t-2C) in
 * ONE launch over disjoint workgroup ranges: one kernel boundary instead of n. */
int sat_lstm_steps_fwd(const SatLstmFwd* steps, int32_t n, void* stream);
int sat_lstm_step_bwd(const SatLstmBwd* args, void* stream);
int sat_lstm_steps_bwd(const SatLstmBwd* steps, int32_t n, void* stream);

/* ---------------------------------------------------------------- dual-source attention step
 * Replaces, for one decoder step, the two attention mechanisms of DualSourceAttentionRNN
 * (modules/module.py:1520-1530) inside TF AttentionWrapper:
 *   mechanism 1: ForwardAttention.__call__ (modules/forward_attention.py:88-122) when
 *                att1_forward = 1, else BahdanauAttention (modules/attentions.py:53-57);
 *   mechanism 2: BahdanauAttention (additive, normalize=False);
 *   contexts   : AttentionWrapper._compute_attention (alignments @ values).
 * Keys/values are the masked memories precomputed once per utterance (memory_layer GEMM).
 * Launches the tile kernel (grid ntiles x B) and the per-utterance combine kernel.
 * Outputs: s_out (softmax alignments = next location-conv input), a_out (alpha = returned
 * alignments), s2_out, contexts [c1 | c2] into ctx (row stride ctx_sb), stats [B][4] for the
 * backward.  e1/e2/part are scratch. */
typedef struct SatAttnStep {
  int32_t B, N, D1, M1, D2, M2, F, KW, NT, ntiles, att1_forward;
  float u;                                  /* forward-attention transition factor (0.5) */
  const float* q; int64_t q_sb;             /* [B][D1 + D2] processed queries */
  const float* K1; const float* V1;         /* [B][N][D1], [B][N][M1] */
  const float* K2; const float* V2;         /* [B][N][D2], [B][N][M2] */
  const int64_t* lengths;                   /* [B] memory lengths */
  const float* s_prev; const float* a_prev; /* [B][N] previous state (att1) */
  const float* v1; const float* b1;         /* attention_variable, attention_bias [D1] */
  const float* convW; const float* convb;   /* location conv [KW][1][F], [F] */
  const float* locW;                        /* location layer [F][D1] */
  const float* v2;                          /* attention_v of mechanism 2 [D2] */
  float* e1; float* e2;                     /* scratch [B][N] */
  float* part; int64_t part_stride;         /* scratch [B][ntiles][part_stride] */
  float* s_out; float* a_out; float* s2_out;/* [B][N] */
  float* ctx; int64_t ctx_sb;               /* [B][M1 + M2] */
  float* stats;                             /* [B][4] or NULL */
  float* loc_out;                           /* [B][N][F] location features (bwd history) or NULL */
  int32_t lpp;                              /* lanes per memory position of the tile kernel:
                                               0 (= 16), 8, 16 or 32 */
  int32_t phases;                           /* 0 or 3: both kernels; 1: tile kernel only;
                                               2: combine only (profiling / split launches) */
} SatAttnStep;

int sat_attn_part_stride(int32_t M1, int32_t M2);
/* q = x @ [W1 | W2] (query_layer of both mechanisms), x [B][K] row stride x_sb */
int sat_attn_query(int32_t B, int32_t K, int32_t N1, int32_t N2, const float* x, int64_t x_sb,
                   const float* W1, const float* W2, float* q, int64_t q_sb, void* stream);
int sat_attn_step_fwd(const SatAttnStep* args, void* stream);

/* Backward of one attention step (reverse time t), one launch.  Inputs: dctx = dL/d[c1|c2] at
 * t (all sources); ctx_t = the forward context [c1|c2] of step t (row stride ctx_sb: the
 * utterance-wide softmax / recursion sums are dots with it, so no cross-tile pass is needed);
 * y_next / df_next = what the step t+1 backward sent back (Y[n] = s_{t+1}[n] dL/dprior[n], the
 * alignment recursion's gradient, dalpha_t[n] = (1-u) Y[n] + u Y[n+1]; and the location-feature
 * gradient [B][N][F]) -- both NULL at the last step; the forward state of step t (s_t = s_out,
 * a_t = a_out, a_prev, s_prev, s2_t, stats, q).  Outputs: y_out, df_out (for step t-1), dqp
 * [B][ntiles][D1+D2] per-tile query-gradient partials (overwritten), de1_out / de2_out [B][N]
 * the energy gradients of step t (history rows for sat_attn_param_grads).  Only the critical
 * path runs per step: parameter gradients are one pass after the loop (sat_attn_param_grads),
 * the value gradients dV = alignments^T dctx one batched GEMM. */
typedef struct SatAttnStepBwd {
  int32_t B, N, D1, M1, D2, M2, F, KW, NT, ntiles, att1_forward;
  float u;
  const float* dctx; int64_t dctx_sb;
  const float* ctx_t; int64_t ctx_sb;
  const float* y_next;
  const float* V1; const float* V2;
  const float* s_t; const float* a_t; const float* a_prev; const float* s_prev; const float* s2_t;
  const float* stats;
  const float* df_next;
  const float* q; int64_t q_sb;
  const float* K1; const float* K2;
  const float* v1; const float* b1; const float* convW; const float* convb; const float* locW;
  const float* v2;
  float* y_out;
  float* df_out;
  float* de1_out; float* de2_out;
  float* dqp;
  int32_t waves;                            /* waves per block: 0 (= 16), 4, 8 or 16 */
} SatAttnStepBwd;

int sat_attn_step_bwd(const SatAttnStepBwd* args, void* stream);

/* All attention-parameter gradients of the T reverse steps in one pass over (t, b, n)
 * (ForwardAttention variables modules/forward_attention.py:16-23,68-78 and the Bahdanau
 * memory/score of attention2): energies recomputed from K1/K2 + the query history q
 * (q_t[b] = q + t*q_tstride + b*q_bstride, [D1 | D2]) + b1 + the location-feature history
 * loc [T][B][N][F]; with the energy-gradient histories de1/de2 [T][B][N] and the
 * location-gradient history df [T][B][N][F] (s_prev: s_{t-1}[b][n] = s_prev + t*s_tstride +
 * b*N + n).  Writes dK1 [B][N][D1], dK2 [B][N][D2] (overwritten) and one partial row per
 * workgroup, pg [sat_attn_param_grad_rows(B, N)][pg_stride] =
 * [dv1 D1 | dW_loc F*D1 | dconvW KW*F | dconvb F | dv2 D2] (F = KW = 0 when !att1_forward),
 * to be column-summed.  tsplit = k > 1 splits the T steps into k ranges run by separate
 * workgroups (the one-wave-per-position grid otherwise leaves its last residency round almost
 * empty): dK1 / dK2 are then [k][B][N][D] scratch whose slab 0 holds the gradient on return,
 * and pg has k * sat_attn_param_grad_rows(B, N) rows (0 or 1: no split). */
typedef struct SatAttnParamGrad {
  int32_t T, B, N, D1, D2, F, KW, att1_forward;
  const float* K1; const float* K2;
  const float* q; int64_t q_tstride, q_bstride;
  const float* b1; const float* v1; const float* locW; const float* v2;
  const float* loc;
  const float* s_prev; int64_t s_tstride;
  const float* de1; const float* de2;
  const float* df;
  float* dK1; float* dK2;
  float* pg; int64_t pg_stride;
  int32_t tsplit;
} SatAttnParamGrad;

int sat_attn_pg_stride(int32_t D1, int32_t D2, int32_t F, int32_t KW);
int sat_attn_param_grad_rows(int32_t B, int32_t N);
int sat_attn_param_grads(const SatAttnParamGrad* args, void* stream);

/* ---------------------------------------------------------------- persistent decoder chain
 * ALL T' steps of the decoder's attention chain in one launch (DualSourceAttentionRNN,
 * modules/module.py:1017-1048: ZoneoutLSTM attention RNN -> query layers -> ForwardAttention
 * modules/forward_attention.py:88-122 + BahdanauAttention -> contexts), teacher-forced inputs
 * X0 [T][B][4U] = prenet(x_t) @ W0[:p] + b0 precomputed.  8 groups x 32 workgroups; each
 * (utterance, 32-position tile) K/V slice stays in LDS and each workgroup's LSTM / query weight
 * columns in registers for the whole decode; steps are separated by in-kernel group barriers
 * (sc1 hand-offs, bounded spins: a timeout sets err[0] != 0 and the kernel drains).
 * Compiled for the self-attention-tacotron shapes (U=256, M1=256, M2=32, D1=224, D2=32, F=5,
 * KW=10), B in {8,16,24,32}, (B/8) * ceil(N/32) <= 32; requires 256 co-resident workgroups.
 * Writes the same histories as the per-step path: REC0 [T+1][B][M1+M2+U] (rows 1..T),
 * C0 [T+1][B][U], H0RAW, G0, Q [T][B][.], S1/AL1 [T+1][B][N] (rows 1..T; row 0 = initial
 * state, set by the caller), S2 [T][B][N], ST [T][B][4], LOC [T][B][N][F] (nullable).
 * Scratch: E, PART, QP (sat_decoder_attention_scratch), ctr [sat_decoder_attention_scratch()]
 * words and err [2] (both zeroed by the call). */
typedef struct SatDecAttnFwd {
  int32_t B, N, T, U, M1, M2, D1, D2, F, KW;
  float u, zc, zh;
  const float* X0; const float* W0r; const float* Wq1; const float* Wq2;
  const float* K1; const float* V1; const float* K2; const float* V2;
  const int64_t* lengths;
  const float* v1; const float* b1; const float* convW; const float* convb; const float* locW;
  const float* v2;
  const float* mask_c; const float* mask_h;
  float* REC0; float* C0; float* H0RAW; float* G0; float* Q;
  float* S1; float* AL1; float* S2; float* ST; float* LOC;
  float* E; float* PART; float* QP; uint32_t* ctr; int32_t* err;
  int64_t* prof;   /* optional [256][16] per-workgroup segment clocks (100 MHz) followed by a
                      [T][256][4] event trace, NULL = off */
  float* ZH;       /* optional [T][B][N][D1+D2]: tanh of every energy pre-activation, kept for
                      sat_decoder_attention_bwd (which then recomputes no transcendental) */
} SatDecAttnFwd;

int sat_decoder_attention_fwd(const SatDecAttnFwd* args, void* stream);
int64_t sat_decoder_attention_scratch(int32_t B, int32_t N, int64_t* e_floats, int64_t* part_floats,
                                      int64_t* qp_floats);

/* Persistent BPTT of the same chain: all T reverse steps of the dual-source attention backward
 * + the attention RNN's reverse step in ONE launch.  Replaces, per step, sat_rowdot (the
 * attention RNN's input gradient) + sat_attn_step_bwd + the attention RNN's sat_lstm_steps_bwd
 * (backward.py decoder_bwd's launch path; reference graph: the TF gradients of
 * modules/module.py:1522-1540 AttentionRNN + forward_attention.py / tf additive attention).
 * Inputs: the forward histories (decoder_forward), DH0 = dL/dh0'_t from LSTM1 (all steps) and
 * RD[:, :, :M1+M2] = LSTM1's dL/dctx_t.  Outputs: DG0, the full dL/dctx_t in RD[:, :, :M1+M2],
 * DE1/DE2, DFH, DQP (the inputs of the post-loop parameter-gradient pass).  Same shape limits
 * as the forward; RDP and YA (sizes from sat_decoder_attention_bwd_scratch) are scratch. */
typedef struct SatDecAttnBwd {
  int32_t B, N, T, U, M1, M2, D1, D2, F, KW;
  float u, zc, zh;
  const float* REC0; const float* C0; const float* G0;
  const float* S1; const float* AL1; const float* S2; const float* ST; const float* LOC;
  const float* V1; const float* V2;
  const float* v1; const float* convW; const float* convb; const float* locW;
  const float* v2;
  const float* W0r; const float* Wq1; const float* Wq2;
  const float* mask_c; const float* mask_h;
  const float* DH0;
  const float* ZH;   /* the forward's energy tanh history (SatDecAttnFwd.ZH), required */
  float* RD; float* DG0; float* DE1; float* DE2; float* DFH; float* DQP;
  float* RDP; float* YA; uint32_t* ctr; int32_t* err;
  int64_t* prof;   /* optional [256][16] per-workgroup segment clocks (100 MHz), NULL = off */
} SatDecAttnBwd;

int sat_decoder_attention_bwd(const SatDecAttnBwd* args, void* stream);
int64_t sat_decoder_attention_bwd_scratch(int32_t B, int32_t N, int64_t* rdp_floats,
                                          int64_t* ya_floats);
/* Query-gradient parts per step the BPTT writes into DQP [T][B][parts][D1+D2]: 1 (dq_t
 * fully reduced) when the one-utterance-per-8-workgroups layout applies (N <= 256;
 * SAT_ATTN_BWD8=0 disables it), else ceil(N / 32) tile partials. */
int32_t sat_decoder_attention_bwd_dq_parts(int32_t B, int32_t N);

/* Persistent decoder LSTM stack: all T steps of DecoderRNNV2's two ZoneoutLSTM(U) layers
 * (ext tacotron2 DecoderRNNV2, built at modules/module.py:1531-1540) in ONE launch, LSTM2 one
 * step behind LSTM1, one in-kernel hand-off per step.  Replaces the per-step
 * sat_lstm_steps_fwd / sat_lstm_steps_bwd launches of the two layers (decoder.py /
 * backward.py launch paths); same arithmetic.  U = 256, B <= 32; the hand-off scratch
 * (forward: xch; backward: ctr) and err [2] are zeroed by the call.
 * Forward inputs: X1 = LSTM1's hoisted input projection + bias [T][B][4U], W1r = LSTM1's
 * recurrent kernel rows [U][U][4], W2 = LSTM2's kernel [2U][U][4] (input rows, then recurrent),
 * b2 [4U], zoneout masks [T][B][U] (all four or none: eval blend).  Histories as the launch path:
 * H*RAW [T][B][U] raw outputs, C*S/H*S [T+1][B][U] states (row 0 = initial state, read),
 * G* [T][B][4U] activated gates. */
typedef struct SatDecLstmFwd {
  int32_t B, T, U;
  float zc, zh;
  const float* X1; const float* W1r; const float* W2; const float* b2;
  const float* mask1_c; const float* mask1_h; const float* mask2_c; const float* mask2_h;
  float* H1RAW; float* C1S; float* H1S; float* G1;
  float* H2RAW; float* C2S; float* H2S; float* G2;
  float* xch;      /* hand-off granules, sat_decoder_lstms_scratch(B) floats, zeroed by the call */
  int32_t* err;
  int64_t* prof;   /* optional [256][4] per-workgroup segment clocks (100 MHz), NULL = off */
} SatDecLstmFwd;

/* Its BPTT: DH2 = dL/dh2'_t [T][B][U] (from the decoder head) -> DG2, DG1 [T][B][4U], the
 * gate gradients of both layers (their input / weight gradients are whole-sequence GEMMs). */
typedef struct SatDecLstmBwd {
  int32_t B, T, U;
  float zc, zh;
  const float* W1r; const float* W2;
  const float* G1; const float* C1S; const float* G2; const float* C2S;
  const float* DH2;
  const float* mask1_c; const float* mask1_h; const float* mask2_c; const float* mask2_h;
  float* DG1; float* DG2;
  uint32_t* ctr;   /* sat_decoder_lstms_bwd_scratch(B) words (tagged gate-gradient exchange
                      slots + placement words), 16-byte aligned, zeroed by the call */
  int32_t* err;
  int64_t* prof;   /* optional [256][4] per-workgroup segment clocks (100 MHz), NULL = off */
} SatDecLstmBwd;

/* ---------------------------------------------------------------- the whole decoder loop
 * SURVEY.md 8(b)'s single C entry for the teacher-forced decoder recurrence: DecoderRNNV2
 * (MultiRNNCell[DualSourceAttentionRNN, ZoneoutLSTM, ZoneoutLSTM], ext tacotron2, built at
 * modules/module.py:1531-1540) driven by TransformerTrainingHelper (modules/helpers.py:13-58)
 * over all T' steps, i.e. what decoder.py decoder_forward orchestrates on the persistent path:
 *   1. sat_decoder_attention_fwd(&attn)   -- attention RNN + query + dual-source attention,
 *                                            all T' steps, one persistent launch;
 *   2. X1 = H0RAW W1x[0:U] + b1 + ctx W1x[U:U+M1+M2]  -- LSTM1's input projection for all
 *      steps as two GEMMs (ctx = REC0 rows 1..T', columns 0..M1+M2; ConcatOutputAndAttention);
 *   3. sat_decoder_lstms_fwd(&lstm)       -- both ZoneoutLSTM layers, one persistent launch.
 * lstm.X1 must point at the X1 buffer [T'][B][4U]; attn.H0RAW / attn.REC0 are read as LSTM1's
 * input.  W1x = LSTM1 kernel input rows [U + M1 + M2][4U] (gate-interleaved), b1 its bias.
 * ws / ws_bytes: GEMM split-K scratch (as SatGemmDesc.ws).  Every buffer is caller-owned. */
typedef struct SatDecoderLoopFwd {
  SatDecAttnFwd attn;
  SatDecLstmFwd lstm;
  const float* W1x; const float* b1;
  void* ws; int64_t ws_bytes;
} SatDecoderLoopFwd;
int sat_decoder_loop_fwd(const SatDecoderLoopFwd* args, void* stream);

/* Its BPTT (backward.py decoder_bwd, persistent path): sat_decoder_lstms_bwd(&lstm) -> DH0 =
 * DG1 W1x[0:U]^T and RD[:, :, 0:M1+M2] = DG1 W1x[U:U+M1+M2]^T (LSTM1's input gradients) ->
 * sat_decoder_attention_bwd(&attn).  attn.DH0 must point at DH0 [T'][B][U] and attn.RD at RD
 * [T'][B][M1+M2+U] (zeroed here first); lstm.DG1 is read as LSTM1's gate gradients. */
typedef struct SatDecoderLoopBwd {
  SatDecLstmBwd lstm;
  SatDecAttnBwd attn;
  const float* W1x;
  float* DH0;
  void* ws; int64_t ws_bytes;
} SatDecoderLoopBwd;
int sat_decoder_loop_bwd(const SatDecoderLoopBwd* args, void* stream);

/* SURVEY.md 8(b)'s names for one ZoneoutLSTM step (ext tacotron2 ZoneoutLSTMCell around TF
 * LSTMCell, modules/module.py:1522-1527): the same entries as sat_lstm_step_fwd / _bwd. */
int sat_zlstm_step_fwd(const SatLstmFwd* args, void* stream);
int sat_zlstm_step_bwd(const SatLstmBwd* args, void* stream);

/* Persistent encoder BiLSTM: all N steps of both directions of ZoneoutCBHG's bidirectional
 * ZoneoutLSTM (modules/module.py:93-110, TF bidirectional_dynamic_rnn with sequence_length;
 * zoneout LSTM cell of ext tacotron2) in ONE launch each way.  Replaces the per-step
 * sat_lstm_steps_fwd / sat_lstm_steps_bwd launches of model.py encoder_fwd and backward.py
 * (same arithmetic: TF LSTMCell gate order i j f o, forget_bias 1.0, steps at or beyond the
 * utterance length copy the state and output 0).  One workgroup per (direction, utterance)
 * holds the whole recurrent matrix in registers, so a step needs no inter-workgroup hand-off.
 * U = 128.  X_fw, X_bw = the hoisted input projections + bias, element (b, n, c) at
 * X + b*x_sb + n*x_sn + c; W_fw, W_bw = recurrent kernel rows [U][U][4]; masks [N][B][U] (all
 * four or none: eval blend); H = raw outputs, direction d at H + b*h_sb + n*h_sn + d*U + u;
 * CS and HS [N+1][B][U] states (forward direction: row 0 read as the initial state, row n+1
 * written at step n; backward direction: row N read, row n written at step n); G [N][B][4U]
 * activated gates. */
typedef struct SatEncLstmFwd {
  int32_t B, N, U;
  float zc, zh;
  const float* X_fw; const float* X_bw; int64_t x_sb, x_sn;
  const float* W_fw; const float* W_bw;
  const float* mc_fw; const float* mh_fw; const float* mc_bw; const float* mh_bw;
  const int64_t* lengths;
  float* H; int64_t h_sb, h_sn;
  float* CS_fw; float* HS_fw; float* CS_bw; float* HS_bw;
  float* G_fw; float* G_bw;
} SatEncLstmFwd;

/* Its BPTT: DY = dL/dH (same layout as H) -> DG_fw, DG_bw [N][B][4U] gate gradients (the input and
 * weight gradients are whole-sequence GEMMs on the host side). */
typedef struct SatEncLstmBwd {
  int32_t B, N, U;
  float zc, zh;
  const float* W_fw; const float* W_bw;
  const float* G_fw; const float* G_bw; const float* CS_fw; const float* CS_bw;
  const float* mc_fw; const float* mh_fw; const float* mc_bw; const float* mh_bw;
  const int64_t* lengths;
  const float* DY; int64_t dy_sb, dy_sn;
  float* DG_fw; float* DG_bw;
} SatEncLstmBwd;

int sat_encoder_lstm_fwd(const SatEncLstmFwd* args, void* stream);
int sat_encoder_lstm_bwd(const SatEncLstmBwd* args, void* stream);

int sat_decoder_lstms_fwd(const SatDecLstmFwd* args, void* stream);
int64_t sat_decoder_lstms_scratch(int32_t B);
int64_t sat_decoder_lstms_bwd_scratch(int32_t B);
int sat_decoder_lstms_bwd(const SatDecLstmBwd* args, void* stream);

/* ---------------------------------------------------------------- elementwise
 * out[b,n,:] = x[b,n,:] * (n < lengths[b])  -- TF _prepare_memory (memory_sequence_length). */
int sat_seq_mask(const float* x, float* out, int32_t B, int32_t N, int32_t C,
                 const int64_t* lengths, void* stream);

/* Embedding lookup (ext tacotron2 Embedding, models/models.py:28,54): out[r] = table[ids[r]-offset];
 * an id outside [offset, offset+V) writes zeros and sets *err = 1 (the reference's
 * tf.assert_* raises InvalidArgumentError).  Backward: fp32 atomic scatter-add. */
int sat_embedding_fwd(const float* table, const int64_t* ids, float* out, int64_t R, int32_t D,
                      int32_t V, int64_t offset, int32_t* err, void* stream);
int sat_embedding_bwd(const float* dout, const int64_t* ids, float* dtable, int64_t R, int32_t D,
                      int32_t V, int64_t offset, void* stream);

/* Column reductions over x [M][C] (row stride ld*): workspace of sat_workspace_colreduce bytes. */
int64_t sat_workspace_colreduce(int32_t M, int32_t C);
/* tf.layers.BatchNormalization (inside ext tacotron2 Conv1d, modules/module.py:46-68):
 * training statistics over every row (biased var), moving averages with `momentum`
 * (mov_* may be NULL); apply y = gamma (x-mean)/sqrt(var+eps) + beta [relu] [+ res];
 * backward: dgamma/dbeta ACCUMULATE, dx = beta_out*dx + BN'(gate(dy)) where gate = the
 * post-ReLU output (NULL if no ReLU); training=0 differentiates the moving-stat (eval) form. */
int sat_bn_stats(const float* x, int64_t ldx, int32_t M, int32_t C, float* mean, float* var,
                 float* mov_mean, float* mov_var, float momentum, void* workspace, void* stream);
int sat_bn_apply(const float* x, int64_t ldx, float* y, int64_t ldy, int32_t M, int32_t C,
                 const float* mean, const float* var, float eps, const float* gamma,
                 const float* beta, int32_t relu, const float* res, int64_t ldr, void* stream);
int sat_bn_bwd(const float* dy, int64_t lddy, const float* x, int64_t ldx, const float* gate,
               int64_t ldg, float* dx, int64_t lddx, int32_t M, int32_t C, const float* mean,
               const float* var, float eps, const float* gamma, float* dgamma, float* dbeta,
               int32_t training, float beta_out, void* workspace, void* stream);
/* out[c] = beta*out[c] + sum_m x[m][c]   (bias gradients) */
int sat_colsum(const float* x, int64_t ldx, int32_t M, int32_t C, float* out, float beta,
               void* workspace, void* stream);
/* Column sums of x scattered into separate parameter gradients (the attention parameters'
 * per-workgroup partial rows, backward.py): for each segment k, columns [col, col+n) go to
 * dst[0..n): dst[j] = beta*dst[j] + sum_m x[m][col+j].  1 <= nseg <= 8. */
typedef struct SatColSegment {
  float* dst;
  int32_t col, n;
} SatColSegment;
int sat_colsum_scatter(const float* x, int64_t ldx, int32_t M, int32_t C,
                       const SatColSegment* segs, int32_t nseg, float beta, void* workspace,
                       void* stream);

/* MaxPooling1D(pool 2, stride 1, SAME) over [B][N][C] (modules/module.py:54,80) and its
 * gradient (first index wins ties, as TF MaxPoolGrad). */
int sat_maxpool2(const float* x, float* y, int32_t B, int32_t N, int32_t C, void* stream);
/* y = BN(x) (+ReLU) as sat_bn_apply over the [B*N][C] rows (contiguous, no residual) AND
 * mp = sat_maxpool2(y) in one pass: the CBHG conv bank's BN and max-pool
 * (modules/module.py:79-80); bit-identical to the two calls. */
int sat_bn_apply_maxpool2(const float* x, float* y, float* mp, int32_t B, int32_t N, int32_t C,
                          const float* mean, const float* var, float eps, const float* gamma,
                          const float* beta, int32_t relu, void* stream);
int sat_maxpool2_bwd(const float* x, const float* dy, float* dx, int32_t B, int32_t N, int32_t C,
                     void* stream);

/* ext tacotron2 HighwayNet combine y = h*t + x*(1-t) (h = ReLU dense, t = sigmoid dense) and
 * its backward to the pre-activations (dh_pre, dt_pre) and the carry path dx. */
int sat_highway_fwd(const float* h, const float* t, const float* x, float* y, int64_t n,
                    void* stream);
/* The same layer after ONE batched GEMM of both pre-activations (h, t hold h_pre, t_pre):
 * h = relu(h), t = sigmoid(t) in place, then y = h*t + x*(1-t). */
int sat_highway_act_fwd(float* h, float* t, const float* x, float* y, int64_t n, void* stream);
int sat_highway_bwd(const float* h, const float* t, const float* x, const float* dy,
                    float* dh_pre, float* dt_pre, float* dx, int64_t n, void* stream);

/* dx = beta*dx + dy * act'(y) [* mask]; act 0 identity, 1 relu, 2 tanh, 3 sigmoid, 4 softsign. */
int sat_act_bwd(const float* dy, const float* y, const float* mask, float* dx, int64_t n,
                int32_t act, float beta, void* stream);
/* out[c][r] = in[r][c]  (weight re-layouts, e.g. query-layer kernels for the per-step rowdot) */
int sat_transpose(const float* in, int64_t ldi, float* out, int64_t ldo, int32_t R, int32_t C,
                  void* stream);
/* y = a*x + b*y */
int sat_axpby(const float* x, float* y, int64_t n, float a, float b, void* stream);
/* z = x + y (n % 4 == 0, 16-byte aligned): a residual sum whose addend is kept for the backward */
int sat_add(const float* x, const float* y, float* z, int64_t n, void* stream);
/* p[i] = bits for n 4-byte words (zero-initialised step buffers and error words inside the
 * captured training step, in place of a framework fill). */
int sat_fill32(void* p, int64_t n, uint32_t bits, void* stream);
/* dst[i*d0 + j*d1 + k] = src[i*s0 + j*s1 + k] for i < n0, j < n1, k < n2 (unit innermost
 * strides): a transposed view made contiguous, or a strided slice copied into a step buffer. */
int sat_copy3d(const float* src, int64_t s0, int64_t s1, float* dst, int64_t d0, int64_t d1,
               int32_t n0, int32_t n1, int32_t n2, void* stream);

/* ScaledDotProductAttentionMechanism softmax (modules/self_attention.py:45-65):
 * P = softmax(scale*S) per row of length L, causal (use_subsequent_mask) masks col > row%Lq,
 * Pd = P * mask (tf.layers.dropout on the probabilities).  Backward gives dS; causal rows read
 * P / dPd only up to the diagonal (dPd beyond it may be unwritten: SatGemmDesc.tri) and get
 * dS = 0 there. */
int sat_softmax_fwd(const float* S, float* P, float* Pd, const float* mask, int64_t R, int32_t L,
                    int32_t Lq, int32_t causal, float scale, void* stream);
int sat_softmax_bwd(const float* P, const float* dPd, const float* mask, float* dS, int64_t R,
                    int32_t L, int32_t Lq, int32_t causal, float scale, void* stream);

/* Loss of models/models.py:159-173: l1_weight * L1(mel, tgt; tmask) + sigmoid xent(stop, done;
 * dmask), tf.losses SUM_BY_NONZERO_WEIGHTS.  out[0..4] = loss, L1, BCE, counts; if dmel/dstop
 * are given, also writes the gradients of out[0].  Deterministic two-pass fp64 reduction over a
 * caller-provided workspace of sat_workspace_loss() bytes. */
int64_t sat_workspace_loss(void);
int sat_loss_fwd_bwd(const float* mel, const float* tgt, const float* tmask, const float* stop,
                     const float* done, const float* dmask, int32_t B, int32_t T, int32_t M,
                     int32_t Tp, float l1_weight, float* out, float* dmel, float* dstop,
                     void* workspace, void* stream);

/* ---------------------------------------------------------------- optimiser
 * models/models.py:175-189 + :283-287 over the whole flat arena in three launches:
 * global norm (fp64 partials), scalar prepare (Noam lr, clip scale, Adam bias correction, reads
 * and increments *global_step on the device), elementwise Adam (TF epsilon-hat form).
 * scalars[4] receives {norm, clip scale, lr, lr_t}.  workspace: sat_workspace_adam() bytes.
 * Health guard: if any of the n_health int32 words at `health` (device; the step's in-kernel
 * error words) is non-zero the whole update is skipped -- params, moments and *global_step stay
 * as they were -- and status[2] (device, nullable) becomes {skipped steps + 1, first error code}.
 * Lets a replayed training graph refuse garbage without a host sync. */
typedef struct SatAdamConfig {
  float lr0, beta1, beta2, eps, clip_norm;   /* clip_norm <= 0 disables clipping */
  int32_t decay, step_factor;
  float grad_scale;   /* grads are used as grad_scale * g (1/world after a SUM all-reduce) */
} SatAdamConfig;

int64_t sat_workspace_adam(void);
int sat_global_norm_sq(const float* g, int64_t n, double* partials, void* stream);
int sat_adam_step(float* params, const float* grads, float* m, float* v, int64_t n,
                  int64_t* global_step, float* scalars, void* workspace,
                  const SatAdamConfig* cfg, const int32_t* health, int32_t n_health,
                  int32_t* status, void* stream);

/* Data-parallel exchange (train.py:67,73 MirroredStrategy -> ONE SUM all-reduce per step over
 * [gradients | BN moving statistics | health tail], sat_amd/dp.py).  pack: tail[i] =
 * |float(health[i])| and bn *= bn_scale (1/world, so the SUM leaves the replicas' mean);
 * unpack after the collective: health[i] = int(tail[i]) (non-zero iff some rank's word was;
 * the code is exact when one rank failed). */
int sat_exchange_pack(const int32_t* health, int32_t n_health, float* bn, int64_t n_bn,
                      float* tail, float bn_scale, void* stream);
int sat_exchange_unpack(const float* tail, int32_t n_health, int32_t* health, void* stream);

/* ---------------------------------------------------------------- dataset records (host)
 * TFRecord framing of the dataset path: datasets/ljspeech/dataset.py:96-112 reads
 * tf.data.TFRecordDataset files written by preprocess/ljspeech.py:23-45 (utils/tfrecord.py:46-49).
 * Host memory, no device work; used by sat_amd/tfrecord.py. */
uint32_t sat_crc32c(const void* data, int64_t n, uint32_t crc);      /* CRC-32C, continuable */
uint32_t sat_tfrecord_masked_crc(const void* data, int64_t n);       /* TF's masked form */
int64_t sat_tfrecord_frame(const void* data, int64_t n, void* out);  /* out: n + 16 bytes */
/* (offset, length) of each payload in a buffer of records (up to cap pairs); returns the record
 * count or a negative SAT_ERR_* on truncation / checksum mismatch (verify != 0) */
int64_t sat_tfrecord_index(const void* buf, int64_t n, int32_t verify, int64_t* spans,
                           int64_t cap);

#ifdef __cplusplus
}
#endif
#endif /* SAT_ABI_H */
