// sat_workspace_size: the caller-owned device scratch one teacher-forced training step needs
// (SURVEY 8(b)), as the sum of every entry's own scratch query, each rounded to 256 bytes.
// Host-only; the per-entry queries stay the authority (a caller may also carve them itself).
#include "sat_common.h"

namespace {
constexpr int64_t kAlign = 256;
int64_t al(int64_t n) { return (n + kAlign - 1) / kAlign * kAlign; }
constexpr int64_t kGemmSplitKBytes = 32ll << 20;   // split-K slab budget per stream (kernels.py)
}  // namespace

extern "C" int64_t sat_workspace_size(const SatDims* d) {
  if (!d || d->B <= 0 || d->N <= 0 || d->Tp <= 0 || d->enc_heads <= 0 || d->dec_heads <= 0 ||
      d->enc_D <= 0 || d->dec_D <= 0 || d->max_cols <= 0) {
    sat::set_error("sat_workspace_size: bad dims");
    return SAT_ERR_ARGUMENT;
  }
  int64_t e = 0, part = 0, qp = 0, rdp = 0, ya = 0;
  const int64_t ctr = sat_decoder_attention_scratch(d->B, d->N, &e, &part, &qp);
  const int64_t bctr = sat_decoder_attention_bwd_scratch(d->B, d->N, &rdp, &ya);
  int64_t total = al(4 * e) + al(4 * part) + al(4 * qp) + al(4 * ctr);           // attention fwd
  total += al(4 * rdp) + al(4 * ya) + al(4 * bctr);                               // attention BPTT
  total += al(4 * sat_decoder_lstms_scratch(d->B)) + al(4 * sat_decoder_lstms_bwd_scratch(d->B));
  const int32_t rows = std::max(d->B * d->N, d->B * d->Tp);
  total += al(sat_workspace_colreduce(rows, d->max_cols));                         // bias / BN
  total += al(sat_workspace_loss()) + al(sat_workspace_adam());
  total += al(sat_mha_scratch_bytes(d->B, d->N, d->enc_D, d->enc_heads, d->enc_D));
  total += al(sat_mha_scratch_bytes(d->B, d->Tp, d->dec_D, d->dec_heads, d->dec_D));
  total += kGemmSplitKBytes;
  return total;
}
