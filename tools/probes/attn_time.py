"""HIP-event time of the two attention-chain launches (sat_decoder_attention_fwd / _bwd), the
attention parameter-gradient pass (sat_attn_param_grads) and the decoder LSTM stack
(sat_decoder_lstms_fwd / _bwd) and the encoder BiLSTM (sat_encoder_lstm_fwd / _bwd) on the
training step's own buffers (B=32, N=200, T'=500, train mode) with whichever library is loaded
(tools only; A/B two builds by running this twice, once with SAT_LIB_OVERRIDE=<other .so>).
Also prints a checksum of the forward's histories and the BPTT outputs so two builds' results
can be compared.

Usage: python tools/probes/attn_time.py [B] [reps]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import _sat_path  # noqa: E402

_sat_path.load()
import torch  # noqa: E402

from sat_amd import _lib, data, engine, hparams  # noqa: E402
from sat_amd import kernels as K  # noqa: E402

KW = {}
NAMES = ("decoder_attention_fwd", "decoder_attention_bwd", "attn_param_grads",
         "decoder_lstms_fwd", "decoder_lstms_bwd", "encoder_lstm_fwd", "encoder_lstm_bwd")
for nm in NAMES:
    orig = getattr(K, nm)

    def rec(_o=orig, _n=nm, **kw):
        KW[_n] = dict(kw)
        _o(**kw)
    setattr(K, nm, rec)
    KW[nm + "_orig"] = orig
B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
hp = hparams.ljspeech_hparams()
m = engine.Tacotron(hp, "cuda", seed=1)
b = data.synthetic_batch(hp, B, N=200, T=1000, shape="max", seed=1)
mk = data.synthetic_masks(hp, B, 200, 500, seed=2)
gb = {k: torch.tensor(v).cuda() for k, v in b.items()}
gm = {k: torch.tensor(v).cuda() for k, v in mk.items()}
out, sv = m.forward(gb, gm, training=True)
m.backward(sv)
torch.cuda.synchronize()
Tp = int(KW["decoder_attention_fwd"]["T"])
RD0 = KW["decoder_attention_bwd"]["RD"].clone()


def timed(nm, reps):
    kw, fn = KW[nm], KW[nm + "_orig"]
    ts = []
    for i in range(reps + 1):
        if nm == "decoder_attention_bwd":
            kw["RD"].copy_(RD0)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn(**kw)
        e1.record()
        torch.cuda.synchronize()
        if i:
            ts.append(e0.elapsed_time(e1) * 1e3)
    if "err" in kw:
        assert int(kw["err"][0].item()) == 0
    return sorted(ts)


for nm in NAMES:
    ts = timed(nm, reps)
    med = ts[len(ts) // 2]
    print(f"{os.path.basename(_lib.LIB_PATH)} {nm}: median {med:.1f} us/launch = {med / Tp:.3f} "
          f"us/step (min {ts[0]:.1f}, max {ts[-1]:.1f})", flush=True)
f, bw = KW["decoder_attention_fwd"], KW["decoder_attention_bwd"]
sums = {k: float(f[k].double().sum()) for k in ("REC0", "Q", "AL1", "S2", "ZH")}
sums.update({k: float(bw[k].double().sum()) for k in ("DG0", "DE1", "RD")})
pg = KW["attn_param_grads"]
sums.update({k: float(pg[k].double().sum()) for k in ("dK1", "dK2", "pg")})
ef, eb = KW["encoder_lstm_fwd"], KW["encoder_lstm_bwd"]
sums.update({"encH": float(ef["H"].double().sum()), "encG": float(ef["G_fw"].double().sum()),
             "encDG": float(eb["DG_fw"].double().sum())})
print("  checksums " + " ".join(f"{k}={v:.9e}" for k, v in sums.items()), flush=True)
