"""Phase clocks of the one-launch free-running decode (sat_decode_persistent) at C5 (B=8, N=200,
500 steps).  Needs the trace build:
    make -C self-attention-tacotron_amd/csrc BUILD=build_trace EXTRA=-DSAT_DP_TRACE=1 \
         OUT=../../tools/probes/libsat_dptrace.so
    SAT_LIB_OVERRIDE=tools/probes/libsat_dptrace.so python tools/probes/dp_profile.py
Thread 0 of every workgroup sums the 100 MHz wall clock spent in each segment; printed as us per
step, mean over the 256 workgroups and for an attention / a non-attention workgroup."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import _sat_path  # noqa: E402

_sat_path.load()
import torch  # noqa: E402

from sat_amd import data, engine, hparams  # noqa: E402
from sat_amd import kernels as K  # noqa: E402
from sat_amd.inference import FreeRunningDecoder  # noqa: E402

SEG = ["loop top->z ready (P1 wait)", "mel|stop", "prenet1 (z fold)", "wait y0", "prenet2",
       "wait p", "attention RNN", "wait h0", "query + LSTM1 rec.", "loc + wait q (attn WGs)",
       "energies + records", "wait records", "alignments + contexts", "LSTM1 + attRNN rec.",
       "wait h1", "LSTM2", "wait h2", "q|k|u + LSTM2 rec.", "cache prefetch + wait qku",
       "scores + partial O", "wait SA records", "z (head output)", "stop test",
       "P5 energies (sub)", "P5 stats (sub)", "P6 headers (sub)"]
B, steps = 8, 500
hp = hparams.ljspeech_hparams()
m = engine.Tacotron(hp, "cuda", seed=1234)
b = data.synthetic_batch(hp, B, N=200, T=1000, shape="max", seed=55)
batch = {k: torch.tensor(v).cuda() for k, v in b.items()}
prof = torch.zeros(256 * 57, dtype=torch.int64, device="cuda")
orig = K.decode_persistent
K.decode_persistent = lambda **kw: orig(**dict(kw, prof=prof))
dec = FreeRunningDecoder(m, max_iters=steps, min_iters=steps, persistent=True)
dec.run(batch)
torch.cuda.synchronize()
prof.zero_()
t0 = time.perf_counter()
dec.run(batch)
torch.cuda.synchronize()
print(f"C5 one-launch (trace build): {1e3 * (time.perf_counter() - t0):.2f} ms per decode")
pr = prof[:256 * 28].view(256, 28).cpu().double() / 100.0 / steps   # us per step
iters = prof[256 * 28:256 * 29].cpu()
print(f"iterations: min {int(iters.min())} max {int(iters.max())}")
mean = pr.mean(0)
# workgroup (g, w) = blockIdx g + 8 w: w = 0 is an attention workgroup, w = 20 is not
wa, wn = 0 + 8 * 0, 0 + 8 * 20
print(f"{'segment':34s} {'mean':>7s} {'attnWG':>7s} {'otherWG':>7s}")
for k, name in enumerate(SEG):
    print(f"{name:34s} {mean[k + 1]:7.3f} {pr[wa, k + 1]:7.3f} {pr[wn, k + 1]:7.3f}")
print(f"{'total':34s} {mean.sum():7.3f} {pr[wa].sum():7.3f} {pr[wn].sum():7.3f}")

# absolute clocks of every workgroup at step 300: skew of each marker over the group-0 workgroups
ab = prof[256 * 29:].view(256, 28).cpu().double() / 100.0
g0 = [8 * w for w in range(32)]
base = ab[g0, 1].min()
print("step 300, group 0: marker  min  median  max (us after the earliest marker 1)")
for k, name in enumerate(SEG):
    col = ab[g0, k + 1] - base
    srt = col.sort().values
    late = int(col.argmax())
    print(f"{name:34s} {srt[0]:7.3f} {srt[16]:7.3f} {srt[-1]:7.3f}  latest w={late}")
