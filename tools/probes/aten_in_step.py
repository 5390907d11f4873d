"""Which PyTorch (aten) GPU launches remain inside one eager training step, and from which line
of the package they come (tools only: torch.profiler with Python stacks).

Usage: python tools/probes/aten_in_step.py [B]   (default B=32, N=200, T=1000)
"""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import _sat_path  # noqa: E402

_sat_path.load()
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from sat_amd import data, engine, hparams, train  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
hp = hparams.ljspeech_hparams()
m = engine.Tacotron(hp, "cuda", seed=1234)
b = data.synthetic_batch(hp, B, N=200, T=1000, shape="max", seed=1000)
batch = {k: torch.tensor(v).cuda() for k, v in b.items()}
tr = train.Trainer(m, B, 200, 500, seed=1234)
tr.batch_lengths = batch["source_length"]
for _ in range(2):
    tr.step(batch)
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
    tr.step(batch)
    torch.cuda.synchronize()

sites = collections.Counter()
dev_k = collections.Counter()
for ev in prof.events():
    if ev.device_type != torch.autograd.DeviceType.CPU:
        if "at::" in ev.name or "copyBuffer" in ev.name or "fillBuffer" in ev.name:
            dev_k[ev.name[:90]] += 1
        continue
    if not ev.name.startswith("aten::") or ev.name in ("aten::empty", "aten::view", "aten::as_strided",
                                                      "aten::empty_strided", "aten::slice",
                                                      "aten::select", "aten::transpose",
                                                      "aten::reshape", "aten::_reshape_alias",
                                                      "aten::unsqueeze", "aten::permute",
                                                      "aten::t", "aten::expand", "aten::alias",
                                                      "aten::detach", "aten::lift_fresh",
                                                      "aten::resolve_conj", "aten::resolve_neg"):
        continue
    if ev.cpu_parent is not None and ev.cpu_parent.name.startswith("aten::"):
        continue          # count the outermost aten op only
    frames = [f for f in (ev.stack or []) if "self-attention-tacotron_amd" in f or "train.py" in f]
    site = frames[0] if frames else "(no package frame)"
    sites[(ev.name, site.split("/")[-1])] += 1
print(f"framework device kernels in one eager step (B={B}): {sum(dev_k.values())}")
for name, n in dev_k.most_common():
    print(f"  {n:3d}  {name}")
print("outermost aten ops (non-view) and their package call sites:")
for (name, site), n in sites.most_common():
    print(f"  {n:3d}  {name:32s} {site}")
