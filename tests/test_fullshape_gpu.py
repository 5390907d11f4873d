"""The hot path at the configured length against the float64 oracle.

north_star bar: mel frames within 1e-4 mean-L1 of the reference over LJSpeech-shape batches of
<= 1000 frames, i.e. 500 recurrent decoder steps -- the length where fp32 drift through the
recurrence and the persistent kernels' <= 1-ulp hand-off tags would
show.  Every case runs the persistent kernels that the bench times (any B <= 32 is eligible).

* C1 (LJSpeech, B=2, N=200, T=1000): eval mode (dropout off, zoneout blend -- the
  teacher-forced ``loss_with_teacher`` computation, models/models.py:208-231) and train mode
  with injected dropout / zoneout masks;
* gradients at B=8, N=200 (7 attention tiles and their halos), T=1000, ragged lengths;
* C2 (B=32, every persistent grid on all 256 CUs) forward in eval mode, and train mode with
  masks including every parameter gradient -- the configuration bench.py times.

Tolerances (written per assertion): mel mean-L1 <= 1e-4 (north_star); loss within 1e-5
relative; stop logits mean-abs <= 1e-4; every parameter gradient within 2e-4 of
max(|g_ref|, 1e-4 max|g|) (fp32 BPTT over 500 steps against float64 autograd; achieved
5.5e-5, profiles/r02_parity_fullshape.jsonl).

* C4 (VCTK multi-speaker, B=32, N=200, T=1000: speaker embedding + MultiSpeakerPreNet,
  modules/multi_speaker_modules.py:11-37, models/models.py:43-46): eval and train with
  injected masks, same bars.
Set SAT_PARITY_REPORT=<file> to append the achieved numbers as JSON lines."""
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _report(name, **vals):
    path = os.environ.get("SAT_PARITY_REPORT")
    if path:
        with open(path, "a") as f:
            f.write(json.dumps({"case": name, **vals}) + "\n")


def _gpu_kinks(sv, O):
    """The HIP forward's branch at the encoder front's piecewise-linear points (prenet / conv
    bank / proj1 ReLU gates, the max-pool window choice) for the oracle (``encoder(kinks=)``)."""
    bank = sv["bank"]
    nxt = torch.cat([bank[:, 1:], bank[:, -1:]], 1)
    k = {"bank": bank > 0, "pool_first": bank >= nxt, "proj1": sv["p1"] > 0}
    for i, x in enumerate(sv["enc_pre"][1:]):
        k[f"prenet{i}"] = x > 0
    return {n: v.double().cpu() for n, v in k.items()}


# at most this many of the encoder front's branch points may be decided differently by the
# HIP forward (fp32) and the oracle (float64) per kind, before the oracle is handed the HIP's
# branches (a systematic mask / max-pool bug must not be absorbed)
KINK_FLIPS_MAX = 16


def _bound_kink_flips(sv, O, p64, hp, b, mk, train):
    """Count the branch points where the HIP forward's decision differs from the oracle's own
    (float64, no substitution) and bound them; the counts go to the parity report."""
    from sat_amd import params
    ours = _gpu_kinks(sv, O)
    with torch.no_grad():
        theirs = O.encoder_front_branches(
            O.to_torch(b)["source"], {k: v.detach() for k, v in p64.items()},
            O.to_torch(params.init_bn_buffers(hp)), hp, None if mk is None else O.to_torch(mk),
            train)
    flips = {k: int((ours[k] != theirs[k]).sum()) for k in ours}
    sizes = {k: int(ours[k].numel()) for k in ours}
    _report("c2_train_kink_flips", flips=flips, sizes=sizes, bar=KINK_FLIPS_MAX)
    assert all(v <= KINK_FLIPS_MAX for v in flips.values()), (flips, sizes)


def _run(cuda, B, N, T, train, shape="max", seed=11, grads=False, preset="ljspeech",
         kinks=False):
    from sat_amd import data, engine, hparams, params
    from sat_amd.decoder import persistent_eligible
    from oracle import sat_oracle as O
    hp = getattr(hparams, f"{preset}_hparams")()
    vals = params.init_params(hp, seed=5)
    b = data.synthetic_batch(hp, B, N=N, T=T, shape=shape, seed=seed)
    Np, Tp = b["source"].shape[1], b["mel"].shape[1] // hp.outputs_per_step
    mk = data.synthetic_masks(hp, B, Np, Tp, seed=seed + 1) if train else None
    m = engine.Tacotron(hp, cuda, init_values=vals)
    assert persistent_eligible(m.d, B, Np)
    gb = {k: torch.tensor(v).to(cuda) for k, v in b.items()}
    gm = None if mk is None else {k: torch.tensor(v).to(cuda) for k, v in mk.items()}
    out, sv = m.forward(gb, gm, training=train, need_grad=grads)
    assert "attn_scratch" in sv["dec"].tensors          # the persistent kernels ran
    if grads:
        m.backward(sv)
    torch.cuda.synchronize()
    sv["dec"].tensors["attn_scratch"].check()
    p64 = {k: v.requires_grad_(grads) for k, v in O.to_torch(vals).items()}
    if kinks:
        _bound_kink_flips(sv, O, p64, hp, b, mk, train)
    with torch.set_grad_enabled(grads):
        ref = O.model_forward(p64, O.to_torch(params.init_bn_buffers(hp)), hp, O.to_torch(b),
                              None if mk is None else O.to_torch(mk), training=train,
                              kinks=_gpu_kinks(sv, O) if kinks else None)
        if grads:
            ref["loss"].backward()
    return hp, m, out, ref, p64, b


def _compare_outputs(name, out, ref, b):
    mel = out["mel"].double().cpu().numpy()
    rmel = ref["mel"].detach().numpy()
    w = b["mel_mask"][..., None].astype(bool) & np.ones_like(rmel, bool)
    l1 = float(np.abs(mel - rmel)[w].mean())
    l1_all = float(np.abs(mel - rmel).mean())
    mx = float(np.abs(mel - rmel).max())
    stop = out["stop"].double().cpu().numpy().reshape(ref["stop"].shape)
    st = float(np.abs(stop - ref["stop"].detach().numpy()).mean())
    loss, rloss = float(out["loss"].item()), float(ref["loss"].detach())
    _report(name, mel_mean_l1=l1, mel_mean_l1_padded=l1_all, mel_max_abs=mx, stop_mean_abs=st,
            loss=loss, loss_ref=rloss)
    assert l1 <= 1e-4, f"{name}: mel mean-L1 {l1:.3e} > 1e-4"
    assert l1_all <= 1e-4
    assert st <= 1e-4, f"{name}: stop mean-abs {st:.3e}"
    assert abs(loss - rloss) <= 1e-5 * max(1.0, abs(rloss)), (loss, rloss)


@pytest.mark.parametrize("train", [False, True], ids=["eval", "train_masks"])
def test_c1_full_length_matches_oracle(cuda, train):
    """C1: B=2, N=200, T=1000 -> 500 decoder steps (modules/forward_attention.py:88-122,
    modules/module.py:743-765), persistent kernels vs the float64 oracle."""
    hp, m, out, ref, _, b = _run(cuda, 2, 200, 1000, train)
    _compare_outputs(f"c1_{'train' if train else 'eval'}", out, ref, b)


def test_c2_full_shape_forward_matches_oracle(cuda):
    """C2: B=32 (four utterances per hand-off group, 7 tiles each), N=200, T=1000, eval."""
    hp, m, out, ref, _, b = _run(cuda, 32, 200, 1000, False, seed=21)
    _compare_outputs("c2_eval", out, ref, b)


@pytest.mark.parametrize("train", [False, True], ids=["eval", "train_masks"])
def test_c4_vctk_full_shape_matches_oracle(cuda, train):
    """C4: VCTK multi-speaker self-attention-tacotron.json at the bench shape (B=32, N=200,
    T=1000 -> 500 steps): speaker rows through the MultiSpeakerPreNet's softsign epilogue and
    zero-batch-stride residual, persistent kernels, vs the float64 oracle."""
    hp, m, out, ref, _, b = _run(cuda, 32, 200, 1000, train, seed=41, preset="vctk")
    assert hp.use_speaker_embedding and m.d.multi_speaker
    assert "speaker_id" in b and int(b["speaker_id"].min()) >= 225
    _compare_outputs(f"c4_{'train' if train else 'eval'}", out, ref, b)


def _compare_grads(name, m, p64, b):
    grads = m.grads_dict()
    gmax = max(float(p.grad.abs().max()) for p in p64.values())
    worst, worst_at, bad = 0.0, None, []
    for pname, p in p64.items():
        g_ref = p.grad.numpy()
        scale = max(np.abs(g_ref).max(), 1e-4 * gmax)
        err = float(np.abs(grads[pname].astype(np.float64) - g_ref).max() / scale)
        if err > worst:
            worst, worst_at = err, pname
        if not err <= 2e-4:
            bad.append((pname, err))
    _report(name, worst_rel_grad_err=worst, worst_param=worst_at, bar=2e-4,
            steps=int(b["mel"].shape[1] // 2))
    assert not bad, bad


def test_gradients_full_length_match_oracle(cuda):
    """BPTT over 500 steps at B=8, N<=200 (ragged; up to 7 tiles with halos), T<=1000, train
    mode with injected masks: loss and every parameter gradient vs float64 autograd."""
    hp, m, out, ref, p64, b = _run(cuda, 8, 200, 1000, True, shape="ljs", seed=31, grads=True)
    assert b["source"].shape[1] > 160 and b["mel"].shape[1] >= 800   # long, ragged batch
    _compare_outputs("grad_b8_outputs", out, ref, b)
    _compare_grads("grad_b8", m, p64, b)


def test_c2_train_gradients_match_oracle(cuda):
    """The benched configuration itself: C2 (B=32, N=200, T=1000 -> 500 steps, every persistent
    grid on all 256 CUs, 32 hand-off groups over the 8 XCDs), train mode with injected dropout /
    zoneout masks: mel, stop and loss vs the float64 oracle, then every parameter gradient of
    the BPTT vs float64 autograd (models/models.py:159-189).

    At this size (6400 positions x 2048 conv-bank channels) a few of the encoder front's ReLU
    gates and max-pool choices land on the other side of their kink in fp32 than in float64,
    and each such flip routes that element's whole gradient differently: the conv-bank / prenet /
    embedding gradients then differ by up to ~3e-2 of their max while every backward stage is
    exact on its own inputs (profiles/r04_cbhg_bwd_stages.txt, tools/probes/enc_kinks.py).  The
    oracle therefore takes the HIP forward's branch at those points (oracle ``encoder(kinks=)``:
    the same sub-gradient), and the bar stays 2e-4 for every parameter."""
    hp, m, out, ref, p64, b = _run(cuda, 32, 200, 1000, True, seed=51, grads=True, kinks=True)
    _compare_outputs("c2_train_outputs", out, ref, b)
    _compare_grads("c2_train_grad", m, p64, b)
