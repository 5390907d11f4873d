"""The oracle reproduces its committed golden vectors (tests/golden/, made by make_golden.py).

This pins the CPU restatement against drift; the reference itself cannot run here and ships no
golden vectors, so agreement with TF is "parity unpinned" (DESIGN.md)."""
import os
import sys

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))

import make_golden as MG  # noqa: E402
from oracle import sat_oracle as O  # noqa: E402

GOLD = {p: np.load(os.path.join(HERE, "golden", c["file"])) for p, c in MG.MODEL_CASES.items()}
OPS = np.load(os.path.join(HERE, "golden", "golden_ops.npz"))


@pytest.mark.parametrize("preset", sorted(MG.MODEL_CASES))
def test_generator_inputs_unchanged(preset):
    G = GOLD[preset]
    hp, vals, batch, masks = MG.model_case(preset)
    names, cks = MG.param_checksums(vals)
    assert list(G["param_names"]) == names
    np.testing.assert_allclose(cks, G["param_checksums"], rtol=1e-12)
    for k, v in batch.items():
        np.testing.assert_array_equal(v, G[f"batch__{k}"])
    for k, v in masks.items():
        np.testing.assert_array_equal(v, G[f"mask__{k}"])


@pytest.mark.parametrize("preset", sorted(MG.MODEL_CASES))
def test_oracle_model_matches_golden(preset):
    G = GOLD[preset]
    hp, vals, batch, masks = MG.model_case(preset)
    for mode in ("eval", "train"):
        r = MG.oracle_model(hp, vals, batch, masks, mode == "train")
        for k in ("loss", "l1", "bce"):
            assert abs(r[k] - float(G[f"{mode}__{k}"])) < 1e-10, (mode, k)
        np.testing.assert_allclose(r["mel"], G[f"{mode}__mel"], atol=1e-10)
        np.testing.assert_allclose(r["stop"], G[f"{mode}__stop"], atol=1e-10)
        np.testing.assert_allclose(r["grad_sum_sumsq"], G[f"{mode}__grad_sum_sumsq"],
                                   rtol=1e-8, atol=1e-12)
        np.testing.assert_allclose(r["grad_head"], G[f"{mode}__grad_head"], rtol=1e-8,
                                   atol=1e-12)


def test_oracle_ops_match_golden():
    T = torch.tensor
    g = OPS
    for mode, (mc, mh) in {"train": (T(g["zlstm_mc"]), T(g["zlstm_mh"])),
                           "eval": (None, None)}.items():
        hr, c2, h2 = O.zoneout_lstm_step(T(g["zlstm_x"]), T(g["zlstm_c"]), T(g["zlstm_h"]),
                                         T(g["zlstm_w"]), T(g["zlstm_b"]), 0.1, 0.1, mc, mh)
        np.testing.assert_allclose(np.stack([hr, c2, h2]), g[f"zlstm_{mode}_out"], atol=1e-14)
    pm = {k[len("mha_p_"):].replace("__", "/"): T(g[k]) for k in g.files if k.startswith("mha_p_")}
    y, a = O.mha(T(g["mha_x"]), pm, "mha", 2, True, None)
    np.testing.assert_allclose(y.numpy(), g["mha_out"], atol=1e-14)
    np.testing.assert_allclose(a.numpy(), g["mha_probs"], atol=1e-14)
    assert np.all(np.triu(g["mha_probs"][0, 0], 1) == 0)          # causal
    np.testing.assert_allclose(
        O.conv1d_same(T(g["conv_x"]), T(g["conv_w"]), T(g["conv_b"])).numpy(), g["conv_out"],
        atol=1e-13)
    np.testing.assert_allclose(O.maxpool2_same(T(g["conv_x"])).numpy(), g["pool_out"])
    loss = O.losses(T(g["loss_mel"]), T(g["loss_stop"]), T(g["loss_tgt"]), T(g["loss_tmask"]),
                    T(g["loss_done"]), T(g["loss_dmask"]))
    np.testing.assert_allclose([float(v) for v in loss], g["loss_out"], atol=1e-14)


def test_golden_even_kernel_same_padding_by_hand():
    """TF SAME with k=10: 4 zeros on the left, 5 on the right."""
    g = OPS
    x, w, b = g["conv_x"], g["conv_w"], g["conv_b"]
    xp = np.concatenate([np.zeros((2, 4, 3)), x, np.zeros((2, 5, 3))], axis=1)
    y = sum(xp[:, j:j + 7, :] @ w[j] for j in range(10)) + b
    np.testing.assert_allclose(y, g["conv_out"], atol=1e-12)
