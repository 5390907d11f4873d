"""Model plugin surface: encoder / decoder / model factories and ``model_fn``.

Mirrors models/models.py:20-378: ``encoder_factory(params, is_training)``,
``decoder_factory(params)``, ``tacotron_model_factory(hparams, model_dir, run_config,
warm_start_from=None)`` keyed by the ``hparams.encoder`` / ``decoder`` / ``tacotron_model``
strings (unknown -> ``ValueError``, as the reference), and the Estimator-shaped
``DualSourceSelfAttentionTacotronModel`` whose ``model_fn(features, labels, mode, params)``
returns an ``EstimatorSpec``:

* TRAIN  -- one full training step on libsat_hip (masks drawn on the device, forward, BPTT,
  [RCCL all-reduce], clip_by_global_norm(1.0) + TF Adam + Noam decay), loss = 0.1 L1 + BCE
  (models/models.py:151-189);
* EVAL   -- ``loss`` of the validation decode (OneHotValidationHelper: softmax feedback, exactly
  T' steps with real attention; models/models.py:86-97) plus the teacher-forced
  ``loss_with_teacher`` metrics (models/models.py:208-235, 305-320); eval semantics (dropout off,
  zoneout blend, BatchNorm moving statistics);
* PREDICT -- free-running inference (BASELINE configs[4]; inference.FreeRunningDecoder: the
  stop-token helper + the KV-cached incremental decoder self-attention), returning the
  reference's predictions dict (models/models.py:252-277).

``features`` / ``labels`` follow the reference's dataset records (``PreprocessedSourceData`` /
``PreprocessedTargetData``, datasets/codes/dataset.py:45-48; ``codes`` is the mel target for
LJSpeech/VCTK), as device tensors or numpy arrays.
"""

from __future__ import annotations

import os
from collections import namedtuple
from typing import Dict, Optional

import numpy as np
import torch

from . import dp
from . import params as PR
from .engine import Tacotron
from .train import StepGraphCache, Trainer


class ModeKeys:
    """tf.estimator.ModeKeys values."""
    TRAIN = "train"
    EVAL = "eval"
    PREDICT = "infer"


PreprocessedSourceData = namedtuple(
    "PreprocessedSourceData", ["id", "key", "source", "source_length", "text"])
PreprocessedTargetData = namedtuple(
    "PreprocessedTargetData", ["id", "key", "codes", "target_length", "done", "code_loss_mask",
                               "binary_loss_mask"])
# VCTK records (datasets/vctk/dataset.py:31-46): source carries speaker_id / age / gender, and
# the target is MelData with spec_loss_mask in place of code_loss_mask.
SourceData = namedtuple(
    "SourceData", ["id", "key", "source", "source_length", "speaker_id", "age", "gender", "text"])
MelData = namedtuple(
    "MelData", ["id", "key", "mel", "mel_width", "target_length", "done", "spec_loss_mask",
                "binary_loss_mask"])
EstimatorSpec = namedtuple("EstimatorSpec", ["mode", "loss", "train_op", "predictions",
                                             "eval_metric_ops"])


class SelfAttentionCBHGEncoder:
    """Configuration of modules/module.py:378-438 as built by encoder_factory
    (models/models.py:325-346); executed by libsat_hip inside the model step."""

    def __init__(self, is_training, **cfg):
        self.is_training = is_training
        self.config = cfg


class DualSourceTransformerDecoder:
    """Configuration of modules/module.py:1455-1562 as built by decoder_factory
    (models/models.py:349-368)."""

    def __init__(self, **cfg):
        self.config = cfg


def encoder_factory(params, is_training):
    if params.encoder == "SelfAttentionCBHGEncoder":
        return SelfAttentionCBHGEncoder(
            is_training, cbhg_out_units=params.cbhg_out_units,
            conv_channels=params.conv_channels, max_filter_width=params.max_filter_width,
            projection1_out_channels=params.projection1_out_channels,
            projection2_out_channels=params.projection2_out_channels,
            num_highway=params.num_highway,
            self_attention_out_units=params.self_attention_out_units,
            self_attention_num_heads=params.self_attention_num_heads,
            self_attention_num_hop=params.self_attention_num_hop,
            prenet_out_units=params.encoder_prenet_out_units,
            drop_rate=params.encoder_prenet_drop_rate,
            zoneout_factor_cell=params.zoneout_factor_cell,
            zoneout_factor_output=params.zoneout_factor_output,
            self_attention_drop_rate=params.self_attention_drop_rate)
    raise ValueError(f"Unknown encoder: {params.encoder}")


def decoder_factory(params):
    if params.decoder == "DualSourceTransformerDecoder":
        return DualSourceTransformerDecoder(
            prenet_out_units=params.decoder_prenet_out_units,
            drop_rate=params.decoder_prenet_drop_rate,
            attention_rnn_out_units=params.attention_out_units,
            decoder_version=params.decoder_version, decoder_out_units=params.decoder_out_units,
            num_mels=params.num_mels, outputs_per_step=params.outputs_per_step,
            max_iters=params.max_iters, n_feed_frame=params.n_feed_frame,
            zoneout_factor_cell=params.zoneout_factor_cell,
            zoneout_factor_output=params.zoneout_factor_output,
            self_attention_out_units=params.decoder_self_attention_out_units,
            self_attention_num_heads=params.decoder_self_attention_num_heads,
            self_attention_num_hop=params.decoder_self_attention_num_hop,
            self_attention_drop_rate=params.decoder_self_attention_drop_rate)
    raise ValueError(f"Unknown decoder: {params.decoder}")


def _to_device(x, dev, dtype):
    if isinstance(x, torch.Tensor):
        return x.to(device=dev, dtype=dtype)
    return torch.as_tensor(np.asarray(x), dtype=dtype, device=dev)


class _PinnedStager:
    """Host -> device upload of a batch without a host-side wait.  A pageable ``as_tensor(...,
    device=)`` blocks the host until the stream has drained (a synchronous copy), so the next
    step's launches only start once the GPU is idle.  Here each array is packed into a pinned
    buffer and copied with ``non_blocking=True`` in stream order; buffers rotate over a small
    ring and a slot is rewritten only after the copy that last read it has finished (its event),
    so the host runs ahead of the device by up to ``depth`` batches."""

    def __init__(self, depth: int = 3):
        self.depth = depth
        self.slots = [dict() for _ in range(depth)]     # name -> pinned uint8 buffer
        self.events = [None] * depth
        self.i = 0

    def upload(self, arrays, dev, dtypes):
        """arrays: name -> numpy / tensor; dtypes: name -> torch dtype.  Returns device tensors."""
        if not torch.cuda.is_available() or torch.device(dev).type != "cuda":
            return {k: _to_device(v, dev, dtypes[k]) for k, v in arrays.items()}
        slot, ev = self.slots[self.i], self.events[self.i]
        if ev is not None:
            ev.synchronize()                             # that slot's last copy is done
        out = {}
        for k, v in arrays.items():
            if isinstance(v, torch.Tensor) and v.is_cuda:
                out[k] = v.to(dtype=dtypes[k])
                continue
            h = torch.as_tensor(np.ascontiguousarray(np.asarray(v))).to(dtypes[k])
            nb = h.numel() * h.element_size()
            buf = slot.get(k)
            if buf is None or buf.numel() < nb:
                buf = torch.empty(max(nb, 1), dtype=torch.uint8, pin_memory=True)
                slot[k] = buf
            pin = buf[:nb].view(h.dtype).view(h.shape)
            pin.copy_(h)
            out[k] = torch.empty(h.shape, dtype=h.dtype, device=dev)
            out[k].copy_(pin, non_blocking=True)
        e = torch.cuda.Event()
        e.record()
        self.events[self.i] = e
        self.i = (self.i + 1) % self.depth
        return out


class DualSourceSelfAttentionTacotronModel:
    """Estimator-shaped model (models/models.py:20-320) over the libsat_hip engine."""

    def __init__(self, params, model_dir=None, config=None, warm_start_from=None,
                 device="cuda", seed: int = 1234,
                 init_values: Optional[Dict[str, np.ndarray]] = None,
                 graph_cache: Optional[int] = None, graph_t_quantum: Optional[int] = None):
        """``graph_cache``: captured training steps kept per padded batch shape (LRU; 0 = every
        TRAIN step eager; default SAT_GRAPH_CACHE or 0); ``graph_t_quantum``: pad T' to a
        multiple of it before the lookup (default SAT_GRAPH_T_QUANTUM or 0 = exact shapes;
        train.StepGraphCache).  Default eager: with the pinned asynchronous upload the eager
        drop-in path keeps the GPU busy (its host issue runs ahead of the device), and it
        measured as fast as the cache's steady state over ragged LJSpeech-like batches (bench
        ``drop_in_ragged_ljs``), without the cache's first-sighting capture cost."""
        encoder_factory(params, True)                        # name checks, as the reference
        if params.decoder not in ("DualSourceDecoder", "DualSourceTransformerDecoder"):
            raise AssertionError(f"decoder must be a dual-source decoder: {params.decoder}")
        decoder_factory(params)
        if params.use_speaker_embedding and params.use_external_speaker_embedding:
            raise AssertionError("only one of speaker_embedding / external_speaker_embedding")
        PR.resolve_dims(params)                              # shapes this build supports
        self.params = params
        self.model_dir = model_dir
        self.config = config
        if warm_start_from is not None:
            raise NotImplementedError("warm start from TF checkpoints is outside the hot path")
        self.engine = Tacotron(params, device, seed=seed, init_values=init_values)
        # data-parallel replicas start from rank 0's weights and statistics
        dp.broadcast_params(self.engine.params)
        dp.broadcast_params(self.engine.bn.buf)
        self._trainer: Optional[Trainer] = None
        self._graphs: Optional[StepGraphCache] = None
        self._stager = _PinnedStager()
        env = os.environ.get
        self.graph_cache = int(env("SAT_GRAPH_CACHE", "0") if graph_cache is None else graph_cache)
        self.graph_t_quantum = int(env("SAT_GRAPH_T_QUANTUM", "0") if graph_t_quantum is None
                                   else graph_t_quantum)
        # dropout / zoneout masks differ per replica (each rank's shard is its own batch)
        self._seed = seed + 1000003 * dp.rank()
        self._eval_decoder = None

    @staticmethod
    def learning_rate_decay(init_rate, global_step, step_factor):
        """models/models.py:283-287 (host form; the device form lives in sat_adam_step)."""
        warmup = 4000.0
        step = float(global_step * step_factor + 1)
        return init_rate * warmup ** 0.5 * min(step * warmup ** -1.5, step ** -0.5)

    def _batch(self, features, labels):
        dev = self.engine.device
        codes = labels.codes if hasattr(labels, "codes") else labels.mel
        cmask = (labels.code_loss_mask if hasattr(labels, "code_loss_mask")
                 else labels.spec_loss_mask)
        arrays = {"source": features.source, "source_length": features.source_length,
                  "mel": codes, "mel_mask": cmask, "done": labels.done,
                  "done_mask": labels.binary_loss_mask, "target_length": labels.target_length}
        if self.params.use_speaker_embedding:                 # models/models.py:69-70
            if getattr(features, "speaker_id", None) is None:
                raise ValueError("use_speaker_embedding=True needs features.speaker_id")
            arrays["speaker_id"] = features.speaker_id
        i64 = ("source", "source_length", "target_length", "speaker_id")
        dtypes = {k: torch.int64 if k in i64 else torch.float32 for k in arrays}
        return self._stager.upload(arrays, dev, dtypes)

    def _get_trainer(self, batch) -> Trainer:
        """ONE trainer (one optimiser state) for every batch shape: its mask views are re-pointed
        per shape inside one arena (Trainer.reshape), so memory stays flat over a stream of
        differently padded batches."""
        B, N = batch["source"].shape
        Tp = batch["mel"].shape[1] // self.params.outputs_per_step
        if self._trainer is None:
            self._trainer = Trainer(self.engine, B, N, Tp, seed=self._seed)
        return self._trainer

    def _predict(self, features) -> EstimatorSpec:
        """PREDICT (models/models.py:84-97, 252-277): free-running decode (inference.py) and
        the reference's predictions dict.  ``codes`` follows the fork's one-hot of the argmax
        over the feature bins of each frame (:99-100); ``mel`` is the raw decoder output
        (code_output_raw) the one-hot is taken from."""
        from .inference import FreeRunningDecoder
        dev = self.engine.device
        batch = {"source": _to_device(features.source, dev, torch.int64),
                 "source_length": _to_device(features.source_length, dev, torch.int64)}
        if self.params.use_speaker_embedding:
            if getattr(features, "speaker_id", None) is None:
                raise ValueError("use_speaker_embedding=True needs features.speaker_id")
            batch["speaker_id"] = _to_device(features.speaker_id, dev, torch.int64)
        out = FreeRunningDecoder(self.engine, max_iters=self.params.max_iters).run(batch)
        mel = out["mel"]
        codes = torch.zeros_like(mel)
        codes.scatter_(2, mel.argmax(dim=2, keepdim=True), 1.0)       # tf.one_hot(argmax)
        preds = {"id": features.id, "key": features.key, "codes": codes, "mel": mel,
                 "stop_token": out["stop"], "alignment": out["alignment1"],
                 "alignment2": out["alignment2"], "source": features.source,
                 "text": getattr(features, "text", None)}
        # decoder self-attention alignments (per hop, per head, transposed as :108-109), then
        # the encoder's (alignment5..8)
        dec = [a[:, h].transpose(1, 2) for a in out["decoder_self_alignments"]
               for h in range(a.shape[1])]
        for i, a in enumerate(dec[:2]):
            preds[f"alignment{3 + i}"] = a
        enc = [a[:, h].transpose(1, 2) for a in out["encoder_self_alignments"]
               for h in range(a.shape[1])]
        for i, a in enumerate(enc[:4]):
            preds[f"alignment{5 + i}"] = a
        preds = {k: v for k, v in preds.items() if v is not None}
        return EstimatorSpec(ModeKeys.PREDICT, loss=None, train_op=None, predictions=preds,
                             eval_metric_ops=None)

    def forced_alignment_pass(self, batch) -> Dict[str, object]:
        """``use_forced_alignment_mode`` (models/models.py:84-97, 118-148): a teacher-forced
        validation pass (eval semantics; equal to the training-branch decoder by
        modules/transformer_test.py:44-90) yields the alignment histories, then a second pass
        decodes with ``force_alignment_dual_source_attention_factory`` mechanisms
        (TeacherForcing*Attention replaying those alignments) under
        ``OneHotValidationHelper(teacher_forcing=False)`` (softmax feedback, exactly T' steps).
        Returns the second pass's outputs (the ones the reference's loss and predictions use)
        with its alignment histories [B, N, T'] and the teacher-forced first pass's."""
        from .attentions import force_alignment_dual_source_attention_factory
        from .inference import FreeRunningDecoder
        hp = self.params
        kinds = (hp.forced_alignment_attention, hp.forced_alignment_attention2)
        for k in kinds:
            if k not in ("teacher_forcing_forward", "teacher_forcing_additive"):
                raise ValueError(f"forced_alignment_attention must be a teacher_forcing kind: {k}")
        force_alignment_dual_source_attention_factory(hp)          # option checks
        with torch.no_grad():
            first, _ = self.engine.forward(batch, None, training=False, need_grad=False)
            a1 = first["alignment1"].permute(1, 0, 2).contiguous()    # [B, T', N]
            a2 = first["alignment2"].permute(1, 0, 2).contiguous()
            dec = FreeRunningDecoder(self.engine, forced_alignments=(a1, a2), feed="softmax")
            out = dec.run(batch)
        out["teacher_alignment1"] = a1.transpose(1, 2)
        out["teacher_alignment2"] = a2.transpose(1, 2)
        return out

    def _loss_of(self, mel, stop, batch):
        """0.1 * codes_loss + binary_loss (models/models.py:159-173) of a decode's outputs."""
        from . import kernels as K
        loss = torch.zeros(8, device=mel.device)
        K.loss_fwd_bwd(mel.contiguous(), batch["mel"], batch["mel_mask"], stop.contiguous(),
                       batch["done"], batch["done_mask"], loss)
        return loss

    def validation_pass(self, batch) -> Dict[str, object]:
        """EVAL's own decode (models/models.py:86-97 with is_validation=True,
        teacher_forcing=False): OneHotValidationHelper (modules/helpers.py:61-108) -- exactly
        T' = T/r steps with real attention, step t+1 fed the per-frame softmax of step t's
        output."""
        from .inference import FreeRunningDecoder
        if self._eval_decoder is None:
            self._eval_decoder = FreeRunningDecoder(self.engine, helper="validation",
                                                    feed="softmax")
        return self._eval_decoder.run(batch)

    def _eval(self, batch) -> EstimatorSpec:
        """EVAL (models/models.py:84-97, 151-173, 208-235, 305-320):
        * ``loss`` / ``code_loss`` / ``done_loss`` of the validation decode (softmax feedback,
          T' steps; under ``use_forced_alignment_mode`` the forced second pass instead);
        * ``loss_with_teacher`` / ``code_loss_with_teacher`` / ``done_loss_with_teacher`` of the
          teacher-forced pass (validation with teacher forcing, equal to the training branch
          in eval mode by modules/transformer_test.py:44-90)."""
        hp = self.params
        with torch.no_grad():
            if getattr(hp, "use_forced_alignment_mode", False):
                out = self.forced_alignment_pass(batch)
            else:
                out = self.validation_pass(batch)
            l = self._loss_of(out["mel"], out["stop"], batch)
            teach, _ = self.engine.forward(batch, None, training=False, need_grad=False)
        code_loss, done_loss = 0.1 * l[1:2], l[2:3]
        loss = code_loss + done_loss                                  # + regularization (0)
        metrics = {"code_loss": code_loss, "done_loss": done_loss,
                   "loss_with_teacher": teach["loss"],
                   "code_loss_with_teacher": 0.1 * teach["l1"],
                   "done_loss_with_teacher": teach["bce"],
                   "alignment1": out["alignment1"], "alignment2": out["alignment2"]}
        return EstimatorSpec(ModeKeys.EVAL, loss=loss, train_op=None,
                             predictions={"mel": out["mel"], "stop_token": out["stop"]},
                             eval_metric_ops=metrics)

    def model_fn(self, features, labels, mode, params=None) -> EstimatorSpec:
        if mode == ModeKeys.PREDICT:
            return self._predict(features)
        batch = self._batch(features, labels)
        if mode == ModeKeys.TRAIN:
            # one captured step per padded batch shape, replayed when the shape comes back
            # (train.StepGraphCache; eager on a first sighting or with graph_cache=0)
            tr = self._get_trainer(batch)
            if self._graphs is None:
                self._graphs = StepGraphCache(tr, self.graph_cache, self.graph_t_quantum)
            out = self._graphs.step(batch)
            return EstimatorSpec(mode, loss=out["loss"], train_op=tr.global_step,
                                 predictions=None, eval_metric_ops=None)
        if mode == ModeKeys.EVAL:
            return self._eval(batch)
        raise ValueError(f"Unknown mode: {mode}")

    # ---- tf.estimator.Estimator-like drivers
    def predict(self, input_fn):
        for features, _ in input_fn():
            yield self.model_fn(features, None, ModeKeys.PREDICT, self.params).predictions

    def train(self, input_fn, steps: int):
        loss = None
        it = iter(input_fn())
        for _ in range(steps):
            features, labels = next(it)
            loss = self.model_fn(features, labels, ModeKeys.TRAIN, self.params).loss
        return loss

    def evaluate(self, input_fn, steps: int = 1):
        tot = 0.0
        it = iter(input_fn())
        for _ in range(steps):
            features, labels = next(it)
            tot += float(self.model_fn(features, labels, ModeKeys.EVAL, self.params).loss.item())
        return {"loss": tot / steps}


def tacotron_model_factory(hparams, model_dir, run_config, warm_start_from=None, **kw):
    if hparams.tacotron_model == "DualSourceSelfAttentionTacotronModel":
        return DualSourceSelfAttentionTacotronModel(hparams, model_dir, config=run_config,
                                                    warm_start_from=warm_start_from, **kw)
    raise ValueError(f"Unknown Tacotron model: {hparams.tacotron_model}")


def synthetic_input_fn(params, batch_size: int, N: int = 200, T: int = 1000, shape="max",
                       seed: int = 0):
    """An input_fn over seeded synthetic batches with the dataset contract of SURVEY.md 8(d)."""
    from . import data

    def input_fn():
        step = 0
        while True:
            b = data.synthetic_batch(params, batch_size, N=N, T=T, seed=seed + step, shape=shape)
            step += 1
            ids = np.arange(batch_size)
            if "speaker_id" in b:
                yield (SourceData(ids, ids, b["source"], b["source_length"], b["speaker_id"],
                                  None, None, None),
                       MelData(ids, ids, b["mel"], params.num_mels, b["target_length"],
                               b["done"], b["mel_mask"], b["done_mask"]))
                continue
            yield (PreprocessedSourceData(ids, ids, b["source"], b["source_length"], None),
                   PreprocessedTargetData(ids, ids, b["mel"], b["target_length"], b["done"],
                                          b["mel_mask"], b["done_mask"]))
    return input_fn
