"""Hyper-parameter surface, drop-in for the reference's ``hparams`` object.

The reference builds one global ``tf.contrib.training.HParams`` (``hparams.py:11-225``) and
overrides it in two layers: ``hparams.parse_json(open(json).read())`` then
``hparams.parse("k=v,...")`` (``train.py:110-115``).  This module keeps the same key names, the
same defaults and the same precedence, without TensorFlow:

* ``HParams(**defaults)`` -- attribute access, ``values()``, ``set_hparam``, ``override_from_dict``;
* ``parse_json(text)``     -- unknown keys raise ``KeyError`` like TF ``set_hparam``;
* ``parse("a=1,b=[1,2]")`` -- values are coerced to the type of the default (TF semantics:
  an int default accepts only ints, a float default accepts ints, bools accept true/false).

The defaults below are grouped by subsystem.  Values and names follow ``hparams.py:13-222``;
keys that only the reference's out-of-scope subsystems read are kept so that every
``examples/*/*.json`` and every ``--hparams`` string the reference accepts is accepted here.
"""

from __future__ import annotations

import ast
import json
from typing import Any, Dict

# --- audio / features  (hparams.py:13-42) ------------------------------------------------------
_AUDIO = {
    "num_mels": 1025, "num_mgcs": 60, "num_freq": 2049, "sample_rate": 48000,
    "frame_length_ms": 50.0, "frame_shift_ms": 12.5, "ref_level_db": 20,
    "average_mel_level_db": [0.0], "stddev_mel_level_db": [0.0], "min_mel_level_db": [0.0],
    "silence_mel_level_db": -3.0,
    "mgc_dim": 60, "mgc_alpha": 0.77, "mgc_gamma": 0.0, "mgc_fft_len": 4096,
    "num_lf0s": 256, "f0_max": 529.0, "f0_min": 66.0, "lf0_loss_factor": 0.5,
}

# --- dataset / model selection  (hparams.py:38-52) ----------------------------------------------
_DATA = {
    "dataset": "codes.dataset.DatasetSource", "num_symbols": 256, "source": "phone",
    "source_file_extension": "source.tfrecord", "target_file_extension": "target.tfrecord",
    "tacotron_model": "DualSourceSelfAttentionTacotronModel",
    "outputs_per_step": 1, "n_feed_frame": 1, "embedding_dim": 256,
}

# --- accent embedding (hparams.py:55-61) -- not used by the LJSpeech/VCTK configs -------------
_ACCENT = {
    "use_accent_type": False, "accent_type_embedding_dim": 32, "num_accent_type": 129,
    "accent_type_offset": 0x3100, "accent_type_unknown": 0x3180,
    "accent_type_prenet_out_units": (32, 16), "encoder_prenet_out_units_if_accent": (224, 112),
}

# --- encoder (hparams.py:63-88) -----------------------------------------------------------------
_ENCODER = {
    "encoder": "SelfAttentionCBHGEncoder",
    "encoder_prenet_drop_rate": 0.5, "cbhg_out_units": 256, "conv_channels": 128,
    "max_filter_width": 16, "projection1_out_channels": 128, "projection2_out_channels": 128,
    "num_highway": 4, "encoder_prenet_out_units": (256, 128),
    "encoder_v2_num_conv_layers": 3, "encoder_v2_kernel_size": 5, "encoder_v2_out_units": 512,
    "encoder_v2_drop_rate": 0.5,
    "self_attention_out_units": 32, "self_attention_num_heads": 2, "self_attention_num_hop": 1,
    "self_attention_encoder_out_units": 32, "self_attention_drop_rate": 0.05,
    "self_attention_transformer_num_conv_layers": 1, "self_attention_transformer_kernel_size": 5,
}

# --- decoder + attention (hparams.py:90-122) ---------------------------------------------------
_DECODER = {
    "decoder": "DualSourceTransformerDecoder",
    "attention": "additive", "forced_alignment_attention": "teacher_forcing_additive",
    "attention2": "additive", "forced_alignment_attention2": "teacher_forcing_additive",
    "attention1_out_units": 224, "attention2_out_units": 32,
    "decoder_prenet_drop_rate": 0.5, "apply_dropout_on_inference": False,
    "decoder_prenet_out_units": (256, 128), "attention_out_units": 256, "decoder_out_units": 256,
    "attention_kernel": 31, "attention_filters": 32, "cumulative_weights": False,
    "use_forward_attention_transition_agent": False,
    "decoder_self_attention_out_units": 256, "decoder_self_attention_num_heads": 2,
    "decoder_self_attention_num_hop": 1, "decoder_self_attention_drop_rate": 0.05,
}

# --- speakers (hparams.py:124-135) ---------------------------------------------------------------
_SPEAKER = {
    "use_speaker_embedding": False, "use_external_speaker_embedding": False,
    "speaker_embedding_projection_out_dim": -1, "embedding_file": "",
    "num_speakers": 1, "speaker_embedding_dim": 16, "speaker_embedding_offset": 0,
    "speaker_for_synthesis": -1, "speaker_embedd_to_prenet": True,
    "speaker_embedd_to_decoder": False, "speaker_embedd_to_postnet": False,
}

# --- post-nets (hparams.py:137-151) -- no post-net is built by DualSourceSelfAttentionTacotronModel
_POSTNET = {
    "post_net_cbhg_out_units": 256, "post_net_conv_channels": 128, "post_net_max_filter_width": 8,
    "post_net_projection1_out_channels": 256, "post_net_projection2_out_channels": 80,
    "post_net_num_highway": 4, "use_postnet_v2": False, "num_postnet_v2_layers": 5,
    "postnet_v2_kernel_size": 5, "postnet_v2_out_channels": 512, "postnet_v2_drop_rate": 0.5,
}

# --- loss / training / eval / predict (hparams.py:153-202) -------------------------------------
_TRAIN = {
    "code_loss_type": "l1",
    "batch_size": 32, "adam_beta1": 0.9, "adam_beta2": 0.999, "adam_eps": 1e-8,
    "initial_learning_rate": 0.002, "decay_learning_rate": True, "learning_rate_step_factor": 1,
    "use_l2_regularization": False, "l2_regularization_weight": 1e-7,
    "save_summary_steps": 50, "save_checkpoints_steps": 50, "keep_checkpoint_max": 20000,
    "keep_checkpoint_every_n_hours": 1, "log_step_count_steps": 1, "alignment_save_steps": 50,
    "save_training_time_metrics": False, "approx_min_target_length": 100,
    "suffle_buffer_size": 64, "batch_bucket_width": 50, "batch_num_buckets": 50,
    "interleave_cycle_length_cpu_factor": 1.0, "interleave_cycle_length_min": 4,
    "interleave_cycle_length_max": 16, "interleave_buffer_output_elements": 200,
    "interleave_prefetch_input_elements": 200, "prefetch_buffer_size": 4,
    "use_cache": False, "cache_file_name": "", "logfile": "log.txt",
    "record_profile": False, "profile_steps": 50,
    "warm_start": False, "ckpt_to_initialize_from": "", "vars_to_warm_start": [".*"],
    "max_iters": 450, "num_evaluation_steps": 5, "keep_eval_results_max_epoch": 10,
    "eval_start_delay_secs": 120, "eval_throttle_secs": 600,
    "use_forced_alignment_mode": False, "predicted_mel_extension": "mfbsp",
}

# --- extensions / text front-end / preprocessing (hparams.py:204-222) --------------------------
_MISC = {
    "use_zoneout_at_encoder": False, "decoder_version": "v1",
    "zoneout_factor_cell": 0.1, "zoneout_factor_output": 0.1,
    "phoneme": "flite", "flite_binary_path": "", "phoneset_path": "",
    "trim_top_db": 30, "trim_frame_length": 1024, "trim_hop_length": 256, "num_silent_frames": 0,
}


def default_values() -> Dict[str, Any]:
    out: Dict[str, Any] = {}
    for group in (_AUDIO, _DATA, _ACCENT, _ENCODER, _DECODER, _SPEAKER, _POSTNET, _TRAIN, _MISC):
        out.update(group)
    return out


def _coerce(name: str, default: Any, value: Any) -> Any:
    """Cast ``value`` to the type of ``default`` the way TF HParams.set_hparam does."""
    if isinstance(default, bool):
        if isinstance(value, bool):
            return value
        if isinstance(value, str) and value.lower() in ("true", "false"):
            return value.lower() == "true"
        if isinstance(value, int) and value in (0, 1):
            return bool(value)
        raise ValueError(f"Could not cast {value!r} to bool for hparam {name}")
    if isinstance(default, int):
        if isinstance(value, bool) or not isinstance(value, int):
            if isinstance(value, float) and value.is_integer():
                return int(value)
            raise ValueError(f"Could not cast {value!r} to int for hparam {name}")
        return value
    if isinstance(default, float):
        if isinstance(value, bool) or not isinstance(value, (int, float)):
            raise ValueError(f"Could not cast {value!r} to float for hparam {name}")
        return float(value)
    if isinstance(default, (list, tuple)):
        if not isinstance(value, (list, tuple)):
            value = [value]
        if len(default) > 0:
            value = [_coerce(name, default[0], v) for v in value]
        return type(default)(value) if isinstance(default, tuple) else list(value)
    if isinstance(default, str):
        if not isinstance(value, str):
            raise ValueError(f"Could not cast {value!r} to str for hparam {name}")
        return value
    return value


class HParams:
    """Minimal TF1 ``HParams`` work-alike (attribute store with typed overrides)."""

    def __init__(self, **kwargs: Any) -> None:
        object.__setattr__(self, "_values", dict(kwargs))

    def __getattr__(self, name: str) -> Any:
        values = object.__getattribute__(self, "_values")
        if name in values:
            return values[name]
        raise AttributeError(name)

    def __setattr__(self, name: str, value: Any) -> None:
        self.set_hparam(name, value)

    def __contains__(self, name: str) -> bool:
        return name in self._values

    def values(self) -> Dict[str, Any]:
        return dict(self._values)

    def set_hparam(self, name: str, value: Any) -> None:
        if name not in self._values:
            raise KeyError(f"Unknown hparam: {name}")
        self._values[name] = _coerce(name, self._values[name], value)

    def add_hparam(self, name: str, value: Any) -> None:
        if name in self._values:
            raise ValueError(f"Hyperparameter name is reserved: {name}")
        self._values[name] = value

    def override_from_dict(self, values_map: Dict[str, Any]) -> "HParams":
        for name, value in values_map.items():
            self.set_hparam(name, value)
        return self

    def parse_json(self, values_json: str) -> "HParams":
        return self.override_from_dict(json.loads(values_json))

    def parse(self, values: str) -> "HParams":
        """``"a=1,b=[1,2],c=foo"`` -> typed overrides (train.py:115)."""
        for name, raw in _split_assignments(values):
            if name not in self._values:
                raise ValueError(f"Unknown hyperparameter type for {name}")
            self.set_hparam(name, _literal(raw))
        return self

    def copy(self) -> "HParams":
        return HParams(**{k: (list(v) if isinstance(v, list) else v) for k, v in self._values.items()})

    def __repr__(self) -> str:
        return f"HParams({len(self._values)} keys)"


def _literal(raw: str) -> Any:
    raw = raw.strip()
    if raw.lower() in ("true", "false"):
        return raw.lower() == "true"
    try:
        return ast.literal_eval(raw)
    except (ValueError, SyntaxError):
        return raw


def _split_assignments(text: str):
    """Split on top-level commas (commas inside [...] belong to list values)."""
    depth, cur, parts = 0, [], []
    for ch in text:
        if ch in "[(":
            depth += 1
        elif ch in "])":
            depth -= 1
        if ch == "," and depth == 0:
            parts.append("".join(cur))
            cur = []
        else:
            cur.append(ch)
    if "".join(cur).strip():
        parts.append("".join(cur))
    for p in parts:
        if "=" not in p:
            raise ValueError(f"Malformed hparam assignment: {p!r}")
        k, v = p.split("=", 1)
        yield k.strip(), v


def create_hparams(json_path: str | None = None, overrides: str | None = None) -> HParams:
    """defaults < JSON file < ``k=v`` string -- the precedence of ``train.py:110-115``."""
    hp = HParams(**default_values())
    if json_path:
        with open(json_path, "r", encoding="utf-8") as f:
            hp.parse_json(f.read())
    if overrides:
        hp.parse(overrides)
    return hp


# The reference exposes a module-level ``hparams`` singleton (hparams.py:11).
hparams = HParams(**default_values())


def hparams_debug_string(hp: HParams | None = None) -> str:
    values = (hp or hparams).values()
    return "Hyperparameters:\n" + "\n".join(f"  {k}: {values[k]}" for k in sorted(values))


# Hot-path overrides carried by examples/ljspeech/self-attention-tacotron.json (mel statistics
# omitted: they feed only the offline dataset normalisation, datasets/ljspeech/dataset.py:131).
LJSPEECH_SELF_ATTENTION_OVERRIDES = {
    "num_mels": 80, "num_freq": 1025, "sample_rate": 22050, "frame_length_ms": 50,
    "frame_shift_ms": 12.5, "initial_learning_rate": 0.0005, "outputs_per_step": 2,
    "max_iters": 500, "attention": "forward", "cumulative_weights": False,
    "attention_kernel": 10, "attention_filters": 5, "use_zoneout_at_encoder": True,
    "decoder_version": "v2", "dataset": "ljspeech.dataset.DatasetSource",
    "target_file_extension": "target.tfrecord", "save_checkpoints_steps": 379,
    "tacotron_model": "DualSourceSelfAttentionTacotronModel",
    "encoder": "SelfAttentionCBHGEncoder", "decoder": "DualSourceTransformerDecoder",
}

# examples/vctk/self-attention-tacotron.json adds multi-speaker keys on top of the same model.
VCTK_SELF_ATTENTION_OVERRIDES = dict(
    LJSPEECH_SELF_ATTENTION_OVERRIDES, num_freq=2049, sample_rate=48000, frame_length_ms=50.0,
    trim_top_db=10, dataset="vctk.dataset.DatasetSource", save_checkpoints_steps=1343,
    use_speaker_embedding=True, num_speakers=152, speaker_embedding_offset=225,
)


def ljspeech_hparams(**extra: Any) -> HParams:
    hp = HParams(**default_values()).override_from_dict(LJSPEECH_SELF_ATTENTION_OVERRIDES)
    return hp.override_from_dict(extra) if extra else hp


def vctk_hparams(**extra: Any) -> HParams:
    hp = HParams(**default_values()).override_from_dict(VCTK_SELF_ATTENTION_OVERRIDES)
    return hp.override_from_dict(extra) if extra else hp
