"""MI355X-native Self-attention Tacotron teacher-forced training path.

Import name: ``sat_amd`` (the directory name is not a Python identifier; ``_sat_path.load()``
registers it).  The hot path runs in ``libsat_hip.so`` (hand-written HIP for gfx950, C-ABI in
``include/sat_abi.h``); this package is the host side that mirrors the reference's plugin
surface (hparams, ``attention_mechanism_factory``, factories, ``model_fn``).
"""

__version__ = "0.1.0"
