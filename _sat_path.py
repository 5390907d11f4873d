"""Register the ``self-attention-tacotron_amd/`` directory as the importable package ``sat_amd``."""

import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "self-attention-tacotron_amd")


def load():
    if "sat_amd" in sys.modules:
        return sys.modules["sat_amd"]
    spec = importlib.util.spec_from_file_location(
        "sat_amd", os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["sat_amd"] = mod
    spec.loader.exec_module(mod)
    return mod
