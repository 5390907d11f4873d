"""The C-ABI boundary without a GPU: libsat_hip.so loads, exports every function that
include/sat_abi.h declares, the ctypes binding covers exactly that set, and the ctypes structs
match the C struct sizes.  No device call is made."""
import ctypes
import os
import re

import pytest

import _sat_path  # noqa: E402

_sat_path.load()
from sat_amd import _lib  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _lib_built():
    return os.path.exists(_lib.LIB_PATH)


def test_header_declares_and_binding_covers_the_same_set():
    h = _lib.header_symbols()
    assert len(h) >= 30
    assert h == _lib.bound_symbols()


@pytest.mark.skipif(not _lib_built(), reason="libsat_hip.so not built (run __graft_entry__.build())")
def test_library_exports_every_header_symbol():
    missing = _lib.header_symbols() - _lib.exported_symbols()
    assert not missing, missing
    lib = _lib.load()
    assert lib.sat_version() > 0
    # the binding's struct layout == the header's == the library's
    import re
    hdr = open(_lib.HEADER_PATH).read()
    assert int(re.search(r"#define SAT_ABI_VERSION (\d+)", hdr).group(1)) == _lib.ABI_VERSION
    assert lib.sat_abi_version() == _lib.ABI_VERSION
    # host-only queries (no device touched)
    assert lib.sat_workspace_adam() > 0
    assert lib.sat_workspace_colreduce(1000, 256) > 0
    assert lib.sat_attn_part_stride(256, 32) >= 8 + 256 + 32
    assert lib.sat_attn_pg_stride(224, 32, 5, 10) % 4 == 0


def _c_sizeof(struct):
    """sizeof(struct) as the C compiler sees include/sat_abi.h (gcc, host only)."""
    import subprocess
    import tempfile
    src = f'#include "sat_abi.h"\n#include <stdio.h>\nint main(){{printf("%zu", sizeof({struct}));}}\n'
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "s.c")
        open(c, "w").write(src)
        exe = os.path.join(d, "s")
        subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", exe], check=True)
        return int(subprocess.run([exe], capture_output=True, text=True, check=True).stdout)


STRUCTS = ["SatGemmDesc", "SatLstmFwd", "SatLstmBwd", "SatAttnStep", "SatAttnStepBwd",
           "SatAttnParamGrad", "SatDecAttnFwd", "SatDecAttnBwd", "SatDecLstmFwd",
           "SatDecLstmBwd", "SatEncLstmFwd", "SatEncLstmBwd", "SatAdamConfig", "SatConvBank", "SatMha", "SatDims", "SatRngSegment", "SatColSegment",
           "SatDecoderLoopFwd", "SatDecoderLoopBwd", "SatDecodePersistent"]


def _c_offsets(struct, fields):
    """offsetof every field as gcc lays out include/sat_abi.h."""
    import subprocess
    import tempfile
    body = "".join(f'printf("%zu\\n", offsetof({struct}, {f}));' for f in fields)
    src = (f'#include "sat_abi.h"\n#include <stdio.h>\n#include <stddef.h>\n'
           f'int main(){{{body}}}\n')
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "s.c")
        open(c, "w").write(src)
        exe = os.path.join(d, "s")
        subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", exe], check=True)
        out = subprocess.run([exe], capture_output=True, text=True, check=True).stdout
    return [int(x) for x in out.split()]


@pytest.mark.parametrize("name", STRUCTS)
def test_ctypes_structs_match_c_layout(name):
    st = getattr(_lib, name)
    assert ctypes.sizeof(st) == _c_sizeof(name)
    fields = [f for f, _ in st._fields_ if not f.startswith("pad")]
    assert [getattr(st, f).offset for f in fields] == _c_offsets(name, fields)


def test_errors_are_reported_not_swallowed():
    """A bad argument returns an error code and a message; check() raises (no silent fallback)."""
    if not _lib_built():
        pytest.skip("libsat_hip.so not built")
    lib = _lib.load()
    d = _lib.SatAttnStepBwd()   # all-zero sizes
    rc = lib.sat_attn_step_bwd(ctypes.byref(d), None)
    assert rc != 0
    assert b"sat_attn_step_bwd" in lib.sat_last_error_string()
    with pytest.raises(_lib.SatLibraryError):
        _lib.check(rc, "sat_attn_step_bwd")


def test_header_cites_reference_interfaces():
    text = open(os.path.join(ROOT, "include", "sat_abi.h")).read()
    cites = re.findall(r"[\w/]+\.py:\d+", text)
    assert len(cites) >= 10


def test_workspace_size_is_the_sum_of_the_entry_queries():
    """sat_workspace_size = every per-entry scratch query, 256-B aligned, + the
    32 MB GEMM split-K budget (host-only arithmetic: no GPU needed)."""
    if not _lib_built():
        pytest.skip("libsat_hip.so not built")
    lib = _lib.load()
    B, N, Tp = 32, 200, 500
    d = _lib.SatDims(B, N, Tp, 4, 4, 256, 256, 2048)
    al = lambda n: (n + 255) // 256 * 256   # noqa: E731
    e, pt, qp, rdp, ya = (ctypes.c_int64() for _ in range(5))
    ctr = lib.sat_decoder_attention_scratch(B, N, ctypes.byref(e), ctypes.byref(pt), ctypes.byref(qp))
    bctr = lib.sat_decoder_attention_bwd_scratch(B, N, ctypes.byref(rdp), ctypes.byref(ya))
    want = sum(al(4 * x) for x in (e.value, pt.value, qp.value, ctr, rdp.value, ya.value, bctr,
                                   lib.sat_decoder_lstms_scratch(B),
                                   lib.sat_decoder_lstms_bwd_scratch(B)))
    want += al(lib.sat_workspace_colreduce(B * Tp, 2048)) + al(lib.sat_workspace_loss()) + \
        al(lib.sat_workspace_adam())
    want += al(lib.sat_mha_scratch_bytes(B, N, 256, 4, 256)) + \
        al(lib.sat_mha_scratch_bytes(B, Tp, 256, 4, 256)) + (32 << 20)
    assert lib.sat_workspace_size(ctypes.byref(d)) == want
    assert lib.sat_workspace_size(ctypes.byref(_lib.SatDims())) < 0


def test_attn_param_grads_rejects_uncompiled_location_widths():
    """F outside the compiled variants is refused before any device work (it used to be read
    with the F = 8 variant's row stride)."""
    if not _lib_built():
        pytest.skip("libsat_hip.so not built")
    lib = _lib.load()
    d = _lib.SatAttnParamGrad()
    d.T, d.B, d.N, d.D1, d.D2, d.F, d.KW, d.att1_forward = 4, 2, 9, 224, 32, 3, 10, 1
    rc = lib.sat_attn_param_grads(ctypes.byref(d), None)
    assert rc != 0
    assert b"location features" in lib.sat_last_error_string()


def test_attn_param_grads_rejects_bad_step_split():
    """tsplit outside 0..8, or above T (an empty step range), is refused before device work."""
    if not _lib_built():
        pytest.skip("libsat_hip.so not built")
    lib = _lib.load()
    for T, ts in ((4, 9), (3, 4), (8, -1)):
        d = _lib.SatAttnParamGrad()
        d.T, d.B, d.N, d.D1, d.D2, d.F, d.KW, d.att1_forward = T, 2, 9, 224, 32, 5, 10, 1
        d.tsplit = ts
        rc = lib.sat_attn_param_grads(ctypes.byref(d), None)
        assert rc != 0
        assert b"tsplit" in lib.sat_last_error_string()


def test_mha_bwd_weight_gradients_all_or_none():
    """sat_mha_bwd refuses a descriptor with only some of the four weight gradients set (all of
    them: inline; none: deferred to sat_mha_bwd_wgrad), before any device work."""
    if not _lib_built():
        pytest.skip("libsat_hip.so not built")
    lib = _lib.load()
    d = _lib.SatMha()
    d.B, d.L, d.W, d.D, d.H, d.out_dim, d.causal = 2, 8, 16, 16, 2, 16, 0
    fake = ctypes.c_void_p(16)
    for f in ("x", "Wq", "Wk", "Wv", "Wo", "q", "k", "v", "P", "o", "dy", "dx", "scratch"):
        setattr(d, f, fake)
    d.scratch_bytes = 1 << 30
    d.dWq = fake                      # only one of four
    rc = lib.sat_mha_bwd(ctypes.byref(d), None)
    assert rc != 0
    assert b"all or none" in lib.sat_last_error_string()
    rc = lib.sat_mha_bwd_wgrad(ctypes.byref(_lib.SatMha()), None)
    assert rc != 0
