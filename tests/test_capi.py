"""CPU: the C-ABI library loads and exports exactly what include/adaptive_amd.h declares, and the
host-side queries (no device work) behave.  No compute calls: there is no GPU here."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "adaptive_amd.h")


def header_functions():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"AA_API\s+[\w\s\*]+?\b(aa_\w+)\s*\(", text)))


@pytest.fixture(scope="module")
def lib():
    from adaptive_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        subprocess.run(["make", "-C", os.path.join(ROOT, "adaptive_amd", "csrc")], check=True)
    return _lib.load()


def test_header_declares_expected_entry_points():
    fns = header_functions()
    for f in ("aa_pack_weights", "aa_encoder_tail", "aa_decode_step", "aa_greedy_decode", "aa_synth_uniform"):
        assert f in fns


def test_library_exports_every_header_symbol(lib):
    from adaptive_amd import _lib
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\sT\s+(aa_\w+)", out))
    assert set(header_functions()) == exported, (set(header_functions()) ^ exported)
    assert set(_lib.SIGNATURES) == exported


def test_dims_and_sizes(lib):
    from adaptive_amd import _lib
    d = _lib.Dims(256, 512, 10123, 2048, 49)
    assert lib.aa_abi_version() == _lib.ABI_VERSION
    assert lib.aa_check_dims(d) == 0
    assert lib.aa_check_dims(_lib.Dims(256, 500, 10123, 2048, 49)) == -2   # hidden % 256
    assert lib.aa_check_dims(_lib.Dims(256, 384, 10123, 2048, 49)) == -2
    assert lib.aa_check_dims(_lib.Dims(256, 512, 10123, 2048, 36)) == -2   # spatial must be 49
    assert lib.aa_packed_bytes(_lib.Dims(256, 500, 10123, 2048, 49)) == 0
    pk = lib.aa_packed_bytes(d)
    # packed weights: encoder tail + decoder + the 104 MB per-token LSTM-input table + bf16 W_m copy
    # incl. the 31.5 MB bf16x3 copy of W_m for beam search and the fragment-order bf16x3 encoder
    # weights of k_enc_v4 / k_enc_heads3 (22 MB)
    assert 215e6 < pk < 235e6
    ws = lib.aa_decode_workspace_bytes(d, 512, 20)
    assert ws > 512 * 49 * 512 * 4  # holds V
    assert lib.aa_decode_workspace_bytes(d, 0, 20) == 0
    assert lib.aa_step_workspace_bytes(d, 4) > 0


def test_argument_errors_without_device_work(lib):
    from adaptive_amd import _lib
    assert lib.aa_greedy_decode(None, None, 1, 1, None, None, None, None, 0, None, 0, None) == -1
    m = _lib.Model(_lib.Dims(256, 512, 10123, 2048, 49), 256, 10)  # fake aligned pointer, too small
    assert lib.aa_greedy_decode(m, None, 1, 1, None, None, None, None, 0, None, 0, None) == -4
    m = _lib.Model(_lib.Dims(256, 512, 10123, 2048, 49), 256 + 16, 10 ** 9)
    assert lib.aa_greedy_decode(m, None, 1, 1, None, None, None, None, 0, None, 0, None) == -5  # 256-B alignment
    m = _lib.Model(_lib.Dims(256, 512, 10123, 2048, 49), 256, 10 ** 9)
    assert lib.aa_greedy_decode(m, None, -1, 1, None, None, None, None, 0, None, 0, None) == -3
    assert lib.aa_greedy_decode(m, None, 0, 20, None, None, None, None, 0, None, 0, None) == 0   # empty batch
    assert lib.aa_greedy_decode(m, None, 4, 20, None, None, None, None, 0, None, 0, None) == -1
    assert b"too small" in lib.aa_error_string(-4)
    # the two-stream form: same argument checks
    assert lib.aa_greedy_decode_aux(m, None, -1, 1, None, None, None, None, 0, None, 0, None, None) == -3
    assert lib.aa_greedy_decode_aux(m, None, 0, 20, None, None, None, None, 0, None, 0, None, None) == 0
    assert lib.aa_greedy_decode_aux(m, 256, 4, 20, None, None, None, 256, 10 ** 9, None, 0, None, None) == -1
    # decode plans: shape and pointer checks before any capture
    h = ctypes.c_void_p()
    assert lib.aa_decode_plan_create(m, 256, 0, 20, 256, None, None, 256, 10 ** 9, 0, ctypes.byref(h)) == -3
    assert lib.aa_decode_plan_create(m, None, 4, 20, 256, None, None, 256, 10 ** 9, 0, ctypes.byref(h)) == -1
    assert lib.aa_decode_plan_create(m, 256, 4, 20, 256, None, None, 256, 10 ** 9, 0, None) == -1
    assert h.value is None


def test_product_path_fails_loudly_without_library(monkeypatch, tmp_path):
    from adaptive_amd import _lib
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "missing.so"))
    with pytest.raises(RuntimeError, match="no CPU fallback|not built"):
        _lib.load()
