"""The drop-in boundary: libsstgpu.so loads on a GPU-less host, exports every
function include/sst.h declares, and fails loudly (no CPU fallback) when no
HIP device is visible.  CPU only."""
import ctypes
import os
import re
import shutil
import subprocess

import numpy as np
import pytest

from conftest import REPO
from spectrseqtools_amd import _native

HEADER = os.path.join(REPO, "include", "sst.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(sst_[a-z_]+)\s*\(", src)))


def test_header_and_exports_agree():
    assert header_functions() == sorted(_native.EXPORTS)


def test_library_exports_every_header_symbol():
    lib = _native.load_library()
    for name in header_functions():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", _native.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (sst_\w+)", out))
    assert set(header_functions()) <= exported


def test_library_targets_gfx950(tmp_path):
    # llvm-objdump --offloading writes the code objects it lists next to its
    # input: run it on a copy in a scratch directory, not on the in-tree library
    lib = tmp_path / "libsstgpu.so"
    shutil.copyfile(_native.LIB_PATH, lib)
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", str(lib)],
                         capture_output=True, text=True, cwd=tmp_path)
    text = out.stdout + out.stderr
    if "gfx" not in text:  # older objdump: fall back to the raw bundle id string
        text = open(_native.LIB_PATH, "rb").read().decode("latin-1")
    assert "gfx950" in text


def test_no_cpu_fallback_without_device():
    lib = _native.load_library()
    if lib.sst_device_count() > 0:
        pytest.skip("a HIP device is visible")
    with pytest.raises(_native.EngineError):
        _native.Engine(0)
    h = ctypes.c_void_p()
    assert lib.sst_ctx_create(0, ctypes.byref(h)) != 0


def test_null_arguments_rejected():
    lib = _native.load_library()
    assert lib.sst_table_build(None, None, 0, 0, 32, None) < 0
    assert lib.sst_is_valid_batch(None, None, None, 0, 1e-5, 1e-3, None) < 0
    assert lib.sst_explain_batch(None, None, None, 0, 1e-5, 1e-3, None, 0, 1, 1, None) < 0
    assert lib.sst_result_stats(None, None) < 0
    assert lib.sst_profile_sample(None, 1) < 0
    assert lib.sst_last_error(None) == b"null context"


def test_budget_conversion():
    # the reference only tests `A > 0` and decrements by one (mass_explanation.py:166-172)
    assert _native._budget(np.inf) == -1
    assert _native._budget(None) == -1
    assert _native._budget(3) == 3
    assert _native._budget(2.5) == 3
    assert _native._budget(-2) == 0
    assert _native._budget(-np.inf) == 0
    arr, s = _native._mods([1, np.inf, 0], 3)
    assert arr.tolist() == [1, -1, 0] and s == 0


def test_library_matches_its_build_record():
    """The shipped libsstgpu.so is the one built from this tree's sources
    (spectrseqtools_amd/build_record.json: the Makefile writes it after every
    link; the loader refuses a library or sources that no longer match)."""
    import json
    import os

    from spectrseqtools_amd import build_record

    if not os.path.exists(build_record.LIB):
        pytest.skip("libsstgpu.so not built")
    assert build_record.check() is None, build_record.check()
    rec = json.load(open(build_record.RECORD))
    assert rec["arch"] == "gfx950" and rec["library"]["bytes"] == os.path.getsize(build_record.LIB)
    assert set(rec["sources"]) >= {"spectrseqtools_amd/csrc/sst_kernels.hip", "include/sst.h"}
