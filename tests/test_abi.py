"""CPU: the C-ABI library builds for gfx950, loads, and exports every symbol
include/sw_amd.h declares; host-side entry points behave (no GPU needed)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import REPO


def declared_functions():
    src = open(os.path.join(REPO, "include", "sw_amd.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    pat = r"^\s*(?:SW_API\s+)?(?:int|int32_t|void\s*\*|const char\s*\*)\s*(sw_\w+)\s*\("
    return sorted(set(re.findall(pat, src, re.M)))


def test_only_the_c_abi_is_exported(sw):
    out = subprocess.run(["nm", "-D", "--defined-only", sw.capi.LIB_PATH], capture_output=True, text=True).stdout
    text = [ln.split()[-1] for ln in out.splitlines() if " T " in ln]
    assert sorted(text) == declared_functions()


def test_header_symbols_exported(sw):
    names = declared_functions()
    assert len(names) >= 18
    L = sw.capi.lib()
    for n in names:
        assert hasattr(L, n), n
    assert sorted(sw.capi.EXPORTED) == names
    out = subprocess.run(["nm", "-D", "--defined-only", sw.capi.LIB_PATH], capture_output=True, text=True).stdout
    for n in names:
        assert re.search(r"\bT %s$" % n, out, re.M), n


def test_library_has_gfx950_code_object(sw):
    data = open(sw.capi.LIB_PATH, "rb").read()
    assert b"gfx950" in data
    assert b"sw_inter" in data and b"sw_intra" in data


def test_encode_matches_oracle(sw, oracle):
    allb = bytes(range(1, 256))
    assert np.array_equal(sw.encode(allb), oracle.encode(allb))


def test_builtin_matrices_match_oracle(sw, oracle):
    for mid in (0, 1, 2, 3):
        assert np.array_equal(sw.builtin_matrix(mid), oracle.matrix(mid))
    with pytest.raises(sw.SWError):
        sw.builtin_matrix(7)


def test_topk(sw):
    s = np.array([5, 9, 9, 1, 7, 9], dtype=np.int32)
    ids, vals = sw.topk(s, 4)
    assert ids.tolist() == [1, 2, 5, 4] and vals.tolist() == [9, 9, 9, 7]
    ids, vals = sw.topk(s[:2], 4)
    assert ids.tolist() == [1, 0, -1, -1]


def test_null_arguments_are_errors_not_crashes(sw):
    L = sw.capi.lib()
    assert L.sw_create(0, None) == -1
    assert L.sw_db_create(None, None, None, 0, None, None) == -1
    assert L.sw_scan(None, None, None, 0, None, None) == -1
    assert L.sw_get_timing(None, None) == -1
    assert L.sw_destroy(None) == 0
    assert "null" in L.sw_last_error().decode()


def test_no_device_is_reported(sw):
    torch = pytest.importorskip("torch")
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(sw.SWError, match="-4"):
        sw.Handle(0)


def test_version(sw):
    assert sw.capi.lib().sw_version() >= 100
