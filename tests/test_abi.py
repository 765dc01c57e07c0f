"""CPU tests of the C-ABI boundary: the library loads, exports exactly what
include/pj.h declares, host-only entry points (sol_file writer) match the
oracle byte for byte, and the CLI's argument contract (:294-303) holds."""
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import ROOT

INF = 100000


def _declared():
    with open(os.path.join(ROOT, "include", "pj.h")) as f:
        text = f.read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w\s\*]+?\b(pj_\w+)\s*\(", text, re.M)))


def test_header_symbols_exported(pj):
    import ctypes
    lib = ctypes.CDLL(pj.LIB_PATH)
    names = _declared()
    assert len(names) >= 20
    for name in names:
        assert hasattr(lib, name), name
    assert set(names) == set(pj.EXPORTS)


def test_library_is_gfx950_code_object(pj):
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-S", pj.LIB_PATH],
                         capture_output=True, text=True)
    assert ".hip_fatbin" in out.stdout
    blob = open(pj.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_no_device_is_loud(pj):
    # In the CPU container there is no GPU: the product path must fail, not fall back.
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("GPU present")
    except ImportError:
        pass
    with pytest.raises(pj.PJError) as e:
        pj.Context(0)
    assert e.value.name == "PJ_ERR_NODEVICE"


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_format_sol_matches_oracle(pj, oracle, seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(0, 50000))
    d = rng.integers(0, 200000, n).astype(np.int32)
    d[rng.random(n) < 0.3] = INF
    assert pj.format_sol(d) == oracle.format_sol(d)


def test_write_sol(pj, oracle, tmp_path):
    rng = np.random.default_rng(5)
    d = rng.integers(0, 100001, 700_001).astype(np.int32)  # spans several writer chunks
    p = tmp_path / "sol.txt"
    pj.write_sol(d, str(p))
    assert p.read_bytes() == oracle.format_sol(d)
    # unopenable path: silent like the reference's ofstream (:617) unless strict
    pj.write_sol(d[:3], str(tmp_path / "no" / "such" / "dir.txt"))
    with pytest.raises(pj.PJError):
        pj.write_sol(d[:3], str(tmp_path / "no" / "such" / "dir.txt"), strict=True)
    pj.write_sol(np.zeros(0, np.int32), str(p))
    assert p.read_bytes() == b"the vector is:\n"


def test_cli_usage_contract(pj):
    for argv in ([], ["a"], ["a", "0"], ["a", "0", "b", "c"]):
        r = subprocess.run([pj.cli_path()] + argv, capture_output=True, text=True)
        assert r.returncode == 255
        assert r.stderr.splitlines() == [
            "to run this program must supply the following command line arguments (in order)",
            "argv[1]---web graph file.",
            "argv[2]---source node number.",
            "argv[3]---file to save the solution.",
        ]
        assert r.stdout == ""


def test_multi_handle_argument_and_device_errors(pj):
    """pj_multi_* on the host: bad arguments are PJ_ERR_ARG, and without a GPU the n-GPU
    handle fails loudly (no CPU fallback) instead of returning a handle."""
    import ctypes
    lib = ctypes.CDLL(pj.LIB_PATH)
    h = ctypes.c_void_p()
    assert lib.pj_multi_create(0, 0, ctypes.byref(h)) == -1  # n_gpus < 1
    assert lib.pj_multi_create(2, 7, ctypes.byref(h)) == -1  # unknown transport
    assert lib.pj_multi_create(1, 0, None) == -1
    assert lib.pj_multi_sssp(None, 0, None, None) == -1
    assert lib.pj_multi_info(None, None) == -1
    assert lib.pj_multi_destroy(None) == 0
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("GPU present")
    except ImportError:
        pass
    from paralleljohnson_amd.partition import Multi
    with pytest.raises(pj.PJError):
        Multi(2, "host")
