"""The C-ABI from plain C (examples/ikg_c_demo.c, built by the csrc Makefile):
no Python, torch or HIP headers in the caller.  CPU: the program links, reads
its inputs and fails loudly without a device.  GPU: it reproduces the
reference KATs (740 / 736 updates, q within 1e-12 of trajectory.json)."""
import ctypes as C
import json
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, PKG

DEMO = os.path.join(PKG, "ikgrasp", "_native", "ikg_c_demo")


def _row(d):
    return np.concatenate([np.array(d["R"], dtype=np.float64).reshape(9), np.array(d["t"], dtype=np.float64)])


def _inputs(tmp_path):
    from ikgrasp import _lib
    from ikgrasp.model import load_nextage
    d = _lib.model_desc(load_nextage())
    desc = tmp_path / "desc.bin"
    desc.write_bytes(bytes(memoryview(d)))
    with open(os.path.join(GOLDEN, "kat.json")) as f:
        kat = json.load(f)
    tg = np.stack([_row(kat["cube_placement"]), _row(kat["cube_placement_target"])])
    targets = tmp_path / "targets.bin"
    targets.write_bytes(tg.tobytes())
    return str(desc), str(targets), kat


def _run(*args):
    return subprocess.run([DEMO, *args], capture_output=True, text=True, timeout=120)


def test_demo_is_built_and_checks_inputs(tmp_path):
    assert os.access(DEMO, os.X_OK), "build with make -C <pkg>/csrc"
    r = _run(str(tmp_path / "missing.bin"), str(tmp_path / "missing.bin"))
    assert r.returncode == 2 and "bad input files" in r.stderr


def test_demo_fails_loudly_without_gpu(tmp_path):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    desc, targets, _ = _inputs(tmp_path)
    r = _run(desc, targets)
    assert r.returncode == 1 and "ikg_solve_batch" in r.stderr and r.stdout == ""


def _parse(out, nq=15):
    rows = [list(map(float, line.split())) for line in out.strip().splitlines()]
    conv = [int(r[0]) for r in rows]
    iters = [int(r[1]) for r in rows]
    q = np.array([r[4:4 + nq] for r in rows])
    return conv, iters, q


@pytest.mark.gpu
@pytest.mark.parametrize("extra", [[], ["f64", "specialize"]])
def test_demo_reproduces_kats(tmp_path, extra):
    desc, targets, kat = _inputs(tmp_path)
    r = _run(desc, targets, *extra)
    assert r.returncode == 0, r.stderr
    conv, iters, q = _parse(r.stdout)
    assert conv == [1, 1] and iters == [740, 736]
    assert np.abs(q[0] - np.array(kat["q0"])).max() <= 1e-12
    assert np.abs(q[1] - np.array(kat["qe"])).max() <= 1e-12


@pytest.mark.gpu
def test_demo_fp32(tmp_path):
    desc, targets, kat = _inputs(tmp_path)
    r = _run(desc, targets, "f32")
    assert r.returncode == 0, r.stderr
    conv, iters, q = _parse(r.stdout)
    assert conv == [1, 1] and abs(iters[0] - 740) <= 2 and abs(iters[1] - 736) <= 2
