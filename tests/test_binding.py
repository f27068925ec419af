"""The C-ABI's structure layouts and the reference-side binding
(examples/ikgrasp_binding.py) -- CPU only.

* A C probe of include/ikgrasp.h (tests/abi_probe.c, built with gcc) prints
  sizeof / offsetof of every field of ikg_model_desc, ikg_params,
  ikg_collision_desc and ikg_frame_kin_out; the ctypes structures of the
  product (ikgrasp/_lib.py) and of the binding must match them field by field.
* The binding's descriptors, built from a RobotWrapper-shaped robot
  (tests/fake_pinocchio.py: Pinocchio 3 `Frame.parentJoint` and 2.x
  `Frame.parent`), equal the product's compiled tables byte for byte.
"""
import ctypes as C
import importlib
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def probe(tmp_path_factory):
    exe = tmp_path_factory.mktemp("abi") / "abi_probe"
    subprocess.run(["gcc", "-std=c99", "-Wall", "-I", os.path.join(ROOT, "include"), "-o", str(exe),
                    os.path.join(ROOT, "tests", "abi_probe.c")], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout
    lay = {}
    for ln in out.splitlines():
        s, f, off, size = ln.split()
        lay.setdefault(s, {})[f] = (int(off), int(size))
    return lay


@pytest.fixture(scope="module")
def binding():
    from ikgrasp import config, tools
    saved = {k: sys.modules.get(k) for k in ("config", "tools")}
    sys.modules["config"], sys.modules["tools"] = config, tools  # the reference's modules, same names
    sys.path.insert(0, os.path.join(ROOT, "examples"))
    try:
        yield importlib.import_module("ikgrasp_binding")
    finally:
        sys.path.remove(os.path.join(ROOT, "examples"))
        for k, v in saved.items():
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v


def _check(struct, lay, rename=None):
    rename = rename or {}
    assert C.sizeof(struct) == lay["SIZEOF"][0], (struct.__name__, C.sizeof(struct), lay["SIZEOF"])
    names = [f[0] for f in struct._fields_]
    assert sorted(rename.get(n, n) for n in names) == sorted(k for k in lay if k != "SIZEOF")
    for n in names:
        fd = getattr(struct, n)
        assert (fd.offset, fd.size) == lay[rename.get(n, n)], (struct.__name__, n)


def test_product_structs_match_the_c_layout(probe):
    from ikgrasp import _lib
    _check(_lib.ModelDesc, probe["ikg_model_desc"])
    _check(_lib.Params, probe["ikg_params"], {"lambda_": "lambda"})
    _check(_lib.CollisionDesc, probe["ikg_collision_desc"])
    _check(_lib.FrameKinOut, probe["ikg_frame_kin_out"])


def test_binding_structs_match_the_c_layout(probe, binding):
    _check(binding.Desc, probe["ikg_model_desc"])
    _check(binding.Params, probe["ikg_params"], {"lam": "lambda"})
    _check(binding.CDesc, probe["ikg_collision_desc"])
    _check(binding.FKOut, probe["ikg_frame_kin_out"])


@pytest.mark.parametrize("pin2", [False, True])
def test_binding_descriptors_equal_the_compiled_tables(binding, pin2):
    from fake_pinocchio import nextage_wrapper
    from ikgrasp import _lib
    from ikgrasp.collision import load_nextage_scene
    from ikgrasp.model import load_nextage
    robot, cube = nextage_wrapper(pin2)
    assert bytes(binding._desc(robot, cube)) == bytes(_lib.model_desc(load_nextage()))
    cd = _lib.collision_desc(load_nextage_scene())
    assert bytes(binding._cdesc(robot)) == bytes(cd)
    assert cd.target_geom == cd.n_geoms - 1  # setcubeplacement's geometryObjects[-1]
