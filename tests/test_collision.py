"""Collision term of `success` on the CPU.

* the product's scene compiler (ikgrasp/collision.py) against the oracle's
  independent parse of the same URDF/SRDF (tests/golden/collision_scene.json);
* the collision oracle against the reference's KAT-5
  (`collision(robot, robot.q0) == True`, lab_instructions.ipynb:252/:262) and
  the KAT solutions (collision-free: their 740/736 iteration counts require
  the stop test to have passed there) and against its own frozen fixtures;
* the DEVICE narrow phase (ikg_collision.hpp stage functions: bounding-sphere
  broad phase, exact sphere tests, boolean GJK for boxes / cylinders) compiled
  for the host by the emulator (test tooling), against the oracle's answers
  (exact sphere/box, separating-axis box/box, GJK for cylinders);
* the collision-continuation semantics (inverse_geometry.py:70, :97-98)
  through the emulator against the oracle's full loop;
* C-ABI validation of ikg_model_set_collision (no GPU calls).

Collision parity beyond KAT-5 / the KAT solutions is pinned only to the
restated hpp-fcl semantics (no hpp-fcl outputs exist in the reference tree).
"""
import ctypes as C
import json
import os

import numpy as np

import helpers
import pytest

from conftest import GOLDEN
from ikgrasp import _lib
from ikgrasp.collision import load_nextage_scene
from ikgrasp.model import load_nextage
from oracle import collision_oracle as co

EMU = helpers.emu_path()


@pytest.fixture(scope="module")
def oscene():
    return co.load_scene(os.path.join(GOLDEN, "collision_scene.json"))


@pytest.fixture(scope="module")
def col_cases():
    return dict(np.load(os.path.join(GOLDEN, "collision_cases.npz")))


@pytest.fixture(scope="module")
def solve_cases():
    return dict(np.load(os.path.join(GOLDEN, "collision_solve_cases.npz")))


@pytest.fixture(scope="module")
def emu():
    if not os.path.exists(EMU):
        pytest.skip("libikgrasp_emu.so not built")
    lib = C.CDLL(EMU)
    vp = C.c_void_p
    lib.ikg_emu_solve.argtypes = [vp, C.c_int, vp, vp, C.c_int64, C.c_int64, vp, vp, vp, vp, vp, vp, C.c_int, vp]
    lib.ikg_emu_collision.argtypes = [vp, vp, C.c_int, vp, vp, C.c_int64, vp]
    md = _lib.model_desc(load_nextage())
    cd = _lib.collision_desc(load_nextage_scene())

    def collision(q, targets, dtype=0):
        npt = np.float64 if dtype == 0 else np.float32
        q = np.ascontiguousarray(q, dtype=npt).reshape(-1, 15)
        tg = np.ascontiguousarray(targets, dtype=npt).reshape(-1, 12)
        out = np.empty(len(q), np.uint8)
        lib.ikg_emu_collision(C.byref(md), C.byref(cd), dtype, q.ctypes.data, tg.ctypes.data, len(q),
                              out.ctypes.data)
        return out.astype(bool)

    def solve(targets, q0, dtype=0, **kw):
        npt = np.float64 if dtype == 0 else np.float32
        tg = np.ascontiguousarray(targets, dtype=npt).reshape(-1, 12)
        B = len(tg)
        q0 = np.ascontiguousarray(np.broadcast_to(q0, (B, 15)), dtype=npt)
        p = _lib.default_params(**kw)
        q = np.empty((B, 15), npt)
        conv = np.empty(B, np.uint8)
        it = np.empty(B, np.int32)
        err = np.empty((B, 2), npt)
        assert 0 == lib.ikg_emu_solve(C.byref(md), dtype, tg.ctypes.data, q0.ctypes.data, 15, B, C.byref(p), q.ctypes.data,
                          conv.ctypes.data, it.ctypes.data, err.ctypes.data, None, 0, C.byref(cd))
        return q, conv.astype(bool), it, err

    return collision, solve


def _row(R, t):
    return np.concatenate([np.asarray(R, dtype=np.float64).reshape(9), np.asarray(t, dtype=np.float64)])


# ---------------------------------------------------------------- scene
def test_product_scene_matches_oracle_parse(oscene):
    ps = load_nextage_scene()
    assert len(ps.geoms) == len(oscene["geoms"]) == 48
    for g, og in zip(ps.geoms, oscene["geoms"]):
        assert g.kind == og["kind"], g.name
        assert g.joint == og["joint"], g.name
        assert g.target == og["target"], g.name
        assert np.abs(g.R - og["R"]).max() <= 1e-12, g.name
        assert np.abs(g.t - og["t"]).max() <= 1e-12, g.name
        assert np.abs(g.dims - og["dims"]).max() <= 1e-12, g.name
    assert sorted(map(tuple, ps.pairs.tolist())) == sorted(oscene["pairs"])
    assert len(ps.pairs) == 745
    # setup_pinocchio.py:58: (obstacle, cube) = (46, 47); the cube is the target geometry
    assert (46, 47) in set(map(tuple, ps.pairs.tolist())) and ps.geoms[47].target


def test_translaterobot_quirk_reproduced():
    """setup_pinocchio.py:28-32 moves geometries 0 and 1 only."""
    ps = load_nextage_scene()
    assert ps.geoms[0].joint == -1 and ps.geoms[1].joint == -1
    # the four base spheres share one URDF height; only sphere 1 got the +0.85
    assert abs(ps.geoms[1].t[2] - ps.geoms[2].t[2] - 0.85) <= 1e-12
    assert all(abs(g.t[2] - ps.geoms[2].t[2]) <= 1e-12 for g in ps.geoms[3:5])
    assert ps.geoms[5].name == "WAIST_0" and ps.geoms[5].joint == -1 and ps.geoms[5].t[2] < 0.85


# ---------------------------------------------------------------- oracle pins
def test_oracle_kat5_and_kat_solutions(oscene, kat):
    cp, cpt = kat["cube_placement"], kat["cube_placement_target"]
    assert co.collision(oscene, np.zeros(15), np.array(cp["R"]), np.array(cp["t"]))  # KAT-5
    assert not co.collision(oscene, np.array(kat["q0"]), np.array(cp["R"]), np.array(cp["t"]))
    assert not co.collision(oscene, np.array(kat["qe"]), np.array(cpt["R"]), np.array(cpt["t"]))


def test_oracle_reproduces_its_fixtures(oscene, col_cases):
    c = col_cases
    for i in range(0, len(c["q"]), 37):
        R, t = c["targets"][i, :9].reshape(3, 3), c["targets"][i, 9:]
        assert co.collision(oscene, c["q"][i], R, t) == c["collision"][i], i


def test_oracle_gjk_agrees_with_sat_on_boxes():
    rng = np.random.default_rng(5)
    box = {"kind": co.BOX}
    agree = 0
    for _ in range(300):
        ha, hb = rng.uniform(0.02, 0.2, 3), rng.uniform(0.02, 0.2, 3)
        Ra, Rb = (np.linalg.qr(rng.normal(size=(3, 3)))[0] for _ in range(2))
        ta, tb = np.zeros(3), rng.uniform(-0.4, 0.4, 3)
        ga, gb = dict(box, dims=ha), dict(box, dims=hb)
        sat = co._box_box(Ra, ta, ha, Rb, tb, hb)
        gjk = co.gjk_intersect(lambda d: co.support(ga, Ra, ta, d), lambda d: co.support(gb, Rb, tb, d), ta - tb)
        agree += sat == gjk
    assert agree == 300


# ---------------------------------------------------------------- device stages on the host
def test_device_narrow_phase_matches_oracle_fp64(emu, col_cases):
    collision, _ = emu
    c = col_cases
    got = collision(c["q"], c["targets"])
    ok = c["robust64"].astype(bool)
    assert ok.sum() >= len(ok) - 2
    assert np.array_equal(got[ok], c["collision"][ok])
    assert c["collision"][0] and got[0]  # KAT-5


def test_device_narrow_phase_matches_oracle_fp32(emu, col_cases):
    collision, _ = emu
    c = col_cases
    got = collision(c["q"], c["targets"], dtype=1)
    ok = c["robust32"].astype(bool)
    assert np.array_equal(got[ok], c["collision"][ok])


def test_collision_semantics_loop_matches_oracle(emu, solve_cases, oracle_cases):
    _, solve = emu
    c = solve_cases
    q, ok, it, err = solve(c["targets"], c["q0"], check_collision=1)
    assert np.array_equal(ok, c["success"])
    assert np.array_equal(it, c["iters"])
    # every converged-but-colliding case ran on to max_iters (inverse_geometry.py:70)
    cont = oracle_cases["converged"] & ~c["success"]
    assert cont.sum() >= 5 and (it[cont] == 1000).all()
    s = c["success"]
    assert np.abs(q[s] - c["q"][s]).max() <= 1e-9
    assert np.abs(err[s] - c["err"][s]).max() <= 1e-10


def test_collision_semantics_kats(emu, kat):
    _, solve = emu
    tg = np.stack([_row(kat["cube_placement"]["R"], kat["cube_placement"]["t"]),
                   _row(kat["cube_placement_target"]["R"], kat["cube_placement_target"]["t"])])
    q, ok, it, err = solve(tg, np.zeros(15), check_collision=1)
    assert ok.all() and it.tolist() == [740, 736]
    assert np.abs(q[0] - kat["q0"]).max() <= 1e-12 and np.abs(q[1] - kat["qe"]).max() <= 1e-12


# ---------------------------------------------------------------- C-ABI
def _model():
    lib = _lib.load()
    d = _lib.model_desc(load_nextage())
    h = C.c_void_p()
    assert lib.ikg_model_create(C.byref(d), C.byref(h)) == 0
    return lib, h


def test_set_collision_accepts_nextage_scene():
    lib, h = _model()
    cd = _lib.collision_desc(load_nextage_scene())
    assert cd.n_geoms == 48 and cd.n_pairs == 745 and cd.target_geom == 47
    assert lib.ikg_model_set_collision(h, C.byref(cd)) == 0
    assert lib.ikg_model_set_collision(h, C.byref(cd)) == 0  # replace
    lib.ikg_model_destroy(h)


@pytest.mark.parametrize("mutate,msg", [
    (lambda d: setattr(d, "n_geoms", 0), "n_geoms"),
    (lambda d: setattr(d, "n_pairs", 5000), "n_pairs"),
    (lambda d: d.kind.__setitem__(3, 9), "kind"),
    (lambda d: d.joint.__setitem__(3, 15), "joint"),
    (lambda d: d.pairs[7].__setitem__(1, 48), "pair"),
    (lambda d: d.pairs[7].__setitem__(1, d.pairs[7][0]), "pair"),
    (lambda d: setattr(d, "target_geom", 60), "target_geom"),
    (lambda d: d.dims[2].__setitem__(0, -1.0), "dims"),
])
def test_set_collision_rejects_bad_scene(mutate, msg):
    lib, h = _model()
    cd = _lib.collision_desc(load_nextage_scene())
    mutate(cd)
    assert lib.ikg_model_set_collision(h, C.byref(cd)) == -1
    assert msg in lib.ikg_last_error().decode()
    lib.ikg_model_destroy(h)


def test_collision_query_without_scene_fails_loudly():
    lib, h = _model()
    q = np.zeros((1, 15))
    tg = np.zeros((1, 12))
    out = np.zeros(1, np.uint8)
    rc = lib.ikg_collision_batch(h, 0, 0, q.ctypes.data, tg.ctypes.data, 1, out.ctypes.data, None,
                                 _lib.IKG_FLAG_HOST_POINTERS)
    assert rc == -1 and "collision scene" in lib.ikg_last_error().decode()
    lib.ikg_model_destroy(h)


def test_check_collision_param_validated():
    p = _lib.default_params()
    assert p.check_collision == 0
    p = _lib.default_params(check_collision=2)
    lib, h = _model()
    tg = np.zeros((1, 12))
    q = np.zeros(15)
    out = np.zeros((1, 15))
    rc = lib.ikg_solve_batch(h, 0, 0, tg.ctypes.data, q.ctypes.data, 0, 1, C.byref(p), out.ctypes.data, None, None,
                             None, None, _lib.IKG_FLAG_HOST_POINTERS)
    assert rc == -1 and "check_collision" in lib.ikg_last_error().decode()
    lib.ikg_model_destroy(h)


def test_scene_json_roundtrip():
    ps = load_nextage_scene()
    from ikgrasp.collision import CollisionScene
    again = CollisionScene.from_json(ps.to_json())
    assert json.loads(again.to_json()) == json.loads(ps.to_json())


@pytest.mark.parametrize("dtype", [0, 1])
def test_ball_certificate_is_sound(col_cases, oscene, dtype):
    """The records scan's inscribed-ball certificate (ikg_collision.hpp
    ball_cert / ball_covers, run here through the host emulator): at colliding
    fixture configurations, every colliding pair gets a certificate, and every
    perturbed configuration it claims still intersects does, by the collision
    oracle's own narrow phase (oracle/collision_oracle.py collide).  The
    certificate must also cover most small perturbations (it exists to skip
    narrow phases)."""
    lib = C.CDLL(EMU)
    vp = C.c_void_p
    lib.ikg_emu_ball_cert.argtypes = [vp, vp, C.c_int, C.c_int, vp, vp, vp, C.c_int64, vp, vp]
    md = _lib.model_desc(load_nextage())
    scene = load_nextage_scene()
    cd = _lib.collision_desc(scene)
    index = {tuple(p): k for k, p in enumerate(scene.pairs.tolist())}
    npt = np.float64 if dtype == 0 else np.float32
    rng = np.random.default_rng(17 + dtype)
    col = np.nonzero(col_cases["collision"] & col_cases["robust64"])[0]
    rng.shuffle(col)
    gs = oscene["geoms"]
    n_cert = n_pairs = n_cov = n_small = n_small_cov = 0
    for i in col[:40]:
        q, tg = col_cases["q"][i], col_cases["targets"][i]
        TR, Tt = tg[:9].reshape(3, 3), tg[9:]
        for a, b in co.colliding_pairs(oscene, q, TR, Tt):
            n_pairs += 1
            scales = np.repeat([1e-5, 1e-4, 1e-3, 1e-2], 8)
            dq = rng.uniform(-1, 1, (len(scales), 15)) * scales[:, None]
            qs = np.ascontiguousarray(q[None] + dq, dtype=npt)
            r = C.c_double()
            cov = np.empty(len(qs), np.uint8)
            qc = np.ascontiguousarray(q, dtype=npt)
            tgc = np.ascontiguousarray(tg, dtype=npt)
            assert lib.ikg_emu_ball_cert(C.byref(md), C.byref(cd), dtype, index[(a, b)], qc.ctypes.data,
                                         tgc.ctypes.data, qs.ctypes.data, len(qs), C.byref(r),
                                         cov.ctypes.data) == 0
            if r.value > 0:
                n_cert += 1
            n_small += 8
            n_small_cov += int(cov[:8].sum())
            for k in np.nonzero(cov)[0]:
                n_cov += 1
                P = co.geom_poses(oscene, qs[k].astype(np.float64), TR, Tt)
                assert co.collide(gs[a], P[a][0], P[a][1], gs[b], P[b][0], P[b][1]), (i, a, b, k, r.value)
    print(f"dtype {dtype}: {n_pairs} colliding pairs, {n_cert} certified, {n_cov} perturbed configurations "
          f"proved (all confirmed), 1e-5 perturbations covered {n_small_cov}/{n_small}")
    assert n_pairs >= 40 and n_cert >= 0.8 * n_pairs
    assert n_small_cov >= 0.5 * n_small
