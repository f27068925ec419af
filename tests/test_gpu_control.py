"""Controller row on the GPU: ikg_frame_kinematics_batch
against the control oracle's fixtures (tests/golden/control_cases.npz) in
WORLD / LOCAL / LOCAL_WORLD_ALIGNED, the drop-in task_space_terms, and
full-size properties (J v = frame velocity, dJ = d/dt J, the LDS tile
assembly across ragged batch tails).

Tolerances: fp64 1e-12 absolute (values are O(1)); fp32 2e-4 absolute
(J, dJ entries up to ~10 at the fixtures' velocities)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

KEYS = ("placement", "velocity", "J", "dJ", "dJv")


@pytest.fixture(scope="module")
def cc():
    return dict(np.load(os.path.join(GOLDEN, "control_cases.npz")))


@pytest.mark.parametrize("rf", [0, 1, 2])
@pytest.mark.parametrize("dtype,tol", [("f64", 1e-12), ("f32", 2e-4)])
def test_frame_kinematics_matches_oracle(solver, cc, rf, dtype, tol):
    r = solver.frame_kinematics(cc["q"], cc["v"], cc["q_des"], cc["v_des"], rf=rf,
                                outputs=KEYS + ("err", "derr"), dtype=dtype)
    for k in KEYS:
        np.testing.assert_allclose(r[k], cc[f"{k}_rf{rf}"], rtol=0, atol=tol * max(1.0, np.abs(cc[f"{k}_rf{rf}"]).max() / 10),
                                   err_msg=k)
    np.testing.assert_allclose(r["err"], cc["err"], rtol=0, atol=tol)
    np.testing.assert_allclose(r["derr"], cc["derr"], rtol=0, atol=tol * 10)


def test_zero_pattern_is_exact(solver, cc):
    """Columns outside a hand's support (head joints, the other arm) are exact zeros."""
    r = solver.frame_kinematics(cc["q"], cc["v"], outputs=("J", "dJ"))
    m = solver.model
    for h in range(2):
        support = {m.root_q, *m.arm_q[h]}
        off = [j for j in range(m.nq) if j not in support]
        for k in ("J", "dJ"):
            assert np.all(r[k][:, 6 * h:6 * h + 6, off] == 0), k
            assert np.all(np.any(r[k][:, 6 * h:6 * h + 6, sorted(support)] != 0, axis=1)), k


def test_output_subsets_agree(solver, cc):
    full = solver.frame_kinematics(cc["q"], cc["v"], outputs=KEYS)
    for k in KEYS:
        part = solver.frame_kinematics(cc["q"], cc["v"], outputs=(k,))
        assert np.array_equal(part[k], full[k]), k


def test_no_velocity_means_zero(solver, cc):
    r = solver.frame_kinematics(cc["q"], None, outputs=KEYS)
    assert np.all(r["velocity"] == 0) and np.all(r["dJ"] == 0) and np.all(r["dJv"] == 0)
    np.testing.assert_allclose(r["J"], cc["J_rf2"], atol=1e-12)


def test_task_space_terms_dropin(cc):
    import ikgrasp
    from ikgrasp import control
    from oracle import control_oracle as co
    robot, _, _, _ = ikgrasp.setuppinocchio(device=0)
    for i in (0, 30, 60):
        J, Jdv, e, ed = control.task_space_terms(robot, cc["q"][i], cc["v"][i], cc["q_des"][i], cc["v_des"][i])
        Jr, Jdvr, er, edr = co.task_space_terms(cc["q"][i], cc["v"][i], cc["q_des"][i], cc["v_des"][i])
        assert J.shape == (12, 15) and Jdv.shape == (12,) and e.shape == (12,) and ed.shape == (12,)
        for a, b in ((J, Jr), (Jdv, Jdvr), (e, er), (ed, edr)):
            np.testing.assert_allclose(a, b, rtol=0, atol=1e-12)


@pytest.mark.parametrize("B", [0, 1, 31, 33, 1000])
def test_ragged_batches_and_positions(solver, cc, B):
    """Every state's output is independent of batch size and position (tile tails)."""
    rng = np.random.default_rng(B)
    idx = rng.integers(0, len(cc["q"]), size=B)
    r = solver.frame_kinematics(cc["q"][idx], cc["v"][idx], outputs=KEYS)
    for k in KEYS:
        assert r[k].shape[0] == B
        if B:
            np.testing.assert_allclose(r[k], cc[f"{k}_rf2"][idx], rtol=0, atol=1e-12 * 10, err_msg=k)


def test_full_size_properties_torch():
    """65,536 random states on device: J v = velocity and dJ = central
    difference of J along v (fp64), through the torch zero-copy path."""
    import torch
    from ikgrasp.solver import IKSolver
    s = IKSolver(device=0)
    g = torch.Generator(device="cuda").manual_seed(0)
    B = 65536
    lo = torch.tensor(s.model.lower, device="cuda")
    hi = torch.tensor(s.model.upper, device="cuda")
    q = lo + (hi - lo) * torch.rand(B, 15, generator=g, device="cuda", dtype=torch.float64)
    v = torch.randn(B, 15, generator=g, device="cuda", dtype=torch.float64)
    r = s.frame_kinematics(q, v, outputs=("velocity", "J", "dJ"))
    jv = torch.einsum("bij,bj->bi", r["J"], v).view(B, 2, 6)
    assert (jv - r["velocity"]).abs().max().item() < 1e-12
    h = 1e-6
    Jp = s.frame_kinematics(q + h * v, v, outputs=("J",))["J"]
    Jm = s.frame_kinematics(q - h * v, v, outputs=("J",))["J"]
    fd = (Jp - Jm) / (2 * h)
    scale = v.abs().amax(dim=1).clamp(min=1.0)[:, None, None]
    assert ((fd - r["dJ"]).abs() / scale).max().item() < 1e-7
    torch.cuda.synchronize()
    s.close()


def test_generic_spec_path(cc):
    """The runtime-axis / placement-rotation path (SpecGeneric): the same
    robot with one arm placement rotation perturbed by 1e-300 (no longer the
    exact identity, so the compiled Nextage specialisation does not apply)."""
    import copy
    from ikgrasp.model import load_nextage
    from ikgrasp.solver import IKSolver
    m = copy.deepcopy(load_nextage())
    j = int(m.arm_q[0][2])
    m.R[j][0, 1], m.R[j][1, 0] = -1e-300, 1e-300
    s = IKSolver(m, device=0)
    for rf in (0, 1, 2):
        r = s.frame_kinematics(cc["q"], cc["v"], cc["q_des"], cc["v_des"], rf=rf, outputs=KEYS + ("err", "derr"))
        for k in KEYS:
            np.testing.assert_allclose(r[k], cc[f"{k}_rf{rf}"], rtol=0, atol=1e-11, err_msg=k)
        np.testing.assert_allclose(r["err"], cc["err"], rtol=0, atol=1e-12)
    s.close()
