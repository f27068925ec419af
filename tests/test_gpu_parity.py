"""HIP kernel parity against the oracle / golden vectors (run on an MI355X).

Tolerances (north star: "within 1e-4 end-effector SE(3) error of the
reference"):
  * fp64: q within 1e-12 of the reference KATs and within 1e-9 of the oracle
    fixtures for converged solves, identical iteration counts and flags;
  * fp32: per-hand end-effector error |log6(M_oracle^-1 M_gpu)| <= 1e-4 and
    iteration counts within +-2 of the fp64 oracle.
"""
import numpy as np
import pytest

import helpers
from oracle import ik_oracle as o

pytestmark = pytest.mark.gpu


def _placement_row(d):
    return np.concatenate([np.array(d["R"], dtype=np.float64).reshape(9), np.array(d["t"], dtype=np.float64)])


# ---------------------------------------------------------------- KATs, drop-in
def test_dropin_reproduces_reference_kats(kat):
    import ikgrasp
    from ikgrasp.config import CUBE_PLACEMENT, CUBE_PLACEMENT_TARGET
    robot, _, _, cube = ikgrasp.setuppinocchio()
    q = robot.q0.copy()
    q0, ok0 = ikgrasp.computeqgrasppose(robot, q, cube, CUBE_PLACEMENT)
    qe, oke = ikgrasp.computeqgrasppose(robot, q, cube, CUBE_PLACEMENT_TARGET)
    assert ok0 and oke
    assert np.abs(q0 - np.array(kat["q0"])).max() <= 1e-12
    assert np.abs(qe - np.array(kat["qe"])).max() <= 1e-12
    assert np.array_equal(q, np.zeros(15))  # qcurrent not mutated (:49)
    # the cube is left at the last target (tools.py:62-68)
    assert np.array_equal(cube.placement.translation, CUBE_PLACEMENT_TARGET.translation)


def test_kat_iteration_counts(solver, kat):
    tg = np.stack([_placement_row(kat["cube_placement"]), _placement_row(kat["cube_placement_target"])])
    sol = solver.solve(tg, np.zeros(15))
    assert sol.iters.tolist() == [740, 736]
    assert sol.converged.all()
    assert (sol.err < 1e-3).all()


# ---------------------------------------------------------------- oracle fixtures
def test_fixture_parity_fp64(solver, oracle_cases):
    c = oracle_cases
    sol = solver.solve(c["targets"], c["q0"], dtype="f64")
    assert np.array_equal(sol.converged, c["converged"])
    assert np.array_equal(sol.iters, c["iters"])
    conv = c["converged"]
    assert np.abs(sol.q[conv] - c["q"][conv]).max() <= 1e-9
    # |e| ~ 1e-3 at convergence; the reference's alpha = theta sin/(2(1-cos))
    # carries ~eps/theta^2 (~1e-10 relative at theta ~ 1e-3) rounding noise of its
    # own, which the kernel's cancellation-free form does not reproduce
    assert np.abs(sol.err[conv] - c["err"][conv]).max() <= 1e-10
    # unconverged solves run the full 1000 updates; the final iterate agrees
    # in end-effector space (null-space drift is not corrected by pinv)
    hands_gpu = solver.fk(sol.q[~conv])
    hands_orc = solver.fk(c["q"][~conv])
    for h in range(2):
        e = helpers.se3_err(hands_orc[:, h, :9].reshape(-1, 3, 3), hands_orc[:, h, 9:],
                            hands_gpu[:, h, :9].reshape(-1, 3, 3), hands_gpu[:, h, 9:])
        assert e.max() <= 1e-6


def test_sensitive_cases_against_exact_loop(solver):
    """Rounding-sensitive random-seed trajectories (tests/golden/
    sensitive_cases.npz): flags and update counts equal the
    32-digit evaluation of the loop; q within 1e-9 of it, or -- where no
    float64 evaluation gets there (case 1: every float64 loop lands ~1e-5
    away) -- no farther than the reference's own answer is plus the reference's
    rounding envelope.  Printed: the kernel's and the reference's distances."""
    import os
    from conftest import GOLDEN
    d = np.load(os.path.join(GOLDEN, "sensitive_cases.npz"))
    for variant in (0, 3):  # AUTO (pair), QUAD
        sol = solver.solve(d["targets"], d["q0"], variant=variant)
        assert np.array_equal(sol.converged, d["converged_exact"]) and np.array_equal(sol.iters, d["iters_exact"])
        gpu = np.abs(sol.q - d["q_exact"]).max(axis=1)
        ref = np.abs(d["q"] - d["q_exact"]).max(axis=1)
        print(f"variant {variant}: kernel vs exact", np.array2string(gpu, precision=2),
              "\n  numpy reference vs exact", np.array2string(ref, precision=2))
        assert (gpu <= np.maximum(1e-9, ref + d["envelope"])).all()


def test_fixture_parity_fp32(solver, oracle_cases):
    c = oracle_cases
    sol = solver.solve(c["targets"], c["q0"], dtype="f32")
    conv = c["converged"] & sol.converged
    # convergence decisions agree
    assert np.array_equal(sol.converged, c["converged"])
    assert np.abs(sol.iters[conv].astype(int) - c["iters"][conv]).max() <= 2
    hands_gpu = solver.fk(sol.q.astype(np.float64))
    hands_orc = solver.fk(c["q"])
    for h in range(2):
        e = helpers.se3_err(hands_orc[conv, h, :9].reshape(-1, 3, 3), hands_orc[conv, h, 9:],
                            hands_gpu[conv, h, :9].reshape(-1, 3, 3), hands_gpu[conv, h, 9:])
        assert e.max() <= 1e-4


def test_fk_kernel_matches_oracle(solver):
    from ikgrasp.workload import random_seeds
    q = random_seeds(solver.model, 64, seed=7)
    hands = solver.fk(q)
    for i in range(0, 64, 7):
        oL, oR = o.fk_hands(q[i])
        assert np.abs(hands[i, 0, :9].reshape(3, 3) - oL[0]).max() < 1e-13
        assert np.abs(hands[i, 0, 9:] - oL[1]).max() < 1e-13
        assert np.abs(hands[i, 1, :9].reshape(3, 3) - oR[0]).max() < 1e-13
        assert np.abs(hands[i, 1, 9:] - oR[1]).max() < 1e-13


# ---------------------------------------------------------------- full-size properties
def _check_reported_errors(solver, sol, targets, tol):
    hands = solver.fk(sol.q.astype(np.float64))
    err = helpers.hand_errors_from_fk(solver.model, hands, targets)
    assert np.abs(err - sol.err).max() <= tol
    assert (err[sol.converged] < 1e-3 + tol).all()


def test_config_b4096_fp64_properties(solver):
    from ikgrasp.workload import uniform_targets
    tg = uniform_targets(4096, seed=0)
    a = solver.solve(tg, np.zeros(15), dtype="f64")
    b = solver.solve(tg, np.zeros(15), dtype="f64")
    for x, y in ((a.q, b.q), (a.iters, b.iters), (a.converged, b.converged), (a.err, b.err)):
        assert np.array_equal(x, y)  # deterministic
    assert (a.iters[~a.converged] == 1000).all()
    assert (a.err[a.converged] < 1e-3).all()
    _check_reported_errors(solver, a, tg, 1e-9)  # two independent log6 evaluations (see fixture test)
    # a sample against the oracle
    for i in np.nonzero(a.converged)[0][:3]:
        q, ok, it, _ = o.computeqgrasppose(np.zeros(15), tg[i, :9].reshape(3, 3), tg[i, 9:])
        assert ok and it == a.iters[i] and np.abs(q - a.q[i]).max() <= 1e-9


def test_config_b65536_fp32_vs_fp64(solver):
    from ikgrasp.workload import uniform_targets
    tg = uniform_targets(65536, seed=1)
    s32 = solver.solve(tg, np.zeros(15), dtype="f32")
    s64 = solver.solve(tg, np.zeros(15), dtype="f64")
    both = s32.converged & s64.converged
    flips = int((s32.converged != s64.converged).sum())
    off = int((np.abs(s32.iters[both].astype(int) - s64.iters[both]) > 2).sum())
    # printed (pytest -s) so the escapes the gates allow are on record; the
    # oracle-side comparison of this config is tests/test_gpu_configs.py
    print(f"C3 fp32 vs fp64 on 65,536: {flips} flag flips, {off} of {int(both.sum())} update counts outside +-2")
    assert flips <= 0.001 * len(tg)  # measured 0 (round 3)
    assert off <= 0.002 * both.sum()  # measured 0 of 26,570
    h32 = solver.fk(s32.q.astype(np.float64))
    h64 = solver.fk(s64.q)
    for h in range(2):
        e = helpers.se3_err(h64[both, h, :9].reshape(-1, 3, 3), h64[both, h, 9:],
                            h32[both, h, :9].reshape(-1, 3, 3), h32[both, h, 9:])
        assert e.max() <= 1e-4
    _check_reported_errors(solver, s32, tg, 2e-5)


def test_config_c4_full_batch_fp64_shards_and_limits(solver):
    """C4 at its full size (1,048,576 targets, fp64) on one GPU.  Size-independent
    properties: the whole batch equals the concatenation of its 8 rank shards
    (the weak-scaling partition of bench.py, bit-exact), every q is inside the URDF
    limits (tools.py:21-22), non-converged problems ran all 1000 updates
    (inverse_geometry.py:56), and the reported errors agree with an independent FK."""
    from ikgrasp.parallel import shard_range
    from ikgrasp.workload import uniform_targets
    B = 1 << 20
    tg = uniform_targets(B, seed=11)
    full = solver.solve(tg, np.zeros(15), dtype="f64")
    assert full.q.shape == (B, 15)
    lo_lim, hi_lim = solver.model.lower, solver.model.upper
    assert ((full.q >= lo_lim - 1e-15) & (full.q <= hi_lim + 1e-15)).all()
    assert (full.iters[~full.converged] == 1000).all()
    assert (full.err[full.converged] < 1e-3).all()
    assert 0.3 < full.converged.mean() < 0.5  # the path.py sampler from q0 = 0
    for r in (0, 3, 7):
        lo, hi = shard_range(B, r, 8)
        part = solver.solve(tg[lo:hi], np.zeros(15), dtype="f64")
        assert np.array_equal(part.q, full.q[lo:hi])
        assert np.array_equal(part.iters, full.iters[lo:hi])
        assert np.array_equal(part.converged, full.converged[lo:hi])
    idx = np.random.default_rng(0).choice(B, 4096, replace=False)
    hands = solver.fk(full.q[idx])
    err = helpers.hand_errors_from_fk(solver.model, hands, tg[idx])
    assert np.abs(err - full.err[idx]).max() <= 1e-9


# ---------------------------------------------------------------- edge cases
def test_batch_position_invariance_and_ragged_sizes(solver):
    from ikgrasp.workload import uniform_targets
    tg = uniform_targets(200, seed=3)
    full = solver.solve(tg, np.zeros(15))
    for B in (1, 2, 31, 33, 65, 127):
        part = solver.solve(tg[-B:], np.zeros(15))
        assert np.array_equal(part.q, full.q[-B:])
        assert np.array_equal(part.iters, full.iters[-B:])


def test_broadcast_q0_equals_explicit(solver):
    from ikgrasp.workload import uniform_targets
    tg = uniform_targets(64, seed=4)
    a = solver.solve(tg, np.zeros(15))
    b = solver.solve(tg, np.zeros((64, 15)))
    assert np.array_equal(a.q, b.q) and np.array_equal(a.iters, b.iters)


@pytest.mark.parametrize("dtype", ["f64", "f32"])
def test_q0_layout_from_random_seeds(solver, dtype):
    """A broadcast q0 and a row per problem give one answer per problem.
    fp32 advances the joint sin/cos by the medium-range rule for every q0
    layout: identical bits.  fp64 keeps two rules for steps of 0.025..0.25 rad
    (exact sincos for a broadcast q0, the medium-range series for rows;
    ikg_device.hpp trig_advance_f1): the same iterates to rounding, compared
    over the first 150 updates, before non-converging solves' chaotic drift --
    identical flags and counts, q within 1e-10 and the end effectors within
    north_star's 1e-4 SE(3) tolerance (measured ~1e-12).  From q0 = 0 (no such
    steps) the two are bit-equal in both dtypes
    (test_broadcast_q0_equals_explicit)."""
    from ikgrasp.workload import random_seeds, uniform_targets
    tg = uniform_targets(256, seed=6)
    ee_max = 0.0
    for seed in random_seeds(solver.model, 4, seed=7):
        a = solver.solve(tg, seed, dtype=dtype, max_iters=150)
        b = solver.solve(tg, np.tile(seed, (256, 1)), dtype=dtype, max_iters=150)
        assert np.array_equal(a.converged, b.converged) and np.array_equal(a.iters, b.iters)
        if dtype == "f32":
            assert np.array_equal(a.q, b.q)
            continue
        assert np.abs(a.q - b.q).max() <= 1e-10
        ha, hb = solver.fk(a.q), solver.fk(b.q)
        for h in range(2):
            e = helpers.se3_err(ha[:, h, :9].reshape(-1, 3, 3), ha[:, h, 9:], hb[:, h, :9].reshape(-1, 3, 3),
                                hb[:, h, 9:])
            ee_max = max(ee_max, float(e.max()))
    print(f"q0 layouts, {dtype}: end-effector SE(3) distance max {ee_max:.2e}")
    assert ee_max <= 1e-4  # north_star: 1e-4 end-effector SE(3) error


def test_empty_batch(solver):
    sol = solver.solve(np.zeros((0, 12)), np.zeros(15))
    assert sol.q.shape == (0, 15)


def test_start_at_solution_returns_seed_unchanged(solver, kat):
    q_sol = np.array(kat["q0"])
    q_sol_off = q_sol.copy()
    q_sol_off[1] = 5.0  # passive head joint outside its limits: untouched with 0 updates
    sol = solver.solve(_placement_row(kat["cube_placement"])[None], q_sol_off)
    assert sol.iters[0] == 0 and sol.converged[0]
    assert np.array_equal(sol.q[0], q_sol_off)


def test_max_iters_zero(solver, kat):
    sol = solver.solve(_placement_row(kat["cube_placement"])[None], np.zeros(15), max_iters=0)
    assert sol.iters[0] == 0 and not sol.converged[0]
    assert np.array_equal(sol.q[0], np.zeros(15))


def test_passive_joints_clamped_after_first_update(solver, kat):
    q0 = np.zeros(15)
    q0[1], q0[2] = 5.0, -5.0  # outside HEAD_JOINT0/1 limits
    sol = solver.solve(_placement_row(kat["cube_placement"])[None], q0)
    ref, ok, it, _ = o.computeqgrasppose(q0, np.eye(3), np.array(kat["cube_placement"]["t"]))
    assert sol.q[0, 1] == o.UPPER[1] and sol.q[0, 2] == o.LOWER[2]
    assert sol.iters[0] == it and np.abs(sol.q[0] - ref).max() <= 1e-9


def test_near_pi_rotation_target(solver):
    # cube yawed by ~pi: the initial hand errors take log3's near-pi branch
    c, s = np.cos(np.pi - 1e-3), np.sin(np.pi - 1e-3)
    tg = np.array([c, -s, 0, s, c, 0, 0, 0, 1, 0.36, -0.05, 1.1])
    sol = solver.solve(tg[None], np.zeros(15), max_iters=60)
    q, ok, it, (nl, nr) = o.computeqgrasppose(np.zeros(15), tg[:9].reshape(3, 3), tg[9:], max_iters=60)
    assert sol.iters[0] == it
    assert np.abs(sol.q[0] - q).max() <= 1e-9


def test_damped_variant_matches_damped_oracle(solver, kat):
    # lambda > 0 is an extension (parity unpinned vs the reference)
    lam = 1e-4
    sol = solver.solve(_placement_row(kat["cube_placement"])[None], np.zeros(15), lam=lam, max_iters=200)
    q, ok, it, _ = o.computeqgrasppose(np.zeros(15), np.eye(3), np.array(kat["cube_placement"]["t"]), lam=lam,
                                       max_iters=200)
    assert sol.iters[0] == it and np.abs(sol.q[0] - q).max() <= 1e-9


# ---------------------------------------------------------------- multi-start
def test_multistart_selects_best_seed(solver):
    from ikgrasp.workload import uniform_targets, random_seeds
    T, S = 6, 40
    tg = uniform_targets(T, seed=11)
    seeds = random_seeds(solver.model, S, seed=12)
    seeds[0] = 0.0  # the reference's own seed (robot.q0)
    ms = solver.solve_multistart(tg, seeds, dtype="f64")
    # expected: every (target, seed) through the batch kernel
    full = solver.solve(np.repeat(tg, S, axis=0), np.tile(seeds, (T, 1)), dtype="f64")
    conv = full.converged.reshape(T, S)
    worst = full.err.max(axis=1).reshape(T, S)
    key = np.where(conv, worst, 1e30 + worst)
    best = key.argmin(axis=1)
    assert np.array_equal(ms.best_seed, best)
    for t in range(T):
        k = t * S + best[t]
        assert np.array_equal(ms.q[t], full.q[k])
        assert ms.converged[t] == full.converged[k] and ms.iters[t] == full.iters[k]


@pytest.mark.parametrize("variant", [1, 2])  # PAIR, PACKED
def test_multistart_single_seed_broadcasts(solver, variant):
    """S = 1 with T > 1: the one seed serves every target (the kernel
    read seed rows past the end of the buffer)."""
    from ikgrasp.workload import uniform_targets, random_seeds
    dtype = "f32" if variant == 2 else "f64"
    tg = uniform_targets(70, seed=21)
    seed = random_seeds(solver.model, 1, seed=22)
    ms = solver.solve_multistart(tg, seed, dtype=dtype, variant=variant)
    ref = solver.solve(tg, seed[0], dtype=dtype, variant=variant)
    assert np.array_equal(ms.q, ref.q) and np.array_equal(ms.iters, ref.iters)
    assert np.array_equal(ms.converged, ref.converged) and (ms.best_seed == 0).all()


def test_non_finite_host_inputs_are_rejected(solver):
    """The device code assumes finite math (-ffinite-math-only): host-pointer
    inputs are checked before staging and a NaN/inf target, q0 row or seed
    fails with IKG_EINVAL naming the array (include/ikgrasp.h Conventions)."""
    from ikgrasp._lib import IkgError
    from ikgrasp.workload import uniform_targets, random_seeds
    tg = uniform_targets(3, seed=23)
    seeds = random_seeds(solver.model, 5, seed=24)
    bad = tg.copy()
    bad[1, 9] = np.nan
    for dtype in ("f64", "f32"):
        with pytest.raises(IkgError, match="targets"):
            solver.solve(bad, np.zeros(15), dtype=dtype)
        with pytest.raises(IkgError, match="targets"):
            solver.solve_multistart(bad, seeds, dtype=dtype)
        q0 = np.zeros((3, 15))
        q0[2, 4] = np.inf
        with pytest.raises(IkgError, match="q0"):
            solver.solve(tg, q0, dtype=dtype)
        sd = seeds.copy()
        sd[3, 7] = -np.inf
        with pytest.raises(IkgError, match="seeds"):
            solver.solve_multistart(tg, sd, dtype=dtype)
    # finite inputs still solve
    ok = solver.solve_multistart(tg, seeds, dtype="f64", max_iters=20)
    assert ok.q.shape == (3, 15)


def test_torch_q0_shapes_are_checked(solver):
    import torch
    from ikgrasp.workload import uniform_targets
    tg = torch.from_numpy(uniform_targets(8, seed=25)).cuda()
    a = solver.solve(tg, torch.zeros(15, dtype=torch.float64))
    b = solver.solve(tg, torch.zeros(1, 15, dtype=torch.float64))  # [1, nq] broadcasts
    assert torch.equal(a.q, b.q)
    for bad in ((2, 15), (8, 14), (8, 15, 1)):
        with pytest.raises(ValueError):
            solver.solve(tg, torch.zeros(*bad, dtype=torch.float64))


def test_problems_per_wave_does_not_change_results(solver):
    from ikgrasp.workload import uniform_targets
    tg = uniform_targets(300, seed=9)
    ref = solver.solve(tg, np.zeros(15), ppw=32)
    for ppw in (1, 3, 4, 16):
        s = solver.solve(tg, np.zeros(15), ppw=ppw)
        assert np.array_equal(s.q, ref.q) and np.array_equal(s.iters, ref.iters) and np.array_equal(s.err, ref.err)


# ---------------------------------------------------------------- quad layout (IKG_VARIANT_QUAD)
def test_fixture_parity_fp64_quad_layout(solver, oracle_cases):
    """The quad layout (8 lanes per problem, ikg_quad.hip) against the fixtures
    with the fp64 gates of test_fixture_parity_fp64."""
    c = oracle_cases
    sol = solver.solve(c["targets"], c["q0"], dtype="f64", variant=3)
    assert np.array_equal(sol.converged, c["converged"])
    assert np.array_equal(sol.iters, c["iters"])
    conv = c["converged"]
    assert np.abs(sol.q[conv] - c["q"][conv]).max() <= 1e-9
    assert np.abs(sol.err[conv] - c["err"][conv]).max() <= 1e-10


def test_quad_layout_matches_pair_layout(solver, kat):
    """Same frame-1 arithmetic in another lane layout: identical flags and update
    counts, q to rounding (fp64), at the headline batch size; KATs within 1e-12."""
    from ikgrasp.workload import uniform_targets
    tg = uniform_targets(4096, seed=0)
    a = solver.solve(tg, np.zeros(15), dtype="f64", variant=1)
    b = solver.solve(tg, np.zeros(15), dtype="f64", variant=3)
    assert np.array_equal(a.converged, b.converged) and np.array_equal(a.iters, b.iters)
    assert np.abs(a.q - b.q).max() <= 1e-9
    kt = np.stack([_placement_row(kat["cube_placement"]), _placement_row(kat["cube_placement_target"])])
    k = solver.solve(kt, np.zeros(15), dtype="f64", variant=3)
    assert k.iters.tolist() == [740, 736]
    assert np.abs(k.q[0] - np.array(kat["q0"])).max() <= 1e-12
    assert np.abs(k.q[1] - np.array(kat["qe"])).max() <= 1e-12
    # ragged batches: the last wave holds 1..7 problems
    for B in (1, 3, 9, 15):
        p = solver.solve(tg[-B:], np.zeros(15), dtype="f64", variant=3)
        assert np.array_equal(p.q, b.q[-B:]) and np.array_equal(p.iters, b.iters[-B:])


def test_quad_variant_rejected_for_damped_solves(solver, kat):
    from ikgrasp._lib import IkgError
    tg = np.stack([_placement_row(kat["cube_placement"])])
    with pytest.raises(IkgError):
        solver.solve(tg, np.zeros(15), dtype="f64", variant=3, lam=1e-3)


# ---------------------------------------------------------------- packed fp32 layout (IKG_VARIANT_PACKED)
@pytest.mark.parametrize("variant", [1, 2, 3])  # PAIR, PACKED, QUAD
def test_fixture_parity_fp32_layouts(solver, oracle_cases, variant):
    c = oracle_cases
    sol = solver.solve(c["targets"], c["q0"], dtype="f32", variant=variant)
    conv = c["converged"] & sol.converged
    assert np.array_equal(sol.converged, c["converged"])
    assert np.abs(sol.iters[conv].astype(int) - c["iters"][conv]).max() <= 2
    hands_gpu = solver.fk(sol.q.astype(np.float64))
    hands_orc = solver.fk(c["q"])
    for h in range(2):
        e = helpers.se3_err(hands_orc[conv, h, :9].reshape(-1, 3, 3), hands_orc[conv, h, 9:],
                            hands_gpu[conv, h, :9].reshape(-1, 3, 3), hands_gpu[conv, h, 9:])
        assert e.max() <= 1e-4
    _check_reported_errors(solver, sol, c["targets"], 2e-5)


def test_packed_layout_matches_pair_layout_at_scale(solver):
    # same fp32 arithmetic in a different lane layout: identical up to the
    # scheduling of the packed instructions (flags and iteration counts
    # identical for >= 99.5%, end effectors within the fp32 tolerance)
    from ikgrasp.workload import uniform_targets
    tg = uniform_targets(8192, seed=11)
    a = solver.solve(tg, np.zeros(15), dtype="f32", variant=1)
    b = solver.solve(tg, np.zeros(15), dtype="f32", variant=2)
    assert (a.converged == b.converged).mean() >= 0.995
    both = a.converged & b.converged
    assert (a.iters[both] == b.iters[both]).mean() >= 0.99
    ha, hb = solver.fk(a.q.astype(np.float64)), solver.fk(b.q.astype(np.float64))
    for h in range(2):
        e = helpers.se3_err(ha[both, h, :9].reshape(-1, 3, 3), ha[both, h, 9:],
                            hb[both, h, :9].reshape(-1, 3, 3), hb[both, h, 9:])
        assert e.max() <= 1e-4


def test_packed_variant_rejected_where_it_does_not_apply(solver, kat):
    from ikgrasp._lib import IkgError
    tg = np.stack([_placement_row(kat["cube_placement"])])
    with pytest.raises(IkgError):
        solver.solve(tg, np.zeros(15), dtype="f64", variant=2)
    with pytest.raises(IkgError):
        solver.solve(tg, np.zeros(15), dtype="f32", variant=2, lam=1e-3)
