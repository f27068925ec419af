"""Vectorised numpy helpers for full-size property checks (test infrastructure).

`log6_batch` restates pin.log6 over a batch; it is used to
re-derive hand errors from FK outputs independently of the kernel's own
reported errors.
"""
import numpy as np


def log6_batch(R, p):
    """R [N,3,3], p [N,3] -> [N,6] = [v; w]."""
    R = np.asarray(R, dtype=np.float64)
    p = np.asarray(p, dtype=np.float64)
    tr = np.trace(R, axis1=1, axis2=2)
    skew = np.stack([R[:, 2, 1] - R[:, 1, 2], R[:, 0, 2] - R[:, 2, 0], R[:, 1, 0] - R[:, 0, 1]], axis=1)
    theta = np.arctan2(0.5 * np.linalg.norm(skew, axis=1), 0.5 * (tr - 1.0))
    with np.errstate(divide="ignore", invalid="ignore"):
        f = np.where(theta > 1e-6, theta / np.sin(theta), 1.0 + theta ** 2 / 6.0) * 0.5
    w = f[:, None] * skew
    near_pi = theta >= np.pi - 1e-2
    if near_pi.any():
        i = np.nonzero(near_pi)[0]
        cphi = np.cos(theta[i] - np.pi)
        beta = theta[i] ** 2 / (1 + cphi)
        tmp = (np.diagonal(R[i], axis1=1, axis2=2) + cphi[:, None]) * beta[:, None]
        sg = np.where(skew[i] > 0, 1.0, -1.0)
        w[i] = sg * np.sqrt(np.maximum(tmp, 0.0))
    t2 = theta ** 2
    with np.errstate(divide="ignore", invalid="ignore"):
        small = theta < 1e-3
        st, ct = np.sin(theta), np.cos(theta)
        alpha = np.where(small, 1 - t2 / 12 - t2 * t2 / 720, theta * st / (2 * (1 - ct)))
        beta = np.where(small, 1.0 / 12 + t2 / 720, 1 / t2 - st / (2 * theta * (1 - ct)))
    wp = np.sum(w * p, axis=1)
    v = alpha[:, None] * p - 0.5 * np.cross(w, p) + (beta * wp)[:, None] * w
    return np.concatenate([v, w], axis=1)


def se3_err(Ra, ta, Rb, tb):
    """|log6(Ma^-1 Mb)| for batches."""
    Rm = np.einsum("nji,njk->nik", Ra, Rb)
    pm = np.einsum("nji,nj->ni", Ra, tb - ta)
    return np.linalg.norm(log6_batch(Rm, pm), axis=1)


def hook_targets(model, targets):
    """[B,12] cube placements -> per-hand target (R [B,2,3,3], t [B,2,3])."""
    CR = targets[:, :9].reshape(-1, 3, 3)
    Ct = targets[:, 9:]
    R = np.einsum("bij,hjk->bhik", CR, model.hook_R)
    t = Ct[:, None, :] + np.einsum("bij,hj->bhi", CR, model.hook_t)
    return R, t


def hand_errors_from_fk(model, hands, targets):
    """hands [B,2,12] (from ikg_fk_batch) + cube targets -> [B,2] |log6| errors."""
    TR, Tt = hook_targets(model, np.asarray(targets, dtype=np.float64))
    out = np.empty((hands.shape[0], 2))
    for h in range(2):
        Rh = hands[:, h, :9].reshape(-1, 3, 3).astype(np.float64)
        th = hands[:, h, 9:].astype(np.float64)
        out[:, h] = se3_err(Rh, th, TR[:, h], Tt[:, h])
    return out


def fk_tables(model, q):
    """FK of compiled model tables (canonical joint axes; DualArmModel): joint
    frames [(R, t)] in q order.  Test infrastructure (numpy)."""
    from oracle import ik_oracle as ik
    oMi = []
    for j in range(model.nq):
        liMi = (model.R[j] @ ik.axis_rotation(int(model.axis[j]), q[j]), model.t[j])
        oMi.append(liMi if model.parents[j] < 0 else ik.se3_mul(oMi[model.parents[j]], liMi))
    return oMi


def hands_from_tables(model, q):
    """[2,12] hand placements from compiled tables."""
    from oracle import ik_oracle as ik
    oMi = fk_tables(model, q)
    out = []
    for h in range(2):
        R, t = ik.se3_mul(oMi[int(model.arm_q[h][-1])], (model.hand_R[h], model.hand_t[h]))
        out.append(np.concatenate([R.reshape(9), t]))
    return np.array(out)


def cpu_threads():
    """CPUs this process may use: the affinity mask capped by a cgroup quota
    (the GPU box gives a job 16 CPUs of a large host)."""
    import os
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
            if q != "max":
                n = min(n, max(1, int(int(q) / int(p))))
    except (OSError, ValueError):
        pass
    return n


def rounding_envelope(targets, q0, q_ref, conv_ref, iters_ref, flags, runs=4, threads=0):
    """How far the float64 loop's answer moves when its FK rounds differently:
    the C oracle (oracle/ikg_oracle.c) with `flags` | JITTER (every FK rotation
    entry moved by 0 / +-1 ulp) for `runs` jitter seeds.  Returns (env [B]:
    the largest |q - q_ref| among runs with the same flag and update count,
    outcomes [B]: the set of (converged, iters) the runs reached)."""
    from oracle import c_oracle
    B = len(targets)
    env = np.zeros(B)
    outcomes = [{(bool(conv_ref[i]), int(iters_ref[i]))} for i in range(B)]
    for s in range(1, runs + 1):
        q, c, it, _ = c_oracle.solve_ex(targets, q0, flags | c_oracle.JITTER, seed=s, threads=threads)
        same = (c == conv_ref) & (it == iters_ref)
        env = np.maximum(env, np.where(same, np.abs(q - q_ref).max(axis=1), 0.0))
        for i in range(B):
            outcomes[i].add((bool(c[i]), int(it[i])))
    return env, outcomes


def report(name, d):
    """Print a comparison's counts and, with IKG_REPORT_DIR set, write them to
    <dir>/<name>.json (profiles/r04/*_vs_oracle.json)."""
    import json
    import os
    print(f"{name}: {json.dumps(d)}")
    out = os.environ.get("IKG_REPORT_DIR")
    if out:
        os.makedirs(out, exist_ok=True)
        with open(os.path.join(out, f"{name}.json"), "w") as f:
            json.dump(d, f, indent=1)


def emu_path():
    """The host emulator of the kernel arithmetic (libikgrasp_emu.so), or the
    build named by IKG_EMU_LIB (tests/test_sanitizers.py runs the emulator
    suites against the ASan/UBSan build)."""
    import os
    env = os.environ.get("IKG_EMU_LIB")
    if env:
        return env
    from ikgrasp import _lib
    return os.path.join(os.path.dirname(_lib.LIB_PATH), "libikgrasp_emu.so")


def _mp_solve(args):
    from oracle import ik_oracle
    t, s = args
    q, ok, it, _ = ik_oracle.computeqgrasppose_mp(s, t[:9].reshape(3, 3), t[9:])
    return q, ok, it


def explain_exceptions(targets, q0s, gq, gc, gi, qo, co, io, flags, threads=0, runs=6, procs=8):
    """Classify the problems where a float64 GPU solve (gq, gc, gi) differs
    from the C oracle's (qo, co, io; evaluated with `flags`) by more than 1e-9
    in q, or in its outcome (flag, update count).  DESIGN.md §2g:

    1. within the oracle's own rounding envelope: the GPU outcome is one the
       oracle reaches under 1-ulp FK jitter (`runs` seeds) and |dq| <= 2x the
       jittered runs' spread;
    2. otherwise arbitrated by the 32-digit loop (oracle/ik_oracle.py
       computeqgrasppose_mp, the exact answer): the GPU outcome equals the
       exact loop's, and the GPU q is within max(1e-9, 2 d) of the exact q,
       d = the larger distance of the oracle's two float64 evaluations
       (reference log6 and cancellation-free log6, both with the QR step) from
       it -- no farther from the truth than float64 itself gets.
    Returns (rows, unexplained): one dict per problem."""
    from concurrent.futures import ProcessPoolExecutor
    import multiprocessing as mpc
    from oracle import c_oracle
    B = len(targets)
    rows, hard = [], []
    if B == 0:
        return rows, []
    env, outc = rounding_envelope(targets, q0s, qo, co, io, flags, runs=runs, threads=threads)
    for i in range(B):
        got = (bool(gc[i]), int(gi[i]))
        same = got == (bool(co[i]), int(io[i]))
        dq = float(np.abs(gq[i] - qo[i]).max()) if same else None
        r = dict(gpu=list(got), oracle=[bool(co[i]), int(io[i])], dq=dq, envelope=float(env[i]))
        if got in outc[i] and (not same or dq <= max(1e-9, 2 * env[i])):
            r["explained_by"] = "oracle rounding envelope"
        else:
            hard.append(i)
        rows.append(r)
    if hard:
        h = np.array(hard)
        with ProcessPoolExecutor(min(procs, len(h)), mp_context=mpc.get_context("spawn")) as ex:
            exact = list(ex.map(_mp_solve, list(zip(targets[h], q0s[h]))))
        q_ref, _, _, _ = c_oracle.solve_ex(targets[h], q0s[h], c_oracle.QR_STEP, threads=threads)
        q_acc, _, _, _ = c_oracle.solve_ex(targets[h], q0s[h], c_oracle.ACC_LOG6 | c_oracle.QR_STEP, threads=threads)
        for k, i in enumerate(h):
            qe, oke, ite = exact[k]
            d64 = max(float(np.abs(q_ref[k] - qe).max()), float(np.abs(q_acc[k] - qe).max()))
            dg = float(np.abs(gq[i] - qe).max())
            ok = (bool(gc[i]), int(gi[i])) == (bool(oke), int(ite)) and dg <= max(1e-9, 2 * d64)
            rows[i].update(exact=[bool(oke), int(ite)], gpu_vs_exact=dg, float64_oracles_vs_exact=d64,
                           explained_by="32-digit loop" if ok else None)
    return rows, [r for r in rows if r.get("explained_by") is None]
