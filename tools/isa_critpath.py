"""Critical path and in-order issue model of the IK update loop (gfx950 ISA).

The per-update bound of a latency-limited wave: the loop's hot blocks (the
update's common path; cold blocks -- exact trig at resyncs, exact acos, the
near-pi axis, the singular-arm call -- listed with --skip) are taken in
execution order and run for several iterations through two models:

  * latency only: every instruction starts when its register operands are
    ready (infinite issue rate) -- the dependent chain of one update, i.e.
    the recurrence bound;
  * in-order issue: one wave issues its instructions in order, a VALU
    instruction at most every `VALU_ISSUE` cycles (the CU's arbiter visits a
    SIMD every 4 cycles; one wave measured 4.6-5.4 cycles per VALU
    instruction, profiles/r02/ubench_issue.txt), each one also waiting for
    its operands -- the per-update cycles one wave per SIMD can reach.

Latencies are the measured gfx950 figures (tools/ubench):
dependent fp64 FMA/MUL/ADD 9 cycles, fp32 10, DPP moves 14 (an exchange adds
14.5 to an FMA chain), transcendental (rcp/sqrt/rsq) 20, other VALU
(moves, selects, compares, integer) 8, SALU 2, scalar loads 64 (off the
chain: their addresses are loop-invariant).  Steady-state cycles per update
are the difference between the end times of the last two simulated
iterations.

    hipcc ... -gline-tables-only --cuda-device-only -S ikg_kernels.hip -o k.s
    python tools/isa_critpath.py k.s <kernel-name-substring> --skip=%bb.15,%bb.17,... [--json out.json]
"""
import json
import re
import sys

VALU_ISSUE = 4.0

LAT = dict(f64=9, f32=10, dpp=14, trans=20, valu=8, salu=2, smem=64, vmem=300, branch=1)


def regs(tok):
    """'v[4:5]' -> ['v4', 'v5']; 'v7' -> ['v7']; 's[0:1]' -> ['s0', 's1']; vcc/exec/scc."""
    tok = tok.strip().lstrip("-").rstrip(",")
    tok = re.sub(r"^\|(.*)\|$", r"\1", tok)
    m = re.match(r"^([vsa])\[(\d+):(\d+)\]$", tok)
    if m:
        return [f"{m.group(1)}{i}" for i in range(int(m.group(2)), int(m.group(3)) + 1)]
    m = re.match(r"^([vsa])(\d+)$", tok)
    if m:
        return [tok]
    if tok in ("vcc", "vcc_lo", "vcc_hi", "exec", "exec_lo", "exec_hi", "scc"):
        return {"vcc": ["vcc_lo", "vcc_hi"], "exec": ["exec_lo", "exec_hi"]}.get(tok, [tok])
    return []


def classify(op, line):
    if op.startswith("s_load") or op.startswith("s_buffer_load"):
        return "smem"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_", "ds_")):
        return "vmem"
    if op.startswith("s_cbranch") or op.startswith("s_branch"):
        return "branch"
    if op.startswith("s_"):
        return "salu"
    if "dpp" in op or "quad_perm" in line or "row_" in line:
        return "dpp"
    if re.search(r"v_(rcp|rsq|sqrt|exp|log|sin|cos)_", op):
        return "trans"
    if re.search(r"_f64", op) and not op.startswith(("v_cmp", "v_cndmask", "v_mov")):
        return "f64"
    if re.search(r"_f32|pk_f32", op) and not op.startswith(("v_cmp", "v_cndmask", "v_mov")):
        return "f32"
    return "valu"


def parse(path, kname):
    L = open(path).read().split("\n")
    labels = [(i, l.split(":")[0]) for i, l in enumerate(L) if re.match(r"^[A-Za-z_]\S*:", l)]
    exact = [i for i, n in labels if n == kname]  # extern "C" kernels (the hipRTC-specialised ones)
    start = exact[0] if exact else next(i for i, n in labels if n.startswith("_Z") and kname in n)
    end = next(i for i in range(start, len(L)) if L[i].startswith(".Lfunc_end"))
    blocks, order, cur = {}, [], "entry"
    loc = "?"
    for ln in L[start + 1:end]:
        lm = re.search(r"\.loc\s.*;\s*(\S+?):(\d+):\d+", ln)
        if lm:
            loc = f"{lm.group(1).split('/')[-1]}:{lm.group(2)}"
            continue
        m = re.match(r"^(\.LBB\S+):", ln) or re.match(r"^; %bb\.(\d+):", ln)
        if m:
            cur = m.group(1) if ln.startswith(".LBB") else f"%bb.{m.group(1)}"
            order.append(cur)
            blocks[cur] = []
            continue
        s = ln.split(";")[0].strip()
        if not s or s.startswith(".") or s.endswith(":"):
            continue
        op = s.split()[0]
        if op in ("s_waitcnt", "s_nop", "s_setprio") or op.startswith("s_waitcnt"):
            continue
        args = s[len(op):].split(",")
        toks = [a.strip().split()[0] if a.strip() else "" for a in args]
        kind = classify(op, s)
        if op.startswith("v_cmp") and "_e32" in op:
            dst, srcs = ["vcc_lo", "vcc_hi"], toks
        elif kind in ("branch",) or op.startswith(("s_cmp", "global_store", "buffer_store", "ds_write")):
            dst, srcs = (["scc"] if op.startswith("s_cmp") else []), toks
        elif op.startswith("v_cndmask") and "_e32" in op:
            dst, srcs = regs(toks[0]), toks[1:] + ["vcc"]
        else:
            dst, srcs = (regs(toks[0]) if toks else []), toks[1:]
        if op.startswith("s_cbranch_vcc"):
            srcs = ["vcc"]
        elif op.startswith("s_cbranch_scc"):
            srcs = ["scc"]
        elif op.startswith("s_cbranch_exec"):
            srcs = ["exec"]
        sr = [r for t in srcs for r in regs(t)]
        if "mac" in op or op.startswith("s_and_saveexec") or op.startswith("s_or_saveexec"):
            sr += dst  # accumulators read their destination
        if op.startswith(("s_and_saveexec", "s_or_saveexec", "s_andn2_saveexec")):
            dst = dst + ["exec_lo", "exec_hi"]
        blocks[cur].append((op, kind, dst, sr, loc))
    return blocks, order


def simulate(seq, iters, issue, stalls=None):
    avail = {}
    t_issue = 0.0
    ends = []
    for it in range(iters):
        t_end = 0.0
        for op, kind, dst, sr, loc in seq:
            ready = max([avail.get(r, 0.0) for r in sr] + [0.0])
            if issue:
                gap = VALU_ISSUE if kind in ("f64", "f32", "dpp", "trans", "valu") else 1.0
                t = max(ready, t_issue + gap)
                if stalls is not None and it == iters - 1 and t > t_issue + gap:
                    stalls[loc] = stalls.get(loc, 0.0) + t - (t_issue + gap)
                t_issue = t
            else:
                t = ready
            done = t + LAT[kind]
            for r in dst:
                avail[r] = done
            t_end = max(t_end, done)
        ends.append(max(t_end, max(avail.values()) if avail else 0.0))
    return ends[-1] - ends[-2]


def main():
    path, kname = sys.argv[1], sys.argv[2]
    skip = set(a for x in sys.argv if x.startswith("--skip=") for a in x[7:].split(","))
    only = [a for x in sys.argv if x.startswith("--blocks=") for a in x[9:].split(",")]
    out = next((x[7:] for x in sys.argv if x.startswith("--json=")), None)
    blocks, order = parse(path, kname)
    hot = only or [b for b in order if b not in skip and b in blocks]
    seq = [ins for b in hot for ins in blocks[b]]
    n = len(seq)
    n_valu = sum(1 for s in seq if s[1] in ("f64", "f32", "dpp", "trans", "valu"))
    crit = simulate(seq, 6, issue=False)
    stalls = {}
    inorder = simulate(seq, 6, issue=True, stalls=stalls)
    top = sorted(stalls.items(), key=lambda kv: -kv[1])[:25]
    res = {"kernel": kname, "blocks": hot, "instructions_per_update": n, "valu_per_update": n_valu,
           "issue_bound_cycles": n_valu * VALU_ISSUE, "critical_path_cycles": crit,
           "in_order_cycles": inorder, "latencies": LAT, "valu_issue_cycles": VALU_ISSUE,
           "kinds": {k: sum(1 for s in seq if s[1] == k) for k in LAT},
           "stall_cycles": sum(stalls.values()), "top_stalls_by_source_line": top}
    print(json.dumps(res, indent=1))
    if out:
        with open(out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
