"""Per-stage instruction census of the IK update loop in a gfx950 assembly file
built with -gline-tables-only (the .loc comments carry the inlining chain).

Each instruction is attributed to the stage of solve_pair (ikg_solve.hpp) it
was inlined from -- trig_advance, arm_fk_error (FK + log6), pinv_step (the
frame-1 solve), the stop test / exchange, arm_update -- and to the innermost
ikg_device.hpp function.  Basic blocks of the loop are listed with their
counts so the cold ones (exact-trig resync, the singular-arm fallback) can be
told from the per-update path.

    hipcc ... -gline-tables-only --cuda-device-only -S ikg_kernels.hip -o k.s
    python tools/isa_stages.py k.s <kernel-name-substring> [--blocks]
"""
import collections
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "..", "motion-planning-and-control-for-dual-manipulator-robot_amd", "csrc")


def function_spans(path):
    """(start line, name) of every function definition in a header, by a
    simple scan: a line at brace depth 0 or 1 (namespace) that opens a body
    after an identifier followed by '('."""
    spans = []
    depth = 0
    pending = None
    for i, ln in enumerate(open(path), 1):
        s = ln.split("//")[0]
        if depth <= 1 or re.search(r"\binline\b", s):
            m = re.search(r"([A-Za-z_]\w*)\s*\(", s)
            if m and not s.strip().startswith(("if", "for", "while", "return", "#", "static_assert")) and \
                    m.group(1) not in ("if", "for", "while", "switch", "sizeof", "decltype", "alignas"):
                pending = (i, m.group(1))
        depth += s.count("{") - s.count("}")
        if pending and "{" in s and depth >= 1:
            spans.append(pending)
            pending = None
        if ";" in s and "{" not in s:
            pending = None if depth <= 1 else pending
    return spans


def func_at(spans, line):
    name = "?"
    for st, n in spans:
        if st <= line:
            name = n
        else:
            break
    return name


_SPANS = {}


def stage_of(chain):
    """chain: list of (file, line) innermost first.  The stage is the
    ikg_device.hpp function solve_pair (ikg_solve.hpp) called, or
    solve_pair:<line> for its own code."""
    if "dev" not in _SPANS:
        _SPANS["dev"] = function_spans(os.path.join(CSRC, "ikg_device.hpp"))
        _SPANS["solve"] = function_spans(os.path.join(CSRC, "ikg_solve.hpp"))
    idx = [i for i, (f, ln) in enumerate(chain)
           if f.endswith("ikg_solve.hpp") and func_at(_SPANS["solve"], ln) == "solve_pair"]
    if not idx:
        return "outside solve_pair"
    i = idx[-1]
    if i == 0:
        return f"solve_pair:{chain[0][1]}"
    f, ln = chain[i - 1]
    if f.endswith("ikg_device.hpp"):
        return func_at(_SPANS["dev"], ln)
    return f"{os.path.basename(f)}:{ln}"


LOC = re.compile(r";\s*(\S+?):(\d+):\d+(.*)$")
CHAIN = re.compile(r"@\[\s*(\S+?):(\d+):\d+")


def main(path, kname, show_blocks):
    dev_spans = function_spans(os.path.join(CSRC, "ikg_device.hpp"))
    L = open(path).read().split("\n")
    start = next(i for i, l in enumerate(L) if re.match(r"^_Z\S*:", l) and kname in l.split(":")[0])
    end = next(i for i in range(start, len(L)) if L[i].startswith(".Lfunc_end"))
    body = L[start:end]
    # blocks
    blocks, order = {}, []
    cur = "entry"
    chain = []
    for ln in body:
        m = re.match(r"^(\.LBB\S+):", ln) or re.match(r"^; %bb\.(\d+):", ln)
        if m:
            cur = m.group(1) if ln.startswith(".LBB") else f"%bb.{m.group(1)}"
            order.append(cur)
            blocks[cur] = []
            continue
        s = ln.strip()
        if s.startswith(".loc"):
            lm = LOC.search(ln)
            if lm:
                chain = [(lm.group(1), int(lm.group(2)))] + [(f, int(n)) for f, n in CHAIN.findall(lm.group(3))]
            continue
        if not s or s.startswith((";", ".", "//")) or s.endswith(":"):
            continue
        op = s.split()[0]
        blocks.setdefault(cur, []).append((op, list(chain)))
    if "entry" in blocks and "entry" not in order:
        order.insert(0, "entry")
    # loop blocks: from the target of the last backward branch to the branch
    pos = {b: i for i, b in enumerate(order)}
    back = []
    for b in order:
        for op, _ in blocks.get(b, []):
            pass
    text_blocks = {}
    cur = "entry"
    for ln in body:
        m = re.match(r"^(\.LBB\S+):", ln)
        if m:
            cur = m.group(1)
        bm = re.match(r"^\s+s_(cbranch_\w+|branch)\s+(\.LBB\S+)", ln)
        if bm and bm.group(2) in pos and cur in pos and pos[bm.group(2)] <= pos[cur]:
            back.append((pos[cur] - pos[bm.group(2)], bm.group(2), cur))
    back.sort(reverse=True)
    # the update loop: the widest backward branch whose span holds arm_update
    # (the singular branch's Jacobi sweeps can be wider and hold none)
    def has_update(h, t):
        return any(stage_of(c) == "arm_update" for b in order[pos[h]:pos[t] + 1] for _, c in blocks.get(b, []))
    _, head, tail = next((x for x in back if has_update(x[1], x[2])), back[0])
    loop = order[pos[head]:pos[tail] + 1]
    tot = collections.Counter()
    fn = collections.Counter()
    kinds = collections.Counter()
    rows = []
    for b in loop:
        ins = blocks.get(b, [])
        st = collections.Counter(stage_of(c) for _, c in ins)
        rows.append((b, len(ins), st.most_common(2)))
    print(f"kernel {body[0].split(':')[0][:90]}")
    print(f"loop {head} .. {tail}: {len(loop)} blocks, {sum(len(blocks.get(b, [])) for b in loop)} instructions")
    if show_blocks:
        for b, n, st in rows:
            print(f"  {b:12s} {n:5d}  {st}")
    skip = set(a for x in sys.argv if x.startswith("--skip=") for a in x[7:].split(","))
    hot = [b for b in loop if b not in skip]
    for b in hot:
        for op, c in blocks.get(b, []):
            st = stage_of(c)
            tot[st] += 1
            inner = next(((f, ln) for f, ln in c if f.endswith("ikg_device.hpp")), None)
            fn[(st, func_at(dev_spans, inner[1]) if inner else "-")] += 1
            k = "valu64" if re.search(r"_f64|_b64|_u64|_i64", op) and op.startswith("v_") else \
                "valu" if op.startswith("v_") else "salu" if op.startswith("s_") else "mem"
            kinds[(st, k)] += 1
    print("per stage (listed blocks):")
    for st, n in tot.most_common():
        ks = {k: kinds[(st, k)] for k in ("valu64", "valu", "salu", "mem") if kinds[(st, k)]}
        print(f"  {st:32s} {n:5d}  {ks}")
    print("per stage / innermost device function:")
    for (st, f), n in fn.most_common(40):
        print(f"  {st:32s} {f:28s} {n:5d}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], "--blocks" in sys.argv)
