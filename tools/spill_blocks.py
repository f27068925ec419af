"""Report, per kernel of a saved gfx950 assembly file, the basic blocks that
hold scratch or AGPR-copy (spill) instructions.  The guarded step's LQ /
Jacobi branch is cold: every spill should sit in the one or two blocks of
that branch, none in the update loop.
    python tools/spill_blocks.py build/ikg_kernels-hip-amdgcn-amd-amdhsa-gfx950.s"""
import re
import sys


def main(path):
    S = open(path).read().split("\n")
    starts = [k for k, l in enumerate(S) if re.match(r"^_ZN3ikg\S*kernel\S*:", l)]
    for i in starts:
        j = next(k for k, l in enumerate(S[i:], i) if l.startswith(".Lfunc_end"))
        blocks, lab = {}, "entry"
        for l in S[i:j]:
            if re.match(r"^\.LBB\S+:", l):
                lab = l.split(":")[0]
            if "accvgpr" in l or "scratch_" in l:
                blocks[lab] = blocks.get(lab, 0) + 1
        if blocks:
            print(f"{S[i][:70]:70s} {len(blocks)} blocks {sum(blocks.values())} ops {dict(list(blocks.items())[:6])}")


if __name__ == "__main__":
    for p in sys.argv[1:]:
        main(p)
