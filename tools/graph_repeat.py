"""Repeat the graph-replay test of the collision solve in one process
(tests/test_gpu_graph.py) and count passes: a replay that differs from direct
launches now and then points at a capture-order problem.
usage: python tools/graph_repeat.py [repeats]"""
import os
import sys

root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(root, "motion-planning-and-control-for-dual-manipulator-robot_amd"))
sys.path.insert(0, os.path.join(root, "tests"))
import test_gpu_graph as t  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 5
ok = 0
for i in range(n):
    try:
        t.test_batch_solve_replays_from_a_graph(True)
        ok += 1
        print("pass", i, flush=True)
    except AssertionError:
        print("FAIL", i, flush=True)
print("passed", ok, "of", n)
sys.exit(0 if ok == n else 1)
