"""The drop-in on a RobotWrapper-shaped robot (SURVEY §8b "Duck typing",
/root/reference/setup_pinocchio.py:73-83): the KATs through
computeqgrasppose(robot, robot.q0, cube, target) with the collision term read
from robot.collision_model, KAT-5 through tools.collision, and
distanceToObstacle equal to ikgrasp's own robot."""
import numpy as np
import pytest

from fake_pinocchio import nextage_wrapper

pytestmark = pytest.mark.gpu


def test_kats_through_a_pinocchio_style_robot(kat):
    import ikgrasp
    from ikgrasp.config import CUBE_PLACEMENT, CUBE_PLACEMENT_TARGET
    from ikgrasp.tools import collision, distanceToObstacle
    robot, cube = nextage_wrapper()
    q0, ok0 = ikgrasp.computeqgrasppose(robot, robot.q0.copy(), cube, CUBE_PLACEMENT)
    assert robot.collision_model.geometryObjects[-1].placement is CUBE_PLACEMENT  # :42 side effect
    qe, oke = ikgrasp.computeqgrasppose(robot, robot.q0, cube, CUBE_PLACEMENT_TARGET)
    assert ok0 and oke
    assert np.abs(q0 - kat["q0"]).max() <= 1e-12 and np.abs(qe - kat["qe"]).max() <= 1e-12
    assert not np.any(robot.q0)  # qcurrent copied, never mutated (:49)
    assert collision(robot, robot.q0)  # KAT-5 (lab_instructions.ipynb:252)
    assert not collision(robot, qe)
    own, _, _, own_cube = ikgrasp.setuppinocchio()
    ikgrasp.tools.setcubeplacement(own, own_cube, CUBE_PLACEMENT_TARGET)
    assert distanceToObstacle(robot, qe) == distanceToObstacle(own, qe)


def test_batched_api_on_a_pinocchio_style_robot(oracle_cases):
    from ikgrasp.inverse_geometry import computeqgrasppose_batch
    robot, cube = nextage_wrapper()
    c = oracle_cases
    q, ok, it = computeqgrasppose_batch(robot, c["q0"], c["targets"], cube=cube, check_collision=False)
    assert np.array_equal(ok, c["converged"]) and np.array_equal(it[ok], c["iters"][ok])
    assert np.abs(q[ok] - c["q"][ok]).max() <= 1e-9


def test_reference_side_binding_reproduces_kats(kat):
    """examples/ikgrasp_binding.py (what a maintainer adds
    next to the reference's inverse_geometry.py) on a RobotWrapper-shaped
    robot: KAT-1/2 with the collision term, the cube side effect, the planner
    distance and the controller terms through the raw C-ABI."""
    import importlib
    import os
    import sys
    from ikgrasp import config, tools
    from ikgrasp.config import CUBE_PLACEMENT, CUBE_PLACEMENT_TARGET
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    saved = {k: sys.modules.get(k) for k in ("config", "tools")}
    sys.modules["config"], sys.modules["tools"] = config, tools
    sys.path.insert(0, os.path.join(root, "examples"))
    try:
        b = importlib.import_module("ikgrasp_binding")
        robot, cube = nextage_wrapper(pin2=False)
        q0, ok0 = b.computeqgrasppose(robot, robot.q0, cube, CUBE_PLACEMENT)
        qe, oke = b.computeqgrasppose(robot, robot.q0, cube, CUBE_PLACEMENT_TARGET)
        assert ok0 and oke
        assert np.abs(q0 - kat["q0"]).max() <= 1e-12 and np.abs(qe - kat["qe"]).max() <= 1e-12
        assert robot.collision_model.geometryObjects[-1].placement is CUBE_PLACEMENT_TARGET
        assert b.distanceToObstacle(robot, qe) == tools.distanceToObstacle(robot, qe)
        J, Jdv, e, ed = b.task_space_terms(qe, np.zeros(15), q0, np.zeros(15))
        assert np.abs(Jdv).max() == 0.0 and np.abs(J[:, 1:3]).max() == 0.0  # zero velocity; head columns
    finally:
        sys.path.remove(os.path.join(root, "examples"))
        for k, v in saved.items():
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v
