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
