"""The drop-in takes the reference's own robot object (SURVEY §8b "Duck
typing"): tables read from a RobotWrapper-shaped object equal the compiled
URDF tables, and its collision model equals the compiled scene."""
import numpy as np
import pytest

from fake_pinocchio import nextage_wrapper


@pytest.mark.parametrize("pin2", [False, True])
def test_model_from_wrapper_equals_compiled_tables(pin2):
    from ikgrasp.model import load_nextage
    from ikgrasp.pinocchio_bridge import model_from_robot
    robot, cube = nextage_wrapper(pin2)
    a, b = model_from_robot(robot, cube), load_nextage()
    assert a.joint_names == b.joint_names and list(a.parents) == list(b.parents)
    assert a.root_q == b.root_q and np.array_equal(a.arm_q, b.arm_q) and np.array_equal(a.axis, b.axis)
    for f in ("R", "t", "lower", "upper", "hand_R", "hand_t", "hook_R", "hook_t"):
        assert np.array_equal(getattr(a, f), getattr(b, f)), f


def test_scene_from_wrapper_equals_compiled_scene():
    from ikgrasp.collision import load_nextage_scene
    from ikgrasp.pinocchio_bridge import scene_from_robot
    robot, _ = nextage_wrapper()
    a, b = scene_from_robot(robot), load_nextage_scene()
    assert np.array_equal(a.pairs, b.pairs)
    assert len(a.geoms) == len(b.geoms) == 48
    for ga, gb in zip(a.geoms, b.geoms):
        assert (ga.name, ga.kind, ga.joint, ga.target) == (gb.name, gb.kind, gb.joint, gb.target)
        assert np.array_equal(ga.R, gb.R) and np.array_equal(ga.t, gb.t) and np.array_equal(ga.dims, gb.dims)


def test_setcubeplacement_on_a_wrapper_sets_the_reference_geometries():
    from ikgrasp.config import CUBE_PLACEMENT_TARGET
    from ikgrasp.tools import setcubeplacement
    robot, cube = nextage_wrapper()
    setcubeplacement(robot, cube, CUBE_PLACEMENT_TARGET)  # tools.py:62-68
    for g in (robot.collision_model.geometryObjects[-1], robot.visual_model.geometryObjects[-1],
              cube.collision_model.geometryObjects[0], cube.visual_model.geometryObjects[-1]):
        assert g.placement is CUBE_PLACEMENT_TARGET


def test_unsupported_joint_and_geometry_fail_loudly():
    from ikgrasp.pinocchio_bridge import scene_from_robot, tree_from_model
    from fake_pinocchio import JointModel, NS
    robot, _ = nextage_wrapper()
    robot.model.joints[3] = JointModel("JointModelPZ", 2)
    with pytest.raises(ValueError, match="not supported"):
        tree_from_model(robot.model)
    robot, _ = nextage_wrapper()
    robot.collision_model.geometryObjects[5].geometry = NS()
    with pytest.raises(ValueError, match="unsupported"):
        scene_from_robot(robot)
