"""Model compiler (URDF -> kernel tables) against the oracle's hand-transcribed
tables and the notebook's joint order."""
import numpy as np
import pytest

from ikgrasp.model import DualArmModel, load_nextage, parse_urdf, rpy_to_matrix
from oracle import ik_oracle as o


def test_compiled_tables_match_oracle(kat):
    m = load_nextage()
    assert m.joint_names == kat["joint_names"]
    assert m.parents == o.PARENT
    assert list(m.axis) == o.AXIS
    assert np.array_equal(m.lower, o.LOWER) and np.array_equal(m.upper, o.UPPER)
    for i, (R, t) in enumerate(o.joint_placements()):
        assert np.array_equal(m.R[i], R) and np.array_equal(m.t[i], t)
    assert np.array_equal(m.hand_R[0], o.FRAME_LEFT[1]) and np.array_equal(m.hand_t[1], o.FRAME_RIGHT[2])
    assert np.array_equal(m.hook_R[1], o.HOOK_RIGHT[0]) and np.array_equal(m.hook_t[0], o.HOOK_LEFT[1])
    assert m.root_q == 0 and m.arm_q.tolist() == [[3, 4, 5, 6, 7, 8], [9, 10, 11, 12, 13, 14]]
    assert m.passive_q == [1, 2]


def test_json_roundtrip():
    m = load_nextage()
    m2 = DualArmModel.from_json(m.to_json())
    assert m2.joint_names == m.joint_names
    for k in ("R", "t", "lower", "upper", "hand_R", "hand_t", "hook_R", "hook_t"):
        assert np.array_equal(getattr(m, k), getattr(m2, k))


def test_rpy_matches_rotation():
    R = rpy_to_matrix(0.3, -0.2, 1.1)
    assert np.allclose(R @ R.T, np.eye(3), atol=1e-15)
    cz, sz = np.cos(1.1), np.sin(1.1)
    cy, sy = np.cos(-0.2), np.sin(-0.2)
    cx, sx = np.cos(0.3), np.sin(0.3)
    Rz = np.array([[cz, -sz, 0], [sz, cz, 0], [0, 0, 1]])
    Ry = np.array([[cy, 0, sy], [0, 1, 0], [-sy, 0, cy]])
    Rx = np.array([[1, 0, 0], [0, cx, -sx], [0, sx, cx]])
    assert np.allclose(R, Rz @ Ry @ Rx, atol=1e-15)


TOY = """<robot name="toy">
  <link name="base"/><link name="a"/><link name="b"/>
  <joint name="j_b" type="revolute"><parent link="base"/><child link="b"/>
    <origin xyz="0 0 1"/><axis xyz="0 1 0"/><limit lower="-1" upper="1"/></joint>
  <joint name="j_a" type="revolute"><parent link="base"/><child link="a"/>
    <origin xyz="1 0 0"/><axis xyz="1 0 0"/><limit lower="-2" upper="2"/></joint>
</robot>"""


def test_urdf_children_sorted_by_joint_name():
    # urdfdom keeps joints in a std::map: siblings are visited alphabetically
    tree = parse_urdf(TOY)
    assert tree.joint_names() == ["j_a", "j_b"]
    assert tree.joints[0].axis == 0 and tree.joints[1].axis == 1


def test_unaligned_axis_compiled_onto_canonical_axis():
    """An unaligned axis (RevoluteUnaligned) is re-expressed on the nearest
    canonical axis (here Z); tests/test_generic_model.py checks the kinematics."""
    tree = parse_urdf(TOY.replace('<axis xyz="0 1 0"/>', '<axis xyz="0 0.6 0.8"/>'))
    j = tree.joints[1]
    assert j.axis == 2 and np.allclose(j.Q @ np.array([0, 0, 1.0]), [0, 0.6, 0.8])


def test_structure_validation_rejects_non_dual_arm():
    tree = parse_urdf(TOY)
    with pytest.raises(KeyError):
        DualArmModel.from_trees(tree, tree, hands=("nope", "nope"))
