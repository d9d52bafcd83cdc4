"""Pin the CPU oracle against the reference's own known-answer tests.

test/testContactModel.cpp (Boost.Test) and test/UnitTest.cpp restated case by case.  The
reference tests predate contactPointRadius = 0.01 and minContacts = 3
(src/Configuration.hpp:56-58), so each KAT runs with the configuration it implicitly
assumes; where the current code gives a different value the current-code value is pinned as
a regression vector ("Staleness").
"""
import ctypes as C
import math

import numpy as np
import pytest

import eslam_abi as A


class FakeMLSAccess:
    """test/testContactModel.cpp:8-38 -- quadrant patches, records every queried point."""

    def __init__(self, oracle, z, stddev, res=None):
        self.z, self.stddev, self.res = z, stddev, res
        self.points = []
        self.cb = oracle.MAPFN(self.get)

    def get(self, user, p, q_mean, q_stdev, mean, stdev):
        pos = (p[0], p[1], p[2])
        self.points.append(pos)
        index = 0
        if pos[1] > 0:
            index += 2
        if pos[0] > 0:
            index += 1
        # SurfacePatch stores float mean/stdev (see DESIGN.md "map")
        mean[0] = float(np.float32(self.z[index]))
        stdev[0] = float(np.float32(self.stddev[index]))
        if self.res is not None:
            return int(self.res[index])
        return 1


def make_model(oracle, points, radius=0.01, min_contacts=3, q=(1.0, 0.0, 0.0, 0.0)):
    cfg = A.default_config()
    cfg.contact_point_radius = radius
    cfg.min_contacts = min_contacts
    cm = oracle.ContactModelS()
    L = oracle.lib()
    L.or_cm_init(C.byref(cm), C.byref(cfg))
    arr = (A.ContactPoint * len(points))()
    for i, (pos, contact, gid) in enumerate(points):
        arr[i].position[:] = list(pos)
        arr[i].contact = contact
        arr[i].group_id = gid
    L.or_cm_set_contact_points(C.byref(cm), len(points), arr, (C.c_double * 4)(*q))
    return cm


def pose(tx=0.0, ty=0.0, tz=0.0, yaw=0.0):
    c, s = math.cos(yaw), math.sin(yaw)
    # Translation3d * AngleAxisd(yaw, UnitZ), Eigen's AngleAxis -> matrix formula
    return (C.c_double * 12)(c, -s, 0.0, tx, s, c, 0.0, ty, 0.0, 0.0, (1.0 - c) + c, tz)


def evaluate(oracle, cm, T, meas_var, access):
    return oracle.lib().or_cm_evaluate_pose(C.byref(cm), T, meas_var, access.cb, None)


# ---- test_eslam_passes_valid_global_position_to_map_accessor (testContactModel.cpp:69-126)
@pytest.mark.parametrize("radius,expect_z", [(0.0, 0.0), (0.01, -0.01)])
def test_passes_valid_global_position_to_map_accessor(oracle, radius, expect_z):
    pts = [((1, 0, 0), 0.5, -1), ((-1, 0, 0), 0.5, -1)]
    cm = make_model(oracle, pts, radius=radius)
    acc = FakeMLSAccess(oracle, [0] * 4, [0] * 4)
    evaluate(oracle, cm, pose(0.25), 1.0, acc)
    assert len(acc.points) >= 2
    assert np.linalg.norm(np.subtract(acc.points[0], (1.25, 0, expect_z))) < 1e-6
    assert np.linalg.norm(np.subtract(acc.points[1], (-0.75, 0, expect_z))) < 1e-6
    acc = FakeMLSAccess(oracle, [0] * 4, [0] * 4)
    evaluate(oracle, cm, pose(0.25, yaw=math.pi / 2), 1.0, acc)
    assert np.linalg.norm(np.subtract(acc.points[0], (0.25, 1, expect_z))) < 1e-6
    assert np.linalg.norm(np.subtract(acc.points[1], (0.25, -1, expect_z))) < 1e-6


def _check_contact_point_selection(cm, positions, z, expected):
    assert cm.ncp == len(expected)
    for i, idx in enumerate(expected):
        p = np.array(positions[idx], dtype=float)
        p[2] = z[idx]
        got = np.array(list(cm.cp[i].point))
        assert np.linalg.norm(got - p) <= 1e-6 * max(np.linalg.norm(p), 1e-300) + 1e-7


NOGROUP = [((-1, -1, 0), 0.5, -1), ((1, -1, 0), 0.5, -1), ((-1, 1, 0), 0.5, -1), ((1, 1, 0), 0.5, -1)]


# ---- test_updatePose_nogroup (testContactModel.cpp:128-190)
@pytest.mark.parametrize("radius", [0.0, 0.01])
def test_update_pose_nogroup(oracle, radius):
    cm = make_model(oracle, NOGROUP, radius=radius)
    positions = [p for p, _, _ in NOGROUP]
    z = [0, 0, 0, 0]
    acc = FakeMLSAccess(oracle, z, [1, 1, 1, 1])
    assert evaluate(oracle, cm, pose(), 1.0, acc) == 1
    _check_contact_point_selection(cm, positions, z, [0, 1, 2, 3])
    if radius == 0.0:
        assert abs(cm.zdelta) < 1e-6                            # BOOST_CHECK_SMALL
    else:
        assert cm.zdelta == pytest.approx(0.01, rel=1e-9)       # current-code value
    assert cm.zvar == pytest.approx(0.5, rel=1e-8)              # BOOST_CHECK_CLOSE 1e-6 %
    assert cm.weight == pytest.approx(1.0, rel=1e-8)

    z = [0, -0.12, -0.12, -0.12]
    acc = FakeMLSAccess(oracle, z, [1, 1e9, 1e9, 1e9])
    assert evaluate(oracle, cm, pose(), 1.0, acc) == 1
    _check_contact_point_selection(cm, positions, z, [0, 1, 2, 3])
    if radius == 0.0:
        assert abs(cm.zdelta) < 1e-6
    else:
        assert cm.zdelta == pytest.approx(0.01, rel=1e-6)
    assert cm.zvar == pytest.approx(2.0, rel=1e-8)
    assert cm.weight == pytest.approx(1.0, rel=1e-8)


# ---- test_lowest_points_without_groups / with_group (testContactModel.cpp:193-279)
def test_lowest_points_without_groups(oracle):
    pts = [((-1, -1, 0.1), 1, -1), ((1, -1, -0.1), 2, -1), ((-1, 1, 0.1), 3, -1), ((1, 1, -0.1), 4, -1)]
    cm = make_model(oracle, pts)
    L = oracle.lib()
    out = (C.c_double * (3 * A.MAX_CONTACTS))()
    n = L.or_cm_lowest_points(C.byref(cm), out)
    assert n == 4
    for i in range(4):
        assert list(out[3 * i:3 * i + 3]) == list(pts[i][0])
    assert list(cm.contact[:4]) == [1, 2, 3, 4]
    L.or_cm_update_contact_state_lph(C.byref(cm))
    assert list(cm.contact[:4]) == [1, 2, 3, 4]


def test_lowest_points_with_group(oracle):
    pts = [((-1, -1, 0.1), 1, 0), ((1, -1, -0.1), 2, 0), ((-1, 1, 0.1), 3, 1), ((1, 1, -0.1), 4, 1)]
    cm = make_model(oracle, pts)
    L = oracle.lib()
    out = (C.c_double * (3 * A.MAX_CONTACTS))()
    n = L.or_cm_lowest_points(C.byref(cm), out)
    assert n == 2
    assert list(out[0:3]) == list(pts[1][0])
    assert list(out[3:6]) == list(pts[3][0])
    assert list(cm.contact[:4]) == [1, 2, 3, 4]
    L.or_cm_update_contact_state_lph(C.byref(cm))
    assert list(cm.contact[:4]) == [0, 1, 0, 1]


GROUPED = [((-1, -1, 0.1), float("nan"), 0), ((1, -1, -0.1), float("nan"), 0),
           ((-1, 1, 0.1), float("nan"), 1), ((1, 1, -0.1), float("nan"), 1)]


# ---- test_updatePose_group (testContactModel.cpp:281-324): stale against the current code.
def test_update_pose_group_current_code(oracle):
    # minContacts = 3 (current default): only 2 grouped points -> BOOST_REQUIRE would fail
    cm = make_model(oracle, GROUPED, radius=0.01, min_contacts=3)
    acc = FakeMLSAccess(oracle, [-0.1] * 4, [1e9, 1, 1e9, 1])
    assert evaluate(oracle, cm, pose(), 1.0, acc) == 0
    assert cm.ncp == 2                      # NaN contact probability passes the gate (Q13)
    # regression vector with minContacts = 2: ratio-weighted group averaging makes every
    # group's zvar ~1.39e9, so getZVar() = 6.95e8 instead of the stale 1.
    cm = make_model(oracle, GROUPED, radius=0.01, min_contacts=2)
    acc = FakeMLSAccess(oracle, [-0.1] * 4, [1e9, 1, 1e9, 1])
    assert evaluate(oracle, cm, pose(), 1.0, acc) == 1
    assert cm.ncp == 2
    for i in range(2):
        assert cm.cp[i].zvar == pytest.approx(1.39e9, rel=0.01)
        assert cm.cp[i].zdiff == pytest.approx(-0.01, abs=2e-3)
    assert cm.zvar == pytest.approx(6.95e8, rel=0.01)
    # the ContactPoint position comes from the group's FIRST valid contact (Q19)
    assert list(cm.cp[0].point)[:2] == [-1.0, -1.0]
    assert list(cm.cp[1].point)[:2] == [-1.0, 1.0]


# ---- test_mapAbsence_group (testContactModel.cpp:326-362)
def test_map_absence_group(oracle):
    cm = make_model(oracle, GROUPED, radius=0.01, min_contacts=1)
    acc = FakeMLSAccess(oracle, [-0.1] * 4, [1e9, 1, 1e9, 1], res=[True, True, True, False])
    assert evaluate(oracle, cm, pose(), 1.0, acc) == 1
    assert cm.ncp == 1


def test_zero_measurement_variance_throws(oracle):
    cm = make_model(oracle, NOGROUP)
    acc = FakeMLSAccess(oracle, [0] * 4, [1] * 4)
    assert evaluate(oracle, cm, pose(), 0.0, acc) == -1   # src/ContactModel.cpp:122-123


def test_group_poisoning_quirk_q7(oracle):
    """A miss on a group's first evaluated point leaves group_valid false for every later
    contact (src/ContactModel.cpp:194-214)."""
    cm = make_model(oracle, NOGROUP, radius=0.0, min_contacts=0)
    acc = FakeMLSAccess(oracle, [0] * 4, [1] * 4, res=[True, False, True, True])
    evaluate(oracle, cm, pose(), 1.0, acc)
    assert cm.ncp == 1                    # contacts 2 and 3 are skipped after the miss
    assert len(acc.points) == 2           # ... and never queried


# ---- UnitTest.cpp surface_param (121-143) + Buckets::bucketIndex
def test_surface_param(oracle):
    L = oracle.lib()
    sx, sy = C.c_double(), C.c_double()
    pts = (C.c_double * 12)(0, 0, 1.0, 1.0, 0, 1.0, 1.0, 1.0, 1.0, 0, 1.0, 1.5)
    L.or_surface_param_from_points(pts, 4, C.byref(sx), C.byref(sy))
    assert sx.value == pytest.approx(-0.25, abs=1e-12)
    assert sy.value == pytest.approx(0.25, abs=1e-12)
    assert L.or_bucket_index(20, -1.0, 1.0, sx.value) == 7
    assert L.or_bucket_index(20, -1.0, 1.0, sy.value) == 12
    pts = (C.c_double * 12)(0, 0, 1.0, 1.0, 0, 1.0, 1.0, 1.0, 1.0, 0, 1.0, 1.0)
    L.or_surface_param_from_points(pts, 4, C.byref(sx), C.byref(sy))
    assert abs(sx.value) < 1e-12 and abs(sy.value) < 1e-12
    assert L.or_bucket_index(20, -1.0, 1.0, sx.value) == 10
    # clamping at both ends
    assert L.or_bucket_index(20, -1.0, 1.0, -5.0) == 0
    assert L.or_bucket_index(20, -1.0, 1.0, 5.0) == 19


def test_surface_param_matches_least_squares(oracle):
    rng = np.random.default_rng(3)
    L = oracle.lib()
    for _ in range(20):
        P = rng.normal(size=(5, 3))
        sx, sy = C.c_double(), C.c_double()
        L.or_surface_param_from_points((C.c_double * 15)(*P.reshape(-1)), 5, C.byref(sx), C.byref(sy))
        M = np.c_[P[:, 0], P[:, 1], np.ones(5)]
        sol = np.linalg.lstsq(M, P[:, 2], rcond=None)[0]
        assert sx.value == pytest.approx(sol[0], rel=1e-9, abs=1e-12)
        assert sy.value == pytest.approx(sol[1], rel=1e-9, abs=1e-12)
