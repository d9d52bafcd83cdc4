"""The reference's contact-model known-answer tests as whole-filter inputs (test infrastructure).

test/testContactModel.cpp evaluates ContactModel::evaluatePose against FakeMLSAccess
(test/testContactModel.cpp:8-38): four quadrant patches, index = (y > 0 ? 2 : 0) + (x > 0 ? 1 : 0),
patch (z[index], stddev[index]), found = res[index].  kat_grid() builds the same quadrants as a
2 x 2-cell MLS grid (cells [-2, 0) and [0, 2) per axis, one patch per cell, none where res is
false), so a one-particle filter at the KAT's pose runs the case through updateWeights -- on the
CPU oracle and through the HIP library's C ABI alike.  The grid and the accessor agree wherever
no coordinate is exactly 0 (the accessor puts 0 in the lower quadrant, floor() in the upper);
every queried point of the cases below is off the axes.  The accessor applies no 3-sigma gate;
every case here passes MLSGrid::getPatch's gate (|z - mean| <= 0.13 < 3 sqrt(stdev^2 + measVar),
measVar = 1).
"""
import numpy as np

import eslam_abi as A

NOGROUP = [((-1, -1, 0), 0.5, -1), ((1, -1, 0), 0.5, -1), ((-1, 1, 0), 0.5, -1), ((1, 1, 0), 0.5, -1)]
GROUPED = [((-1, -1, 0.1), float("nan"), 0), ((1, -1, -0.1), float("nan"), 0),
           ((-1, 1, 0.1), float("nan"), 1), ((1, 1, -0.1), float("nan"), 1)]

# name: (contacts, z[4], stddev[4], res[4], radius, minContacts, expected)
# expected: ncp, accepted, and where the reference pins them the contact model's outputs
# weight / zdelta / zvar (getWeight / getZDelta / getZVar)
CASES = {
    # test_updatePose_nogroup (testContactModel.cpp:152-170); radius 0 = the test's assumption
    "nogroup_flat_r0": (NOGROUP, [0, 0, 0, 0], [1, 1, 1, 1], None, 0.0, 3,
                        dict(ncp=4, accepted=1, weight=1.0, zdelta=0.0, zvar=0.5)),
    # the same with the current contactPointRadius = 0.01: zDelta = +0.01 (current-code value)
    "nogroup_flat_r001": (NOGROUP, [0, 0, 0, 0], [1, 1, 1, 1], None, 0.01, 3,
                          dict(ncp=4, accepted=1, weight=1.0, zdelta=0.01, zvar=0.5)),
    # testContactModel.cpp:171-189: three quadrants at -0.12 with stdev 1e9
    "nogroup_steps_r0": (NOGROUP, [0, -0.12, -0.12, -0.12], [1, 1e9, 1e9, 1e9], None, 0.0, 3,
                         dict(ncp=4, accepted=1, weight=1.0, zdelta=0.0, zvar=2.0)),
    # test_updatePose_group (testContactModel.cpp:281-324) under the current minContacts = 3:
    # two grouped points, rejected (NaN contact probability passes the gate, Q13)
    "group_min3": (GROUPED, [-0.1] * 4, [1e9, 1, 1e9, 1], None, 0.01, 3, dict(ncp=2, accepted=0)),
    # the same with minContacts = 2: ratio-weighted group averages, zVar ~ 6.95e8
    "group_min2": (GROUPED, [-0.1] * 4, [1e9, 1, 1e9, 1], None, 0.01, 2,
                   dict(ncp=2, accepted=1, zvar=6.95e8)),
    # test_mapAbsence_group (testContactModel.cpp:326-362): quadrant 3 has no patch
    "map_absence_group": (GROUPED, [-0.1] * 4, [1e9, 1, 1e9, 1], [True, True, True, False], 0.01, 1,
                          dict(ncp=1, accepted=1)),
    # Q7: a miss on contact 1 poisons every later contact (src/ContactModel.cpp:194-214)
    "poison_q7": (NOGROUP, [0, 0, 0, 0], [1, 1, 1, 1], [True, False, True, True], 0.0, 0,
                  dict(ncp=1, accepted=1)),
}


def kat_grid(z, stddev, res=None):
    """FakeMLSAccess(z, stddev, res) as a 2 x 2 grid; cell (m, n) = quadrant m + 2 n."""
    res = [True] * 4 if res is None else list(res)
    cell_start = [0]
    mean, sd = [], []
    for q in range(4):                         # cell index n * width + m == quadrant index
        if res[q]:
            mean.append(z[q])
            sd.append(stddev[q])
        cell_start.append(len(mean))
    return A.GridArrays(2, 2, (2.0, 2.0), (-2.0, -2.0), np.array(cell_start, dtype=np.uint32),
                        np.array(mean, dtype=np.float32), np.array(sd, dtype=np.float32))


def kat_setup(name):
    """(config, grid, step input, one-particle state, expected) of a KAT case: the particle sits
    at the origin with zSigma = 1 and measurementError = 0, so measVar = 1 as in the tests."""
    contacts, z, sd, res, radius, min_contacts, expected = CASES[name]
    cfg = A.default_config()
    cfg.particle_count = 1
    cfg.contact_point_radius = radius
    cfg.min_contacts = min_contacts
    cfg.measurement_error = 0.0
    cfg.min_effective = 0                      # no resample: the state stays the KAT's
    st = A.StepInput()
    st.body2odometry_rot[:] = [1.0, 0.0, 0.0, 0.0]
    st.n_contacts = len(contacts)
    st.ltc_count = 1
    for i, (pos, contact, gid) in enumerate(contacts):
        st.contacts[i].position[:] = list(pos)
        st.contacts[i].contact = contact
        st.contacts[i].group_id = gid
    pa = A.ParticleArrays(1)
    pa.zsigma[:] = 1.0
    pa.weight[:] = 1.0
    pa.floating[:] = 1
    return cfg, kat_grid(z, sd, res), st, pa, expected
