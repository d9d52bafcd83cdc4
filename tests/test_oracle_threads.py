"""The oracle's OpenMP per-particle loops (or_set_threads) give the same bits as one thread.

The multi-threaded oracle exists only for the CPU baseline's labelled multi-core figure
(bench.py --cpu-threads, SURVEY §8d "oracle-OpenMP (correct)"); it must not change a result.
"""
import numpy as np
import pytest

import eslam_abi as A
import oracle_ffi as O
import synthetic as S


def run(threads, sum_mode, rough, n=20000, steps=4):
    cfg = S.bench_config(A.default_config(), n)
    f = O.OracleFilter(cfg, sum_mode)
    f.set_threads(threads)
    f.set_map(S.rough_map(cells=200) if rough else S.flat_map(cells=200))
    f.init_gaussian(n, [0.0, 0.0, 0.0], [0.1, 0.1, 0.1], 0.18, 1.001)
    infos = []
    for st in S.step_stream(steps, tilt=rough):
        f.step(st)
        i = f.info()
        infos.append(tuple(i.as_dict().values()))
    pa = f.download()
    return infos, [np.array(a, copy=True) for a in (pa.x, pa.y, pa.orientation, pa.zpos, pa.zsigma, pa.weight, pa.mprob,
                                                        pa.floating, pa.n_contact_points)]


@pytest.mark.parametrize("sum_mode", [O.SUM_CONTRACT, O.SUM_REFERENCE])
@pytest.mark.parametrize("rough", [False, True])
def test_threads_bit_identical(sum_mode, rough):
    i1, p1 = run(1, sum_mode, rough)
    i4, p4 = run(4, sum_mode, rough)
    assert i1 == i4
    for a, b in zip(p1, p4):
        assert a.tobytes() == b.tobytes()
