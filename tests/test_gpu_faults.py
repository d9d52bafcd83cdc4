"""A cross-block wait of the resample scan that gives up poisons the filter:
nothing further is written and every later call fails until the filter is re-initialised.
The debug spin limit 0 forces the path (eslam_gpu_debug_set_spin_limit)."""
import pytest

import eslam_abi as A
import eslam_amd
import oracle_ffi as O
import synthetic as S
from parity_util import assert_bit_identical

pytestmark = pytest.mark.gpu


def _filter(n, grid):
    cfg = S.bench_config(A.default_config(), n)       # resample forced every update
    gpu = eslam_amd.GpuFilter(cfg, device=0)
    gpu.set_map(grid)
    gpu.init_gaussian(n, [0.0, 0.0, 0.0], [0.1, 0.1, 0.1], 0.18, 1.001)
    return gpu, cfg


@pytest.mark.parametrize("n", [4096, 300_000])
def test_timeout_poisons_filter_until_reinit(n):
    grid = S.flat_map(cells=200)
    stream = S.step_stream(4)
    gpu, cfg = _filter(n, grid)
    gpu.step(stream[0])
    gpu.sync()
    gpu.debug_set_spin_limit(0)
    gpu.step(stream[1])                   # the waits give up inside this launch
    with pytest.raises(eslam_amd.EslamError, match="cross-block wait gave up"):
        gpu.sync()
    for call in (lambda: gpu.step(stream[2]), gpu.download, gpu.weights_sum, gpu.sync):
        with pytest.raises(eslam_amd.EslamError, match="re-initialised"):
            call()
    # starting over clears the fault; with the normal limit the filter equals the oracle again
    gpu.debug_set_spin_limit(1 << 18)
    gpu.init_gaussian(n, [0.0, 0.0, 0.0], [0.1, 0.1, 0.1], 0.18, 1.001)
    orc = O.OracleFilter(cfg, O.SUM_CONTRACT)
    orc.set_map(grid)
    orc.init_gaussian(n, [0.0, 0.0, 0.0], [0.1, 0.1, 0.1], 0.18, 1.001)
    # the GPU's event counters advanced through the poisoned steps: the oracle takes over the
    # GPU's fresh particles and RNG state
    orc.upload(gpu.download())
    orc.set_rng_state(gpu.rng_state())
    for st in stream[2:]:
        assert gpu.step(st) == orc.step(st)
    gpu.sync()
    assert_bit_identical(gpu.download(), orc.download(), "after re-init")
