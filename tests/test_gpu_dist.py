"""Multi-rank GPU path: libeslam_gpu sharded over several processes (eslam_gpu_set_comm)
against the one-process CPU oracle, bit for bit.  On a one-GPU box the ranks share the
card: gloo with host staging for 2 and 3 ranks, and RCCL on device buffers with one rank
(the full exchange sequence -- statistics all_gather, totals, counts, all_to_all_v --
runs through RCCL to itself), both through the torch.distributed callbacks and over the
library's own RCCL communicator (eslam_gpu_set_comm_rccl)."""
import pytest

from test_dist_cpu import assert_same, launch, merge, single_oracle

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,n_global,world", [("forced", 5000, 2), ("natural", 2500, 2), ("upload", 2000, 2),
                                                 ("upload", 700, 3)])
def test_sharded_gpu_gloo_equals_single(oracle, tmp_path, name, n_global, world):
    want = single_oracle(name, n_global)
    got = merge(launch("gpu", name, n_global, world, str(tmp_path), mem="host", timeout=400))
    assert_same(got, want, f"gpu {name} N={n_global} world={world}")


@pytest.mark.parametrize("name,n_global", [("forced", 5000), ("upload", 2000)])
def test_sharded_gpu_rccl_one_rank(oracle, tmp_path, name, n_global):
    want = single_oracle(name, n_global)
    got = merge(launch("gpu", name, n_global, 1, str(tmp_path), mem="device", timeout=400))
    assert_same(got, want, f"gpu rccl {name} N={n_global}")


@pytest.mark.parametrize("name,n_global", [("forced", 5000), ("upload", 2000)])
def test_sharded_gpu_native_rccl_one_rank(oracle, tmp_path, name, n_global):
    want = single_oracle(name, n_global)
    got = merge(launch("gpu", name, n_global, 1, str(tmp_path), mem="rccl", timeout=400))
    assert_same(got, want, f"gpu native rccl {name} N={n_global}")


@pytest.mark.parametrize("mem,world", [("host", 2), ("rccl", 1)])
def test_sharded_gpu_two_row_chunks(oracle, tmp_path, mem, world):
    """1.05M particles: canonical summation chunks of two rows (dm_chunk_rows = 2), which
    the small cases above never reach, through gloo (2 ranks) and the library's RCCL."""
    import eslam_abi as A
    n_global = 1050000
    assert A.chunk_rows(n_global) == 2
    want = single_oracle("forced", n_global)
    got = merge(launch("gpu", "forced", n_global, world, str(tmp_path), mem=mem, timeout=280))
    assert_same(got, want, f"gpu {mem} forced N={n_global} world={world}")
