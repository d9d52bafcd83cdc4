"""Multi-rank GPU path: libeslam_gpu sharded over several processes (eslam_gpu_set_comm)
against the one-process CPU oracle, bit for bit.  On a one-GPU box the ranks share the
card: gloo with host staging for 2 and 3 ranks, and RCCL on device buffers with one rank
(the full exchange sequence -- statistics all_gather, totals, counts, all_to_all_v --
runs through RCCL to itself), both through the torch.distributed callbacks and over the
library's own RCCL communicator (eslam_gpu_set_comm_rccl)."""
import numpy as np
import pytest

from test_dist_cpu import assert_same, launch, merge, single_oracle

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,n_global,world", [("forced", 5000, 2), ("natural", 2500, 2), ("upload", 2000, 2),
                                                 ("upload", 700, 3), ("hash", 3000, 2), ("hash", 1500, 3),
                                                 ("maps", 3000, 2), ("maps", 1500, 3),
                                                 ("burst", 5000, 2), ("burst", 7001, 3), ("edit", 3000, 2),
                                                 ("edit", 1500, 3), ("heirloom", 2000, 2), ("heirloom", 1500, 3),
                                                 ("chunks", 3000, 2), ("chunks", 1500, 3)])
def test_sharded_gpu_gloo_equals_single(oracle, tmp_path, name, n_global, world):
    want = single_oracle(name, n_global)
    got = merge(launch("gpu", name, n_global, world, str(tmp_path), mem="host", timeout=400))
    assert_same(got, want, f"gpu {name} N={n_global} world={world}")


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_records_equal_single_context(gpu_mod, tmp_path, world):
    """logDebug on a sharded filter (src/PoseEstimator.cpp:285-287,322-325): the PoseParticle
    records with their cpoints, meas_pos and meas_theta, downloaded after every update by every
    rank (a collective: records of ancestors that sat on another rank are fetched from it),
    concatenated over 2 / 3 gloo ranks, equal the one-context filter's records bit for bit --
    and particles did descend from ancestors on other ranks.  The one-context records equal the
    oracle's capture (test_gpu_records.py)."""
    import eslam_abi as A
    from dist_scenarios import run_scenario, scenario_config
    n_global = 6000
    cfg = scenario_config("records", n_global)
    f = gpu_mod.GpuFilter(cfg)
    want = run_scenario(f, "records", n_global, 0, n_global, info_fn=lambda g: g.sync())
    f.close()
    got = merge(launch("gpu", "records", n_global, world, str(tmp_path), mem="host", timeout=400))
    assert_same(got, want, f"gpu records N={n_global} world={world}")
    g = A.shard_bounds(n_global, world)
    owner = np.searchsorted(g, np.arange(n_global), side="right") - 1
    moved = sum(int(np.count_nonzero(owner[want[k].astype(np.int64)] != owner)) for k in want if k.endswith("/anc"))
    assert moved > 0
    assert any(want[k].any() for k in want if k.endswith("/rec_n_cpoints"))


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_getter_on_one_rank_then_destroy(oracle, tmp_path, world):
    """A rank-local getter on rank 0 only after deferred updates, then every rank destroys its
    context (include/eslam_gpu.h, SPMD order): no rank hangs in the deferred exchange, and
    rank 0 holds the single filter's particles."""
    want = single_oracle("getter0", 5000)
    parts = launch("gpu", "getter0", 5000, world, str(tmp_path), mem="host", timeout=300)
    hi = len(parts[0]["last/x"])
    for key, v in parts[0].items():
        assert np.array_equal(v.view(np.uint8), want[key][:hi].view(np.uint8)), key
    assert all(not p for p in parts[1:])


@pytest.mark.parametrize("name,n_global", [("forced", 5000), ("upload", 2000)])
def test_sharded_gpu_rccl_one_rank(oracle, tmp_path, name, n_global):
    want = single_oracle(name, n_global)
    got = merge(launch("gpu", name, n_global, 1, str(tmp_path), mem="device", timeout=400))
    assert_same(got, want, f"gpu rccl {name} N={n_global}")


@pytest.mark.parametrize("name,n_global", [("forced", 5000), ("upload", 2000), ("hash", 3000), ("maps", 2000)])
def test_sharded_gpu_native_rccl_one_rank(oracle, tmp_path, name, n_global):
    want = single_oracle(name, n_global)
    got = merge(launch("gpu", name, n_global, 1, str(tmp_path), mem="rccl", timeout=400))
    assert_same(got, want, f"gpu native rccl {name} N={n_global}")


@pytest.mark.parametrize("mem,world", [("host", 2), ("rccl", 1)])
def test_sharded_gpu_two_row_chunks(oracle, tmp_path, mem, world):
    """525k particles: canonical summation chunks of two rows (dm_chunk_rows = 2), which
    the small cases above never reach, through gloo (2 ranks) and the library's RCCL."""
    import eslam_abi as A
    n_global = 525000
    assert A.chunk_rows(n_global) == 2
    want = single_oracle("forced", n_global)
    got = merge(launch("gpu", "forced", n_global, world, str(tmp_path), mem=mem, timeout=280))
    assert_same(got, want, f"gpu {mem} forced N={n_global} world={world}")


@pytest.mark.timeout(1200)
def test_config3_eight_ranks_equal_single_context(oracle, tmp_path):
    """BASELINE configs[3]'s decomposition on one GPU: 16M particles as 8 ranks x 2M (gloo,
    host staging; the ranks share the card; the summation chunk sized by a rank), 3 steps of the bench workload with a forced
    resample each.  Every rank's shard equals the same slice of ONE 16M-particle context bit
    for bit (all fields, the last resample's ancestors as global indices), every rank reports
    the single context's update info, best index and RNG state, and the single context's last
    resample passes the stratified-resample properties (src/ParticleFilter.hpp:85-108)."""
    import eslam_abi as A
    import eslam_amd
    from dist_scenarios import CONFIG3_STEPS, FIELDS, digest, run_config3, scenario_config
    from parity_util import check_resample_properties
    n_global, world = 16 * 1024 * 1024, 8
    parts = launch("gpu", "config3", n_global, world, str(tmp_path), mem="host", timeout=900)
    cfg = scenario_config("config3", n_global)
    assert cfg.sum_chunk_rows == 7                 # sized by a rank's 2M (dm_chunk_rows(16M) = 13)
    f = eslam_amd.GpuFilter(cfg)
    rec, fields, anc, best, rng = run_config3(f, n_global, 0, n_global, info_fn=lambda g: g.sync())
    bounds = A.shard_bounds(n_global, world, cfg.sum_chunk_rows)
    for r, p in enumerate(parts):
        lo, hi = bounds[r], bounds[r + 1]
        assert tuple(p["range"]) == (lo, hi)
        for fld in FIELDS:
            assert str(p[f"sha/{fld}"]) == digest(fields[fld][lo:hi]), f"rank {r}: {fld} differs"
        assert str(p["sha/anc"]) == digest(anc[lo:hi].astype(np.uint32)), f"rank {r}: ancestors differ"
        assert np.array_equal(p["centroid"].view(np.uint64), rec["centroid"].view(np.uint64)), f"rank {r}: centroid"
        for k in range(CONFIG3_STEPS):
            assert np.array_equal(p[f"s{k}/info"].view(np.uint64), rec[f"s{k}/info"].view(np.uint64)), (r, k)
        assert int(p["best"][0]) == int(best[0]) and int(p["rng"][0]) == int(rng[0])
    assert rec[f"s{CONFIG3_STEPS - 1}/info"][6] == 1.0        # resampled
    after = A.ParticleArrays(n_global)
    for fld in FIELDS:
        getattr(after, fld)[:] = fields[fld]
    check_resample_properties(anc, after, n_global)
    f.close()


@pytest.mark.timeout(1500)
def test_config4_eight_ranks_equal_single_context(oracle, tmp_path):
    """BASELINE configs[4]'s decomposition on one GPU: 64M particles with per-particle maps as
    8 ranks x 8M (gloo, host staging; the ranks share the card), 3 steps of bench.py
    --local-maps' workload (rough map unmapped beyond x = 0.3 m, a scan merged into every
    particle's map after each step, forced resample).  Every rank's shard equals the same slice
    of ONE 64M-particle context bit for bit (all fields, the last resample's ancestors as
    global indices, the maps of 64 sampled particles -- a migrated particle carries its store),
    every rank reports the single context's update info, best index and RNG state, and the
    single context's last resample passes the stratified-resample properties."""
    import eslam_abi as A
    import eslam_amd
    from dist_scenarios import CONFIG3_STEPS, FIELDS, digest, map_samples, run_config3, scenario_config
    from parity_util import check_resample_properties
    n_global, world = 64 * 1024 * 1024, 8
    parts = launch("gpu", "config4", n_global, world, str(tmp_path), mem="host", timeout=1200)
    cfg = scenario_config("config4", n_global)
    f = eslam_amd.GpuFilter(cfg)
    rec, fields, anc, best, rng = run_config3(f, n_global, 0, n_global, info_fn=lambda g: g.sync(), name="config4")
    bounds = A.shard_bounds(n_global, world, cfg.sum_chunk_rows)
    seen = 0
    for r, p in enumerate(parts):
        lo, hi = bounds[r], bounds[r + 1]
        assert tuple(p["range"]) == (lo, hi)
        for fld in FIELDS:
            assert str(p[f"sha/{fld}"]) == digest(fields[fld][lo:hi]), f"rank {r}: {fld} differs"
        assert str(p["sha/anc"]) == digest(anc[lo:hi].astype(np.uint32)), f"rank {r}: ancestors differ"
        for k in range(CONFIG3_STEPS):
            assert np.array_equal(p[f"s{k}/info"].view(np.uint64), rec[f"s{k}/info"].view(np.uint64)), (r, k)
        assert int(p["best"][0]) == int(best[0]) and int(p["rng"][0]) == int(rng[0])
        for g in map_samples(n_global):
            if lo <= g < hi:
                assert str(p[f"map/{g}"]) == str(rec[f"map/{g}"]), f"rank {r}: map of particle {g} differs"
                seen += 1
    assert seen == len(map_samples(n_global))
    assert rec[f"s{CONFIG3_STEPS - 1}/info"][6] == 1.0        # resampled
    after = A.ParticleArrays(n_global)
    for fld in FIELDS:
        getattr(after, fld)[:] = fields[fld]
    check_resample_properties(anc, after, n_global)
    f.close()
