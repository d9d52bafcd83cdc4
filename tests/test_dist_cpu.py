"""Multi-rank path on the CPU: the oracle's sharded mode (the CPU statement of the
multi-GPU decomposition) over gloo, world sizes 2 and 3, through the same eslam_comm
callbacks (slam-eslam_amd/eslam_dist.TorchComm) the GPU library uses.  A sharded run
concatenated over the ranks equals the one-process filter bit for bit."""
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle_ffi as O
from dist_scenarios import run_scenario, scenario_config

HERE = os.path.dirname(os.path.abspath(__file__))


def launch(kind, name, n_global, world, tmp, mem="host", timeout=240):
    """Run the ranks; they meet through a FileStore in `tmp` (no rendezvous port to race for)."""
    store = os.path.join(tmp, f"store_{kind}_{name}_{world}_{mem}")
    if os.path.exists(store):
        os.remove(store)
    procs, outs = [], []
    for r in range(world):
        out = os.path.join(tmp, f"{kind}_{name}_{world}_{r}.npz")
        env = dict(os.environ, RANK=str(r), LOCAL_RANK="0", WORLD_SIZE=str(world), ESLAM_DIST_STORE=store,
                   OMP_NUM_THREADS="1")
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "dist_worker.py"), kind, name, str(n_global),
                                       out, mem], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
        outs.append(out)
    logs = []
    for p in procs:
        try:
            o, _ = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        logs.append(o.decode(errors="replace"))
    bad = [f"--- rank {r} (exit {p.returncode}) ---\n{log[-2500:]}" for r, (p, log) in enumerate(zip(procs, logs))
           if p.returncode != 0]
    assert not bad, "\n".join(bad)
    return [dict(np.load(o)) for o in outs]


def merge(parts):
    """Concatenate the per-rank arrays; scalars (info, sums, best, rng) must agree."""
    out = {}
    for key in parts[0]:
        vals = [p[key] for p in parts]
        if "/" in key and not key.endswith("/info"):
            out[key] = np.concatenate(vals)
        else:
            for v in vals[1:]:
                assert np.array_equal(v.view(np.uint8), vals[0].view(np.uint8)), f"{key} differs between ranks"
            out[key] = vals[0]
    return out


def assert_same(got, want, label):
    assert set(got) == set(want), f"{label}: keys {sorted(set(got) ^ set(want))}"
    for key in want:
        g, w = got[key], want[key]
        assert g.shape == w.shape, f"{label} {key}: shape {g.shape} != {w.shape}"
        assert np.array_equal(np.ascontiguousarray(g).view(np.uint8), np.ascontiguousarray(w).view(np.uint8)), \
            f"{label} {key}: differs at {np.count_nonzero(g != w)} entries"


def single_oracle(name, n_global):
    cfg = scenario_config(name, n_global)
    f = O.OracleFilter(cfg, O.SUM_CONTRACT)
    return run_scenario(f, name, n_global, 0, n_global, info_fn=lambda g: g.info())


@pytest.mark.parametrize("name,n_global,world", [("forced", 3000, 2), ("natural", 2500, 2), ("upload", 2000, 2),
                                                 ("forced", 1000, 3), ("upload", 700, 3), ("hash", 2000, 2),
                                                 ("hash", 1500, 3), ("maps", 3000, 2), ("maps", 1500, 3),
                                                 ("burst", 3000, 2), ("edit", 3000, 2), ("edit", 1000, 3),
                                                 ("heirloom", 2000, 2), ("heirloom", 1500, 3),
                                                 ("chunks", 3000, 2), ("chunks", 1500, 3)])
def test_sharded_oracle_equals_single(oracle, tmp_path, name, n_global, world):
    want = single_oracle(name, n_global)
    got = merge(launch("oracle", name, n_global, world, str(tmp_path)))
    assert_same(got, want, f"{name} N={n_global} world={world}")
    if name == "maps":
        # particles (and their own maps) did migrate between ranks
        import eslam_abi as A
        g = A.shard_bounds(n_global, world)
        owner = np.searchsorted(g, np.arange(n_global), side="right") - 1
        moved = sum(int(np.count_nonzero(owner[want[k].astype(np.int64)] != owner)) for k in want if k.endswith("/anc"))
        assert moved > 0


def test_shard_bounds_chunk_aligned():
    import eslam_abi as A
    for n in (64, 1000, 262144 * 3 + 5, 4 * 1024 * 1024 * 8):
        for w in (1, 2, 3, 8):
            if -(-n // (64 * A.chunk_rows(n))) < w:
                continue
            g = A.shard_bounds(n, w)
            csz = 64 * A.chunk_rows(n)
            assert g[0] == 0 and g[-1] == n and all(g[r] % csz == 0 for r in range(w))
            assert all(g[r + 1] > g[r] for r in range(w))


def test_shard_bounds_with_a_fixed_chunk():
    """eslam_config.sum_chunk_rows (ABI 8): an explicit chunk overrides dm_chunk_rows, and the
    shard starts follow it (configs[3]: 16M over 8 ranks in a rank's 7-row chunks)."""
    import eslam_abi as A
    assert A.chunk_rows(16 * 1024 * 1024) == 13 and A.chunk_rows(16 * 1024 * 1024, 7) == 7
    assert A.chunk_rows(2 * 1024 * 1024) == 7
    g = A.shard_bounds(16 * 1024 * 1024, 8, 7)
    assert g[0] == 0 and g[-1] == 16 * 1024 * 1024
    assert all(b % (64 * 7) == 0 for b in g[:-1]) and all(g[r + 1] > g[r] for r in range(8))
    assert A.shard_bounds(3000, 2, 3) != A.shard_bounds(3000, 2) or A.chunk_rows(3000) == 3
