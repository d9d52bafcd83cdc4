"""One rank of a multi-rank test: runs a scenario on its shard and saves what it holds.

    RANK=r WORLD_SIZE=w MASTER_ADDR=127.0.0.1 MASTER_PORT=p \
        python tests/dist_worker.py {oracle|gpu} SCENARIO N_GLOBAL OUT.npz [host|device]

oracle: the CPU oracle's sharded mode over gloo (host-memory callbacks);
gpu:    libeslam_gpu sharded over gloo (host staging) or, with 'device', RCCL on device
        buffers through the torch.distributed callbacks, or, with 'rccl', over the library's
        own RCCL communicator (eslam_gpu_set_comm_rccl; one rank per GPU).
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "slam-eslam_amd"))

import numpy as np  # noqa: E402


def main():
    kind, name, n_global, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
    mem = sys.argv[5] if len(sys.argv) > 5 else "host"
    import torch
    import torch.distributed as dist
    import eslam_abi as A
    import eslam_dist
    from dist_scenarios import run_scenario, scenario_config
    rank = int(os.environ["RANK"])
    # rendezvous through a file the launcher names (no TCP port to race for); env:// otherwise
    store = os.environ.get("ESLAM_DIST_STORE")
    init = dict(init_method="file://" + store, rank=rank, world_size=int(os.environ["WORLD_SIZE"])) if store else {}
    if kind == "gpu" and mem in ("device", "rccl"):
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
        dist.init_process_group("nccl", **init)
    else:
        dist.init_process_group("gloo", **init)
    comm = eslam_dist.TorchComm(device_memory=(mem in ("device", "rccl")))
    cfg = scenario_config(name, n_global)
    bounds = A.shard_bounds(n_global, comm.nranks, cfg.sum_chunk_rows)
    lo, hi = bounds[rank], bounds[rank + 1]
    if kind == "oracle":
        import oracle_ffi as O
        f = O.OracleFilter(cfg, O.SUM_CONTRACT)
        f.set_comm(comm, n_global)
        rec = run_scenario(f, name, n_global, lo, hi, info_fn=lambda g: g.info())
    else:
        dev = int(os.environ.get("LOCAL_RANK", "0"))
        if mem == "rccl":
            f = eslam_dist.RcclShardedGpuFilter(cfg, n_global, rank, comm.nranks, device=dev)
        else:
            f = eslam_dist.ShardedGpuFilter(cfg, n_global, comm, device=dev)
        if name in ("config3", "config4"):
            from dist_scenarios import digest, run_config3
            # the ranks share one GPU: a rank's waits between its own blocks may outlast another
            # rank's long kernels (the 8M-particle map pools' initialisation), so they get
            # seconds instead of the default ~60 ms before the filter is declared faulted
            f.debug_set_spin_limit(1 << 24)
            rec, fields, anc, best, rng = run_config3(f, n_global, lo, hi, info_fn=lambda g: g.sync(), name=name)
            for fld, v in fields.items():
                rec[f"sha/{fld}"] = np.array(digest(v))
            rec["sha/anc"] = np.array(digest(anc.astype(np.uint32)))
            rec["best"] = best
            rec["rng"] = rng
            rec["range"] = np.array([lo, hi])
        else:
            try:
                rec = run_scenario(f, name, n_global, lo, hi, info_fn=lambda g: g.sync())
            except Exception as e:
                if comm.error is not None:       # the collective's own failure, not the library's report of it
                    raise RuntimeError(f"rank {rank}: {e}") from comm.error
                raise
        f.close()
    if comm.error is not None:
        raise comm.error
    np.savez(out, **rec)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
