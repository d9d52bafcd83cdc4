"""bench.py's launch contract on a host without enough GPUs (CPU only): `--gpus N` must fail
non-zero rather than measure fewer GPUs and report them as N."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_bench(args, **env_over):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_over)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, cwd=ROOT,
                          capture_output=True, text=True, timeout=300)


def test_gpus_beyond_visible_fails():
    import torch
    if torch.cuda.device_count() >= 2:
        import pytest
        pytest.skip("host has 2 or more GPUs")
    r = run_bench(["--gpus", "2", "--steps", "1", "--warmup", "0"])
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert r.stdout.strip() == ""                   # no JSON line claiming any GPU count
    assert "--gpus 2 but only" in r.stderr


def test_world_size_mismatch_fails():
    r = run_bench(["--gpus", "2", "--steps", "1", "--warmup", "0"], WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert r.stdout.strip() == ""
    assert "--gpus 2 but WORLD_SIZE=3" in r.stderr


def test_multi_gpu_default_is_weak_scaling():
    """--gpus N keeps the one-GPU line's per-GPU work (configs[2]'s 4M particles per rank);
    configs[3] (16M over 8 GPUs) is named when asked for explicitly."""
    sys.path.insert(0, ROOT)
    import bench
    assert "weak-scaled to 8 GPUs (32M global)" in bench.workload_name(4 * 1024 * 1024, 8, False)
    assert bench.workload_name(4 * 1024 * 1024, 1, False) == "configs[2]"
    assert bench.workload_name(2 * 1024 * 1024, 8, False) == "configs[3]"
    assert bench.workload_name(262144, 1, False) == "configs[1]"
