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
