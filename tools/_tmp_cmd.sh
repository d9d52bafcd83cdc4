cd $GRAFT_REPO_ROOT
bash tools/gpu_round.sh tests || exit 1
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/bench_fin.log 2>&1 || exit 1
python - <<'PY' > gpurun_out/notiming.log 2>&1
import sys, time
sys.path.insert(0, 'slam-eslam_amd'); sys.path.insert(0, 'tests')
import eslam_abi as A, eslam_amd, synthetic as S
n = 4 * 1024 * 1024
grid = S.flat_map(cells=1000)
stream = S.step_stream(60)
cfg = S.bench_config(A.default_config(), n)
f = eslam_amd.GpuFilter(cfg)
f.set_map(grid); f.init_gaussian(n, [0, 0, 0], [0.1, 0.1, 0.1], 0.18, 1.001)
for st in stream[:10]: f.step(st)
f.sync()
for timing in (False, True, False):
    f.enable_timing(timing)
    t0 = time.perf_counter()
    for st in stream[10:50]: f.step(st)
    f.sync()
    dt = (time.perf_counter() - t0) / 40
    print("timing", timing, "ms/step", round(dt * 1e3, 4), f.kernel_times() if timing else "")
PY
