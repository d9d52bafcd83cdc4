# GPU test session: the named test files (default: all -m gpu tests), one pytest process
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu "$@" > gpurun_out/pytest_gpu.log 2>&1
rc=$?
grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -3
grep -E "^(FAILED|ERROR)" gpurun_out/pytest_gpu.log | head -20
exit $rc
