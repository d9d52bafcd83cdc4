cd "$(dirname "$0")/.."
for lib in slam-eslam_amd/lib/libeslam_gpu*.so; do
  echo "== $lib"
  ESLAM_GPU_LIB=$PWD/$lib timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['kernel_ms'])" || exit 1
done
