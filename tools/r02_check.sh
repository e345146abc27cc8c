#!/usr/bin/env bash
# Round-2 GPU check (run on the GPU box from the repo root): pytest -m gpu, then one bench line per
# BASELINE config on one GPU. Every GPU step has its own time limit; the first failure ends the script.
set -u -o pipefail
OUT=gpurun_out/${1:-r02}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --durations=15 --timeout 240 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
for args in "" "--config 3" "--config 4 --steps 5 --warmup 1" "--config 5 --steps 32 --warmup 1"; do
  echo "== bench $args"
  timeout -k 10 300 python bench.py $args > "$OUT/bench_$(echo "$args" | tr -d ' -').log" 2>&1 || { echo "bench $args failed"; tail -20 "$OUT/bench_$(echo "$args" | tr -d ' -').log"; exit 1; }
  tail -1 "$OUT/bench_$(echo "$args" | tr -d ' -').log"
done
