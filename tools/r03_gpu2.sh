#!/usr/bin/env bash
# Round-3 re-entry check: the whole GPU suite, smoke() and the default bench line at the current HEAD.
set -u -o pipefail
OUT=gpurun_out/r03_gpu${GPU_TAG:-2}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --durations=15 \
  > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
  || { echo "smoke failed"; tail -20 "$OUT/smoke.log"; exit 1; }
timeout -k 10 300 python bench.py > "$OUT/bench_default.log" 2>&1 || { echo "bench failed"; tail -20 "$OUT/bench_default.log"; exit 1; }
tail -1 "$OUT/bench_default.log" | cut -c1-600
echo "gpu2 done"
