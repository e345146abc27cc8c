#!/usr/bin/env bash
# The driver's round-end commands on the final tree: the GPU suite, smoke() and the default bench line
# (python3 bench.py --gpus 1 --steps 20 --warmup 5).
set -u -o pipefail
OUT=gpurun_out/r03_final
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
  || { echo "pytest failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -2 "$OUT/smoke.log"
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.log" 2>&1 || { tail -20 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log" | cut -c1-400
