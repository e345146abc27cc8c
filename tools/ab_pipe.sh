#!/usr/bin/env bash
# A/B of pipelined frames (tools/abtest.sh variants): pytest -m gpu on the in-tree build, then per config
# the variants frame by frame and pipelined. Usage: tools/ab_pipe.sh <outdir> <rounds> [configs...]
set -u -o pipefail
OUT=gpurun_out/${1:-ab}
R=${2:-2}
shift 2 || true
CONFIGS=${*:-2 3 5}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
for c in $CONFIGS; do
  case $c in 4) extra="--steps 3 --warmup 1";; 5) extra="--steps 16 --warmup 1";; *) extra="--steps 30 --warmup 3";; esac
  for mode in "--frame-by-frame" ""; do
    echo "== config $c $mode"
    timeout -k 10 900 tools/abtest.sh run "$R" --config "$c" $extra $mode --no-cpu-baseline --no-reuse-leg \
      2>&1 | tee -a "$OUT/ab.log" || exit 1
  done
done
