#!/usr/bin/env bash
# A/B round 11: deferred tiger tests, larger thresholds / waits.
set -u -o pipefail
OUT=gpurun_out/r03_ab11
mkdir -p "$OUT"
COMMON="--no-cpu-baseline --no-ops --no-reuse-leg --no-fbf-leg"
bash tools/abtest.sh run 2 --config 5 --steps 32 --warmup 8 $COMMON 2>&1 | tee "$OUT/c5.log" || exit 1
bash tools/abtest.sh run 2 --config 2 --scene tiger --steps 20 --warmup 20 $COMMON 2>&1 | tee "$OUT/tiger.log" || exit 1
bash tools/abtest.sh run 1 --config 5 --steps 16 --warmup 3 --frame-by-frame $COMMON 2>&1 | tee "$OUT/c5fbf.log" || exit 1
echo "ab11 done"
