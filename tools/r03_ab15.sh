#!/usr/bin/env bash
# A/B round 15: the sphere kernel at 6 waves with four-tile claims: waves 5/6, deferral threshold 24/32/40/off.
set -u -o pipefail
OUT=gpurun_out/r03_ab15
mkdir -p "$OUT"
COMMON="--no-cpu-baseline --no-ops --no-reuse-leg --no-fbf-leg"
bash tools/abtest.sh run 3 --config 2 --steps 20 --warmup 20 $COMMON 2>&1 | tee "$OUT/c2.log" || exit 1
bash tools/abtest.sh run 1 --config 2 --steps 20 --warmup 5 --frame-by-frame $COMMON 2>&1 | tee "$OUT/c2fbf.log" || exit 1
echo "ab15 done"
