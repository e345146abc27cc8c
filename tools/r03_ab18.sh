#!/usr/bin/env bash
# A/B round 18: deferred hypercube cell tests (RT4_DEFER_HYPER / _WAIT) on config 3; config 5 unchanged check.
set -u -o pipefail
OUT=gpurun_out/r03_ab18
mkdir -p "$OUT"
COMMON="--no-cpu-baseline --no-ops --no-reuse-leg --no-fbf-leg"
bash tools/abtest.sh run 3 --config 3 --steps 20 --warmup 20 $COMMON 2>&1 | tee "$OUT/c3.log" || exit 1
bash tools/abtest.sh run 1 --config 3 --steps 20 --warmup 5 --frame-by-frame $COMMON 2>&1 | tee "$OUT/c3fbf.log" || exit 1
echo "ab18 done"
