#!/usr/bin/env bash
# A/B round 9: the sphere kernel with multi-tile claims instead of deferred exact tests.
set -u -o pipefail
OUT=gpurun_out/r03_ab9
mkdir -p "$OUT"
COMMON="--no-cpu-baseline --no-ops --no-reuse-leg --no-fbf-leg"
bash tools/abtest.sh run 3 --config 2 --steps 20 --warmup 20 $COMMON 2>&1 | tee "$OUT/c2.log" || exit 1
echo "ab9 done"
