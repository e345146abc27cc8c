#!/usr/bin/env bash
# A/B round 14: the deferred-sphere kernel with multi-tile claims at 6 waves/SIMD (room for the claim state);
# then the warmup dependence of the timed rate (clock ramp).
set -u -o pipefail
OUT=gpurun_out/r03_ab14
mkdir -p "$OUT"
COMMON="--no-cpu-baseline --no-ops --no-reuse-leg --no-fbf-leg"
bash tools/abtest.sh run 3 --config 2 --steps 20 --warmup 20 $COMMON 2>&1 | tee "$OUT/c2.log" || exit 1
bash tools/r03_warm.sh
echo "ab14 done"
