#!/usr/bin/env bash
# A/B round 5: sphere kernel waves/SIMD with the deferral (RT4_WAVES_SPHERE), deferral threshold 40.
set -u -o pipefail
OUT=gpurun_out/r03_ab5
mkdir -p "$OUT"
COMMON="--no-cpu-baseline --no-ops --no-reuse-leg --no-fbf-leg"
bash tools/abtest.sh run 4 --config 2 --steps 20 --warmup 20 $COMMON 2>&1 | tee "$OUT/c2.log" || exit 1
echo "ab5 done"
