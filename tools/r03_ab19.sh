#!/usr/bin/env bash
# A/B round 19: exact-sphere deferral threshold / wait at the sphere kernel's 6-wave, four-tile configuration.
set -u -o pipefail
OUT=gpurun_out/r03_ab19
mkdir -p "$OUT"
COMMON="--no-cpu-baseline --no-ops --no-reuse-leg --no-fbf-leg"
bash tools/abtest.sh run 3 --config 2 --steps 20 --warmup 20 $COMMON 2>&1 | tee "$OUT/c2.log" || exit 1
echo "ab19 done"
