#!/usr/bin/env bash
# A/B round 10: deferred tiger tests (RT4_DEFER_TIGER threshold / RT4_DEFER_TIGER_WAIT) on the open tiger scenes.
set -u -o pipefail
OUT=gpurun_out/r03_ab10
mkdir -p "$OUT"
COMMON="--no-cpu-baseline --no-ops --no-reuse-leg --no-fbf-leg"
bash tools/abtest.sh run 2 --config 5 --steps 32 --warmup 8 $COMMON 2>&1 | tee "$OUT/c5.log" || exit 1
bash tools/abtest.sh run 2 --config 2 --scene tiger --steps 20 --warmup 20 $COMMON 2>&1 | tee "$OUT/tiger.log" || exit 1
bash tools/abtest.sh run 1 --config 2 --scene cylinder4d --steps 20 --warmup 20 $COMMON 2>&1 | tee "$OUT/cyl.log" || exit 1
bash tools/abtest.sh run 1 --config 2 --steps 20 --warmup 20 $COMMON 2>&1 | tee "$OUT/c2.log" || exit 1
echo "ab10 done"
