#!/usr/bin/env bash
# A/B round 13: a lone idle lane waits for a second one before the refill (RT4_REFILL_AGE).
set -u -o pipefail
OUT=gpurun_out/r03_ab13
mkdir -p "$OUT"
COMMON="--no-cpu-baseline --no-ops --no-reuse-leg --no-fbf-leg"
bash tools/abtest.sh run 3 --config 2 --steps 20 --warmup 20 $COMMON 2>&1 | tee "$OUT/c2.log" || exit 1
bash tools/abtest.sh run 2 --config 3 --steps 20 --warmup 20 $COMMON 2>&1 | tee "$OUT/c3.log" || exit 1
bash tools/abtest.sh run 1 --config 5 --steps 32 --warmup 8 $COMMON 2>&1 | tee "$OUT/c5.log" || exit 1
echo "ab13 done"
