#!/usr/bin/env bash
# A/B round 7: tiles per queue atomic (RT4_CLAIM_TILES 1 / 2 / 4).
set -u -o pipefail
OUT=gpurun_out/r03_ab7
mkdir -p "$OUT"
COMMON="--no-cpu-baseline --no-ops --no-reuse-leg --no-fbf-leg"
bash tools/abtest.sh run 3 --config 2 --steps 20 --warmup 20 $COMMON 2>&1 | tee "$OUT/c2.log" || exit 1
bash tools/abtest.sh run 2 --config 3 --steps 20 --warmup 20 $COMMON 2>&1 | tee "$OUT/c3.log" || exit 1
bash tools/abtest.sh run 2 --config 2 --steps 20 --warmup 3 --frame-by-frame $COMMON 2>&1 | tee "$OUT/c2fbf.log" || exit 1
bash tools/abtest.sh run 1 --config 5 --steps 32 --warmup 8 $COMMON 2>&1 | tee "$OUT/c5.log" || exit 1
bash tools/abtest.sh run 1 --config 4 --steps 20 --warmup 3 $COMMON 2>&1 | tee "$OUT/c4.log" || exit 1
echo "ab7 done"
