#!/usr/bin/env bash
# A/B round 2: deferral threshold / wait sweep (RT4_DEFER_EXACT, RT4_DEFER_WAIT), per-kernel phase refill policy vs all kernels.
set -u -o pipefail
OUT=gpurun_out/r03_ab2
mkdir -p "$OUT"
COMMON="--no-cpu-baseline --no-ops --no-reuse-leg --no-fbf-leg"
bash tools/abtest.sh run 3 --config 2 --steps 20 --warmup 20 $COMMON 2>&1 | tee "$OUT/c2.log" || exit 1
bash tools/abtest.sh run 2 --config 2 --scene room --steps 5 --warmup 5 $COMMON 2>&1 | tee "$OUT/room.log" || exit 1
bash tools/abtest.sh run 2 --config 3 --steps 20 --warmup 20 $COMMON 2>&1 | tee "$OUT/c3.log" || exit 1
bash tools/abtest.sh run 1 --config 4 --steps 3 --warmup 1 $COMMON 2>&1 | tee "$OUT/c4.log" || exit 1
bash tools/abtest.sh run 1 --config 5 --steps 32 --warmup 8 $COMMON 2>&1 | tee "$OUT/c5.log" || exit 1
echo "ab2 done"
