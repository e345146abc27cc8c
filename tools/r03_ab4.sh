#!/usr/bin/env bash
# A/B round 4: which kernels get the lockstep rules (RT4_PHASE_REFILL 3 = closed rooms, 1 = + tiger kernels, 0 = none).
set -u -o pipefail
OUT=gpurun_out/r03_ab4
mkdir -p "$OUT"
COMMON="--no-cpu-baseline --no-ops --no-reuse-leg --no-fbf-leg"
bash tools/abtest.sh run 2 --config 5 --steps 32 --warmup 8 $COMMON 2>&1 | tee "$OUT/c5.log" || exit 1
bash tools/abtest.sh run 2 --config 2 --scene tiger --steps 10 --warmup 5 $COMMON 2>&1 | tee "$OUT/tiger.log" || exit 1
bash tools/abtest.sh run 2 --config 2 --scene room --steps 10 --warmup 5 $COMMON 2>&1 | tee "$OUT/room.log" || exit 1
bash tools/abtest.sh run 1 --config 4 --steps 20 --warmup 3 $COMMON 2>&1 | tee "$OUT/c4.log" || exit 1
bash tools/abtest.sh run 1 --config 2 --steps 20 --warmup 20 $COMMON 2>&1 | tee "$OUT/c2.log" || exit 1
echo "ab4 done"
