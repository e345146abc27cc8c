#!/usr/bin/env bash
# A/B round 3: wave clock (RT4_WAVE_CLOCK) on the phase-refill kernels: config 4 pipelined (20 frames) and frame by
# frame, config 5, the room and the one-space tiger.
set -u -o pipefail
OUT=gpurun_out/r03_ab3
mkdir -p "$OUT"
COMMON="--no-cpu-baseline --no-ops --no-reuse-leg --no-fbf-leg"
bash tools/abtest.sh run 2 --config 4 --steps 20 --warmup 3 $COMMON 2>&1 | tee "$OUT/c4.log" || exit 1
bash tools/abtest.sh run 1 --config 4 --steps 3 --warmup 1 --frame-by-frame $COMMON 2>&1 | tee "$OUT/c4fbf.log" || exit 1
bash tools/abtest.sh run 2 --config 5 --steps 32 --warmup 8 $COMMON 2>&1 | tee "$OUT/c5.log" || exit 1
bash tools/abtest.sh run 2 --config 2 --scene room --steps 10 --warmup 5 $COMMON 2>&1 | tee "$OUT/room.log" || exit 1
bash tools/abtest.sh run 2 --config 2 --scene tiger --steps 10 --warmup 5 $COMMON 2>&1 | tee "$OUT/tiger.log" || exit 1
echo "ab3 done"
