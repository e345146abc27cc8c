#!/usr/bin/env bash
# A/B round 17: all_primitives kernel waves/SIMD 5 / 6 / 7 (config 5, pipelined and frame by frame).
set -u -o pipefail
OUT=gpurun_out/r03_ab17
mkdir -p "$OUT"
COMMON="--no-cpu-baseline --no-ops --no-reuse-leg --no-fbf-leg"
bash tools/abtest.sh run 3 --config 5 --steps 32 --warmup 8 $COMMON 2>&1 | tee "$OUT/c5.log" || exit 1
bash tools/abtest.sh run 1 --config 5 --steps 8 --warmup 3 --frame-by-frame $COMMON 2>&1 | tee "$OUT/c5fbf.log" || exit 1
echo "ab17 done"
