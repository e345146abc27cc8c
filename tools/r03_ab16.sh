#!/usr/bin/env bash
# A/B round 16: waves/SIMD bounds of the hypercube (EXACT), mirror-room (MIRROR) and all_primitives (ALLPRIM)
# kernels with round 3's scheduling code.
set -u -o pipefail
OUT=gpurun_out/r03_ab16
mkdir -p "$OUT"
COMMON="--no-cpu-baseline --no-ops --no-reuse-leg --no-fbf-leg"
bash tools/abtest.sh run 2 --config 3 --steps 20 --warmup 20 $COMMON 2>&1 | tee "$OUT/c3.log" || exit 1
bash tools/abtest.sh run 1 --config 5 --steps 32 --warmup 8 $COMMON 2>&1 | tee "$OUT/c5.log" || exit 1
bash tools/abtest.sh run 1 --config 4 --steps 10 --warmup 3 $COMMON 2>&1 | tee "$OUT/c4.log" || exit 1
echo "ab16 done"
