#!/usr/bin/env bash
# Historical (round 3, kept for the logged measurements): RT4_PIPE_MIRROR, the knob this script varies, was
# removed in r03-v35 when the mirror room started pipelining; rebuilding it now gives one binary.
# A/B: phase-aligned refill (RT4_PHASE_REFILL) x config-4 pipelining (RT4_PIPE_MIRROR), deferred exact sphere
# tests (RT4_DEFER_EXACT / RT4_DEFER_WAIT), every BASELINE config; lane statistics of config 2 (pending histogram).
set -u -o pipefail
OUT=gpurun_out/r03_ab1
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
true \
  > "$OUT/ls_sphere.log" 2>&1 || { echo "lanestats failed"; tail -20 "$OUT/ls_sphere.log"; exit 1; }
cat "$OUT/ls_sphere.log"
COMMON="--no-cpu-baseline --no-ops --no-reuse-leg --no-fbf-leg"
bash tools/abtest.sh run 2 --config 4 --steps 3 --warmup 1 $COMMON 2>&1 | tee "$OUT/c4.log" || exit 1
bash tools/abtest.sh run 2 --config 2 --steps 20 --warmup 20 $COMMON 2>&1 | tee "$OUT/c2.log" || exit 1
bash tools/abtest.sh run 2 --config 3 --steps 20 --warmup 20 $COMMON 2>&1 | tee "$OUT/c3.log" || exit 1
bash tools/abtest.sh run 2 --config 5 --steps 32 --warmup 8 $COMMON 2>&1 | tee "$OUT/c5.log" || exit 1
echo "ab1 done"
