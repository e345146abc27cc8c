#!/usr/bin/env bash
# Round 6: where config 2's clock goes. For each sampler-table placement (RT4_WLUT_ALLOC:
# default coarse-grained, fine, uncached) and each launch shape (the bench's 20 + 20 frames; 20 warmup frames then
# 128 frames = two 64-frame dispatches) this runs
#   1. bench.py alone (kernel ms per frame from HIP events, no profiler),
#   2. a PMC pass with the clock and VALU counters per dispatch (GRBM_GUI_ACTIVE, SQ_BUSY_CYCLES, SQ_INSTS_VALU,
#      SQ_THREAD_CYCLES_VALU),
#   3. a PMC pass with the fabric request sizes (TCC_EA0_RDREQ, _32B, TCC_BUBBLE) and
#   4. a PMC pass with the L2 hit rate and the fabric read latency (TCC_HIT/MISS, TCC_EA0_RDREQ_LEVEL),
# and tools/clock_summary.py prints one row per dispatch. Usage (GPU box, repo root):
#   tools/clock_probe.sh <tag> [placements...] [-- extra bench args]
set -u
TAG=$1; shift
PLACES=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do PLACES+=("$1"); shift; done
[ $# -gt 0 ] && shift
EXTRA="$*"
[ ${#PLACES[@]} -eq 0 ] && PLACES=(default uncached fine)
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/clock_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
PY=$(command -v python3)
BASE="--config 2 --no-cpu-baseline --no-ops --no-reuse-leg --no-fbf-leg --no-sections-leg --no-steady-leg $EXTRA"
for place in "${PLACES[@]}"; do
  if [ "$place" = default ]; then unset RT4_WLUT_ALLOC; else export RT4_WLUT_ALLOC=$place; fi
  for shape in "20 20" "128 20"; do
    set -- $shape
    name=${place}_s$1
    ARGS="$BASE --steps $1 --warmup $2"
    timeout -k 10 120 "$PY" "$ROOT/bench.py" $ARGS > "$OUT/$name.bench.log" 2>&1 || { echo "bench $name failed"; exit 1; }
    k=0
    for pmc in "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU" \
               "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum" \
               "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum"; do
      k=$((k + 1))
      timeout -k 10 180 rocprofv3 --kernel-trace --pmc $pmc -d "$OUT/${name}_p$k" -o p --output-format csv -- \
        "$PY" "$ROOT/bench.py" $ARGS > "$OUT/${name}_p$k.log" 2>&1 || { echo "pmc $name pass $k failed"; exit 1; }
    done
    echo "$name done"
  done
done
unset RT4_WLUT_ALLOC
"$PY" "$ROOT/tools/clock_summary.py" "$OUT" > "$OUT/summary.txt" && cat "$OUT/summary.txt"
