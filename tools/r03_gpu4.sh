#!/usr/bin/env bash
# Full check of a kernel version on one MI355X: GPU suite, smoke, bench-shape profiles of configs 2-5 (kernel
# trace + PMC), then every config's bench line with its same-shape profile in place.
# Usage: GPU_TAG=<tag> VER=<r03vNN> bash tools/r03_gpu4.sh
set -u -o pipefail
TAG=${GPU_TAG:-4}
VER=${VER:-r03v34}
OUT=gpurun_out/r03_gpu$TAG
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --durations=15 \
  > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
  || { echo "smoke failed"; tail -20 "$OUT/smoke.log"; exit 1; }
tail -2 "$OUT/smoke.log"
bash tools/profile_configs.sh "$VER" 2 3 4 5 || exit 1
PD=profiles/${VER/v/_v}
mkdir -p "$PD"
for c in 2 3 4 5; do
  cp "gpurun_out/prof_${VER}_config$c/summary.json" "$PD/pmc_config$c.json"
  ks=$(find "gpurun_out/prof_${VER}_config$c" -name "*kernel_stats.csv" -print -quit)
  [ -n "$ks" ] && cp "$ks" "$PD/trace_kernel_stats_config$c.csv"
done
timeout -k 10 300 python bench.py > "$OUT/bench_default.log" 2>&1 || { echo "bench failed"; tail -20 "$OUT/bench_default.log"; exit 1; }
tail -1 "$OUT/bench_default.log" | cut -c1-300
for c in 3 4 5; do
  case $c in 5) st=32;; *) st=20;; esac
  timeout -k 10 400 python bench.py --config $c --steps $st > "$OUT/bench_c$c.log" 2>&1 || { echo "bench $c failed"; tail -20 "$OUT/bench_c$c.log"; exit 1; }
  tail -1 "$OUT/bench_c$c.log" | cut -c1-300
done
echo "gpu$TAG done"
