#!/usr/bin/env bash
# PC sampling of bench.py's trace kernel (rocprofv3 beta). Usage: tools/pcsample.sh <tag> [method] [unit] [interval]
set -u
TAG=${1:-run}; METHOD=${2:-stochastic}; UNIT=${3:-cycles}; IV=${4:-1048576}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pcs_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method "$METHOD" --pc-sampling-unit "$UNIT" \
  --pc-sampling-interval "$IV" -d "$OUT" -o pcs --output-format csv -- "$(command -v python3)" "$ROOT/bench.py" \
  --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/log.txt" 2>&1
echo "pcsample $METHOD/$UNIT rc=$?"
