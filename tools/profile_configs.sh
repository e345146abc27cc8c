#!/usr/bin/env bash
# rocprofv3 kernel trace + PMC passes (tools/profile.sh) for every BASELINE config on one GPU at the bench's
# launch shape: warmup = steps, so that every trace dispatch holds the same frames as the timed one (20
# frames per pipelined dispatch for configs 2-4, 32 for config 5; pmc_summary.py reports per frame), then
# one summary per config (tools/pmc_summary.py). Usage (on the GPU box): tools/profile_configs.sh <tag> [configs...]
set -u
TAG=$1; shift
CONFIGS=${*:-2 3 4 5}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
for c in $CONFIGS; do
  case $c in
    5) steps="--steps 32 --warmup 32" ;;
    *) steps="--steps 20 --warmup 20" ;;
  esac
  bash "$ROOT/tools/profile.sh" "${TAG}_config$c" --config "$c" $steps --no-cpu-baseline --no-ops --no-reuse-leg \
    --no-fbf-leg --no-sections-leg --no-steady-leg || exit 1
  python3 "$ROOT/tools/pmc_summary.py" "$ROOT/gpurun_out/prof_${TAG}_config$c" > /dev/null || exit 1
  echo "config $c profiled"
done
