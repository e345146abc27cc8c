#!/usr/bin/env bash
# PMC passes (VALU issue / lane utilisation / cycles) for several scenes. Usage: tools/pmc_scenes.sh <tag> scene...
set -u
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
for sc in "$@"; do
  for pass in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH" \
              "SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"; do
    name=$(echo "$pass" | cut -d' ' -f2)
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc $pass -d "$ROOT/gpurun_out/pmc_${TAG}_${sc}/pmc_$name" -o p --output-format csv \
      -- "$(command -v python3)" "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --scene "$sc" > /dev/null 2>&1 || exit 1
  done
  timeout -k 10 300 rocprofv3 --kernel-trace -d "$ROOT/gpurun_out/pmc_${TAG}_${sc}/trace" -o t --output-format csv \
      -- "$(command -v python3)" "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --scene "$sc" > "$ROOT/gpurun_out/pmc_${TAG}_${sc}/bench.log" 2>&1 || exit 1
  echo "done $sc"
done
