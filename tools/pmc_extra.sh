#!/usr/bin/env bash
# Extra PMC passes (instruction fetch, scalar cache, LDS waits) over bench.py; each pass its own run.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc_extra
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
PY=$(command -v python3)
ARGS="--steps 3 --warmup 1 --no-cpu-baseline ${*:-}"
run() {
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc "$@" -d "$OUT/$name" -o "$name" --output-format csv -- "$PY" "$ROOT/bench.py" $ARGS > "$OUT/$name.log" 2>&1
  echo "pass $name rc=$?"
}
run sq SQ_IFETCH SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES || exit 1
run icache SQC_ICACHE_MISSES SQC_ICACHE_HITS || exit 1
run dcache SQC_DCACHE_MISSES SQC_DCACHE_HITS || exit 1
