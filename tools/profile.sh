#!/usr/bin/env bash
# rocprofv3 passes over bench.py (run on the GPU box from the repo root):
#   1. kernel trace + stats (per-kernel average duration; must agree with bench.py's kernel_ms)
#   2..n. PMC passes, each its own run with --kernel-trace only (MI355X_MICROARCH.md §rocprofv3 PMC slots)
# Usage: tools/profile.sh <tag> [bench args...]
set -u
TAG=${1:-run}
shift || true
ARGS=${*:-"--steps 5 --warmup 1 --no-cpu-baseline"}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
PY=$(command -v python3)

run() {  # name, rocprof args...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" -d "$OUT/$name" -o "$name" --output-format csv -- "$PY" "$ROOT/bench.py" $ARGS \
    > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "pass $name rc=$rc"
  return $rc
}

run trace --kernel-trace --stats || exit 1
run pmc_inst --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH || exit 1
run pmc_cyc --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT || exit 1
run pmc_thr --kernel-trace --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA || true
run pmc_fetch --kernel-trace --pmc FETCH_SIZE || exit 1
run pmc_write --kernel-trace --pmc WRITE_SIZE || exit 1
run pmc_tcc --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum || true
# mean fabric read latency (Little's law: requests in flight summed per cycle / requests), which tells an
# Infinity-Cache-served gather (~545 cycles idle) from an HBM-served one (~900; MI355X_MICROARCH.md)
run pmc_lat --kernel-trace --pmc TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum || true
# request sizes of the fabric reads (FETCH_SIZE = 128 B x bubble + 64 B x the rest + 32 B x 32B requests)
run pmc_req --kernel-trace --pmc TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum TCC_EA0_RDREQ_sum || true
# fp32 operations the kernel executed (round 6): the FLOP counters (calibrated on gfx950 by
# tools/flops_calib.hip: EXEC-masked lane counts or wave counts x 64, profiles/r06/flops_calib.txt) and the
# instruction mix
run pmc_flops --kernel-trace --pmc SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FLOPS_FP32_TRANS SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU || true
echo "profile $TAG done"
