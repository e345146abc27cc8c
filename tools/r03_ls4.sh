#!/usr/bin/env bash
# Lane statistics of the tiger kernels' tiger test (configs 4, 5 and the one-space tiger).
set -u -o pipefail
OUT=gpurun_out/r03_ls4
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1 RT4_AB_TOLERANT=1 RT4_LIB=$PWD/4d_ray_tracing_amd/lib_ls/librt4.so
run() {
  local n=$1; shift
  timeout -k 10 300 python tools/lanestats.py "$@" > "$OUT/$n.log" 2>&1 || { echo "$n failed"; tail -20 "$OUT/$n.log"; exit 1; }
  grep -v amdgpu.ids "$OUT/$n.log"
}
run allprims all_primitives 16 8 3840 2160 4 pipelined
run mirrors tiger_two_mirrors 16 12 3840 2160 4 pipelined
run tiger tiger 16 8 1920 1080 10 pipelined
