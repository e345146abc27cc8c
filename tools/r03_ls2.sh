#!/usr/bin/env bash
# Lane statistics of the r03-v36 kernels (lib_ls: -DRT4_LANESTATS): configs 2, 3, the mirror room and all_primitives.
set -u -o pipefail
OUT=gpurun_out/r03_ls2
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1 RT4_AB_TOLERANT=1 RT4_LIB=$PWD/4d_ray_tracing_amd/lib_ls/librt4.so
run() {  # name, lanestats args
  local n=$1; shift
  timeout -k 10 300 python tools/lanestats.py "$@" > "$OUT/$n.log" 2>&1 || { echo "$n failed"; tail -20 "$OUT/$n.log"; exit 1; }
  grep -v amdgpu.ids "$OUT/$n.log"
}
run sphere sphere 16 8 1920 1080 20 pipelined
run hypercube hypercube 16 8 1920 1080 20 pipelined
run mirrors tiger_two_mirrors 16 12 3840 2160 8 pipelined
run allprims all_primitives 16 8 3840 2160 4 pipelined
echo "ls2 done"
