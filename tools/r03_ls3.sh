#!/usr/bin/env bash
# Lane statistics of the hypercube kernel's pending-cell loop (config 3).
set -u -o pipefail
OUT=gpurun_out/r03_ls3
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1 RT4_AB_TOLERANT=1 RT4_LIB=$PWD/4d_ray_tracing_amd/lib_ls/librt4.so
timeout -k 10 300 python tools/lanestats.py hypercube 16 8 1920 1080 20 pipelined > "$OUT/hypercube.log" 2>&1 || { tail -20 "$OUT/hypercube.log"; exit 1; }
grep -v amdgpu.ids "$OUT/hypercube.log"
