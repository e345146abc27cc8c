#!/usr/bin/env bash
# Lane statistics of the sphere kernel (config 2, 20 frames pipelined) with 1 and 2 tiles per claim.
set -u -o pipefail
OUT=gpurun_out/r03_ls5
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1 RT4_AB_TOLERANT=1
for v in ls ls2; do
  RT4_LIB=$PWD/4d_ray_tracing_amd/lib_$v/librt4.so timeout -k 10 300 python tools/lanestats.py sphere 16 8 1920 1080 20 pipelined > "$OUT/sphere_$v.log" 2>&1 || { tail -20 "$OUT/sphere_$v.log"; exit 1; }
  grep -v amdgpu.ids "$OUT/sphere_$v.log"
done
