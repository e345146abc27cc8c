#!/usr/bin/env bash
# Phase shares of the trace loop (-DRT4_STAMPS build, frame by frame): configs 2 and 3.
set -u -o pipefail
OUT=gpurun_out/r03_st
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1 RT4_AB_TOLERANT=1
for sc in sphere hypercube; do
  timeout -k 10 300 python tools/stamps.py $sc 16 8 > "$OUT/$sc.log" 2>&1 || { tail -20 "$OUT/$sc.log"; exit 1; }
  grep -v amdgpu.ids "$OUT/$sc.log"
done
