#!/usr/bin/env bash
# Where are the sampler-table gathers served? tools/mall_probe.hip: uniform random 4-B
# gathers over tables of 2 MiB .. 4 GiB, plain (rates) and under two PMC passes (L2 hit/miss, fabric read
# requests and their mean latency by Little's law, per size). Build first: hipcc -O3 --offload-arch=gfx950
# -o tools/build/mall_probe tools/mall_probe.hip
set -u -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r03_mall
mkdir -p "$OUT"
BIN=$ROOT/tools/build/mall_probe
timeout -k 10 120 "$BIN" 256 > "$OUT/probe.json" 2>&1 || { echo "probe failed"; cat "$OUT/probe.json"; exit 1; }
cat "$OUT/probe.json"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum \
  -d "$OUT/pmc_lat" -o pmc_lat --output-format csv -- "$BIN" 256 > "$OUT/pmc_lat.log" 2>&1 \
  || { echo "pmc_lat failed"; tail -20 "$OUT/pmc_lat.log"; exit 1; }
echo "mall done"
