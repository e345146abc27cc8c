#!/usr/bin/env bash
# Round-2 kernel check + profiles (GPU box, repo root): pytest -m gpu, set_scene probe, stamps,
# one bench line per BASELINE config, then rocprofv3 kernel trace + PMC passes per config.
# Usage: tools/r02_v28.sh <tag>. Each GPU step has its own time limit; the first failure ends it.
set -u -o pipefail
TAG=${1:-r02v28}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
bash tools/r02_check.sh "$TAG" || exit 1
timeout -k 10 120 python tools/setscene_probe.py > "$OUT/setscene_probe.log" 2>&1 || { tail -20 "$OUT/setscene_probe.log"; exit 1; }
cat "$OUT/setscene_probe.log"
timeout -k 10 120 python tools/stamps.py sphere > "$OUT/stamps_sphere.log" 2>&1 || { tail -20 "$OUT/stamps_sphere.log"; exit 1; }
cat "$OUT/stamps_sphere.log"
timeout -k 10 1500 bash tools/profile_configs.sh "$TAG" 2 3 4 5 || exit 1
