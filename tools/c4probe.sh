#!/usr/bin/env bash
set -u -o pipefail
for extra in "" "--spp 16" "--width 1920 --height 1080" "--format f16" "--scene tiger --width 1920 --height 1080" "--scene all_primitives --spp 64 --bounces 12 --width 1920 --height 1080"; do
  for mode in "--frame-by-frame" ""; do
    out=$(timeout -k 10 200 python bench.py --config 4 --steps 3 --warmup 1 --no-cpu-baseline --no-reuse-leg --no-ops $extra $mode 2>/dev/null | tail -1) || { echo "fail $extra $mode"; exit 1; }
    python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(f'{sys.argv[2]:>60s} {sys.argv[3]:>16s} kernel {d[\"kernel_ms\"]:.3f} ms  {d[\"intersections_per_step\"]:.0f}')" "$out" "$extra" "$mode"
  done
done
