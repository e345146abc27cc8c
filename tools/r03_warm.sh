#!/usr/bin/env bash
# Does the timed rate depend on how long the GPU ran before (clock ramp)? Config 3 and 2 at several warmups.
set -u -o pipefail
OUT=gpurun_out/r03_warm
mkdir -p "$OUT"
for c in 3 2; do
  for w in 3 5 20 100 3; do
    timeout -k 10 300 python bench.py --config $c --steps 20 --warmup $w --no-cpu-baseline --no-ops --no-reuse-leg --no-fbf-leg > "$OUT/c${c}_w$w.log" 2>&1 || { tail -5 "$OUT/c${c}_w$w.log"; exit 1; }
    python3 -c "import json,sys; d=json.loads([l for l in open('$OUT/c${c}_w$w.log') if l.startswith('{')][-1]); print('config $c warmup $w', round(d['kernel_ms'],4), round(d['ms_per_step'],4))"
  done
done
