#!/usr/bin/env bash
# Clock of the config-4 trace launches, frame by frame vs pipelined (rocprofv3 GRBM counters).
set -u -o pipefail
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
for mode in "--frame-by-frame" ""; do
  tag=c4clk$( [ -n "$mode" ] && echo fbf || echo pipe )
  mkdir -p "$ROOT/gpurun_out/$tag"
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d "$ROOT/gpurun_out/$tag/pmc_clk" -o pmc_clk --output-format csv -- \
    python3 "$ROOT/bench.py" --config 4 --steps 3 --warmup 0 --no-cpu-baseline --no-reuse-leg --no-ops $mode > "$ROOT/gpurun_out/$tag/pmc_clk.log" 2>&1 || exit 1
  python3 - "$ROOT/gpurun_out/$tag" <<'PY'
import csv, glob, sys
from collections import defaultdict
d = sys.argv[1]
f = glob.glob(d + "/pmc_clk/*counter_collection.csv")[0]
rows = defaultdict(dict)
for r in csv.DictReader(open(f)):
    if "rt4_trace_kernel" in r["Kernel_Name"]:
        rows[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
        rows[r["Dispatch_Id"]]["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
for k, v in rows.items():
    print(d.split("/")[-1], k, f"{v['ns']/1e6:.2f} ms  clock {v['GRBM_GUI_ACTIVE']/8/v['ns']:.3f} GHz  busy/wave {v['SQ_WAVE_CYCLES']/max(1,v['SQ_BUSY_CYCLES']):.1f}")
PY
done
