#!/usr/bin/env python3
"""Per-dispatch clock, VALU and fabric figures of a tools/clock_probe.sh run (round 6).

For every run <placement>_s<steps> of the probe and every trace-kernel dispatch of it (in launch order: the warmup
call's 20-frame dispatch, then the timed call's 20 or 2 x 64 frames):
  clock      = GRBM_GUI_ACTIVE / 8 XCDs / duration             (GHz; MI355X_MICROARCH.md DVFS note)
  util       = SQ_THREAD_CYCLES_VALU / (64 x SQ_INSTS_VALU)      (VALU lane utilisation)
  issue      = 2 x SQ_INSTS_VALU / (1024 SIMDs x clock x duration)
  fc         = SQ_THREAD_CYCLES_VALU / (duration x 7.864e13)    (frac_counters: lane-ops over the 2.4 GHz ceiling)
  us/frame   = duration / frames of the dispatch
  req/frame, 32B share, 128B share, L2 hit, fabric latency (cycles, Little's law) from the TCC passes.
The bench line of the same run without a profiler gives kernel_ms (HIP events) for comparison.
Usage: python tools/clock_summary.py gpurun_out/clock_<tag>"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

PEAK_LANE_OPS = 256 * 4 * 32 * 2.4e9


def dispatches(d):
    """[{counter: value, 'ns': duration}] per trace-kernel dispatch, in dispatch order."""
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        return []
    per = defaultdict(dict)
    with open(f[0]) as fh:
        for r in csv.DictReader(fh):
            if "rt4_trace_kernel" not in r.get("Kernel_Name", ""):
                continue
            key = int(r.get("Dispatch_Id") or r.get("Correlation_Id"))
            per[key][r["Counter_Name"]] = per[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            per[key]["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return [per[k] for k in sorted(per)]


def bench_line(path):
    if not os.path.exists(path):
        return None
    lines = [l for l in open(path) if l.startswith("{")]
    return json.loads(lines[-1]) if lines else None


def frames_of(steps, n):
    seq = [20] + ([20] if steps == 20 else [64, 64])
    return seq[:n] + [None] * (n - len(seq))


def main():
    d = sys.argv[1]
    runs = sorted({os.path.basename(p)[:-len(".bench.log")] for p in glob.glob(os.path.join(d, "*.bench.log"))})
    rows = []
    print(f"{'run':18s} {'disp':>4s} {'frames':>6s} {'us/frame':>9s} {'GHz':>5s} {'util':>6s} {'issue':>6s} {'fc':>6s} "
          f"{'Mreq/fr':>8s} {'32B':>5s} {'128B':>5s} {'L2hit':>6s} {'lat':>6s}")
    for run in runs:
        steps = int(run.rsplit("_s", 1)[1])
        b = bench_line(os.path.join(d, run + ".bench.log"))
        p = [dispatches(os.path.join(d, f"{run}_p{k}")) for k in (1, 2, 3)]
        n = max(len(x) for x in p)
        for i, fr in enumerate(frames_of(steps, n)):
            c = {}
            for x in p:
                if i < len(x):
                    for k, v in x[i].items():
                        if k != "ns":
                            c[k] = v
            ns = p[0][i]["ns"] if i < len(p[0]) else None
            row = {"run": run, "dispatch": i, "frames": fr, "ns": ns, "counters": c}
            if ns and fr:
                row["us_per_frame"] = ns / fr / 1e3
            if ns and "GRBM_GUI_ACTIVE" in c:
                clk = c["GRBM_GUI_ACTIVE"] / 8 / ns
                row["clock_ghz"] = clk
                if "SQ_INSTS_VALU" in c and "SQ_THREAD_CYCLES_VALU" in c:
                    row["util"] = c["SQ_THREAD_CYCLES_VALU"] / (64 * c["SQ_INSTS_VALU"])
                    row["issue"] = 2 * c["SQ_INSTS_VALU"] / (1024 * clk * ns)
                    row["frac_counters"] = c["SQ_THREAD_CYCLES_VALU"] / (ns * 1e-9 * PEAK_LANE_OPS)
            rq = c.get("TCC_EA0_RDREQ_sum")
            if rq and fr:
                row["mreq_per_frame"] = rq / fr / 1e6
                row["req32_share"] = c.get("TCC_EA0_RDREQ_32B_sum", 0) / rq
                row["req128_share"] = c.get("TCC_BUBBLE_sum", 0) / rq
                if "TCC_EA0_RDREQ_LEVEL_sum" in c:
                    row["fabric_latency_cycles"] = c["TCC_EA0_RDREQ_LEVEL_sum"] / rq
            if "TCC_HIT_sum" in c:
                row["l2_hit"] = c["TCC_HIT_sum"] / max(1.0, c["TCC_HIT_sum"] + c.get("TCC_MISS_sum", 0))
            rows.append(row)

            def f(k, fmt):
                v = row.get(k)
                return format(v, fmt) if v is not None else "-"
            print(f"{run:18s} {i:4d} {str(fr):>6s} {f('us_per_frame', '9.1f')} {f('clock_ghz', '5.2f')} "
                  f"{f('util', '6.3f')} {f('issue', '6.3f')} {f('frac_counters', '6.3f')} {f('mreq_per_frame', '8.2f')} "
                  f"{f('req32_share', '5.2f')} {f('req128_share', '5.2f')} {f('l2_hit', '6.3f')} "
                  f"{f('fabric_latency_cycles', '6.0f')}")
        if b:
            print(f"{run:18s} bench (no profiler): kernel_ms {b['kernel_ms']:.4f} per frame, "
                  f"{b['value'] / 1e9:.2f} G int/s, {b['frames_per_launch']} frames per launch")
            rows.append({"run": run, "bench_kernel_ms": b["kernel_ms"], "bench_value": b["value"]})
    json.dump(rows, open(os.path.join(d, "summary.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
