#!/usr/bin/env python3
"""Summarise a tools/profile.sh run: per-kernel average duration and PMC-derived metrics.

Usage: python tools/pmc_summary.py gpurun_out/prof_<tag> [kernel-substring]
Writes <dir>/summary.json and prints it. Counter semantics (rocprofv3 -L on gfx950):
  SQ_INSTS_VALU            VALU wave-instructions issued (all SEs)
  SQ_THREAD_CYCLES_VALU    VALU thread-cycles (x active lanes)  -> lane utilisation
  SQ_ACTIVE_INST_VALU      quad-cycles waves spend on VALU
  SQ_WAVE_CYCLES / SQ_BUSY_CYCLES / GRBM_GUI_ACTIVE            -> occupancy, clock
  FETCH_SIZE / WRITE_SIZE  KiB from/to the memory side; FETCH_SIZE doubled on gfx950
                           (MI355X_MICROARCH.md §HBM: it reports 1/2 of wide coalesced reads)
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

CUS, SIMDS_PER_CU, LANES = 256, 4, 64


def kernel_rows(path, sub):
    with open(path) as f:
        for r in csv.DictReader(f):
            if sub in r.get("Kernel_Name", ""):
                yield r


def main():
    d = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else "rt4_trace_kernel"
    out = {"dir": d, "kernel": sub}
    tr = glob.glob(os.path.join(d, "trace", "*kernel_trace.csv"))
    if tr:
        durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in kernel_rows(tr[0], sub)]
        if durs:
            out["dispatches"] = len(durs)
            out["avg_ns"] = sum(durs) / len(durs)
            out["min_ns"] = min(durs)
            out["max_ns"] = max(durs)
            rows = list(kernel_rows(tr[0], sub))
            out["vgpr"] = int(rows[0]["VGPR_Count"])
            out["sgpr"] = int(rows[0]["SGPR_Count"])
            out["scratch"] = int(rows[0]["Scratch_Size"])
            out["lds"] = int(rows[0]["LDS_Block_Size"])
    counters = defaultdict(list)
    durations = defaultdict(list)
    for f in glob.glob(os.path.join(d, "pmc_*", "*counter_collection.csv")):
        for r in kernel_rows(f, sub):
            counters[r["Counter_Name"]].append(float(r["Counter_Value"]))
            durations[r["Counter_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    c = {k: sum(v) / len(v) for k, v in counters.items()}
    out["counters"] = c
    m = {}
    if "SQ_INSTS_VALU" in c and "SQ_WAVES" in c:
        m["valu_insts_per_wave"] = c["SQ_INSTS_VALU"] / c["SQ_WAVES"]
    if "SQ_THREAD_CYCLES_VALU" in c and "SQ_INSTS_VALU" in c:
        # calibrated on gfx950 (tools/calib_util.py): a fully active wave64 VALU instruction adds ~64
        # thread-cycles, so utilisation = THREAD_CYCLES / (INSTS * 64)
        m["valu_lane_utilisation"] = c["SQ_THREAD_CYCLES_VALU"] / (c["SQ_INSTS_VALU"] * 64)
    if "GRBM_GUI_ACTIVE" in c:
        dur = sum(durations["GRBM_GUI_ACTIVE"]) / len(durations["GRBM_GUI_ACTIVE"])
        m["clock_ghz"] = c["GRBM_GUI_ACTIVE"] / 8 / dur  # summed over 8 XCDs (MI355X_MICROARCH.md DVFS note)
        m["pmc_pass_duration_ns"] = dur
    if "SQ_INSTS_VALU" in c and "GRBM_GUI_ACTIVE" in c:
        dur = sum(durations["SQ_INSTS_VALU"]) / len(durations["SQ_INSTS_VALU"])
        clk = m.get("clock_ghz", 2.4) * 1e9
        # each wave64 VALU instruction needs 2 cycles of one SIMD-32
        m["valu_issue_frac"] = c["SQ_INSTS_VALU"] * 2 / (CUS * SIMDS_PER_CU * clk * dur * 1e-9)
    if "SQ_WAVE_CYCLES" in c and "SQ_BUSY_CYCLES" in c:
        # SQ_WAVE_CYCLES counts quad-cycles per resident wave, SQ_BUSY_CYCLES cycles summed over the 32 shader engines
        # (round 6: the earlier expression lacked both factors and read ~50 waves/SIMD)
        m["avg_waves_per_simd"] = c["SQ_WAVE_CYCLES"] * 4 / (CUS * SIMDS_PER_CU * c["SQ_BUSY_CYCLES"] / 32)
    if "SQ_ACTIVE_INST_VALU" in c and "SQ_WAVE_CYCLES" in c:
        m["valu_share_of_wave_cycles"] = c["SQ_ACTIVE_INST_VALU"] / c["SQ_WAVE_CYCLES"]
    if "SQ_WAIT_ANY" in c and "SQ_WAVE_CYCLES" in c:
        m["wait_any_share"] = c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"]
        m["wait_inst_any_share"] = c.get("SQ_WAIT_INST_ANY", 0) / c["SQ_WAVE_CYCLES"]
        m["active_any_share"] = c.get("SQ_ACTIVE_INST_ANY", 0) / c["SQ_WAVE_CYCLES"]
    if "FETCH_SIZE" in c:
        m["hbm_read_bytes_corrected"] = c["FETCH_SIZE"] * 1024 * 2
    if "WRITE_SIZE" in c:
        m["hbm_write_bytes"] = c["WRITE_SIZE"] * 1024
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        m["hbm_bytes_per_launch"] = m["hbm_read_bytes_corrected"] + m["hbm_write_bytes"]
    if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
        m["l2_hit_rate"] = c["TCC_HIT_sum"] / max(1.0, c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
    if "TCC_EA0_RDREQ_sum" in c and "TCC_EA0_RDREQ_DRAM_sum" in c:
        # L2 misses sent to the fabric, and the part of them that reached DRAM (the rest: MALL hits)
        m["fabric_read_requests"] = c["TCC_EA0_RDREQ_sum"]
        m["dram_read_share"] = c["TCC_EA0_RDREQ_DRAM_sum"] / max(1.0, c["TCC_EA0_RDREQ_sum"])
    if "TCC_EA0_RDREQ_LEVEL_sum" in c and "TCC_EA0_RDREQ_sum" in c:
        # Little's law over the L2's fabric read interface (TCC cycles): the mean latency of an L2 miss
        m["ea_read_latency_cycles"] = c["TCC_EA0_RDREQ_LEVEL_sum"] / max(1.0, c["TCC_EA0_RDREQ_sum"])
    if "TCC_EA0_RDREQ_32B_sum" in c and "TCC_BUBBLE_sum" in c and "TCC_EA0_RDREQ_sum" in c:
        # request sizes (the FETCH_SIZE expression of rocprofv3 -L): 128 B bubbles, 32 B requests, 64 B the rest
        r, r32, bub = c["TCC_EA0_RDREQ_sum"], c["TCC_EA0_RDREQ_32B_sum"], c["TCC_BUBBLE_sum"]
        m["fabric_read_bytes"] = bub * 128 + (r - bub - r32) * 64 + r32 * 32
        m["fabric_req_32b_share"] = r32 / max(1.0, r)
        m["fabric_req_128b_share"] = bub / max(1.0, r)
        if "hbm_write_bytes" in m:
            # memory-side bytes of the launch from the request sizes (no gfx950 x2 correction: that one is for
            # wide coalesced reads; these are 64-B requests, profiles/r04_ab.txt)
            m["traffic_bytes_per_launch"] = m["fabric_read_bytes"] + m["hbm_write_bytes"]
    out["derived"] = m
    for log in ("trace.log", os.path.join("trace", "..", "bench.log")):
        lp = os.path.join(d, log)
        if os.path.exists(lp):
            lines = [l for l in open(lp) if l.startswith("{")]
            if lines:
                b = json.loads(lines[-1])
                fpl = b.get("frames_per_launch", 1)
                if fpl > 1 and out.get("avg_ns"):  # pipelined frames (bench --warmup 0): one dispatch = fpl frames
                    out["frames_per_dispatch"] = fpl
                    out["avg_ns"] /= fpl
                    for k in ("min_ns", "max_ns"):
                        out[k] /= fpl
                    for k in list(c):
                        c[k] /= fpl
                    for k in ("hbm_read_bytes_corrected", "hbm_write_bytes", "hbm_bytes_per_launch", "fabric_read_requests",
                              "fabric_read_bytes", "traffic_bytes_per_launch"):
                        if k in m:
                            m[k] /= fpl
                out["config"] = b["config"]
                out["bench"] = {k: b[k] for k in ("value", "kernel_ms", "intersections_per_step")}
                if out.get("avg_ns"):
                    out["bench"]["kernel_ms_vs_trace"] = b["kernel_ms"] / (out["avg_ns"] * 1e-6)
                n = b["intersections_per_step"]
                if "SQ_INSTS_VALU" in c:
                    m["valu_lane_slots_per_intersection"] = c["SQ_INSTS_VALU"] * 64 / n
                break
    json.dump(out, open(os.path.join(d, "summary.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
