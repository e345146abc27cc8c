#!/usr/bin/env python3
"""Timeline of overlapped single-frame launches from a rocprofv3 kernel trace: the last N trace
and fold dispatches, their durations, how long each fold starts after its trace ends, and the span per frame.
Usage: python tools/fbf_timeline.py <kernel_trace.csv> [N]"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    tr = [r for r in rows if "rt4_trace_kernel" in r["Kernel_Name"]][-n:]
    fo = [r for r in rows if "rt4_fold_frames_kernel" in r["Kernel_Name"]][-n:]
    t0 = int(tr[0]["Start_Timestamp"])
    us = lambda r, k: (int(r[k]) - t0) / 1e3
    print(f"{'frame':>5} {'queue':>5} {'trace start':>11} {'end':>9} {'dur':>7} | {'fold start':>10} {'dur':>7} {'wait':>7}")
    for i, (t, f) in enumerate(zip(tr, fo)):
        print(f"{i:5d} {t['Queue_Id']:>5} {us(t, 'Start_Timestamp'):11.1f} {us(t, 'End_Timestamp'):9.1f} "
              f"{us(t, 'End_Timestamp') - us(t, 'Start_Timestamp'):7.1f} | {us(f, 'Start_Timestamp'):10.1f} "
              f"{us(f, 'End_Timestamp') - us(f, 'Start_Timestamp'):7.1f} {us(f, 'Start_Timestamp') - us(t, 'End_Timestamp'):7.1f}")
    span = us(fo[-1], "End_Timestamp")
    td = [us(t, "End_Timestamp") - us(t, "Start_Timestamp") for t in tr]
    fd = [us(f, "End_Timestamp") - us(f, "Start_Timestamp") for f in fo]
    print(f"span {span:.1f} us -> {span / len(tr):.1f} us/frame; trace mean {sum(td) / len(td):.1f} us, "
          f"fold mean {sum(fd) / len(fd):.1f} us")


if __name__ == "__main__":
    main()
