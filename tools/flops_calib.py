#!/usr/bin/env python3
"""Reads a rocprofv3 --pmc run of tools/flops_calib.hip and prints, per (operation, active lanes), each counter
divided by the known lane-operations of the dispatch (BLOCKS x THREADS / EVERY x ITERS). A counter that counts
executed lane operations reads 1 per add/mul/sqrt (2 per fma if it counts FLOPs) at every lane count; one that
counts wave instructions x 64 grows as 64 / active lanes per wave.
Usage: python tools/flops_calib.py <rocprofv3 output dir>"""
import csv
import glob
import re
import sys
from collections import defaultdict

ITERS, BLOCKS, THREADS = 4096, 2048, 256
OPS = {0: "fma", 1: "add", 2: "mul", 3: "sqrt"}


def main():
    f = glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True)[0]
    per = defaultdict(dict)
    with open(f) as fh:
        for r in csv.DictReader(fh):
            m = re.search(r"calib_kernel(?:ILi(\d)ELi(\d+)E|<(\d), (\d+)>)", r["Kernel_Name"])
            if m:
                op, every = (m.group(1), m.group(2)) if m.group(1) else (m.group(3), m.group(4))
                per[(int(op), int(every))][r["Counter_Name"]] = float(r["Counter_Value"])
    names = sorted({k for v in per.values() for k in v})
    print("op   lanes/wave " + " ".join(f"{n.replace('SQ_INSTS_VALU_', '').replace('SQ_', ''):>14s}" for n in names))
    for (op, every), c in sorted(per.items()):
        lane_ops = BLOCKS * THREADS // every * ITERS
        print(f"{OPS[op]:5s}{64 // every:6d}     " + " ".join(f"{c.get(n, 0) / lane_ops:14.4f}" for n in names))


if __name__ == "__main__":
    main()
