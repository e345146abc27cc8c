#!/usr/bin/env python3
"""Static instruction mix of a kernel's trace loop (the basic blocks hipcc marks "in Loop ... Depth>=1") from a
hipcc -S listing (make -C 4d_ray_tracing_amd/csrc asm): VALU, and the scalar side split into exec-mask
bookkeeping of divergent branches, branches, waits/nops, scalar memory and other SALU. The divergent regions
(s_and_saveexec ... s_or_b64 exec) are listed by the VALU they guard, so small ones stand out.
Usage: python tools/loop_mix.py <file.s> <kernel-substring>"""
import collections
import re
import sys


def kernel_body(path, sub):
    s = open(path).read()
    for m in re.finditer(r"^(\S*rt4\w*):\s*;\s*@", s, re.M):
        if sub in m.group(1):
            return m.group(1), s[m.end():s.index(".Lfunc_end", m.end())].splitlines()
    raise SystemExit(f"no kernel matching {sub}")


def kind(op, line):
    if op.startswith("v_"):
        return "valu"
    if op.startswith(("ds_", "global_", "buffer_", "scratch_", "flat_")):
        return "vmem/lds"
    if op.startswith("s_load") or op.startswith("s_buffer_load"):
        return "smem"
    if op.startswith("s_cbranch") or op == "s_branch":
        return "branch"
    if op in ("s_waitcnt", "s_nop", "s_barrier"):
        return "wait/nop"
    if "exec" in line and op.startswith("s_"):
        return "exec mask"
    if op.startswith("s_"):
        return "salu other"
    return "other"


def main():
    name, lines = kernel_body(sys.argv[1], sys.argv[2])
    depth = 0
    mix = collections.Counter()
    regions = []  # (line, guarded VALU)
    open_regions = {}
    for i, ln in enumerate(lines):
        if re.match(r"^(\.LBB|; %bb)", ln):
            m = re.search(r"Depth=(\d+)", ln)
            depth = int(m.group(1)) if m else 0
            continue
        t = ln.strip()
        if not t or t.startswith((";", ".")):
            continue
        op = t.split()[0]
        if depth == 0:
            continue
        mix[kind(op, t)] += 1
        m = re.search(r"s_and_saveexec_b64 (s\[\d+:\d+\])", t)
        if m:
            open_regions[m.group(1)] = [i, 0]
        m = re.search(r"s_or_b64 exec, exec, (s\[\d+:\d+\])", t)
        if m and m.group(1) in open_regions:
            regions.append(tuple(open_regions.pop(m.group(1))))
        if op.startswith("v_"):
            for r in open_regions.values():
                r[1] += 1
    total = sum(mix.values())
    print(name)
    print(f"trace-loop instructions (static): {total}")
    for k, n in mix.most_common():
        print(f"  {k:>12s} {n:5d}  {n / total * 100:5.1f} %")
    small = [r for r in regions if r[1] <= 8]
    print(f"divergent regions (s_and_saveexec .. s_or_b64 exec) in the loop: {len(regions)}, "
          f"guarding <= 8 VALU: {len(small)}")
    for ln, v in sorted(small):
        print(f"  line {ln:5d}: {v} VALU")


if __name__ == "__main__":
    main()
