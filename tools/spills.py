#!/usr/bin/env python3
"""Where a kernel's register spills sit (hipcc -S listing, `make -C 4d_ray_tracing_amd/csrc asm`): every scratch
access with the loop depth of its basic block (the "in Loop: Header=... Depth=N" label comments), so a spill in
the trace loop can be told from one in the set-up or the final flush.
Usage: python tools/spills.py <file.s> <kernel-substring>"""
import re
import sys


def kernel_body(path, sub):
    s = open(path).read()
    for m in re.finditer(r"^(\S*rt4\w*):\s*;\s*@", s, re.M):
        if sub in m.group(1):
            return m.group(1), s[m.end():s.index(".Lfunc_end", m.end())].splitlines()
    raise SystemExit(f"no kernel matching {sub}")


def main():
    name, lines = kernel_body(sys.argv[1], sys.argv[2])
    depth, n_in, n_out = 0, 0, 0
    print(name)
    for i, ln in enumerate(lines):
        if re.match(r"^(\.LBB|; %bb)", ln):
            m = re.search(r"Depth=(\d+)", ln)
            depth = int(m.group(1)) if m else 0
        if "scratch_" in ln or "buffer_store" in ln or "buffer_load" in ln:
            where = f"loop depth {depth}" if depth else "outside the loops"
            print(f"  line {i:5d}  {where:18s}  {ln.strip()}")
            if depth:
                n_in += 1
            else:
                n_out += 1
    print(f"{n_in} scratch accesses inside loops, {n_out} outside")


if __name__ == "__main__":
    main()
