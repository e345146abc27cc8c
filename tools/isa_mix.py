#!/usr/bin/env python3
"""Static instruction mix of one kernel in a hipcc -S listing (make -C 4d_ray_tracing_amd/csrc asm).
Usage: python tools/isa_mix.py <file.s> <kernel-substring> [top]"""
import collections
import re
import sys


def body(path, sub):
    s = open(path).read()
    for m in re.finditer(r"^(\S*rt4\w*):\s*;\s*@", s, re.M):
        if sub in m.group(1):
            end = s.index(".Lfunc_end", m.end())
            return m.group(1), s[m.end():end]
    raise SystemExit(f"no kernel matching {sub}")


def main():
    name, b = body(sys.argv[1], sys.argv[2])
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 50
    ins = [l.split()[0] for l in b.splitlines() if l.startswith("\t") and not l.startswith(("\t.", "\t;"))]
    c = collections.Counter(ins)
    print(name)
    print(len(ins), "instructions;", sum(n for k, n in c.items() if k.startswith("v_")), "VALU;",
          sum(n for k, n in c.items() if k.startswith("s_")), "SALU/branch")
    for k, n in c.most_common(top):
        print(f"{n:5d} {k}")


if __name__ == "__main__":
    main()
