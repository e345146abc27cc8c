#!/usr/bin/env python3
"""Scratch (spill) accesses of every trace kernel in a built librt4.so, split into those inside a loop and
those outside (no trace kernel may touch scratch inside its trace loop).

The device code object is taken from the library's .hip_fatbin section (llvm-objcopy, clang-offload-bundler)
and disassembled (llvm-objdump). A loop is the address range of a backward branch: [target, branch]. A
scratch instruction inside any such range of its kernel counts as "in a loop".

Usage: python tools/codegen_check.py [--joins-only] [librt4.so | --object code.o]   (one line per trace kernel)
  --object     check a device code object (ELF) directly, e.g. llc's output for tools/codegen_repro/*.ll.gz
  --joins-only fail only on join-block copies (the stress builds may spill in their loops)
Exit status 1 when a kernel fails a check: the csrc Makefile runs this after linking each library, so a build
whose trace kernels touch scratch in a loop or hold the copy pattern fails.

The reduced reproducer of the fault: tools/codegen_repro/allprim_r05.ll.gz is the device
LLVM IR of the one all_primitives trace kernel (LUT, no reuse) of the round-5 source that miscomputed on the
MI355X (the bitwise cull at 6 waves/SIMD, commit f7bc3cd, profiles/r05/codegen/repro.log), cut out of the module
with opt's internalize + globaldce. `make -C 4d_ray_tracing_amd/csrc repro` runs
  gunzip -c tools/codegen_repro/allprim_r05.ll.gz | llc -O3 -mtriple=amdgcn-amd-amdhsa -mcpu=gfx950 -filetype=obj
and requires this detector to flag the result; a ROCm update whose llc no longer produces the pattern shows there
first, on the CPU."""
import os
import re
import subprocess
import sys
import tempfile

LLVM = os.environ.get("ROCM_LLVM_BIN", "/opt/rocm/lib/llvm/bin")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEFAULT_LIB = os.path.join(ROOT, "4d_ray_tracing_amd", "lib", "librt4.so")


def disassemble_object(co):
    return subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co], check=True,
                          capture_output=True, text=True).stdout


def disassemble(lib):
    with tempfile.TemporaryDirectory() as d:
        fat, co = os.path.join(d, "fat.bin"), os.path.join(d, "dev.co")
        subprocess.run([f"{LLVM}/llvm-objcopy", "--dump-section", f".hip_fatbin={fat}", lib, os.path.join(d, "x.so")],
                       check=True, capture_output=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True, capture_output=True)
        return subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co], check=True,
                              capture_output=True, text=True).stdout


HEAD = re.compile(r"^[0-9a-f]+ <(\S+)>:$")
ADDR = re.compile(r"//\s*([0-9A-F]+):")
TARGET = re.compile(r"<(\S+)\+0x([0-9a-f]+)>")


def kernels(dis):
    """{kernel symbol: [(offset, text), ...]} for the trace kernels."""
    out, cur, base = {}, None, 0
    for ln in dis.splitlines():
        m = HEAD.match(ln)
        if m:
            cur = m.group(1) if "rt4_trace_kernel" in m.group(1) else None
            base = None
            if cur:
                out[cur] = []
            continue
        if cur is None:
            continue
        a = ADDR.search(ln)
        if not a:
            continue
        addr = int(a.group(1), 16)
        if base is None:
            base = addr
        out[cur].append((addr - base, ln.strip()))
    return out


# Spill traffic: scratch (flat scratch or MUBUF) stores and reloads, and moves between VGPRs and AGPRs. The trace
# kernels use no MFMA, so any AGPR access is the register allocator parking a VGPR in the accumulation registers of
# gfx950's unified register file (.amdhsa_accum_offset), its first spill target before scratch.
SPILL = ("scratch_", "buffer_store", "buffer_load", "v_accvgpr_write", "v_accvgpr_read", "v_accvgpr_mov")


def scratch_report(insts):
    """(spill accesses inside a loop, outside any loop) of one kernel; a loop is a backward branch's range."""
    loops = []
    for off, text in insts:
        if text.startswith(("s_branch", "s_cbranch")):
            t = TARGET.search(text)
            if t and int(t.group(2), 16) <= off:
                loops.append((int(t.group(2), 16), off))
    inside, outside = 0, 0
    for off, text in insts:
        if text.startswith(SPILL):
            if any(lo <= off <= hi for lo, hi in loops):
                inside += 1
            else:
                outside += 1
    return inside, outside


_R = r"[va](?:\[\d+:\d+\]|\d+)"  # a VGPR or AGPR, single or a range
# register-to-register moves of a lane's value: VGPR copies (32/64-bit), the packed 64-bit copy (v_pk_mov_b32 takes one
# dword from each source pair, so it is a copy whenever both sources are registers), and AGPR reads/writes/moves
VCOPY = re.compile(r"^(?:v_mov_b(?:32|64)(?:_e32|_e64)?\s+v(?:\[\d+:\d+\]|\d+),\s*v(?:\[\d+:\d+\]|\d+)"
                   r"|v_pk_mov_b32\s+" + _R + r",\s*" + _R + r",\s*" + _R + r"(?:\s+op_sel:\[\d,\d\])?"
                   r"|v_accvgpr_(?:read|write|mov)_b32(?:_e64)?\s+" + _R + r",\s*" + _R + r")$")
RELOAD = ("scratch_load", "buffer_load")  # a reload of a split or spilled value
CONTROL = ("s_branch", "s_cbranch", "s_and_saveexec", "s_or_saveexec", "s_andn2_saveexec", "s_xor_b64 exec",
           "s_mov_b64 exec", "s_and_b64 exec", "s_andn2_b64 exec", "s_endpgm", "s_setpc", "s_swappc")


def split_copies_before_join(insts):
    """Register-to-register copies (VGPR, packed 64-bit or AGPR moves) or reloads (scratch, MUBUF) placed in a join
    block ahead of its EXEC restore
    (s_or_b64 exec, exec, s[..]).
    They run only for the lanes of the branch that falls into the block; the lanes the restore re-enables skip them,
    so a live-range split whose copy-out lands there and whose copy-back runs after the restore hands those lanes
    another variable's value. Returns the offsets of such blocks."""
    starts = {0}
    for k, (off, text) in enumerate(insts):
        if text.startswith(("s_branch", "s_cbranch")):
            t = TARGET.search(text)
            if t:
                starts.add(int(t.group(2), 16))
            if k + 1 < len(insts):
                starts.add(insts[k + 1][0])
    found = []
    for k, (off, text) in enumerate(insts):
        if off not in starts:
            continue
        copies = 0
        for off2, t2 in insts[k:]:
            if off2 != off and off2 in starts:
                break
            if t2.startswith("s_or_b64 exec, exec, s["):
                if copies:
                    found.append(off)
                break
            if t2.startswith(CONTROL):
                break
            t2c = t2.split("//")[0].strip()
            if VCOPY.match(t2c) or t2c.startswith(RELOAD):  # a register copy or a reload of a split
                copies += 1
    return found


def short_name(sym):
    m = re.search(r"rt4_trace_kernelILj(\d+)ELb(\d)ELb(\d)E", sym)
    if not m:
        return sym
    return f"K={m.group(1)} lut={m.group(2)} reuse={m.group(3)}"


def report(lib=DEFAULT_LIB, obj=None):
    """[(kernel, scratch accesses in loops, outside, join blocks with copies ahead of the EXEC restore)] for every
    trace kernel of lib (or of the device code object obj)."""
    ks = kernels(disassemble_object(obj) if obj else disassemble(lib))
    return [(short_name(k), *scratch_report(v), len(split_copies_before_join(v))) for k, v in sorted(ks.items())]


if __name__ == "__main__":
    argv = sys.argv[1:]
    joins_only = "--joins-only" in argv
    argv = [a for a in argv if a != "--joins-only"]
    obj = argv[argv.index("--object") + 1] if "--object" in argv else None
    lib = argv[0] if argv and not obj else DEFAULT_LIB
    rows = report(lib, obj)
    if not rows:
        print(f"no trace kernels found in {obj or lib}")
        sys.exit(2)
    bad_loop = bad_join = 0
    for name, inside, outside, joins in rows:
        print(f"{name:40s} scratch accesses in loops {inside:3d}, outside {outside:3d}; copies ahead of a join's "
              f"EXEC restore {joins}")
        bad_loop += inside != 0
        bad_join += joins != 0
    print(f"{bad_loop} trace kernels with scratch accesses inside a loop, {bad_join} with copies ahead of a join's "
          f"EXEC restore")
    sys.exit(1 if bad_join or (bad_loop and not joins_only) else 0)
