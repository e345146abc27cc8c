"""Code-generation invariants of the built libraries, on the CPU.

At 6 waves/SIMD the tiger kernels ran at the register limit, and the compiler's live-range splitting could place
register copies in a join block ahead of its EXEC restore (s_or_b64 exec, exec, s[..]): lanes re-enabled by the
restore skip the copy-out but run the copy-back and receive another variable's value. Builds that differed only in
the machine scheduler (-amdgpu-sched-strategy=iterative-ilp) or in a pure-predicate rewrite of the sphere cull then
computed other images and counts on the MI355X (profiles/r05_ab.txt). The shipped library keeps every trace kernel
off scratch inside its trace loop, and no build may hold such copies. tools/codegen_check.py reads the gfx950 code
object out of each library and checks both."""
import gzip
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import codegen_check  # noqa: E402

PKG = os.path.join(ROOT, "4d_ray_tracing_amd")
PRODUCT = os.path.join(PKG, "lib", "librt4.so")
STRESS = [os.path.join(PKG, d, "librt4.so") for d in ("lib_alt/ilp", "lib_alt/cull", "lib_native")]

HAVE_LLVM = all(os.path.exists(os.path.join(codegen_check.LLVM, t)) for t in ("llvm-objdump", "llvm-objcopy", "llc"))
REPRO_IR = os.path.join(ROOT, "tools", "codegen_repro", "allprim_r05.ll.gz")


def _require(lib):
    """A library that is not built skips its test; one that is built must be checked: missing ROCm llvm tools then
    fail the test instead of skipping it."""
    if not os.path.exists(lib):
        pytest.skip(f"{lib} not built (__graft_entry__.build())")
    assert HAVE_LLVM, f"{lib} is built but the ROCm llvm tools under {codegen_check.LLVM} are missing: cannot check it"


def test_product_kernels_no_loop_scratch_no_join_copies():
    _require(PRODUCT)
    rows = codegen_check.report(PRODUCT)
    assert len(rows) >= 50, rows  # every trace kernel instantiation of the kernel table
    assert [r for r in rows if r[1] != 0] == [], "scratch accesses inside a trace loop"
    assert [r for r in rows if r[3] != 0] == [], "register copies ahead of a join's EXEC restore"


@pytest.mark.parametrize("lib", STRESS, ids=lambda p: os.path.relpath(os.path.dirname(p), PKG))
def test_stress_builds_no_join_copies(lib):
    # the stress builds may spill in the loop (the iterative-ilp one does); what must never appear is the copy
    # pattern that miscomputed
    _require(lib)
    rows = codegen_check.report(lib)
    assert [r for r in rows if r[3] != 0] == []


def test_llc_repro_is_flagged(tmp_path):
    """The reduced reproducer: the device IR of the round-5 all_primitives kernel that miscomputed
    on the MI355X (profiles/r05/codegen/repro.log). This image's llc must still place register copies ahead of a
    join's EXEC restore in it, and the detector must flag exactly that kernel; the day a ROCm update's llc stops, this
    test says so on the CPU."""
    if not HAVE_LLVM:
        pytest.skip("ROCm llvm tools not installed")
    ll = tmp_path / "k.ll"
    ll.write_bytes(gzip.decompress(open(REPRO_IR, "rb").read()))
    obj = tmp_path / "k.o"
    subprocess.run([os.path.join(codegen_check.LLVM, "llc"), "-O3", "-mtriple=amdgcn-amd-amdhsa", "-mcpu=gfx950",
                    "-filetype=obj", str(ll), "-o", str(obj)], check=True, capture_output=True)
    rows = codegen_check.report(obj=str(obj))
    assert [r[0] for r in rows] == ["K=33817407 lut=1 reuse=0"], rows
    assert rows[0][3] >= 1, rows  # the copy pattern
    assert rows[0][1] > 0, rows   # and the loop spills it comes with


def _insts(lines):
    return [(4 * k, t) for k, t in enumerate(lines)]


def test_detector_flags_copies_ahead_of_exec_restore():
    # the shape found in the broken all_primitives builds: a rotation of three registers ahead of the restore
    bad = _insts([
        "s_cbranch_execz 3 // <k+0xc>",
        "v_add_f32_e32 v1, v2, v3",
        "s_or_b64 exec, exec, s[6:7]",
        "v_mov_b32_e32 v51, v38",  # 0xc: the join block the branch skips to
        "v_mov_b32_e32 v38, v44",
        "v_mov_b32_e32 v77, 0x3c08839e",
        "s_or_b64 exec, exec, s[10:11]",
        "v_mov_b32_e32 v44, v38",
        "s_endpgm",
    ])
    assert codegen_check.split_copies_before_join(bad) == [0xC]


def test_detector_passes_copies_after_exec_restore_and_constants():
    ok = _insts([
        "s_cbranch_execz 3 // <k+0x10>",
        "v_add_f32_e32 v1, v2, v3",
        "s_or_b64 exec, exec, s[6:7]",
        "v_mov_b32_e32 v77, 0x3c08839e",  # a constant ahead of the restore: no lane's value is moved
        "s_or_b64 exec, exec, s[10:11]",
        "v_mov_b32_e32 v51, v38",          # after the restore: every lane of the join copies
        "s_endpgm",
    ])
    assert codegen_check.split_copies_before_join(ok) == []


@pytest.mark.parametrize("copy", [
    "v_mov_b64_e32 v[38:39], v[44:45]",
    "v_pk_mov_b32 v[68:69], v[14:15], v[16:17] op_sel:[1,0]",  # the 64-bit packed copy
    "v_accvgpr_write_b32 a3, v38",                             # a VGPR parked in an AGPR
    "v_accvgpr_read_b32 v38, a3",                              # and read back
    "v_accvgpr_mov_b32 a4, a3",
    "scratch_load_dword v38, off, s33 offset:4",               # a reload from scratch
    "buffer_load_dword v38, off, s[0:3], 0 offset:8",          # a reload through a MUBUF spill slot
])
def test_detector_flags_each_copy_form(copy):
    # one positive control per form a live-range split or spill can take ahead of the restore
    bad = _insts([
        "s_cbranch_execz 2 // <k+0x8>",
        "v_add_f32_e32 v1, v2, v3",
        copy,                                # 0x8: the join block the branch skips to
        "s_or_b64 exec, exec, s[10:11]",
        "s_endpgm",
    ])
    assert codegen_check.split_copies_before_join(bad) == [0x8]


def test_detector_counts_agpr_spills_in_loops():
    insts = _insts([
        "v_accvgpr_write_b32 a0, v1",        # before the loop
        "v_add_u32_e32 v0, 1, v0",            # loop head at 0x4
        "v_accvgpr_read_b32 v1, a0",          # inside: an AGPR spill reload
        "buffer_store_dword v2, off, s[0:3], 0",
        "s_cbranch_scc1 65532 // <k+0x4>",
    ])
    assert codegen_check.scratch_report(insts) == (2, 1)


def test_detector_loop_ranges():
    insts = _insts([
        "v_mov_b32_e32 v0, 0",
        "scratch_store_dword off, v0, off",  # before the loop
        "v_add_u32_e32 v0, 1, v0",            # loop head at 0x8
        "scratch_load_dword v1, off, off",    # inside
        "s_cbranch_scc1 65532 // <k+0x8>",    # backward branch
        "scratch_load_dword v1, off, off",    # after
    ])
    assert codegen_check.scratch_report(insts) == (1, 2)


@pytest.mark.skipif(shutil.which("make") is None, reason="no make")
def test_makefile_names_the_stress_builds():
    mk = open(os.path.join(PKG, "csrc", "Makefile")).read()
    assert "iterative-ilp" in mk and "RT4_CULL_BITWISE" in mk and "RT4_GUARD_WRITES" in mk
    # every library is checked after it is linked, and the repro target runs llc on the committed IR
    assert mk.count("$(call check_codegen,$@") == 4 and "allprim_r05.ll.gz" in mk
