"""Code-generation invariants of the built libraries, on the CPU.

At 6 waves/SIMD the tiger kernels ran at the register limit, and the compiler's live-range splitting could place
register copies in a join block ahead of its EXEC restore (s_or_b64 exec, exec, s[..]): lanes re-enabled by the
restore skip the copy-out but run the copy-back and receive another variable's value. Builds that differed only in
the machine scheduler (-amdgpu-sched-strategy=iterative-ilp) or in a pure-predicate rewrite of the sphere cull then
computed other images and counts on the MI355X (profiles/r05_ab.txt). The shipped library keeps every trace kernel
off scratch inside its trace loop, and no build may hold such copies. tools/codegen_check.py reads the gfx950 code
object out of each library and checks both."""
import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import codegen_check  # noqa: E402

PKG = os.path.join(ROOT, "4d_ray_tracing_amd")
PRODUCT = os.path.join(PKG, "lib", "librt4.so")
STRESS = [os.path.join(PKG, d, "librt4.so") for d in ("lib_alt/ilp", "lib_alt/cull", "lib_native")]

needs_llvm = pytest.mark.skipif(not os.path.exists(os.path.join(codegen_check.LLVM, "llvm-objdump")),
                                reason="ROCm llvm tools not installed")


def _require(lib):
    if not os.path.exists(lib):
        pytest.skip(f"{lib} not built (__graft_entry__.build())")


@needs_llvm
def test_product_kernels_no_loop_scratch_no_join_copies():
    _require(PRODUCT)
    rows = codegen_check.report(PRODUCT)
    assert len(rows) >= 50, rows  # every trace kernel instantiation of the kernel table
    assert [r for r in rows if r[1] != 0] == [], "scratch accesses inside a trace loop"
    assert [r for r in rows if r[3] != 0] == [], "register copies ahead of a join's EXEC restore"


@needs_llvm
@pytest.mark.parametrize("lib", STRESS, ids=lambda p: os.path.relpath(os.path.dirname(p), PKG))
def test_stress_builds_no_join_copies(lib):
    # the stress builds may spill in the loop (the iterative-ilp one does); what must never appear is the copy
    # pattern that miscomputed
    _require(lib)
    rows = codegen_check.report(lib)
    assert [r for r in rows if r[3] != 0] == []


@needs_llvm
def test_repro_build_is_flagged():
    """make repro: the bitwise-cull source with round 4's register use, the build whose all_primitives kernels
    miscomputed on the MI355X (profiles/r05/codegen/repro.log). The detector must flag it (a positive control on a
    real code object; the build is optional: make -C 4d_ray_tracing_amd/csrc repro)."""
    lib = os.path.join(PKG, "lib_repro", "librt4.so")
    _require(lib)
    flagged = [r[0] for r in codegen_check.report(lib) if r[3] != 0]
    assert flagged and all(name.startswith("K=33817407") for name in flagged), flagged


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
