"""Host-side C++ of librt4 (rt4_host.cpp: scene .frag loader, properties.txt parser, camera, PPM
writer) under AddressSanitizer + UndefinedBehaviorSanitizer, CPU only (GPU sanitizers are not
available on the MI355X pool). tools/host_fuzz.cpp parses every repo scene and properties.txt, every
prefix of each, and 3000 seeded byte mutations of each; any sanitizer report fails the run."""
import glob
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(600)
def test_host_code_under_asan_ubsan(tmp_path):
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    exe = tmp_path / "host_fuzz"
    subprocess.check_call(["g++", "-std=c++17", "-g", "-O1", "-fsanitize=address,undefined",
                           "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer",
                           "-I", os.path.join(ROOT, "include"), "-o", str(exe),
                           os.path.join(ROOT, "tools", "host_fuzz.cpp"),
                           os.path.join(ROOT, "4d_ray_tracing_amd", "csrc", "rt4_host.cpp")])
    inputs = [os.path.join(ROOT, "properties.txt")] + sorted(glob.glob(os.path.join(ROOT, "scenes", "*.frag")))
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:exitcode=86",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1:exitcode=87")
    r = subprocess.run([str(exe), str(tmp_path)] + inputs, capture_output=True, text=True, env=env, timeout=540)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "host_fuzz ok" in r.stdout
