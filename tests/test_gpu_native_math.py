"""Native-math mode on the MI355X: lib_native/librt4.so, the kernel built with
-DRT4_NATIVE_MATH (ocml acosf/asinf/sinf/cosf, the shader's multiply-adds unfused, the exact shortcuts
compiled out), against the deterministic kernel and against the native CPU oracle (glibc) on BASELINE
configs 1-3 at their full shapes and configs 4-5 (tiger, union, cylinders) on row bands. SURVEY.md 8(c): "native-math mode: pixel fraction within 1e-4 plus mean
error, reported". A sensitivity report of the images to the built-ins' definition (the GL reference's
driver-defined acos/asin/sin/cos, shader.frag:50,129,137,211-217), not a parity test."""
import json
import os

import pytest

from native_math import CONFIGS, config_region, divergence

pytestmark = pytest.mark.gpu

THREADS = max(1, min(16, os.cpu_count() or 1))


def gpu_frame(rt4, library, scene, u, reg):
    import torch

    t = rt4.Tracer(device=0, flags=rt4.FLAG_SAMPLER_LUT, scene=scene, library=library)
    try:
        fr = torch.zeros((reg.h, reg.w, 4), dtype=torch.float32, device="cuda")
        cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
        t.render_device(u, reg, fr.data_ptr(), reg.w, cnt.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        return fr.cpu().numpy(), int(cnt.item())
    finally:
        t.close()


@pytest.mark.parametrize("config", [1, 2, 3, 4, 5])
def test_native_ocml_kernel_vs_deterministic(rt4, oracle, config):
    native_lib = rt4.load_variant(os.path.join(os.path.dirname(rt4.LIB_PATH), "..", "lib_native", "librt4.so"))
    name, W, H, spp, bounces, _ = CONFIGS[config]
    scene = rt4.Scene.named(name)
    u = rt4.make_uniforms(W, H, samples=spp, reflections=bounces, seed=12345)
    reg = config_region(rt4, config)
    det, n_det = gpu_frame(rt4, None, scene, u, reg)
    nat, n_nat = gpu_frame(rt4, native_lib, scene, u, reg)
    cpu_nat, n_cpu = oracle.render(scene.desc, u, reg, threads=THREADS, native=True)[:2]
    d1 = divergence(det, nat, n_det, n_nat)
    d2 = divergence(cpu_nat, nat, n_cpu, n_nat)
    print(f"config {config} native ocml kernel vs deterministic kernel: {json.dumps(d1)}")
    print(f"config {config} native ocml kernel vs native glibc oracle: {json.dumps(d2)}")
    for d in (d1, d2):
        assert d["frac_within_1e-4"] >= 0.999
        assert d["mean_abs_error"] < 1e-5
    assert (nat[..., 3] == 1.0).all() and (nat[..., :3] >= 0).all() and (nat[..., :3] < 1).all()
