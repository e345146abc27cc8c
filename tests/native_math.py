"""Native-math sensitivity report — TEST INFRASTRUCTURE ONLY.

The reference is a GLSL 330 shader whose built-ins (acos, asin, sin, cos, and whether a*b + c is fused)
are defined by whatever GL driver runs it; it cannot run here, so image parity is
pinned to rt4's one deterministic definition. This module measures how far the images
move when that definition is swapped for plain library built-ins with the shader's expressions unfused:
  * CPU: oracle/build/librt4_oracle_native.so (glibc acosf/asinf/sinf/cosf) vs the deterministic oracle;
  * GPU: lib_native/librt4.so (ocml, exact shortcuts compiled out) vs the deterministic kernel and vs the
    native oracle (two different native libms, as two GL drivers would differ).
Reported per BASELINE config (SURVEY.md 8(c)'s fallback definition): the fraction of pixels whose
RGB channels are all within 1e-4, the mean and max absolute channel error, the bit-identical pixel
fraction and the intersection counts. Configs 1-3 at their full frames; configs 4 and 5 (the tiger, the
union and the cylinders: the transcendental-heavy intersectors, shader.frag:211-217, :251-294, :317-341) on
four 8-row bands spread over the 3840x2160 frame (32 rows, 1/67.5 of it), one frame each (config 5: one
16-spp frame in fp32, so that only the built-ins differ).
"""
import numpy as np

CONFIGS = {  # BASELINE configs: scene, frame W x H, spp, bounces, rows (y0, band rows, band step, h)
    1: ("sphere", 256, 256, 1, 2, None),
    2: ("sphere", 1920, 1080, 16, 8, None),
    3: ("hypercube", 1920, 1080, 16, 8, None),
    4: ("tiger_two_mirrors", 3840, 2160, 64, 12, (266, 8, 540, 32)),
    5: ("all_primitives", 3840, 2160, 16, 8, (266, 8, 540, 32)),
}


def config_region(rt4, config):
    """The rendered region of a config: the whole frame, or its row bands (rt4_region band layout)."""
    _, W, H, _, _, rows = CONFIGS[config]
    if rows is None:
        return rt4.region(W, H)
    y0, band_rows, band_step, h = rows
    return rt4.region(W, h, 0, y0, band_rows, band_step)


def divergence(a, b, n_a=None, n_b=None):
    """Pixel statistics of two RGBA float32 frames (RGB only)."""
    e = np.abs(a[..., :3].astype(np.float64) - b[..., :3].astype(np.float64))
    pix = e.max(axis=-1)
    out = {
        "pixels": int(pix.size),
        "frac_within_1e-4": float((pix <= 1e-4).mean()),
        "frac_bit_identical": float((pix == 0).mean()),
        "mean_abs_error": float(e.mean()),
        "max_abs_error": float(e.max()),
    }
    if n_a is not None:
        out["intersections"] = [int(n_a), int(n_b)]
    return out
