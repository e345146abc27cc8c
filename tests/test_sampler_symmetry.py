"""could the 32 MiB sampler table (rt4.h RT4_FLAG_SAMPLER_LUT: w_by_volume of all 2^23 rand()
values, shader.frag:141-150) be served from half its size through the S^3 symmetry w(1 - v) = -w(v)? The identity
holds for the exact inverse of volume_by_w (shader.frag:136-138 is odd about w = 0, v = 1/2), but the table stores
the reference's Newton iterate, whose last bits depend on its start (w = 0), its one-sided finite difference (the
sign branch of :146) and its stopping rule. Exhaustively on the CPU (all 2^23 - 1 pairs m <-> 2^23 - m,
profiles/r05_ab.txt): only 33.4 % of the pairs are exact negatives, the rest differ by up to 3216 ulp, so a half
table would need an exception list of 5.6 M entries: rejected. This test pins the finding on a sample of pairs."""
import numpy as np

RT4_EVAL_W_BY_VOLUME = 5  # rt4.h rt4_eval_fn


def test_w_by_volume_antisymmetry_fails_for_most_pairs(oracle):
    m = np.arange(1, 1 << 23, 61, dtype=np.uint32)  # ~137 k pairs spread over the whole domain
    v = (m.astype(np.float64) * 2.0 ** -23).astype(np.float32)
    vm = ((np.uint32(1 << 23) - m).astype(np.float64) * 2.0 ** -23).astype(np.float32)  # 1 - v, exactly
    assert np.all(v.astype(np.float64) + vm.astype(np.float64) == 1.0)
    w, _ = oracle.eval_array(RT4_EVAL_W_BY_VOLUME, v)
    wm, _ = oracle.eval_array(RT4_EVAL_W_BY_VOLUME, vm)
    exact = wm.view(np.uint32) == (-w).view(np.uint32)
    assert 0.30 < exact.mean() < 0.37, exact.mean()  # exhaustive: 0.334
    ulp = np.abs(wm.astype(np.float64) + w.astype(np.float64)) / np.spacing(np.abs(w)).astype(np.float64)
    assert ulp.max() > 100  # exhaustive: 3216
