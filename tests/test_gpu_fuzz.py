"""Randomised extractor parity (seeded): image sizes, feature budgets, scale factors and level counts drawn
over the ranges ORB-SLAM2 configurations use and beyond (odd widths, short and tall images, few levels,
scale factors up to 1.6), each compared bit-exactly with the oracle.  Cases the geometry rejects (a level
without a single 30-px FAST cell, src/ORBextractor.cc:941-949 would divide by zero) must be rejected by
both the oracle and the extractor."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N_CASES = 40


# A level's keypoint budget is bounded by the quadtree's LDS node arrays (include/orbx.h, orbx_capacity):
# the random budgets stay below it; test_level_budget_beyond_quadtree_capacity covers the rejection.
MAX_LEVEL_BUDGET = 1400


def _level0_share(scale, nl):
    f = 1.0 / scale
    return (1 - f) / (1 - f ** nl) if nl > 1 else 1.0


def _cases():
    rng = np.random.default_rng(2026)
    out = []
    for i in range(N_CASES):
        w = int(rng.integers(96, 1400))
        h = int(rng.integers(80, 800))
        nfeat = int(rng.integers(100, 3000))
        scale = float(rng.choice([1.1, 1.2, 1.25, 1.3, 1.4, 1.6]))
        nl = int(rng.integers(1, 9))
        ini = int(rng.integers(10, 30))
        mn = int(rng.integers(3, ini))
        nfeat = min(nfeat, int(MAX_LEVEL_BUDGET / _level0_share(scale, nl)))
        out.append((i, w, h, nfeat, scale, nl, ini, mn))
    return out


@pytest.mark.parametrize("case", _cases(), ids=lambda c: "c%d_%dx%d_n%d_s%.2f_l%d" % c[:6])
def test_random_extractor_case(orbref, cuda, case):
    import orbx
    import orbx_synth
    from test_gpu_parity import assert_same_keypoints
    i, w, h, nfeat, scale, nl, ini, mn = case
    img = orbx_synth.gen_image(900 + i, w, h)
    p = orbref.make_params(nfeat, scale, nl, ini, mn)
    sizes = orbref.level_sizes(p, w, h)
    # every level needs one FAST cell of 30 px inside its 16-px border (EDGE_THRESHOLD - 3) on both axes
    # and a quadtree root: nIni = round(width / height) of the region inside the border must be >= 1 (:650)
    valid = all((lw - 19 + 3 - 16) >= 30 and (lh - 19 + 3 - 16) >= 30 and (lw - 32) >= 0.5 * (lh - 32)
                for lw, lh in sizes)
    ex = orbx.ORBextractor(nfeat, scale, nl, ini, mn)
    if not valid:
        with pytest.raises(orbx.OrbxError):
            ex(img)
        return
    ref = orbref.extract(img, p)
    kps, desc = ex(img)
    assert_same_keypoints(kps, ref.keypoints, desc, ref.descriptors, "case %s" % (case,))
    pyr = ex.mvImagePyramid
    for l in range(nl):
        assert np.array_equal(pyr[l], ref.pyramid[l]), "case %s level %d" % (case, l)


def test_level_budget_beyond_quadtree_capacity(orbref, cuda):
    """One level asked to keep 2600 keypoints: the quadtree's node arrays (about 90 B of LDS per node) would
    not fit a workgroup's 160 KB, so the extractor rejects the geometry instead of running it."""
    import orbx
    import orbx_synth
    ex = orbx.ORBextractor(2600, 1.2, 1, 20, 7)
    with pytest.raises(orbx.OrbxError):
        ex(orbx_synth.gen_image(5, 1036, 207))
    ok = orbx.ORBextractor(1400, 1.2, 1, 20, 7)   # within the budget: runs and matches the oracle
    img = orbx_synth.gen_image(5, 1036, 207)
    from test_gpu_parity import assert_same_keypoints
    ref = orbref.extract(img, orbref.make_params(1400, 1.2, 1, 20, 7), want_pyramid=False)
    kps, desc = ok(img)
    assert_same_keypoints(kps, ref.keypoints, desc, ref.descriptors, "1 level, 1400")


@pytest.mark.parametrize("batch", [1, 2, 8, 9, 23])
def test_batch_sizes_across_the_latency_threshold(orbref, cuda, batch):
    """Batches of up to 8 frames run FAST one cell per wave, describe one keypoint per wave and every quadtree
    level in one launch; larger ones run 3 cells / 4 keypoints per wave and per-level launches.  Both forms,
    and the boundary between them, give the oracle's result for every frame."""
    import orbx
    import orbx_synth
    from test_gpu_parity import _run_batch, assert_same_keypoints
    frames = np.stack([orbx_synth.gen_image(700 + f, 752, 480) for f in range(batch)])
    ex = orbx.ORBextractor(1000, 1.2, 8, 20, 7)
    p = orbref.make_params(1000, 1.2, 8, 20, 7)
    _, _, _, _, klist, dlist = _run_batch(ex, frames, cuda)
    for f in range(batch):
        ref = orbref.extract(frames[f], p, want_pyramid=False)
        assert_same_keypoints(klist[f], ref.keypoints, dlist[f], ref.descriptors, "batch %d frame %d" % (batch, f))
