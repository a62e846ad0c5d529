"""Randomised extractor parity (seeded): image sizes, feature budgets, scale factors and level counts drawn
over the ranges ORB-SLAM2 configurations use and beyond (odd widths, short and tall images, few levels,
scale factors up to 1.6), each compared bit-exactly with the oracle.  Cases the geometry rejects (a level
without a single 30-px FAST cell, src/ORBextractor.cc:941-949 would divide by zero) must be rejected by
both the oracle and the extractor."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N_CASES = 40


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


def test_level_budget_past_lds_node_arrays(orbref, cuda):
    """One level asked to keep 2600 keypoints: the quadtree's node list (about 90 B per node) does not fit a
    workgroup's 160 KB of LDS, so that level's node arrays run from global memory (LevelGeom::qt_glob), with
    the same result as the oracle; 1400 still runs from LDS.  Both through the host call and a batch."""
    import orbx
    import orbx_synth
    from test_gpu_parity import _run_batch, assert_same_keypoints
    noise = np.random.default_rng(8).integers(0, 256, (207, 1036), dtype=np.uint8)   # ~18k candidates
    for img in (orbx_synth.gen_image(5, 1036, 207), noise):
        for nfeat in (2600, 1400, 6000):
            ex = orbx.ORBextractor(nfeat, 1.2, 1, 20, 7)
            ref = orbref.extract(img, orbref.make_params(nfeat, 1.2, 1, 20, 7), want_pyramid=False)
            kps, desc = ex(img)
            assert_same_keypoints(kps, ref.keypoints, desc, ref.descriptors, "1 level, %d" % nfeat)
            assert len(ref.keypoints) > min(nfeat, 1000)
    frames = np.stack([orbx_synth.gen_image(60 + f, 1036, 207) for f in range(11)])
    ex = orbx.ORBextractor(2600, 1.2, 1, 20, 7)
    _, _, _, _, klist, dlist = _run_batch(ex, frames, cuda)
    p = orbref.make_params(2600, 1.2, 1, 20, 7)
    for f in range(len(frames)):
        ref = orbref.extract(frames[f], p, want_pyramid=False)
        assert_same_keypoints(klist[f], ref.keypoints, dlist[f], ref.descriptors, "batch frame %d" % f)


def test_initialisation_extractor_8000_at_1080p(orbref, cuda):
    """Tracking's monocular initialisation extractor is ORBextractor(2 * nFeatures, ...) (src/Tracking.cc:133):
    at config 5's 4000 features that is 8000, about 1,738 keypoints at level 0, past the LDS node arrays.
    Extraction (host call and a 9-frame batch, i.e. per-level launches) and SearchForInitialization on the
    result both match the oracle."""
    import torch
    import orbx
    import orbx_synth
    from test_gpu_parity import _run_batch, assert_same_keypoints
    p = orbref.make_params(8000, 1.2, 8, 20, 7)
    ex = orbx.ORBextractor(8000, 1.2, 8, 20, 7)
    img = orbx_synth.gen_image(77, 1920, 1080)
    ref = orbref.extract(img, p, want_pyramid=False)
    kps, desc = ex(img)
    assert_same_keypoints(kps, ref.keypoints, desc, ref.descriptors, "host 8000")
    assert (ref.keypoints["octave"] == 0).sum() > 1700
    big = orbx_synth.gen_image(78, 2000, 1100)   # 9 consecutive frames of a slow pan
    frames = np.stack([big[2 * f:2 * f + 1080, 3 * f:3 * f + 1920] for f in range(9)])
    imgs, dk, dd, dc, klist, dlist = _run_batch(ex, frames, cuda)
    refs = [orbref.extract(frames[f], p, want_pyramid=False) for f in range(len(frames))]
    for f in range(len(frames)):
        assert_same_keypoints(klist[f], refs[f].keypoints, dlist[f], refs[f].descriptors, "batch frame %d" % f)
    pa = torch.tensor([0, 1, 4], dtype=torch.int32, device=cuda)
    pb = torch.tensor([1, 2, 5], dtype=torch.int32, device=cuda)
    m = orbx.ORBmatcher(0.9, True)
    m12, nm = m.search_for_initialization_batch(dk, dd, dc, pa, pb, 1080, 1920, 100)
    torch.cuda.synchronize()
    m12, nm = m12.cpu().numpy(), nm.cpu().numpy()
    for i, (a, b) in enumerate(zip(pa.tolist(), pb.tolist())):
        want_n, want_m, _ = orbref.search_for_initialization(refs[a].keypoints, refs[a].descriptors,
                                                             refs[b].keypoints, refs[b].descriptors, 1920, 1080,
                                                             window=100, nnratio=0.9, check_ori=True)
        assert nm[i] == want_n, "pair %d: %d matches vs oracle %d" % (i, nm[i], want_n)
        assert np.array_equal(m12[i, :len(want_m)], want_m)
    assert nm[0] > 100


def test_phase2_nodes_past_16_bit_sizes(orbref, cuda):
    """A tiny budget on a 2000 x 2000 noise image: about 400k FAST candidates meet at the single root, whose
    four children (about 100k each) go straight into phase 2 (4 + 3 * 4 > N), so phase 2 sorts nodes of more
    than 0xFFFF keypoints, past the packed (size, creation) key (csrc/orbx_extract.hip, SH_BIG); the
    (size, creation) order must still be the oracle's."""
    import orbx
    from test_gpu_parity import assert_same_keypoints
    img = np.random.default_rng(3).integers(0, 256, (2000, 2000), dtype=np.uint8)
    for nfeat in (6, 10, 15):
        ex = orbx.ORBextractor(nfeat, 1.2, 1, 20, 7)
        ref = orbref.extract(img, orbref.make_params(nfeat, 1.2, 1, 20, 7), want_pyramid=False)
        kps, desc = ex(img)
        assert_same_keypoints(kps, ref.keypoints, desc, ref.descriptors, "noise, %d" % nfeat)


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
