"""Extractor parameter edges the fuzz cases (tests/test_gpu_fuzz.py) do not draw, each bit-exact against the oracle:
FAST thresholds with minThFAST >= iniThFAST (the retry at src/ORBextractor.cc:982-987 then keeps at most what
the first pass kept) and thresholds down to 1, feature budgets of 1-9 (the per-level shares of
src/ORBextractor.cc:427-440 round to zero or one, but DistributeOctTree splits the root before it tests the
node count, so the oracle keeps 4 keypoints per level, 32 at 640 x 480), a scale factor of 2, and a level 0 at
the 4096-px side the packed coordinates allow."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _check(orbref, img, nfeat, scale, nl, ini, mn, tag, batch_frames=None, cuda=None):
    import orbx
    from test_gpu_parity import _run_batch, assert_same_keypoints
    p = orbref.make_params(nfeat, scale, nl, ini, mn)
    ex = orbx.ORBextractor(nfeat, scale, nl, ini, mn)
    ref = orbref.extract(img, p, want_pyramid=False)
    kps, desc = ex(img)
    assert_same_keypoints(kps, ref.keypoints, desc, ref.descriptors, tag)
    if batch_frames is not None:
        _, _, _, _, klist, dlist = _run_batch(ex, batch_frames, cuda)
        for f in range(len(batch_frames)):
            r = orbref.extract(batch_frames[f], p, want_pyramid=False)
            assert_same_keypoints(klist[f], r.keypoints, dlist[f], r.descriptors, "%s batch frame %d" % (tag, f))
    return ref


@pytest.mark.parametrize("ini,mn", [(20, 20), (12, 30), (5, 1), (1, 1), (60, 40), (90, 7)])
def test_fast_threshold_edges(orbref, cuda, ini, mn):
    import orbx_synth
    img = orbx_synth.gen_image(41, 752, 480)
    frames = np.stack([orbx_synth.gen_image(42 + f, 752, 480) for f in range(10)])
    ref = _check(orbref, img, 1000, 1.2, 8, ini, mn, "ini %d min %d" % (ini, mn), frames, cuda)
    assert len(ref.keypoints) > 0


@pytest.mark.parametrize("nfeat", [1, 2, 5, 9])
def test_tiny_feature_budgets(orbref, cuda, nfeat):
    import orbx_synth
    img = orbx_synth.gen_image(51, 640, 480)
    frames = np.stack([orbx_synth.gen_image(52 + f, 640, 480) for f in range(9)])
    _check(orbref, img, nfeat, 1.2, 8, 20, 7, "nfeat %d" % nfeat, frames, cuda)


def test_scale_factor_two(orbref, cuda):
    import orbx_synth
    # three levels: KITTI's fourth at scale 2 (155 x 47) has no 30-px FAST cell, which the extractor rejects
    frames = orbx_synth.kitti_sequence(9, start=3)
    ref = _check(orbref, frames[0], 2000, 2.0, 3, 20, 7, "scale 2", frames, cuda)
    assert (ref.keypoints["octave"] == 2).sum() > 0


def test_level0_at_the_4096_px_side(orbref, cuda):
    """4096 x 320: level 0's keypoint x reaches 4096 - 19, the largest a 12-bit packed x holds (the split
    the geometry picks up to 4096 x 4096, orbx_geom.hpp pack_kp), on every level and through both the host call
    and a batch."""
    import orbx_synth
    img = orbx_synth.gen_image(61, 4096, 320)
    frames = np.stack([orbx_synth.gen_image(62 + f, 4096, 320) for f in range(9)])
    ref = _check(orbref, img, 4000, 1.2, 8, 20, 7, "4096 wide", frames, cuda)
    assert ref.keypoints["x"].max() > 4000


def test_buffer_range_check_covers_soffset(cuda):
    """k_fast_cells' first staging passes (fast_issue0) load a partial last pass's rows past the cell ROI through
    a buffer descriptor sized to end at the ROI's last byte, with the pass's row offset in the scalar offset.
    That is memory-safe only if gfx950's range check tests voffset + soffset against num_records, so that those
    loads return zeros without touching memory.  tools/probes/buffer_oob.hip pins it: a 64-byte descriptor over
    nonzero data, loads at soffset 0 / 64 / 256."""
    import ctypes
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    path = os.path.join(root, "tools", "probes", "liboob_probe.so")
    assert os.path.exists(path), "liboob_probe.so missing: run __graft_entry__.build()"
    lib = ctypes.CDLL(path)
    r = (ctypes.c_uint32 * (3 * 64))()
    assert lib.oob_probe_run(r) == 0
    v = np.frombuffer(r, dtype=np.uint32).reshape(3, 64)
    want0 = np.where(np.arange(64) < 16, 0x1000 + np.arange(64), 0).astype(np.uint32)
    assert np.array_equal(v[0], want0), v[0]                   # the descriptor's 16 dwords, zeros past them
    assert not v[1].any() and not v[2].any(), (v[1], v[2])     # soffset moves every lane past num_records


def test_border_patches_of_levels_with_little_row_padding(orbref, cuda):
    """describe stages a level >= 1 border keypoint's patch by buffer-descriptor DMA only when the level's row
    padding (pitch - width) is at least 16 bytes, so that a 16-byte chunk straddling the level's end never drops a
    pixel; levels with less take the reflect-101 byte path.  1224 x 400: level 1 is 1020 px wide in a 1024-byte
    pitch (4 bytes of padding), level 2 850 in 896 (46), so both paths run in one frame, with the default
    threshold's keypoints along every edge, bit-exact through the host call and a 10-frame batch."""
    import orbx_synth
    img = orbx_synth.gen_image(71, 1224, 400)
    frames = np.stack([orbx_synth.gen_image(72 + f, 1224, 400) for f in range(10)])
    ref = _check(orbref, img, 2000, 1.2, 8, 20, 7, "1224 x 400", frames, cuda)
    lv1 = ref.keypoints[ref.keypoints["octave"] == 1]
    assert len(lv1) > 0
