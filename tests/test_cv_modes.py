"""SURVEY.md Appendix A's alternative OpenCV builds: the oracle's modes against independent
numpy restatements written from OpenCV's published source (CPU), and the GPU in each mode it implements against
the oracle in the same mode (-m gpu), bit-exact.

  resize  ORBX_RESIZE_SSE2: VResizeLinearVec_32s8u's vertical pass, ((mulhi16(h0 >> 4, b0) + mulhi16(h1 >> 4, b1)
          + 2) >> 2), on all but a 0..4-px row tail (A.2; src/ORBextractor.cc:1361)
  blur    ORBX_BLUR_SSE2: SymmColumnVec_32s8u's float column pass, half-to-even rounding on all but the row's
          width % 4 tail; ORBX_BLUR_BITEXACT: 3.4.6+ / 4.x's fixed-point kernel [18 34 48 56 48 34 18] (A.3; :1301-1306)
  trig    correctly rounded cos / sin of the BRIEF angle (A.5; :146-148), oracle only

OpenCV itself is absent here, so these pin the restatements against each other, not against a real OpenCV build
(parity unpinned)."""
import math

import numpy as np
import pytest


# ---- numpy restatements ------------------------------------------------------------------------------------------
def _simd_end_np(w):
    x = 0
    while x <= w - 16:
        x += 16
    while x < w - 4:
        x += 4
    return x


def _resize_np(src, dw, dh, sse2):
    """cv::resize INTER_LINEAR u8: float32 source coordinates, cvRound'ed 11-bit coefficients."""
    sh, sw = src.shape
    sx_ = (np.arange(dw) + 0.5) * (sw / dw) - 0.5
    fx = sx_.astype(np.float32)
    ix = np.floor(fx).astype(np.int64)
    fx = (fx - ix.astype(np.float32)).astype(np.float32)
    lo = ix < 0
    fx[lo], ix[lo] = 0, 0
    hi = ix >= sw - 1
    fx[hi], ix[hi] = 0, sw - 1
    a0 = np.rint((np.float32(1) - fx) * np.float32(2048)).astype(np.int64)
    a1 = np.rint(fx * np.float32(2048)).astype(np.int64)
    x1 = np.minimum(ix + 1, sw - 1)
    S = src.astype(np.int64)
    H = S[:, ix] * a0 + S[:, x1] * a1                      # [sh, dw]
    out = np.empty((dh, dw), np.uint8)
    xs = _simd_end_np(dw) if sse2 else 0
    for dy in range(dh):
        fy = np.float32((dy + 0.5) * (sh / dh) - 0.5)
        sy = int(math.floor(fy))
        fy = np.float32(fy - np.float32(sy))
        b0 = int(np.rint((np.float32(1) - fy) * np.float32(2048)))
        b1 = int(np.rint(fy * np.float32(2048)))
        h0 = H[min(max(sy, 0), sh - 1)]
        h1 = H[min(max(sy + 1, 0), sh - 1)]
        sc = (h0 * b0 + h1 * b1 + (1 << 21)) >> 22
        ss = (((h0 >> 4) * b0 >> 16) + ((h1 >> 4) * b1 >> 16) + 2) >> 2
        out[dy] = np.clip(np.where(np.arange(dw) < xs, ss, sc), 0, 255)
    return out


def _blur_np(img, kernel, sse2):
    h, w = img.shape
    k = np.asarray(kernel, np.int64)
    pad = np.pad(img.astype(np.int64), 3, mode="reflect")   # reflect == OpenCV BORDER_REFLECT_101
    rows = sum(k[i] * pad[:, i:i + w] for i in range(7))     # [h + 6, w]
    T = sum(k[j] * rows[j:j + h] for j in range(7))          # [h, w]
    scalar = np.clip((T + (1 << 15)) >> 16, 0, 255)
    if not sse2:
        return scalar.astype(np.uint8)
    f = (k[3:7].astype(np.float32) / np.float32(65536))
    s = rows[3:3 + h].astype(np.float32) * f[0] + np.float32(0)
    for j in (1, 2, 3):
        s = s + (rows[3 + j:3 + j + h] + rows[3 - j:3 - j + h]).astype(np.float32) * f[j]
    simd = np.clip(np.rint(s), 0, 255)                      # _mm_cvtps_epi32: half to even
    cols = np.arange(w) < (w & ~3)
    return np.where(cols[None, :], simd, scalar).astype(np.uint8)


# ---- CPU: oracle modes against the restatements ------------------------------------------------------------------
def test_resize_simd_end(orbref):
    for w in list(range(1, 70)) + [346, 416, 499, 598, 718, 862, 1034, 1241]:
        assert orbref.resize_simd_end(w) == _simd_end_np(w), w
    assert [orbref.resize_simd_end(w) for w in (16, 17, 20, 21)] == [16, 16, 16, 20]


@pytest.mark.parametrize("mode", [0, 1])
def test_resize_modes_match_restatement(orbref, mode):
    rng = np.random.default_rng(5 + mode)
    for sw, sh, dw, dh in [(640, 480, 533, 400), (1241, 376, 1034, 313), (83, 61, 69, 51), (60, 40, 50, 33),
                           (64, 48, 32, 24)]:
        src = rng.integers(0, 256, (sh, sw), dtype=np.uint8)
        got = orbref.resize_linear(src, dw, dh, mode)
        assert np.array_equal(got, _resize_np(src, dw, dh, mode == 1)), (sw, sh, dw, dh)


def test_resize_sse2_differs_only_by_one_and_not_in_the_tail(orbref):
    rng = np.random.default_rng(8)
    src = rng.integers(0, 256, (376, 1241), dtype=np.uint8)
    a = orbref.resize_linear(src, 1034, 313, 0).astype(int)
    b = orbref.resize_linear(src, 1034, 313, 1).astype(int)
    d = b - a
    xs = orbref.resize_simd_end(1034)
    assert set(np.unique(d)) <= {-1, 0}                     # the SIMD form truncates twice: never above
    assert (d != 0).mean() > 0.1 and not d[:, xs:].any()
    c = np.full((40, 64), 173, np.uint8)                     # constant stays constant in both
    assert (orbref.resize_linear(c, 53, 33, 1) == 173).all()


def test_blur_kernels(orbref):
    assert orbref.blur_kernel(orbref.BLUR_SCALAR).tolist() == [18, 34, 49, 55, 49, 34, 18]
    assert orbref.blur_kernel(orbref.BLUR_SSE2).tolist() == [18, 34, 49, 55, 49, 34, 18]
    # getGaussianKernelBitExact (sigma 2) + getGaussianKernelFixedPoint_ED at 8 fraction bits, restated
    vals = [math.exp(x * x * (-0.125 / 4.0)) for x in (-6, -4, -2)]
    mul = 1.0 / (2 * sum(vals) + 1)
    err, side = 0.0, []
    for v in vals:
        adj = v * mul * 256 + err
        r = round(adj)
        err = adj - r
        side.append(r)
    want = side + [256 - 2 * sum(side)] + side[::-1]
    assert orbref.blur_kernel(orbref.BLUR_BITEXACT).tolist() == want == [18, 34, 48, 56, 48, 34, 18]


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_blur_modes_match_restatement(orbref, mode):
    rng = np.random.default_rng(11)
    diffs = 0
    k = orbref.blur_kernel(mode)
    for h, w in [(61, 83), (40, 64), (120, 203), (97, 31)]:
        for _ in range(6):
            img = rng.integers(0, 256, (h, w), dtype=np.uint8)
            got = orbref.gaussian_blur7(img, mode)
            assert np.array_equal(got, _blur_np(img, k, mode == 1)), (h, w)
            diffs += int((got != orbref.gaussian_blur7(img, 0)).sum())
    if mode == 1:   # ties at T % 2^16 == 2^15 above an even quotient are rare (~1 pixel in 2^17) but do occur
        big = rng.integers(0, 256, (400, 640), dtype=np.uint8)
        got = orbref.gaussian_blur7(big, 1)
        assert np.array_equal(got, _blur_np(big, k, True))
        diffs += int((got != orbref.gaussian_blur7(big, 0)).sum())
        assert diffs > 0
    elif mode == 2:
        assert diffs > 0
    else:
        assert diffs == 0


def test_trig_modes_agree_on_axes(orbref):
    blur = np.random.default_rng(3).integers(0, 256, (64, 64), dtype=np.uint8)
    for ang in (0.0, 90.0, 180.0, 270.0, 45.0):
        a = orbref.brief(blur, 32.0, 32.0, ang, orbref.TRIG_GLIBC)
        b = orbref.brief(blur, 32.0, 32.0, ang, orbref.TRIG_CR)
        assert np.array_equal(a, b), ang


def test_extract_mode_none_is_canonical(orbref):
    import orbx_synth
    img = orbx_synth.gen_image(7, 320, 240)
    p = orbref.make_params(300, 1.2, 8, 20, 7)
    a = orbref.extract(img, p)
    b = orbref.extract(img, p, modes=(0, 0, 0))
    assert np.array_equal(a.keypoints, b.keypoints) and np.array_equal(a.descriptors, b.descriptors)
    c = orbref.extract(img, p, modes=(1, 0, 0))
    assert any(not np.array_equal(x, y) for x, y in zip(a.pyramid[1:], c.pyramid[1:]))
    assert np.array_equal(a.pyramid[0], c.pyramid[0])


# ---- GPU: each device mode against the oracle in the same mode ---------------------------------------------------
MODES = [(1, 0), (0, 1), (0, 2), (1, 1), (1, 2)]


@pytest.mark.gpu
@pytest.mark.parametrize("resize,blur", MODES)
@pytest.mark.parametrize("batch", [2, 10])
def test_gpu_modes_parity(orbref, cuda, resize, blur, batch):
    """KITTI frames through the batch entry point: 2 frames run the small-batch kernels (fused pyramid, one
    keypoint per describe wave), 10 the large-batch ones (one pyramid launch per level, four keypoints per
    wave).  Pyramid bytes, FAST candidates, keypoints and descriptors equal the oracle's in the same mode."""
    import orbx
    import orbx_synth
    from test_gpu_parity import _run_batch, assert_same_keypoints
    frames = orbx_synth.kitti_sequence(batch, start=40)
    ex = orbx.ORBextractor(2000, 1.2, 8, 20, 7)
    ex.set_cv_modes(resize, blur)
    p = orbref.make_params(2000, 1.2, 8, 20, 7)
    sizes = orbref.level_sizes(p, 1241, 376)
    _, _, _, _, klist, dlist = _run_batch(ex, frames, cuda)
    canon_diff = 0
    for f in range(batch):   # every frame: blur SSE2 changes ~0.07% of KITTI descriptors (its rounding ties)
        ref = orbref.extract(frames[f], p, modes=(resize, blur, 0))
        pyr = ex.debug_pyramid(f, sizes)
        for l, (a, b) in enumerate(zip(pyr, ref.pyramid)):
            bad = np.argwhere(a != b)
            assert bad.size == 0, "modes %s f%d pyramid level %d differs at %s" % ((resize, blur), f, l, bad[:3])
        for l in range(8):
            assert np.array_equal(ex.debug_candidates(f, l), orbref.level_candidates(ref.pyramid[l])), (f, l)
        assert_same_keypoints(klist[f], ref.keypoints, dlist[f], ref.descriptors, "modes %s f%d" % ((resize, blur), f))
        can = orbref.extract(frames[f], p, want_pyramid=False)
        canon_diff += len(can.keypoints) != len(ref.keypoints) or not np.array_equal(can.descriptors, ref.descriptors)
    if batch == 10 or (resize, blur) != (0, 1):
        assert canon_diff > 0   # the mode changed the output (else this test would not test it)


@pytest.mark.gpu
@pytest.mark.parametrize("resize,blur", MODES)
def test_gpu_modes_host_path(orbref, cuda, resize, blur):
    """The per-frame host entry point (orbx_extract, replayed as a hipGraph) in each mode, and a switch back to
    the canonical modes on the same handle (the graph is re-captured)."""
    import orbx
    import orbx_synth
    from test_gpu_parity import assert_same_keypoints
    img = orbx_synth.gen_image(77, 640, 480)
    ex = orbx.ORBextractor(1000, 1.2, 8, 20, 7)
    p = orbref.make_params(1000, 1.2, 8, 20, 7)
    kps, desc = ex(img)
    can = orbref.extract(img, p, want_pyramid=False)
    assert_same_keypoints(kps, can.keypoints, desc, can.descriptors, "canonical")
    ex.set_cv_modes(resize, blur)
    kps, desc = ex(img)
    ref = orbref.extract(img, p, modes=(resize, blur, 0))
    assert_same_keypoints(kps, ref.keypoints, desc, ref.descriptors, "modes %s" % ((resize, blur),))
    for l, (a, b) in enumerate(zip(ex.mvImagePyramid, ref.pyramid)):
        assert np.array_equal(a, b), l
    ex.set_cv_modes(0, 0)
    kps, desc = ex(img)
    assert_same_keypoints(kps, can.keypoints, desc, can.descriptors, "canonical again")


@pytest.mark.gpu
def test_set_cv_modes_rejects_unknown(cuda):
    import orbx
    ex = orbx.ORBextractor(500)
    with pytest.raises(orbx.OrbxError):
        ex.set_cv_modes(2, 0)
    with pytest.raises(orbx.OrbxError):
        ex.set_cv_modes(0, 3)
