"""The two capability limits this library has and the reference does not (INTEGRATION.md "Deviations"):

- image sides up to 4096 pixels (keypoint coordinates packed in 12 bits on the device; the reference's
  ORBextractor::operator(), src/ORBextractor.cc:1248-1334, takes any size);
- at most 8192 keypoints per frame for the vocabulary transform, the SearchByBoW / SearchForTriangulation
  searches and the projection searches (LDS-resident per-frame sorts; src/ORBmatcher.cc:45-129, 159-288 and
  TemplatedVocabulary::transform have no limit).

Both sides of each limit are pinned: the largest accepted size runs (bit-exact against the oracle where an
extraction is involved), one past it returns ORBX_EINVAL instead of wrong results.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_image_side_limit(orbref, cuda):
    import orbx
    import orbx_synth
    ex = orbx.ORBextractor(1000, 1.2, 8, 20, 7)
    # (a level taller than wide gives nIni = 0, where the reference divides by zero: -1 for any size)
    cap = lambda r, c: orbx.lib.orbx_capacity(ex._h, r, c)   # the raw C value (-1 = refused)
    assert cap(376, 4096) > 0 and cap(4096, 4096) > 0
    assert cap(376, 4097) == -1 and cap(4097, 4097) == -1
    img = orbx_synth.gen_image(17, 4096, 300)
    kps, desc = ex(img)
    ref = orbref.extract(img, orbref.make_params(1000, 1.2, 8, 20, 7), want_pyramid=False)
    assert len(kps) == len(ref.keypoints) > 500
    for f in ("x", "y", "size", "response", "octave"):
        assert np.array_equal(kps[f], ref.keypoints[f]), f
    assert np.array_equal(desc, ref.descriptors)
    import ctypes
    wide = np.zeros((300, 4097), np.uint8)
    kbuf = np.zeros((64, 7), np.int32)
    dbuf = np.zeros((64, 32), np.uint8)
    n = ctypes.c_int(-1)
    rc = orbx.lib.orbx_extract(ex._h, wide.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), 300, 4097, 4097,
                               kbuf.ctypes.data_as(ctypes.c_void_p), 64,
                               dbuf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), ctypes.byref(n))
    assert rc == orbx.EINVAL and n.value == -1


def _tiny_vocabulary():
    import orbx
    rng = np.random.default_rng(3)
    parent = np.array([0, 0, 0], np.int32)
    is_leaf = np.array([0, 1, 1], np.uint8)
    desc = rng.integers(0, 256, (3, 32), dtype=np.uint8)
    return orbx.ORBVocabulary.from_arrays(2, 1, parent, is_leaf, desc, np.ones(3))


def test_vocabulary_transform_limit(cuda):
    import orbx
    voc = _tiny_vocabulary()
    d = np.random.default_rng(4).integers(0, 256, (8193, 32), dtype=np.uint8)
    words, weights, (fn, fp, fi) = voc.transform(d[:8192])
    assert fp[-1] == 8192 and np.isclose(weights.sum(), 1.0)
    with pytest.raises(orbx.OrbxError) as e:
        voc.transform(d)
    assert e.value.code == orbx.EINVAL


def _keypoints(n, seed):
    import orbx
    rng = np.random.default_rng(seed)
    k = np.zeros(n, orbx.KEYPOINT_DTYPE)
    k["x"] = rng.uniform(0, 1241, n)
    k["y"] = rng.uniform(0, 376, n)
    k["angle"] = rng.uniform(0, 360, n)
    k["size"], k["response"], k["octave"], k["class_id"] = 31.0, 1.0, 0, -1
    return k, rng.integers(0, 256, (n, 32), dtype=np.uint8)


def test_bow_search_limit(cuda):
    import orbx
    m = orbx.ORBmatcher(0.75, True)
    k, d = _keypoints(8193, 5)
    one_node = lambda n: (np.array([7], np.int32), np.array([0, n], np.int32), np.arange(n, dtype=np.int32))
    kf = (k[:100], d[:100], one_node(100), np.ones(100, np.uint8))
    n, match = m.SearchByBoW_KF_F(kf, (k[:8192], d[:8192], one_node(8192)))
    assert len(match) == 8192 and n >= 0
    with pytest.raises(orbx.OrbxError) as e:
        m.SearchByBoW_KF_F(kf, (k, d, one_node(8193)))
    assert e.value.code == orbx.EINVAL


def test_projection_search_limits(cuda):
    import orbx
    m = orbx.ORBmatcher(0.8, True)
    k, d = _keypoints(8193, 6)
    scale = [1.2 ** i for i in range(8)]
    grid = (0.0, 0.0, np.float32(64) / np.float32(1241), np.float32(48) / np.float32(376))
    pts = np.zeros(0, orbx.PROJ_POINT_DTYPE)
    for n in (8192, 8193):
        args = (k[:n], d[:n], np.full(n, -1, np.float32), np.zeros(n, np.uint8), grid, scale, pts,
                np.zeros((0, 32), np.uint8))
        if n == 8192:
            assert m.SearchByProjection(*args)[0] == 0
        else:
            with pytest.raises(orbx.OrbxError) as e:
                m.SearchByProjection(*args)
            assert e.value.code == orbx.EINVAL
    prm = orbx.pose_params((718.856, 718.856, 607.19, 185.22), (0, 1241, 0, 376), scale)
    pose = np.hstack([np.eye(3), np.zeros((3, 1))]).astype(np.float32)
    mp = np.zeros(0, orbx.MAP_POINT_DTYPE)
    for n in (8192, 8193):
        args = (orbx.PROJ_SIM3, k[:n], d[:n], np.full(n, -1, np.float32), np.zeros(n, np.uint8), pose, mp,
                np.zeros((0, 32), np.uint8), prm)
        if n == 8192:
            assert m.project_search(*args)[0] == 0
        else:
            with pytest.raises(orbx.OrbxError) as e:
                m.project_search(*args)
            assert e.value.code == orbx.EINVAL
