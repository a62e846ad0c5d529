"""The two capability limits this library has and the reference does not (INTEGRATION.md "Deviations"):

- image sizes whose sides' bit widths sum to 24 or less, e.g. up to 4096 x 4096 or 8192 x 2048 (keypoint
  coordinates packed in 24 bits on the device, split between x and y by the image's shape; the reference's
  ORBextractor::operator(), src/ORBextractor.cc:1248-1334, takes any size; round 5 capped both sides at 4096);
- at most ORBM_MAX_FEATURES (16384) keypoints per frame for the SearchByBoW / SearchForTriangulation
  searches and the projection searches, and ORBV_MAX_FEATURES (65536) for the vocabulary transform (per-frame
  state in a workgroup's LDS, or past 8192 features in global memory; src/ORBmatcher.cc:45-129, 159-288 and
  TemplatedVocabulary::transform have no limit).

Both sides of each limit are pinned: the largest accepted size runs (bit-exact against the oracle where an
extraction is involved), one past it returns ORBX_EINVAL instead of wrong results.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _check_extract(orbref, ex, img, nfeat, cuda, batch_frames=None):
    from test_gpu_parity import _run_batch, assert_same_keypoints
    p = orbref.make_params(nfeat, 1.2, 8, 20, 7)
    ref = orbref.extract(img, p, want_pyramid=False)
    kps, desc = ex(img)
    assert len(ref.keypoints) > 500
    assert_same_keypoints(kps, ref.keypoints, desc, ref.descriptors, "%dx%d host" % (img.shape[1], img.shape[0]))
    if batch_frames is not None:
        _, _, _, _, klist, dlist = _run_batch(ex, batch_frames, cuda)
        for f in range(len(batch_frames)):
            r = orbref.extract(batch_frames[f], p, want_pyramid=False)
            assert_same_keypoints(klist[f], r.keypoints, dlist[f], r.descriptors, "batch frame %d" % f)
    return ref


def test_image_size_limit(orbref, cuda):
    """sizes past the old 4096-px side run bit-exact (4097 x 600 and 8192 x 512, through the
    host call and a 10-frame batch: the large-batch kernels); the packed coordinates' 24 bits bound the size."""
    import ctypes
    import orbx
    import orbx_synth
    ex = orbx.ORBextractor(2000, 1.2, 8, 20, 7)
    # (a level taller than wide gives nIni = 0, where the reference divides by zero: -1 for any size)
    cap = lambda r, c: orbx.lib.orbx_capacity(ex._h, r, c)   # the raw C value (-1 = refused)
    assert cap(376, 4096) > 0 and cap(4096, 4096) > 0 and cap(376, 4097) > 0 and cap(2048, 8192) > 0
    assert cap(4097, 4097) == -1 and cap(2049, 8192) == -1 and cap(600, 16385) == -1
    for (w, h, seed) in ((4097, 600, 17), (8192, 512, 18)):
        img = orbx_synth.gen_image(seed, w, h)
        frames = np.stack([orbx_synth.gen_image(seed * 10 + f, w, h) for f in range(10)])
        ref = _check_extract(orbref, ex, img, 2000, cuda, frames)
        assert ref.keypoints["x"].max() > 0.97 * w   # keypoints reach past x = 4096 - 19
    tall = np.zeros((300, 4097), np.uint8)   # empty but valid: 0 keypoints
    kbuf = np.zeros((64, 7), np.int32)
    dbuf = np.zeros((64, 32), np.uint8)
    n = ctypes.c_int(-1)
    big = np.zeros((4097, 4097), np.uint8)
    rc = orbx.lib.orbx_extract(ex._h, big.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), 4097, 4097, 4097,
                               kbuf.ctypes.data_as(ctypes.c_void_p), 64,
                               dbuf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), ctypes.byref(n))
    assert rc == orbx.EINVAL and n.value == -1
    rc = orbx.lib.orbx_extract(ex._h, tall.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), 300, 4097, 4097,
                               kbuf.ctypes.data_as(ctypes.c_void_p), 64,
                               dbuf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), ctypes.byref(n))
    assert rc == orbx.OK and n.value == 0


def _tiny_vocabulary():
    import orbx
    rng = np.random.default_rng(3)
    parent = np.array([0, 0, 0], np.int32)
    is_leaf = np.array([0, 1, 1], np.uint8)
    desc = rng.integers(0, 256, (3, 32), dtype=np.uint8)
    return orbx.ORBVocabulary.from_arrays(2, 1, parent, is_leaf, desc, np.ones(3))


def test_vocabulary_transform_limit(orbref, cuda):
    """Past the LDS sort (8192 features) the transform sorts in global memory: 16384 and 20000 descriptors
    bit-exact against the oracle; ORBV_MAX_FEATURES + 1 refused."""
    import orbx
    import test_voc
    v, imgs = test_voc._vocab(5, 8, 3, 4, 200)
    gv = orbx.ORBVocabulary.from_arrays(v.k, v.L, v.parent, v.is_leaf, v.desc, v.weight, v.scoring, v.weighting)
    rng = np.random.default_rng(4)
    base = np.concatenate(imgs)
    for n in (8192, 16384, 20000):
        src = rng.integers(0, len(base), n)
        q = np.packbits(np.unpackbits(base[src], axis=1) ^ (rng.random((n, 256)) < 0.03), axis=1)
        for levelsup in (1, 3):
            test_voc._same(gv.transform(q, levelsup), orbref.voc_transform(v, q, levelsup))
    voc = _tiny_vocabulary()
    d = np.random.default_rng(4).integers(0, 256, (orbx.ORBV_MAX_FEATURES + 1, 32), dtype=np.uint8)
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


def test_bow_search_limit(orbref, cuda):
    """A view of ORBM_MAX_FEATURES features, all in one vocabulary node (the per-wave "matched" bitmap spans
    all of them), for SearchByBoW(KF, F) and (KF, KF): bit-exact against the oracle; one more refused."""
    import orbx
    import test_bow
    N = orbx.ORBM_MAX_FEATURES
    rng = np.random.default_rng(11)
    k1, d1, _ = test_bow._random_side(rng, 300, 1)
    k2, d2, _ = test_bow._random_side(rng, N, 1)   # unrelated descriptors, and one noisy copy of each view1 one
    at = rng.choice(N, 300, replace=False)
    d2[at] = np.packbits(np.unpackbits(d1, axis=1) ^ (rng.random((300, 256)) < 0.04), axis=1)
    k2["angle"][at] = k1["angle"] + np.float32(30.0)
    fv1, fv2 = _one_node_fv(300), _one_node_fv(N)
    mp1 = (rng.random(300) < 0.9).astype(np.uint8)
    mp2 = (rng.random(N) < 0.9).astype(np.uint8)
    m = orbx.ORBmatcher(0.75, True)
    n, mm = m.SearchByBoW_KF_F((k1, d1, fv1, mp1), (k2, d2, fv2))
    wn, wm = orbref.search_by_bow_kf_f(k1, d1, mp1, fv1, k2, d2, fv2, 0.75, True)
    assert n == wn and n > 50 and np.array_equal(mm, wm)
    n, mm = m.SearchByBoW_KF_KF((k1, d1, fv1, mp1), (k2, d2, fv2, mp2))
    wn, wm = orbref.search_by_bow_kf_kf(k1, d1, mp1, fv1, k2, d2, mp2, fv2, 0.75, True)
    assert n == wn and n > 50 and np.array_equal(mm, wm)
    k, d = _keypoints(N + 1, 5)
    with pytest.raises(orbx.OrbxError) as e:
        m.SearchByBoW_KF_F((k1, d1, fv1, mp1), (k, d, _one_node_fv(N + 1)))
    assert e.value.code == orbx.EINVAL


def _one_node_fv(n):
    return (np.array([7], np.int32), np.array([0, n], np.int32), np.arange(n, dtype=np.int32))


def test_projection_search_large_frames(orbref, cuda):
    """SearchByProjection(F, local MapPoints) and the pose-projection searches on frames of ORBM_MAX_FEATURES
    keypoints (past 8192 the replay keeps its MapPoint-per-feature array in the output row in global memory):
    bit-exact against the oracle."""
    import orbx
    import test_proj
    import test_pose_search as tps
    N = orbx.ORBM_MAX_FEATURES
    kps, desc, ur, cl, grid, pts, pdesc = test_proj.scene(7, n_kp=N, n_mp=24000, W=1241, H=376)
    n, mt = orbx.ORBmatcher(0.8).SearchByProjection(kps, desc, ur, cl, grid, test_proj.SCALE, pts, pdesc, 3.0)
    wn, wm = orbref.search_by_projection(kps, desc, ur, cl, grid, test_proj.SCALE, pts, pdesc, 3.0, 0.8)
    assert n == wn and n > 1000 and np.array_equal(mt, wm)
    for mode in ("last_frame", "sim3"):
        sc = tps.scene(3, n_kp=N, n_mp=24000, sim3_scale=1.7 if mode == "sim3" else 1.0)
        pp = tps.params(**tps.CASES[mode][0])
        kps, desc, ur, cl, pose, Scw, pts, pdesc = sc
        ps = Scw.ravel() if mode == "sim3" else pose
        mtc = orbx.ORBmatcher(0.9, bool(pp.check_ori))
        n, mt = mtc.project_search(tps.MODE_ID[mode], kps, desc, ur, cl, ps, pts, pdesc,
                                   orbx.PoseParams.from_buffer_copy(pp))
        wn, wm = tps.run_oracle(mode, sc, pp)
        assert n == wn and n > 100 and np.array_equal(mt, wm), mode


def test_projection_search_limits(cuda):
    import orbx
    m = orbx.ORBmatcher(0.8, True)
    N = orbx.ORBM_MAX_FEATURES
    k, d = _keypoints(N + 1, 6)
    scale = [1.2 ** i for i in range(8)]
    grid = (0.0, 0.0, np.float32(64) / np.float32(1241), np.float32(48) / np.float32(376))
    pts = np.zeros(0, orbx.PROJ_POINT_DTYPE)
    for n in (N, N + 1):
        args = (k[:n], d[:n], np.full(n, -1, np.float32), np.zeros(n, np.uint8), grid, scale, pts,
                np.zeros((0, 32), np.uint8))
        if n == N:
            assert m.SearchByProjection(*args)[0] == 0
        else:
            with pytest.raises(orbx.OrbxError) as e:
                m.SearchByProjection(*args)
            assert e.value.code == orbx.EINVAL
    prm = orbx.pose_params((718.856, 718.856, 607.19, 185.22), (0, 1241, 0, 376), scale)
    pose = np.hstack([np.eye(3), np.zeros((3, 1))]).astype(np.float32)
    mp = np.zeros(0, orbx.MAP_POINT_DTYPE)
    for n in (N, N + 1):
        args = (orbx.PROJ_SIM3, k[:n], d[:n], np.full(n, -1, np.float32), np.zeros(n, np.uint8), pose, mp,
                np.zeros((0, 32), np.uint8), prm)
        if n == N:
            assert m.project_search(*args)[0] == 0
        else:
            with pytest.raises(orbx.OrbxError) as e:
                m.project_search(*args)
            assert e.value.code == orbx.EINVAL
