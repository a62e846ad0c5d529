"""Vocabulary-node searches, SURVEY.md §8a rows a12/a13:
  SearchByBoW(KeyFrame*, Frame&)        src/ORBmatcher.cc:159-288
  SearchByBoW(KeyFrame*, KeyFrame*)     src/ORBmatcher.cc:590-723
  SearchForTriangulation                src/ORBmatcher.cc:725-891 (+ CheckDistEpipolarLine :140-157)

CPU: the C oracle against a pure-Python restatement written from the reference
text (small random cases with many distance ties, so first-min / last-<= and the
greedy skip are exercised), plus hand-built known answers.
GPU: liborbx (host path and batched device path) against the oracle on KITTI-like
frame pairs with FeatureVectors from a vocabulary trained with DBoW2's recipe
(orbx_synth.Vocabulary; ORBvoc.txt is absent).  Bar: match arrays
and nmatches identical.
"""
import numpy as np
import pytest

F32 = np.float32
KP = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"), ("response", "<f4"),
               ("octave", "<i4"), ("class_id", "<i4")])
SCALE = np.array([1.2 ** i for i in range(8)], np.float32)
SIGMA2 = SCALE * SCALE


# ---------------------------------------------------------------- Python restatement

def _ham(a, b):
    return int(np.unpackbits(np.bitwise_xor(a, b)).sum())


def _shared(fv1, fv2):
    n1, p1, i1 = fv1
    n2, p2, i2 = fv2
    d2 = {int(n): k for k, n in enumerate(n2)}
    for k, n in enumerate(n1):
        if int(n) in d2:
            j = d2[int(n)]
            yield list(i1[p1[k]:p1[k + 1]]), list(i2[p2[j]:p2[j + 1]])


def _bin(a1, a2):
    rot = F32(F32(a1) - F32(a2))
    if rot < 0.0:
        rot = F32(rot + F32(360.0))
    v = float(F32(rot * F32(F32(1.0) / F32(30))))
    b = int(np.floor(v + 0.5)) if v - np.floor(v) != 0.5 else int(np.floor(v)) + 1
    return 0 if b == 30 else b


def _rot_filter(bins, match):
    hist = [0] * 30
    for b in bins.values():
        hist[b] += 1
    m1 = m2 = m3 = 0
    i1 = i2 = i3 = -1
    for i, s in enumerate(hist):
        if s > m1:
            m3, m2, m1, i3, i2, i1 = m2, m1, s, i2, i1, i
        elif s > m2:
            m3, m2, i3, i2 = m2, s, i2, i
        elif s > m3:
            m3, i3 = s, i
    if F32(m2) < F32(0.1) * F32(m1):
        i2 = i3 = -1
    elif F32(m3) < F32(0.1) * F32(m1):
        i3 = -1
    for k, b in bins.items():
        if b not in (i1, i2, i3):
            match[k] = -1


def py_bow(mode, k1, d1, mp1, fv1, k2, d2, mp2, fv2, nnratio, check_ori):
    n_out = len(k2) if mode == "kf_f" else len(k1)
    match = np.full(n_out, -1, np.int32)
    matched2 = set()
    bins = {}
    for L1, L2 in _shared(fv1, fv2):
        for i1 in L1:
            if not mp1[i1]:
                continue
            b1, b2, bi = 256, 256, -1
            for i2 in L2:
                if mode == "kf_f" and match[i2] >= 0:
                    continue
                if mode == "kf_kf" and (i2 in matched2 or not mp2[i2]):
                    continue
                d = _ham(d1[i1], d2[i2])
                if d < b1:
                    b2, b1, bi = b1, d, i2
                elif d < b2:
                    b2 = d
            ok = (b1 <= 50) if mode == "kf_f" else (b1 < 50)
            if ok and F32(b1) < F32(nnratio) * F32(b2):
                if mode == "kf_f":
                    match[bi] = i1
                    slot = bi
                else:
                    match[i1] = bi
                    matched2.add(bi)
                    slot = i1
                if check_ori:
                    bins[slot] = _bin(k1["angle"][i1], k2["angle"][bi])
    if check_ori:
        _rot_filter(bins, match)
    return int((match >= 0).sum()), match


def _fma(a, b, c):
    return F32(np.float64(F32(a)) * np.float64(F32(b)) + np.float64(F32(c)))   # exact product, one rounding


def py_triang(k1, d1, mp1, ur1, fv1, k2, d2, mp2, ur2, fv2, F, ex, ey, only_stereo, check_ori):
    F = np.asarray(F, np.float32).reshape(9)
    match = np.full(len(k1), -1, np.int32)
    bins = {}
    for L1, L2 in _shared(fv1, fv2):
        for i1 in L1:
            if mp1[i1]:
                continue
            s1 = ur1[i1] >= 0
            if only_stereo and not s1:
                continue
            x1, y1 = F32(k1["x"][i1]), F32(k1["y"][i1])
            best, bi = 50, -1
            for i2 in L2:
                if mp2[i2]:
                    continue
                s2 = ur2[i2] >= 0
                if only_stereo and not s2:
                    continue
                d = _ham(d1[i1], d2[i2])
                if d > 50 or d > best:
                    continue
                x2, y2, o2 = F32(k2["x"][i2]), F32(k2["y"][i2]), int(k2["octave"][i2])
                if not s1 and not s2:
                    dx, dy = F32(F32(ex) - x2), F32(F32(ey) - y2)
                    if _fma(dx, dx, F32(dy * dy)) < F32(F32(100) * SCALE[o2]):
                        continue
                a = F32(_fma(x1, F[0], F32(y1 * F[3])) + F[6])
                b = F32(_fma(x1, F[1], F32(y1 * F[4])) + F[7])
                c = F32(_fma(y1, F[5], F32(x1 * F[2])) + F[8])
                num = F32(_fma(b, y2, F32(a * x2)) + c)
                den = _fma(a, a, F32(b * b))
                if den == 0:
                    continue
                dsq = F32(F32(num * num) / den)
                if float(dsq) < 3.84 * float(SIGMA2[o2]):
                    best, bi = d, i2
            if bi >= 0:
                match[i1] = bi
                if check_ori:
                    bins[i1] = _bin(k1["angle"][i1], k2["angle"][bi])
    if check_ori:
        _rot_filter(bins, match)
    return int((match >= 0).sum()), match


# ---------------------------------------------------------------- synthetic inputs

def _random_side(rng, n, nnodes, base=None, noise=6, width=640, height=480):
    """n keypoints/descriptors; with `base`, descriptors are noisy copies of base's (matches exist)."""
    k = np.zeros(n, KP)
    k["x"] = rng.uniform(20, width - 20, n).astype(np.float32)
    k["y"] = rng.uniform(20, height - 20, n).astype(np.float32)
    k["angle"] = rng.uniform(0, 360, n).astype(np.float32)
    k["octave"] = rng.integers(0, 8, n)
    k["class_id"] = -1
    if base is None:
        d = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    else:
        src = rng.integers(0, len(base), n)
        bits = np.unpackbits(base[src], axis=1)
        flips = rng.random(bits.shape) < noise / 256.0
        d = np.packbits(bits ^ flips, axis=1)
        d[::5] = base[src[::5]]                       # exact duplicates: distance ties
        k["angle"] = np.where(rng.random(n) < 0.8, F32(30.0), k["angle"]).astype(np.float32)
    node_of = rng.integers(0, nnodes, n) * 3 + 7      # sparse ascending ids
    ids = np.unique(node_of)
    order = np.argsort(node_of, kind="stable")
    ptr = np.concatenate([[0], np.cumsum([(node_of == i).sum() for i in ids])]).astype(np.int32)
    return k, d, (ids.astype(np.int32), ptr, order.astype(np.int32))


def _translation_F(dx, dy):
    # epipolar lines parallel to the image translation (dx, dy): F12 = [e]_x with e = (dx, dy, 0)
    return np.array([[0, 0, dy], [0, 0, -dx], [-dy, dx, 0]], np.float32)


# ---------------------------------------------------------------- CPU: oracle vs restatement

@pytest.mark.parametrize("seed", [0, 1, 2])
@pytest.mark.parametrize("ratio", [0.6, 0.75, 0.9])
def test_oracle_search_by_bow_matches_restatement(orbref, seed, ratio):
    rng = np.random.default_rng(seed)
    k1, d1, fv1 = _random_side(rng, 300, 12)
    k2, d2, fv2 = _random_side(rng, 280, 12, base=d1)
    mp1 = (rng.random(300) < 0.8).astype(np.uint8)
    mp2 = (rng.random(280) < 0.8).astype(np.uint8)
    for co in (True, False):
        n, m = orbref.search_by_bow_kf_f(k1, d1, mp1, fv1, k2, d2, fv2, ratio, co)
        pn, pm = py_bow("kf_f", k1, d1, mp1, fv1, k2, d2, None, fv2, ratio, co)
        assert n == pn and np.array_equal(m, pm) and n > 0
        n, m = orbref.search_by_bow_kf_kf(k1, d1, mp1, fv1, k2, d2, mp2, fv2, ratio, co)
        pn, pm = py_bow("kf_kf", k1, d1, mp1, fv1, k2, d2, mp2, fv2, ratio, co)
        assert n == pn and np.array_equal(m, pm) and n > 0


@pytest.mark.parametrize("seed", [0, 3])
@pytest.mark.parametrize("only_stereo", [False, True])
def test_oracle_triangulation_matches_restatement(orbref, seed, only_stereo):
    rng = np.random.default_rng(seed)
    k1, d1, fv1 = _random_side(rng, 300, 10)
    k2, d2, fv2 = _random_side(rng, 300, 10, base=d1)
    k2["x"], k2["y"] = k1["x"][:300] - 3, k1["y"][:300] - 1     # roughly on the epipolar lines
    mp1 = (rng.random(300) < 0.3).astype(np.uint8)
    mp2 = (rng.random(300) < 0.3).astype(np.uint8)
    ur1 = np.where(rng.random(300) < 0.5, F32(100), F32(-1)).astype(np.float32)
    ur2 = np.where(rng.random(300) < 0.5, F32(100), F32(-1)).astype(np.float32)
    F = _translation_F(-3, -1) + rng.normal(0, 1e-3, (3, 3)).astype(np.float32)
    for ex, ey in ((1e6, 1e6), (320.0, 240.0)):
        n, m = orbref.search_for_triangulation(k1, d1, mp1, ur1, fv1, k2, d2, mp2, ur2, fv2, F, ex, ey, SCALE,
                                               SIGMA2, only_stereo, True)
        pn, pm = py_triang(k1, d1, mp1, ur1, fv1, k2, d2, mp2, ur2, fv2, F, ex, ey, only_stereo, True)
        assert n == pn and np.array_equal(m, pm)


def _one_node(n):
    return (np.array([5], np.int32), np.array([0, n], np.int32), np.arange(n, dtype=np.int32))


def test_kat_greedy_skip_and_ratio(orbref):
    # KF features 0 and 1 are both closest to F feature 0: KF 0 takes it (first in node
    # order), KF 1 must then fall back to F feature 1 (already-matched targets skipped)
    base = np.zeros((3, 32), np.uint8)
    base[1, :2] = 0xFF          # 16 bits away from 0
    base[2, :] = 0xFF           # 256 away from 0
    kf = np.zeros(2, KP)
    f = np.zeros(3, KP)
    dkf = np.stack([base[0], base[0]])
    n, m = orbref.search_by_bow_kf_f(kf, dkf, np.ones(2, np.uint8), _one_node(2), f, base, _one_node(3), 0.9, False)
    assert n == 2 and list(m) == [0, 1, -1]
    # ratio test: best 0, second 16 passes at 0.9; best 16 vs second 256 passes; a 30/31 split fails
    d2 = np.zeros((2, 32), np.uint8)
    d2[0, :4] = 0xFF
    d2[0, 4] = 0xC0           # 34 bits
    d2[1, :4] = 0xFF
    d2[1, 4] = 0xE0           # 35 bits
    n, m = orbref.search_by_bow_kf_f(kf[:1], dkf[:1], np.ones(1, np.uint8), _one_node(1), f[:2], d2, _one_node(2),
                                     0.9, False)
    assert n == 0 and list(m) == [-1, -1]


def test_kat_triangulation_keeps_last_equal(orbref):
    # two identical candidates on the epipolar line: the reference's `dist > bestDist` skip keeps the LAST one
    d = np.zeros((3, 32), np.uint8)
    k1 = np.zeros(1, KP)
    k1["x"], k1["y"] = 100, 100
    k2 = np.zeros(3, KP)
    k2["x"] = [97, 79, 58]        # (100, 100) + t * (-3, -1), t = 1, 7, 14
    k2["y"] = [99, 93, 86]
    F = _translation_F(-3, -1)
    n, m = orbref.search_for_triangulation(k1, d[:1], np.zeros(1, np.uint8), np.full(1, -1, np.float32),
                                           _one_node(1), k2, d, np.zeros(3, np.uint8), np.full(3, -1, np.float32),
                                           _one_node(3), F, 1e6, 1e6, SCALE, SIGMA2, False, False)
    assert n == 1 and list(m) == [2]
    # epipole right next to candidate 2 -> it is rejected by the "too close to the epipole" test
    n, m = orbref.search_for_triangulation(k1, d[:1], np.zeros(1, np.uint8), np.full(1, -1, np.float32),
                                           _one_node(1), k2, d, np.zeros(3, np.uint8), np.full(3, -1, np.float32),
                                           _one_node(3), F, 60.0, 87.0, SCALE, SIGMA2, False, False)
    assert n == 1 and list(m) == [1]


def test_kat_no_shared_nodes(orbref):
    rng = np.random.default_rng(0)
    k1, d1, fv1 = _random_side(rng, 50, 4)
    k2, d2, _ = _random_side(rng, 50, 4, base=d1)
    fv2 = (np.array([1000], np.int32), np.array([0, 50], np.int32), np.arange(50, dtype=np.int32))
    n, m = orbref.search_by_bow_kf_f(k1, d1, np.ones(50, np.uint8), fv1, k2, d2, fv2, 0.9, True)
    assert n == 0 and np.all(m == -1)


# ---------------------------------------------------------------- GPU

def _kitti_sides(orbref, nfeat=2000, seed=0):
    import orbx_synth
    frames = orbx_synth.kitti_sequence(3, start=40)
    p = orbref.make_params(nfeat, 1.2, 8, 20, 7)
    r = [orbref.extract(f, p, want_pyramid=False) for f in frames]
    voc = orbx_synth.Vocabulary.train([x.descriptors for x in r], 10, 3, seed)
    rng = np.random.default_rng(seed)
    out = []
    for x in r:
        n = len(x.keypoints)
        out.append({"kps": x.keypoints, "desc": x.descriptors, "fv": voc.feature_vector(x.descriptors, 1),
                    "has_mp": (rng.random(n) < 0.7).astype(np.uint8),
                    "u_right": np.where(rng.random(n) < 0.3, F32(200), F32(-1)).astype(np.float32)})
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("ratio,co", [(0.7, True), (0.75, True), (0.9, False)])
def test_gpu_search_by_bow_parity(orbref, cuda, ratio, co):
    import orbx
    s = _kitti_sides(orbref)
    m = orbx.ORBmatcher(ratio, co)
    a, b = s[0], s[1]
    n, mm = m.SearchByBoW_KF_F((a["kps"], a["desc"], a["fv"], a["has_mp"]), (b["kps"], b["desc"], b["fv"]))
    wn, wm = orbref.search_by_bow_kf_f(a["kps"], a["desc"], a["has_mp"], a["fv"], b["kps"], b["desc"], b["fv"],
                                       ratio, co)
    assert n == wn and n > 50 and np.array_equal(mm, wm)
    n, mm = m.SearchByBoW_KF_KF((a["kps"], a["desc"], a["fv"], a["has_mp"]),
                                (b["kps"], b["desc"], b["fv"], b["has_mp"]))
    wn, wm = orbref.search_by_bow_kf_kf(a["kps"], a["desc"], a["has_mp"], a["fv"], b["kps"], b["desc"], b["has_mp"],
                                        b["fv"], ratio, co)
    assert n == wn and n > 50 and np.array_equal(mm, wm)


@pytest.mark.gpu
@pytest.mark.parametrize("only_stereo", [False, True])
def test_gpu_triangulation_parity(orbref, cuda, only_stereo):
    import orbx
    s = _kitti_sides(orbref, seed=1)
    a, b = s[0], s[1]
    mp1 = (a["has_mp"] == 0).astype(np.uint8)        # triangulation searches features WITHOUT MapPoints
    mp2 = (b["has_mp"] == 0).astype(np.uint8)
    F = _translation_F(-3, -1)
    m = orbx.ORBmatcher(0.6, True)
    for ex, ey in ((1e6, 1e6), (600.0, 180.0)):
        n, mm = m.SearchForTriangulation((a["kps"], a["desc"], a["fv"], mp1, a["u_right"]),
                                         (b["kps"], b["desc"], b["fv"], mp2, b["u_right"]), F, ex, ey, SCALE,
                                         SIGMA2, only_stereo)
        wn, wm = orbref.search_for_triangulation(a["kps"], a["desc"], mp1, a["u_right"], a["fv"], b["kps"],
                                                 b["desc"], mp2, b["u_right"], b["fv"], F, ex, ey, SCALE, SIGMA2,
                                                 only_stereo, True)
        assert n == wn and n > 5 and np.array_equal(mm, wm)


@pytest.mark.gpu
def test_gpu_bow_batch_device(orbref, cuda):
    import torch
    import orbx
    s = _kitti_sides(orbref, seed=2)
    pairs = [(0, 1), (1, 2), (0, 2)]
    F = _translation_F(-3, -1)
    for mode in (orbx.BOW_KF_F, orbx.BOW_KF_KF, orbx.TRIANGULATION):
        tps = [orbx.triang_params(F, 1e6, 1e6, SCALE, SIGMA2)] * len(pairs) if mode == orbx.TRIANGULATION else None
        side = lambda d: dict(d, has_mp=(d["has_mp"] == 0).astype(np.uint8)) if mode == orbx.TRIANGULATION else d
        bb = orbx.BowBatch(mode, [side(s[i]) for i, _ in pairs], [side(s[j]) for _, j in pairs], tps)
        match, nm = bb.run(0.75, True)
        torch.cuda.synchronize()
        match, nm = match.cpu().numpy(), nm.cpu().numpy()
        for p, (i, j) in enumerate(pairs):
            a, b = side(s[i]), side(s[j])
            if mode == orbx.BOW_KF_F:
                wn, wm = orbref.search_by_bow_kf_f(a["kps"], a["desc"], a["has_mp"], a["fv"], b["kps"], b["desc"],
                                                   b["fv"], 0.75, True)
            elif mode == orbx.BOW_KF_KF:
                wn, wm = orbref.search_by_bow_kf_kf(a["kps"], a["desc"], a["has_mp"], a["fv"], b["kps"], b["desc"],
                                                    b["has_mp"], b["fv"], 0.75, True)
            else:
                wn, wm = orbref.search_for_triangulation(a["kps"], a["desc"], a["has_mp"], a["u_right"], a["fv"],
                                                         b["kps"], b["desc"], b["has_mp"], b["u_right"], b["fv"], F,
                                                         1e6, 1e6, SCALE, SIGMA2, False, True)
            assert nm[p] == wn, (mode, p)
            assert np.array_equal(match[p, :len(wm)], wm), (mode, p)


@pytest.mark.gpu
def test_gpu_bow_large_nodes_and_edges(orbref, cuda):
    """Nodes with > 64 (and > 2x64) candidates take several passes; empty / disjoint vocabularies."""
    import orbx
    rng = np.random.default_rng(7)
    k1, d1, _ = _random_side(rng, 400, 1)
    k2, d2, _ = _random_side(rng, 400, 1, base=d1)
    fv_big = (np.array([3, 9], np.int32), np.array([0, 150, 400], np.int32), np.arange(400, dtype=np.int32))
    mp = np.ones(400, np.uint8)
    m = orbx.ORBmatcher(0.9, True)
    n, mm = m.SearchByBoW_KF_F((k1, d1, fv_big, mp), (k2, d2, fv_big))
    wn, wm = orbref.search_by_bow_kf_f(k1, d1, mp, fv_big, k2, d2, fv_big, 0.9, True)
    assert n == wn and n > 20 and np.array_equal(mm, wm)
    n, mm = m.SearchByBoW_KF_KF((k1, d1, fv_big, mp), (k2, d2, fv_big, mp))
    wn, wm = orbref.search_by_bow_kf_kf(k1, d1, mp, fv_big, k2, d2, mp, fv_big, 0.9, True)
    assert n == wn and np.array_equal(mm, wm)
    fv_other = (np.array([4], np.int32), np.array([0, 400], np.int32), np.arange(400, dtype=np.int32))
    n, mm = m.SearchByBoW_KF_F((k1, d1, fv_big, mp), (k2, d2, fv_other))
    assert n == 0 and np.all(mm == -1)
    empty = (np.zeros(0, np.int32), np.zeros(1, np.int32), np.zeros(0, np.int32))
    n, mm = m.SearchByBoW_KF_KF((k1, d1, empty, mp), (k2, d2, fv_big, mp))
    assert n == 0 and np.all(mm == -1)
