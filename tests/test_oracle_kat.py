"""Known-answer tests that pin the CPU oracle (oracle/orbref.c).

The reference ships no tests or golden vectors and cannot be
built here (no OpenCV), so the oracle is pinned by:
  * every constant table / geometry figure the reference's code determines
    (per-level budgets, umax, scale factors, level sizes, cell grids, quadtree
    roots, patch sizes) — values cross-checked with SURVEY.md Appendix B;
  * hand-derived answers for each OpenCV primitive (FAST ring, resize ramp,
    Gaussian impulse, fastAtan2 axes, BRIEF at angle 0, Hamming);
  * an independent pure-Python restatement of DistributeOctTree
    (src/ORBextractor.cc:644-907) on small random sets;
  * hand-built SearchForInitialization cases (eviction, ratio test, window).
"""
import math

import numpy as np
import pytest


# ---------------------------------------------------------------- a1 tables
@pytest.mark.parametrize("nfeat,expect", [
    (2000, [434, 362, 302, 251, 209, 175, 145, 122]),
    (1000, [217, 181, 151, 126, 105, 87, 73, 60]),
    (1200, [261, 217, 181, 151, 126, 105, 87, 72]),
    (4000, [869, 724, 603, 503, 419, 349, 291, 242]),
])
def test_features_per_level(orbref, nfeat, expect):
    t = orbref.tables(orbref.make_params(nfeat))
    assert list(t.nfeat_level)[:8] == expect
    assert sum(expect) == nfeat


def test_umax_and_scales(orbref):
    t = orbref.tables(orbref.make_params(2000))
    assert list(t.umax) == [15, 15, 15, 15, 14, 14, 14, 13, 13, 12, 11, 10, 9, 8, 6, 3]
    # disc of the intensity centroid: 749 pixels (SURVEY a7 quotes 789; the umax table gives 749)
    assert 31 + 2 * sum(2 * u + 1 for u in list(t.umax)[1:16]) == 749
    want = [1.0, 1.2000000477, 1.4400000572, 1.7280001640, 2.0736002922, 2.4883203506, 2.9859845638, 3.5831816196]
    assert np.allclose(list(t.scale)[:8], want, rtol=0, atol=5e-10)
    assert [int(31 * np.float32(s)) for s in list(t.scale)[:8]] == [31, 37, 44, 53, 64, 77, 92, 111]
    for l in range(8):
        assert t.sigma2[l] == np.float32(np.float32(t.scale[l]) * np.float32(t.scale[l]))
        assert t.inv_scale[l] == np.float32(np.float32(1.0) / np.float32(t.scale[l]))


@pytest.mark.parametrize("W,H,sizes,px,nini,cells", [
    (1241, 376, [(1241, 376), (1034, 313), (862, 261), (718, 218), (598, 181), (499, 151), (416, 126), (346, 105)],
     1444097, 4, 1220),
    (640, 480, [(640, 480), (533, 400), (444, 333), (370, 278), (309, 231), (257, 193), (214, 161), (179, 134)],
     950532, 1, 815),
    (752, 480, [(752, 480), (627, 400), (522, 333), (435, 278), (363, 231), (302, 193), (252, 161), (210, 134)],
     1117367, 2, 982),
    (1920, 1080, [(1920, 1080), (1600, 900), (1333, 750), (1111, 625), (926, 521), (772, 434), (643, 362),
                  (536, 301)], 6419321, 2, 6257),
])
def test_geometry_appendix_b(orbref, W, H, sizes, px, nini, cells):
    p = orbref.make_params(1000)
    got = orbref.level_sizes(p, W, H)
    assert got == sizes
    assert sum(w * h for w, h in got) == px
    assert round(np.float32(W - 32) / np.float32(H - 32)) == nini
    assert sum(orbref.level_cells(w, h) for w, h in got) == cells


def test_kitti_level0_cells(orbref):
    # level 0 of KITTI scans 39 of 40 columns x 11 rows of 31x32 cells (Appendix C.1)
    assert orbref.level_cells(1241, 376) == 429


# ---------------------------------------------------------------- fastAtan2
def test_fast_atan2_axes_and_accuracy(orbref):
    assert orbref.fast_atan2(0.0, 1.0) == 0.0
    assert orbref.fast_atan2(1.0, 0.0) == 90.0
    assert orbref.fast_atan2(0.0, -1.0) == 180.0
    assert orbref.fast_atan2(-1.0, 0.0) == 270.0
    assert orbref.fast_atan2(0.0, 0.0) == 0.0
    rng = np.random.default_rng(0)
    for y, x in rng.integers(-5000, 5000, size=(2000, 2)):
        a = orbref.fast_atan2(float(y), float(x))
        ref = math.degrees(math.atan2(y, x)) % 360.0
        d = abs(a - ref)
        assert 0.0 <= a < 360.0 + 1e-3 and min(d, 360 - d) < 0.01


# ---------------------------------------------------------------- FAST
def _ring_image(v, darker_arc, delta, size=11):
    img = np.full((size, size), v, np.uint8)
    ring = [(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3), (0, -3), (-1, -3), (-2, -2),
            (-3, -1), (-3, 0), (-3, 1), (-2, 2), (-1, 3)]
    c = size // 2
    for k in darker_arc:
        x, y = ring[k % 16]
        img[c + y, c + x] = v - delta
    return img


@pytest.mark.parametrize("arc,expect", [(range(0, 9), True), (range(5, 14), True), (range(0, 8), False),
                                        (range(12, 21), True)])
def test_fast_ring(orbref, arc, expect):
    img = _ring_image(120, arc, 30)
    kps = orbref.fast(img, 20)
    hit = [k for k in kps if k[0] == 5 and k[1] == 5]
    assert bool(hit) == expect
    if expect:
        assert hit[0][2] == 29   # cornerScore = arc min of |v - x| (30) - 1


def test_fast_brighter_and_threshold(orbref):
    img = 255 - _ring_image(120, range(3, 12), 40)   # brighter arc of +40 around 135
    kps = orbref.fast(img, 20)
    assert any(k[0] == 5 and k[1] == 5 and k[2] == 39 for k in kps)
    assert not any(k[0] == 5 and k[1] == 5 for k in orbref.fast(img, 40))   # needs > t strictly


def test_fast_nms_plateau_removes_both(orbref):
    # two equal-score corners side by side: strict '>' NMS keeps neither
    img = np.full((12, 13), 100, np.uint8)
    img[3:9, 3:10] = 100
    img[6, 6] = img[6, 7] = 200
    kps = orbref.fast(img, 20)
    assert not any(k[1] == 6 and k[0] in (6, 7) for k in kps)


# ---------------------------------------------------------------- resize
def test_resize_ramp_and_constant(orbref):
    src = np.tile((16 * np.arange(8)).astype(np.uint8), (8, 1))
    out = orbref.resize_linear(src, 4, 4)
    assert np.array_equal(out[0], [8, 40, 72, 104])
    c = np.full((376, 1241), 173, np.uint8)
    assert np.all(orbref.resize_linear(c, 1034, 313) == 173)


# ---------------------------------------------------------------- blur
def test_blur_kernel_integer_path(orbref):
    c = np.full((20, 20), 100, np.uint8)
    # kernel [18 34 49 55 49 34 18] sums to 257: (100*257^2 + 2^15) >> 16 = 101
    assert np.all(orbref.gaussian_blur7(c) == 101)
    imp = np.zeros((15, 15), np.uint8)
    imp[7, 7] = 255
    b = orbref.gaussian_blur7(imp)
    k = np.array([18, 34, 49, 55, 49, 34, 18])
    want = (255 * np.outer(k, k) + (1 << 15)) >> 16
    assert np.array_equal(b[4:11, 4:11], want)
    assert b.sum() == want.sum()
    # reflect-101 at the border: an impulse in the corner reflects inward
    imp2 = np.zeros((15, 15), np.uint8)
    imp2[0, 0] = 255
    b2 = orbref.gaussian_blur7(imp2)
    assert b2[0, 0] == (255 * 55 * 55 + (1 << 15)) >> 16
    assert b2[1, 0] == (255 * 49 * 55 + (1 << 15)) >> 16


# ---------------------------------------------------------------- BRIEF
def _pattern():
    import os
    p = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "orb-slam-_amd", "csrc",
                     "orb_pattern.inc")
    txt = "".join(l for l in open(p) if not l.lstrip().startswith(("/*", "*")))
    v = np.array([int(x) for x in txt.replace("\n", "").split(",") if x.strip()], np.int32)
    return v.reshape(256, 4)


def test_brief_angle_zero(orbref):
    rng = np.random.default_rng(3)
    blur = rng.integers(0, 256, size=(60, 60), dtype=np.uint8)
    d = orbref.brief(blur, 30.0, 29.0, 0.0)
    pat = _pattern()
    bits = (blur[29 + pat[:, 1], 30 + pat[:, 0]] < blur[29 + pat[:, 3], 30 + pat[:, 2]]).astype(np.uint8)
    assert np.array_equal(np.packbits(bits, bitorder="little"), d)


def test_brief_rotation_90(orbref):
    # angle 90: cos = -4.37e-8, sin = 1 -> sample (x', y') = (round(-y), round(x))
    rng = np.random.default_rng(4)
    blur = rng.integers(0, 256, size=(60, 60), dtype=np.uint8)
    d = orbref.brief(blur, 30.0, 30.0, 90.0)
    pat = _pattern()
    v1 = blur[30 + pat[:, 0], 30 - pat[:, 1]]
    v2 = blur[30 + pat[:, 2], 30 - pat[:, 3]]
    assert np.array_equal(np.packbits((v1 < v2).astype(np.uint8), bitorder="little"), d)


# ---------------------------------------------------------------- Hamming
def test_descriptor_distance(orbref):
    z = np.zeros(32, np.uint8)
    o = np.full(32, 255, np.uint8)
    assert orbref.descriptor_distance(z, o) == 256
    assert orbref.descriptor_distance(z, z) == 0
    one = z.copy()
    one[17] = 8
    assert orbref.descriptor_distance(z, one) == 1
    rng = np.random.default_rng(5)
    for _ in range(50):
        a, b = rng.integers(0, 256, size=(2, 32), dtype=np.uint8)
        assert orbref.descriptor_distance(a, b) == int(np.unpackbits(a ^ b).sum())


# ---------------------------------------------------------------- DistributeOctTree
def py_distribute(xys, minX, maxX, minY, maxY, N):
    """Independent restatement of src/ORBextractor.cc:644-907 with std::list
    emulated by a python list; size ties broken by creation order."""
    seq = [0]

    class Node:
        def __init__(self, x0, x1, y0, y1, keys):
            self.x0, self.x1, self.y0, self.y1, self.keys = x0, x1, y0, y1, keys
            self.no_more = len(keys) == 1
            self.seq = None

    def divide(n):
        hx = int(math.ceil(np.float32(n.x1 - n.x0) / np.float32(2)))
        hy = int(math.ceil(np.float32(n.y1 - n.y0) / np.float32(2)))
        mx, my = n.x0 + hx, n.y0 + hy
        ch = [Node(n.x0, mx, n.y0, my, []), Node(mx, n.x1, n.y0, my, []), Node(n.x0, mx, my, n.y1, []),
              Node(mx, n.x1, my, n.y1, [])]
        for k in n.keys:
            x, y = xys[k][0], xys[k][1]
            q = (0 if y < my else 2) if x < mx else (1 if y < my else 3)
            ch[q].keys.append(k)
        for c in ch:
            c.no_more = len(c.keys) == 1
        return ch

    nIni = int(round(float(np.float32(maxX - minX) / np.float32(maxY - minY))))
    hX = np.float32(np.float32(maxX - minX) / np.float32(nIni))
    nodes = [Node(int(np.float32(hX * np.float32(i))), int(np.float32(hX * np.float32(i + 1))), 0, maxY - minY, [])
             for i in range(nIni)]
    for k, (x, y, s) in enumerate(xys):
        nodes[min(int(np.float32(x) / hX), nIni - 1)].keys.append(k)
    lst = [n for n in nodes if n.keys]
    for n in lst:
        n.no_more = len(n.keys) == 1

    def push_front(c):
        c.seq = seq[0]
        seq[0] += 1
        lst.insert(0, c)

    finish = False
    while not finish:
        prev = len(lst)
        vec = []
        n_exp = 0
        for n in [m for m in lst if not m.no_more]:
            for c in divide(n):
                if c.keys:
                    push_front(c)
                    if len(c.keys) > 1:
                        n_exp += 1
                        vec.append(c)
            lst.remove(n)
        if len(lst) >= N or len(lst) == prev:
            finish = True
        elif len(lst) + 3 * n_exp > N:
            while not finish:
                prev = len(lst)
                pv = sorted(vec, key=lambda c: (len(c.keys), c.seq))
                vec = []
                for n in reversed(pv):
                    for c in divide(n):
                        if c.keys:
                            push_front(c)
                            if len(c.keys) > 1:
                                vec.append(c)
                    lst.remove(n)
                    if len(lst) >= N:
                        break
                if len(lst) >= N or len(lst) == prev:
                    finish = True
    out = []
    for n in lst:
        best = n.keys[0]
        for k in n.keys[1:]:
            if xys[k][2] > xys[best][2]:
                best = k
        out.append(best)
    return out


@pytest.mark.parametrize("seed,n,N,w,h", [(0, 40, 10, 200, 120), (1, 300, 50, 400, 150), (2, 1000, 120, 500, 160),
                                          (3, 60, 100, 300, 100), (4, 500, 37, 640, 480), (5, 2000, 434, 1241, 376)])
def test_distribute_matches_python_restatement(orbref, seed, n, N, w, h):
    rng = np.random.default_rng(seed)
    qw, qh = w - 32, h - 32
    pts = set()
    while len(pts) < n:
        pts.add((int(rng.integers(3, qw - 4)), int(rng.integers(3, qh - 4))))
    pts = sorted(pts, key=lambda p: (p[1], p[0]))
    xys = np.array([(x, y, int(rng.integers(7, 12))) for x, y in pts], np.int32)   # many score ties
    got = orbref.distribute(xys, w, h, N)
    want = py_distribute([tuple(r) for r in xys], 16, w - 16, 16, h - 16, N)
    assert list(got) == want


def test_distribute_keeps_all_when_budget_exceeds(orbref):
    xys = np.array([(10, 10, 9), (100, 50, 8), (200, 80, 7)], np.int32)
    got = orbref.distribute(xys, 300, 150, 50)
    assert sorted(got) == [0, 1, 2]


def test_distribute_first_max_wins(orbref):
    # two keypoints that end in one node (N=1 stops after the first split round) with equal score
    xys = np.array([(10, 10, 9), (11, 10, 9)], np.int32)
    assert list(orbref.distribute(xys, 100, 100, 1)) == [0]


# ---------------------------------------------------------------- SearchForInitialization
def _kp(pts, angles=None):
    from orbref import KEYPOINT_DTYPE
    k = np.zeros(len(pts), KEYPOINT_DTYPE)
    for i, (x, y, o) in enumerate(pts):
        k[i] = (x, y, 31, 0.0 if angles is None else angles[i], 20, o, -1)
    return k


def test_search_init_window_and_skip(orbref):
    k1 = _kp([(100, 100, 0), (110, 100, 0), (400, 300, 1)])
    k2 = _kp([(101, 100, 0), (300, 300, 0)])
    d1 = np.zeros((3, 32), np.uint8)
    d1[1, 0] = 1
    d2 = np.zeros((2, 32), np.uint8)
    d2[1] = 255
    n, m12, prev = orbref.search_for_initialization(k1, d1, k2, d2, 640, 480)
    # A -> a (dist 0); B's only window candidate a is already matched at 0 <= 1: skipped
    assert n == 1 and list(m12) == [0, -1, -1]
    assert tuple(prev[0]) == (101.0, 100.0)


def test_search_init_eviction_and_ratio(orbref):
    k1 = _kp([(100, 100, 0), (105, 100, 0)])
    k2 = _kp([(102, 100, 0), (150, 120, 0)])
    d1 = np.zeros((2, 32), np.uint8)
    d1[0, :1] = 0x1F          # A: dist 5 to a
    d1[1, :1] = 0x07          # B: dist 3 to a (evicts A)
    d2 = np.zeros((2, 32), np.uint8)
    d2[1, :8] = 0xFF          # b far from both (64 bits)
    n, m12, _ = orbref.search_for_initialization(k1, d1, k2, d2, 640, 480)
    assert n == 1 and list(m12) == [-1, 0]
    # ratio test: best 10, second 11 -> 10 < 0.9*11 fails
    d1 = np.zeros((1, 32), np.uint8)
    d2 = np.zeros((2, 32), np.uint8)
    d2[0, :2] = [0xFF, 0x03]
    d2[1, :2] = [0xFF, 0x07]
    n, m12, _ = orbref.search_for_initialization(k1[:1], d1, k2, d2, 640, 480)
    assert n == 0 and list(m12) == [-1]


def test_search_init_window_follows_prev_matched(orbref):
    """The window is centred on vbPrevMatched[i1], not on F1's keypoint (src/ORBmatcher.cc:456-460),
    and a match moves vbPrevMatched[i1] to F2's keypoint (:580-584)."""
    k1 = _kp([(100, 100, 0)])
    k2 = _kp([(101, 100, 0), (402, 301, 0)])
    d1 = np.zeros((1, 32), np.uint8)
    d2 = np.zeros((2, 32), np.uint8)
    d2[0, 0] = 0x01                                   # a: distance 1 (near F1's keypoint)
    d2[1, 0] = 0x03                                   # b: distance 2 (near vbPrevMatched)
    n, m12, prev = orbref.search_for_initialization(k1, d1, k2, d2, 640, 480)
    assert n == 1 and list(m12) == [0] and tuple(prev[0]) == (101.0, 100.0)
    n, m12, prev = orbref.search_for_initialization(k1, d1, k2, d2, 640, 480,
                                                    prev_xy=np.array([[400, 300]], np.float32))
    assert n == 1 and list(m12) == [1] and tuple(prev[0]) == (402.0, 301.0)
    # no match: vbPrevMatched keeps its value
    n, m12, prev = orbref.search_for_initialization(k1, d1, k2, d2, 640, 480,
                                                    prev_xy=np.array([[250, 200]], np.float32))
    assert n == 0 and list(m12) == [-1] and tuple(prev[0]) == (250.0, 200.0)


def test_search_init_frame_bounds(orbref):
    """Frame::PosInGrid drops keypoints outside the grid (src/Frame.cc:504-518): an undistorted
    keypoint at x = -20 is unreachable with bounds 0..640 but found with the undistorted corners'
    bounds -30..650 (ComputeImageBounds, src/Frame.cc:563-621)."""
    k1 = _kp([(5, 100, 0)])
    k2 = _kp([(-20, 100, 0)])
    d = np.zeros((1, 32), np.uint8)
    n, m12, _ = orbref.search_for_initialization(k1, d, k2, d, 640, 480)
    assert n == 0 and list(m12) == [-1]
    n, m12, prev = orbref.search_for_initialization(k1, d, k2, d, 640, 480, bounds=(-30.0, 650.0, -25.0, 505.0))
    assert n == 1 and list(m12) == [0] and tuple(prev[0]) == (-20.0, 100.0)
    # bounds (0, cols, 0, rows) are the default
    a = orbref.search_for_initialization(k1, d, k2, d, 640, 480, bounds=(0.0, 640.0, 0.0, 480.0))
    b = orbref.search_for_initialization(k1, d, k2, d, 640, 480)
    assert a[0] == b[0] and np.array_equal(a[1], b[1])
