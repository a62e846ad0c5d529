"""DistributeOctTree (src/ORBextractor.cc:644-907) restated on path codes: the formulation the
device kernel K3 uses (csrc/orbx_extract.hip, k_qt_paths), checked here on the CPU against the
node-list oracle (oracle/orbref.c, orbref_distribute) on every level of real frames and on
random, clustered and tie-heavy candidate sets.

Every split in DistributeOctTree (ExtractorNode::DivideNode, :569-629) halves a node's x range at
UL.x + ceil((UR.x - UL.x) / 2) and its y range likewise, independently.  So the sequence of
left/right decisions a keypoint meets is a function of its x alone (given its root, x / hX, :679)
and the top/bottom decisions of its y alone: per level, two tables give every keypoint its whole
path down the tree, x and y digits interleaved below the root (quadrant q = right + 2 * bottom,
n1..n4 = 0..3).  Sorted by that key, the keypoints of any node at any depth are one contiguous run.

Phase 1 splits every node with more than one keypoint, so after round d the nodes are exactly the
non-empty depth-d cells (a node kept for holding one keypoint has the same key set as its depth-d
cell).  With fd[i] = the shallowest depth at which sorted keys i-1 and i lie in different cells:
  L_d     = #{i : fd[i] <= d}                       (nodes after round d)
  nexp_d  = L_d - #{i : max(fd[i], fd[i+1]) <= d}    (nodes with more than one keypoint, :746-790)
which settles where phase 1 stops (:793-803) without replaying the rounds.  The list order follows
from the push_front of children in parent-list order: after round D the list is
  reverse(B_D) ++ S_{D-1} ++ ... ++ S_1 ++ S_0
where B_d is the round's children in creation order and S_b the single-keypoint nodes created in
round b (in the round-b list order, S_0 the roots in order); reverse(B_b) visits digit j ascending
iff b - j is odd (the root like digit 1, ascending iff b is even).  Phase 2 (:805-874) splits nodes
by (size, creation) from the largest and stops at N; it runs on the runs of the sorted keys.
"""
import numpy as np
import pytest

F32 = np.float32


def _ceil_half(w):
    return int(np.ceil(F32(w) / F32(2)))


def _depth(npts):
    """Splits until every interval holds at most one integer coordinate (DivideNode on one axis)."""
    if npts <= 1:
        return 0
    h = _ceil_half(npts - 1)
    return 1 + max(_depth(h), _depth(npts - h))


def path_tables(w, h):
    """Per-level tables: xkey[x] = root << 2D | x digits at the even bit positions, ykey[y] = y digits
    at the odd positions (digit j of D at bits 2(D - j) + {0, 1}); x, y relative to the 16-pixel border
    (minBorderX / minBorderY, :1003-1008).  Returns (xkey, ykey, D, rootbits, nIni)."""
    qw, qh = (w - 16) - 16, (h - 16) - 16
    nIni = int(np.round(F32(qw) / F32(qh)))                  # :650 (float32 division, round)
    hX = F32(qw) / F32(nIni)                                 # :653
    roots = [(int(hX * F32(i)), int(hX * F32(i + 1))) for i in range(nIni)]   # Point2i truncation, :666-669
    D = max(max(_depth(x1 - x0 + 1) for x0, x1 in roots), _depth(qh + 1))
    rootbits = max(1, int(nIni - 1).bit_length())
    xkey = np.zeros(w, np.uint64)
    for x in range(w):
        r = min(int(F32(x) / hX), nIni - 1)                  # :681
        x0, x1 = roots[r]
        code = r
        for _ in range(D):
            mid = x0 + _ceil_half(x1 - x0)
            bit = 1 if x >= mid else 0
            code = (code << 2) | bit
            if bit:
                x0 = mid
            else:
                x1 = mid
        xkey[x] = code
    ykey = np.zeros(h, np.uint64)
    for y in range(h):
        y0, y1 = 0, qh
        code = 0
        for _ in range(D):
            mid = y0 + _ceil_half(y1 - y0)
            bit = 1 if y >= mid else 0
            code = (code << 2) | (bit << 1)
            if bit:
                y0 = mid
            else:
                y1 = mid
        ykey[y] = code
    return xkey, ykey, D, rootbits, nIni


def distribute_pathcode(cands, w, h, N):
    """Indices of the kept candidates in the reference's output order (== orbref.distribute)."""
    n = len(cands)
    if n == 0:
        return np.zeros(0, np.int32)
    xkey, ykey, D, rootbits, nIni = path_tables(w, h)
    x, y, score = (cands[:, k].astype(np.int64) for k in range(3))
    key = xkey[x] | ykey[y]
    order = np.argsort(key, kind="stable")
    sk = key[order]
    top = 2 * D + rootbits

    def digit(k, j):   # digit j (1..D) of key k
        return int(k >> np.uint64(2 * (D - j))) & 3

    # fd[i]: first depth at which sorted keys i-1 and i differ (0: another root); fd[0] = fd[n] = 0
    fd = np.zeros(n + 1, np.int64)
    for i in range(1, n):
        dif = int(sk[i - 1] ^ sk[i])
        hb = dif.bit_length() - 1                             # highest differing bit
        fd[i] = 0 if hb >= 2 * D else D - hb // 2
    mx = np.maximum(fd[:n], fd[1:])
    Lc = lambda d: int((fd[:n] <= d).sum())
    Mc = lambda d: int((mx <= d).sum())
    # phase 1, :710-803 (round 1 always runs)
    Dp, phase2 = None, False
    for d in range(1, D + 2):
        Ld, Lp = Lc(d), Lc(d - 1)
        nexp = Ld - Mc(d)
        if Ld >= N or Ld == Lp:
            Dp = d
            break
        if Ld + 3 * nexp > N:
            Dp, phase2 = d, True
            break
    assert Dp is not None
    Dp = min(Dp, D)   # past D nothing changes (every run is a single key)
    # nodes after round Dp: the depth-Dp runs
    starts = [i for i in range(n) if fd[i] <= Dp]
    nodes = []
    for k, s in enumerate(starts):
        e = starts[k + 1] if k + 1 < len(starts) else n
        b = Dp if e - s > 1 else int(max(fd[s], fd[s + 1]))
        root = int(sk[s] >> np.uint64(2 * D))
        tk = root ^ ((1 << rootbits) - 1 if b % 2 else 0)
        for j in range(1, b + 1):
            tk = (tk << 2) | (digit(sk[s], j) ^ (3 if (b - j) % 2 == 0 else 0))
        tk <<= 2 * (D - b)
        nodes.append(dict(s=s, c=e - s, depth=b if e - s == 1 else Dp, born=b, lkey=(Dp - b, tk)))
    nodes.sort(key=lambda nd: nd["lkey"])   # the list after round Dp
    seq = 0
    for nd in reversed(nodes):              # creation order within group 0 = reverse list order
        nd["seq"] = seq
        seq += 1
    lst = nodes

    def divide(nd):
        s, c, dp = nd["s"], nd["c"], nd["depth"]
        kids = []
        lo = s
        for q in range(4):
            hi = lo
            while hi < s + c and (dp + 1 > D or digit(sk[hi], dp + 1) == q):
                hi += 1
            if dp + 1 > D:   # no digits left: all keys in child 0 (cannot happen for distinct keys)
                hi = s + c if q == 0 else lo
            kids.append(dict(s=lo, c=hi - lo, depth=dp + 1))
            lo = hi
        return kids

    if phase2:
        vec = [nd for nd in nodes if nd["lkey"][0] == 0 and nd["c"] > 1]
        vec.sort(key=lambda nd: nd["seq"])
        while True:
            prev_size = len(lst)
            prevv = sorted(vec, key=lambda nd: (nd["c"], nd["seq"]))
            vec = []
            done = False
            for j in range(len(prevv) - 1, -1, -1):
                par = prevv[j]
                front = []
                for kid in divide(par):
                    if kid["c"] > 0:
                        kid["seq"] = seq
                        seq += 1
                        front.insert(0, kid)   # push_front in n1..n4 order
                        if kid["c"] > 1:
                            vec.append(kid)
                lst = front + [nd for nd in lst if nd is not par]
                if len(lst) >= N:
                    break
            if len(lst) >= N or len(lst) == prev_size:
                break
    out = []
    for nd in lst:   # :882-906, first max wins (original index order)
        idx = order[nd["s"]:nd["s"] + nd["c"]]
        best = min(idx, key=lambda i: (-score[i], i))
        out.append(best)
    return np.array(out, np.int32)


def _random_cands(rng, w, h, n, clustered=False, scores=4):
    qw, qh = w - 32, h - 32
    if clustered:
        cx, cy = rng.integers(0, qw), rng.integers(0, qh)
        xs = np.clip(rng.normal(cx, 6, 4 * n).astype(np.int64), 0, qw - 1)
        ys = np.clip(rng.normal(cy, 6, 4 * n).astype(np.int64), 0, qh - 1)
    else:
        xs, ys = rng.integers(0, qw, 4 * n), rng.integers(0, qh, 4 * n)
    _, u = np.unique(ys * 8192 + xs, return_index=True)
    u = rng.permutation(u)[:n]
    c = np.stack([xs[u], ys[u], rng.integers(1, 1 + scores, len(u))], axis=1).astype(np.int32)
    return c


@pytest.mark.parametrize("seed", range(12))
def test_random_sets(orbref, seed):
    rng = np.random.default_rng(seed)
    for w, h in ((640, 480), (1241, 376), (120, 90), (1920, 1080), (400, 600)):
        for n, N in ((0, 10), (1, 5), (2, 1), (7, 3), (60, 20), (300, 120), (900, 434), (3000, 434)):
            for clustered in (False, True):
                c = _random_cands(rng, w, h, n, clustered, scores=int(rng.integers(1, 6)))
                want = orbref.distribute(c, w, h, N)
                got = distribute_pathcode(c, w, h, N)
                assert np.array_equal(got, want), (w, h, n, N, clustered)


def test_real_levels(orbref):
    import orbx_synth
    p = orbref.make_params(2000, 1.2, 8, 20, 7)
    t = orbref.tables(p)
    for f in orbx_synth.kitti_sequence(2, start=30):
        r = orbref.extract(f, p)
        for l in range(8):
            lev = r.pyramid[l]
            hh, ww = lev.shape
            c = orbref.level_candidates(lev)
            N = t.nfeat_level[l]
            assert np.array_equal(distribute_pathcode(c, ww, hh, N), orbref.distribute(c, ww, hh, N)), l


def test_table_depth_fits_the_packed_key():
    """The device key is (root, D digits, score) in 32 bits (k_qt_paths takes a level when
    rootbits + 2 D + 8 <= 32): every KITTI / EuRoC / TUM / 1080p level qualifies."""
    for w0, h0 in ((1241, 376), (752, 480), (640, 480), (1920, 1080)):
        for l in range(8):
            s = 1.2 ** l
            w, h = int(round(w0 / s)), int(round(h0 / s))
            _, _, D, rb, _ = path_tables(w, h)
            assert rb + 2 * D + 8 <= 32, (w0, h0, l, D, rb)
