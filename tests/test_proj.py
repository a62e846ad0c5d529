"""Projection search, SURVEY.md §8f row 3:
  ORBmatcher::SearchByProjection(Frame& F, const vector<MapPoint*>&, th)  src/ORBmatcher.cc:45-129
  (Tracking::SearchLocalPoints, src/Tracking.cc:1234-1244) over Frame::GetFeaturesInArea.

The per-MapPoint inputs are what Frame::isInFrustum leaves in the MapPoint (projection,
predicted level, viewing cosine, in-view flag) plus Observations() > 0.  Scenes are made
so that many MapPoints compete for the same features: the in-call claims (the greedy part
of the reference) decide the result.
CPU: the C oracle against a pure-Python restatement.  GPU: host and batched device paths
against the oracle, match arrays and nmatches identical.
"""
import numpy as np
import pytest

SCALE = np.array([np.float32(1.2) ** i for i in range(8)], np.float32)


def py_search(kps, desc, uright, claimed, grid, scale, pts, pdesc, th, nnratio):
    minx, miny, winv, hinv = (np.float32(g) for g in grid)
    F32 = np.float32
    n = len(kps)
    cells = {}
    for i in range(n):
        px = int(np.floor(float(F32(F32(kps["x"][i] - minx) * winv)) + 0.5))
        py = int(np.floor(float(F32(F32(kps["y"][i] - miny) * hinv)) + 0.5))
        if 0 <= px < 64 and 0 <= py < 48:
            cells.setdefault((px, py), []).append(i)
    cl = claimed.astype(bool).copy()
    match = np.full(n, -1, np.int32)
    nm = 0
    ham = lambda a, b: int(np.unpackbits(a ^ b).sum())
    for m, P in enumerate(pts):
        if not (P["flags"] & 1):
            continue
        level = int(P["level"])
        r = F32(2.5) if float(P["view_cos"]) > 0.998 else F32(4.0)
        if th != 1.0:
            r = F32(r * F32(th))
        rr = F32(r * scale[level])
        x, y = F32(P["proj_x"]), F32(P["proj_y"])
        cx0 = max(0, int(np.floor(float(F32(F32(F32(x - minx) - rr) * winv)))))
        if cx0 >= 64:
            continue
        cx1 = min(63, int(np.ceil(float(F32(F32(F32(x - minx) + rr) * winv)))))
        if cx1 < 0:
            continue
        cy0 = max(0, int(np.floor(float(F32(F32(F32(y - miny) - rr) * hinv)))))
        if cy0 >= 48:
            continue
        cy1 = min(47, int(np.ceil(float(F32(F32(F32(y - miny) + rr) * hinv)))))
        if cy1 < 0:
            continue
        b1, l1, b2, l2, bi = 256, -1, 256, -1, -1
        for ix in range(cx0, cx1 + 1):
            for iy in range(cy0, cy1 + 1):
                for idx in cells.get((ix, iy), []):
                    o = int(kps["octave"][idx])
                    if o < level - 1 or o > level:
                        continue
                    if not (abs(F32(kps["x"][idx] - x)) < rr and abs(F32(kps["y"][idx] - y)) < rr):
                        continue
                    if cl[idx]:
                        continue
                    if uright[idx] > 0 and F32(abs(F32(P["proj_xr"] - uright[idx]))) > rr:
                        continue
                    d = ham(pdesc[m], desc[idx])
                    if d < b1:
                        b2, b1, l2, l1, bi = b1, d, l1, o, idx
                    elif d < b2:
                        l2, b2 = o, d
        if b1 <= 100:
            if l1 == l2 and F32(b1) > F32(F32(nnratio) * F32(b2)):
                continue
            match[bi] = m
            cl[bi] = bool(P["flags"] & 2)
            nm += 1
    return nm, match


def scene(seed, n_kp=600, n_mp=900, W=640, H=480):
    """Keypoints on a coarse lattice with descriptors in clusters; several MapPoints per
    keypoint neighbourhood with descriptors near the cluster centre."""
    import orbref
    rng = np.random.default_rng(seed)
    kps = np.zeros(n_kp, orbref.KEYPOINT_DTYPE)
    kps["x"] = (rng.integers(2, (W - 4) // 4, n_kp) * 4 + rng.random(n_kp)).astype(np.float32)
    kps["y"] = (rng.integers(2, (H - 4) // 4, n_kp) * 4 + rng.random(n_kp)).astype(np.float32)
    kps["octave"] = rng.integers(0, 8, n_kp)
    kps["x"] = np.minimum(kps["x"], W - 1)
    proto = rng.integers(0, 256, (40, 32), dtype=np.uint8)
    owner = rng.integers(0, 40, n_kp)
    flip = lambda src, p: np.packbits(np.unpackbits(src, axis=-1) ^ (rng.random(src.shape[:-1] + (256,)) < p),
                                      axis=-1)
    desc = flip(proto[owner], 0.05)
    uright = np.where(rng.random(n_kp) < 0.3, kps["x"] - rng.uniform(0, 40, n_kp), -1).astype(np.float32)
    claimed = (rng.random(n_kp) < 0.1).astype(np.uint8)
    pts = np.zeros(n_mp, orbref.PROJ_DTYPE)
    tgt = rng.integers(0, n_kp, n_mp)
    pts["proj_x"] = kps["x"][tgt] + rng.normal(0, 3, n_mp).astype(np.float32)
    pts["proj_y"] = kps["y"][tgt] + rng.normal(0, 3, n_mp).astype(np.float32)
    pts["proj_xr"] = np.where(uright[tgt] > 0, uright[tgt] + rng.normal(0, 3, n_mp), 0).astype(np.float32)
    pts["view_cos"] = rng.uniform(0.99, 1.0, n_mp).astype(np.float32)
    pts["level"] = np.clip(kps["octave"][tgt] + rng.integers(0, 2, n_mp), 0, 7)
    pts["flags"] = (rng.random(n_mp) < 0.9).astype(np.int32) | ((rng.random(n_mp) < 0.8).astype(np.int32) << 1)
    pdesc = flip(proto[owner[tgt]], 0.08)
    grid = (0.0, 0.0, np.float32(64) / np.float32(W), np.float32(48) / np.float32(H))
    return kps, desc, uright, claimed, grid, pts, pdesc


@pytest.mark.parametrize("seed", [0, 1, 2])
@pytest.mark.parametrize("th", [1.0, 3.0, 5.0])
def test_oracle_matches_restatement(orbref, seed, th):
    kps, desc, ur, cl, grid, pts, pdesc = scene(seed)
    n, m = orbref.search_by_projection(kps, desc, ur, cl, grid, SCALE, pts, pdesc, th, 0.8)
    pn, pm = py_search(kps, desc, ur, cl, grid, SCALE, pts, pdesc, th, 0.8)
    assert n == pn and np.array_equal(m, pm)
    assert n > 100


def test_claims_change_the_result(orbref):
    """Two MapPoints with the same descriptor at the same spot: the first takes the feature, the
    second (Observations() > 0 claim) must fall back to the next feature; with the first
    MapPoint's Observations() == 0 the feature stays free and the second overwrites it."""
    kps = np.zeros(2, orbref.KEYPOINT_DTYPE)
    kps["x"], kps["y"] = [100, 102], [100, 100]
    desc = np.zeros((2, 32), np.uint8)
    desc[1, 0] = 0x0F
    pts = np.zeros(2, orbref.PROJ_DTYPE)
    pts["proj_x"], pts["proj_y"], pts["view_cos"], pts["flags"] = 100, 100, 1.0, 3
    pdesc = np.zeros((2, 32), np.uint8)
    grid = (0.0, 0.0, np.float32(64) / 640, np.float32(48) / 480)
    ur = np.full(2, -1, np.float32)
    n, m = orbref.search_by_projection(kps, desc, ur, np.zeros(2, np.uint8), grid, SCALE, pts, pdesc, 1.0, 0.8)
    assert n == 2 and list(m) == [0, 1]
    pts["flags"][0] = 1                                     # first MapPoint has no observations
    n, m = orbref.search_by_projection(kps, desc, ur, np.zeros(2, np.uint8), grid, SCALE, pts, pdesc, 1.0, 0.8)
    assert n == 2 and list(m) == [1, -1]


@pytest.mark.gpu
@pytest.mark.parametrize("seed,th", [(0, 1.0), (1, 3.0), (2, 5.0), (3, 1.0)])
def test_gpu_search_by_projection_host(orbref, cuda, seed, th):
    import orbx
    kps, desc, ur, cl, grid, pts, pdesc = scene(seed)
    n, m = orbx.ORBmatcher(0.8).SearchByProjection(kps, desc, ur, cl, grid, SCALE, pts, pdesc, th)
    wn, wm = orbref.search_by_projection(kps, desc, ur, cl, grid, SCALE, pts, pdesc, th, 0.8)
    assert n == wn and np.array_equal(m, wm)


@pytest.mark.gpu
def test_gpu_search_by_projection_batch(orbref, cuda):
    import ctypes
    import torch
    import orbx
    scenes = [scene(s, n_kp=500 + 50 * s, n_mp=700 + 40 * s) for s in range(4)]
    B = len(scenes)
    cap = max(len(s[0]) for s in scenes)
    pcap = max(len(s[5]) for s in scenes)
    kps = np.zeros((B, cap), orbx.KEYPOINT_DTYPE)
    desc = np.zeros((B, cap, 32), np.uint8)
    ur = np.zeros((B, cap), np.float32)
    cl = np.zeros((B, cap), np.uint8)
    pts = np.zeros((B, pcap), orbx.PROJ_POINT_DTYPE)
    pdesc = np.zeros((B, pcap, 32), np.uint8)
    counts = np.array([len(s[0]) for s in scenes], np.int32)
    npts = np.array([len(s[5]) for s in scenes], np.int32)
    for b, (k, d, u, c, g, p, pd) in enumerate(scenes):
        kps[b, :len(k)] = k
        desc[b, :len(k)] = d
        ur[b, :len(k)] = u
        cl[b, :len(k)] = c
        pts[b, :len(p)] = p
        pdesc[b, :len(p)] = pd
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(cuda)
    dk, dd, du, dc = T(kps.view(np.int32).reshape(B, cap, 7)), T(desc), T(ur), T(cl)
    dp, dpd, dn, dnp = T(pts.view(np.int32).reshape(B, pcap, 6)), T(pdesc), T(counts), T(npts)
    match = torch.empty((B, cap), dtype=torch.int32, device=cuda)
    nm = torch.empty((B,), dtype=torch.int32, device=cuda)
    prm = orbx.proj_params(scenes[0][4], SCALE, 3.0, 0.8)
    P = lambda t: ctypes.c_void_p(t.data_ptr())
    rc = orbx.lib.orbm_search_by_projection_device(P(dk), P(dd), P(du), P(dc), P(dn), B, cap, P(dp), P(dpd), P(dnp),
                                                    pcap, ctypes.byref(prm), P(match), P(nm),
                                                    ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc == 0
    torch.cuda.synchronize()
    for b, (k, d, u, c, g, p, pd) in enumerate(scenes):
        wn, wm = orbref.search_by_projection(k, d, u, c, g, SCALE, p, pd, 3.0, 0.8)
        assert int(nm[b]) == wn
        assert np.array_equal(match[b, :len(k)].cpu().numpy(), wm)


def _chain_scene(orbref):
    """Fourteen MapPoints at one spot with one descriptor, twelve features around it at Hamming
    distances 0, 3, 6, ...: each MapPoint takes the next feature, so the later ones find more
    than the first eight candidates of their window claimed."""
    kps = np.zeros(12, orbref.KEYPOINT_DTYPE)
    kps["x"], kps["y"] = 100.0 + np.arange(12), 100.0
    desc = np.zeros((12, 32), np.uint8)
    for i in range(12):
        desc[i, :i] = 0xFF                                  # distance 8*i
    pts = np.zeros(14, orbref.PROJ_DTYPE)
    pts["proj_x"], pts["proj_y"], pts["view_cos"], pts["flags"] = 105.5, 100.0, 1.0, 3
    pdesc = np.zeros((14, 32), np.uint8)
    grid = (0.0, 0.0, np.float32(64) / 640, np.float32(48) / 480)
    return kps, desc, np.full(12, -1, np.float32), np.zeros(12, np.uint8), grid, pts, pdesc


def test_claim_chain(orbref):
    kps, desc, ur, cl, grid, pts, pdesc = _chain_scene(orbref)
    n, m = orbref.search_by_projection(kps, desc, ur, cl, grid, SCALE, pts, pdesc, 3.0, 0.99)
    assert n == 12 and list(m) == list(range(12))
    pn, pm = py_search(kps, desc, ur, cl, grid, SCALE, pts, pdesc, 3.0, 0.99)
    assert pn == n and np.array_equal(pm, m)


@pytest.mark.gpu
def test_gpu_claim_chain(orbref, cuda):
    """The replay runs out of its candidate list and scans the window again."""
    import orbx
    kps, desc, ur, cl, grid, pts, pdesc = _chain_scene(orbref)
    n, m = orbx.ORBmatcher(0.99).SearchByProjection(kps, desc, ur, cl, grid, SCALE, pts, pdesc, 3.0)
    assert n == 12 and list(m) == list(range(12))
