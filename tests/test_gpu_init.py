"""SearchForInitialization with its full reference signature (src/ORBmatcher.cc:417-588):
vbPrevMatched in / out and the Frame grid bounds, through the host entry point
(orbm_search_for_initialization) and the batched device one (orbm_search_for_initialization_device).

Tracking::MonocularInitialization (src/Tracking.cc:586-700) keeps mvbPrevMatched across attempts:
it starts as the initial frame's keypoints (:599-602) and every SearchForInitialization against a
later frame moves the matched entries to that frame's keypoints (:580-584), so a retry after a
failed Initializer::Initialize centres its windows elsewhere.  The bounds are Frame's static
mnMinX..mnMaxY (ComputeImageBounds, src/Frame.cc:563-621), the undistorted image corners when the
camera has distortion (k1 != 0, e.g. Examples/RGB-D/TUM1.yaml).  Bar: bit-exact matches, counts and
updated vbPrevMatched (float equality) against oracle/orbref.c.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

W, H = 1241, 376

# Examples/Monocular/TUM1.yaml (Camera.fx .. Camera.k3): pincushion, the bounds shrink inside the image
TUM1 = dict(fx=517.306408, fy=516.469215, cx=318.643040, cy=255.313989, k1=0.262383, k2=-0.953104,
            p1=-0.005358, p2=0.002628, k3=1.163314)
# Examples/Monocular/EuRoC.yaml: barrel, the undistorted corners (and edge keypoints) leave 0..752 x 0..480
EUROC = dict(fx=458.654, fy=457.296, cx=367.215, cy=248.375, k1=-0.28340811, k2=0.07395907, p1=0.00019359,
             p2=1.76187114e-05, k3=0.0)
CAMS = {"tum1": (TUM1, 640, 480), "euroc": (EUROC, 752, 480)}


def undistort(xy, cam):
    """cv::undistortPoints(..., K, D, noArray(), K) as Frame::UndistortKeyPoints / ComputeImageBounds call it:
    OpenCV 3.x's 5 fixed-point iterations.  Only used to build realistic mvKeysUn / bounds inputs; parity
    compares the GPU with the oracle on whatever float32 values come out."""
    x0 = (xy[:, 0].astype(np.float64) - cam["cx"]) / cam["fx"]
    y0 = (xy[:, 1].astype(np.float64) - cam["cy"]) / cam["fy"]
    x, y = x0.copy(), y0.copy()
    k1, k2, p1, p2, k3 = cam["k1"], cam["k2"], cam["p1"], cam["p2"], cam["k3"]
    for _ in range(5):
        r2 = x * x + y * y
        icd = 1.0 / (1 + ((k3 * r2 + k2) * r2 + k1) * r2)
        dx = 2 * p1 * x * y + p2 * (r2 + 2 * x * x)
        dy = p1 * (r2 + 2 * y * y) + 2 * p2 * x * y
        x, y = (x0 - dx) * icd, (y0 - dy) * icd
    return np.stack([x * cam["fx"] + cam["cx"], y * cam["fy"] + cam["cy"]], axis=1).astype(np.float32)


def image_bounds(cols, rows, cam):
    """Frame::ComputeImageBounds (src/Frame.cc:592-612): min / max over the undistorted corners."""
    c = undistort(np.array([[0, 0], [cols, 0], [0, rows], [cols, rows]], np.float32), cam)
    return (float(min(c[0, 0], c[2, 0])), float(max(c[1, 0], c[3, 0])),
            float(min(c[0, 1], c[1, 1])), float(max(c[2, 1], c[3, 1])))


def _extract(frames, nfeat, cuda):
    import torch
    import orbx
    ex = orbx.ORBextractor(nfeat, 1.2, 8, 20, 7)
    imgs = torch.from_numpy(np.ascontiguousarray(frames)).to(cuda)
    B, rows, cols = imgs.shape
    cap = ex.capacity(rows, cols)
    kps = torch.empty((B, cap, 7), dtype=torch.int32, device=cuda)
    desc = torch.empty((B, cap, 32), dtype=torch.uint8, device=cuda)
    counts = torch.empty((B,), dtype=torch.int32, device=cuda)
    ex.extract_batch_device(imgs, kps, desc, counts)
    ex.sync(torch.cuda.current_stream())
    klist = orbx.keypoints_from_device(kps, counts)
    d = desc.cpu().numpy()
    c = counts.cpu().numpy()
    return kps, desc, counts, klist, [d[f, :c[f]].copy() for f in range(B)]


def _xy(k):
    return np.ascontiguousarray(np.stack([k["x"], k["y"]], axis=1).astype(np.float32))


def _check(tag, got_n, got_m, got_prev, want):
    wn, wm, wprev = want
    assert got_n == wn, "%s: %d matches vs oracle %d" % (tag, got_n, wn)
    assert np.array_equal(got_m, wm), "%s: vnMatches12 differs at %s" % (tag, np.nonzero(got_m != wm)[0][:5])
    bad = np.nonzero((got_prev != wprev).any(axis=1))[0]
    assert bad.size == 0, "%s: vbPrevMatched differs at %s" % (tag, bad[:5])


def test_retry_sequence_host_and_device(orbref, cuda):
    """The initial frame stays F1 while F2 advances (frames 12 apart, 36 px of motion each), and
    vbPrevMatched carries over between attempts, as after failed Initialize calls: by the third
    attempt the scene has moved 108 px, past the 100 px window around F1's own keypoints."""
    import torch
    import orbx
    import orbx_synth
    frames = orbx_synth.kitti_sequence(37, start=3)[::12]
    kps, desc, counts, klist, dlist = _extract(frames, 2000, cuda)
    cap = kps.shape[1]
    m = orbx.ORBmatcher(0.9, True)
    k0, d0 = klist[0], dlist[0]
    n0 = len(k0)
    prev_host = _xy(k0)
    prev_want = _xy(k0)
    prev_dev = torch.zeros((1, cap, 2), dtype=torch.float32, device=cuda)
    prev_dev[0, :n0] = torch.from_numpy(_xy(k0)).to(cuda)
    pa = torch.tensor([0], dtype=torch.int32, device=cuda)
    moved = 0
    differs_from_first_attempt = 0
    for f in range(1, len(frames)):
        want = orbref.search_for_initialization(k0, d0, klist[f], dlist[f], W, H, window=100, nnratio=0.9,
                                                check_ori=True, prev_xy=prev_want)
        first = orbref.search_for_initialization(k0, d0, klist[f], dlist[f], W, H)
        differs_from_first_attempt += int(not np.array_equal(first[1], want[1]))
        n, m12 = m.SearchForInitialization((k0, d0), (klist[f], dlist[f], (W, H)), prev_host, 100)
        _check("host f%d" % f, n, m12, prev_host, want)
        pb = torch.tensor([f], dtype=torch.int32, device=cuda)
        dm12, dnm = m.search_for_initialization_batch(kps, desc, counts, pa, pb, H, W, 100,
                                                      bounds=(0.0, W, 0.0, H), prev_matched=prev_dev)
        torch.cuda.synchronize()
        _check("device f%d" % f, int(dnm.item()), dm12.cpu().numpy()[0, :n0], prev_dev.cpu().numpy()[0, :n0], want)
        moved += int((want[2] != prev_want).any(axis=1).sum())
        prev_want = want[2]
        assert want[0] > 50
    assert moved > 100
    assert differs_from_first_attempt > 0, "the carried-over vbPrevMatched never changed a result"


def test_batch_pairs_with_their_own_prev(orbref, cuda):
    """One device call, four pairs, each with its own vbPrevMatched (F1's keypoints shifted by up to
    +-60 px, so windows cross grid cells and image borders)."""
    import torch
    import orbx
    import orbx_synth
    frames = orbx_synth.kitti_sequence(5, start=11)
    kps, desc, counts, klist, dlist = _extract(frames, 2000, cuda)
    cap = kps.shape[1]
    rng = np.random.default_rng(7)
    pairs = [(0, 1), (1, 2), (0, 3), (2, 4)]
    prev = np.zeros((len(pairs), cap, 2), np.float32)
    for p, (a, _) in enumerate(pairs):
        n = len(klist[a])
        prev[p, :n] = _xy(klist[a]) + rng.uniform(-60, 60, (n, 2)).astype(np.float32)
    prev_dev = torch.from_numpy(prev).to(cuda)
    pa = torch.tensor([a for a, _ in pairs], dtype=torch.int32, device=cuda)
    pb = torch.tensor([b for _, b in pairs], dtype=torch.int32, device=cuda)
    for co in (True, False):
        m = orbx.ORBmatcher(0.9, co)
        pd = prev_dev.clone()
        m12, nm = m.search_for_initialization_batch(kps, desc, counts, pa, pb, H, W, 100, bounds=(0.0, W, 0.0, H),
                                                    prev_matched=pd)
        torch.cuda.synchronize()
        m12, nm, pd = m12.cpu().numpy(), nm.cpu().numpy(), pd.cpu().numpy()
        for p, (a, b) in enumerate(pairs):
            n = len(klist[a])
            want = orbref.search_for_initialization(klist[a], dlist[a], klist[b], dlist[b], W, H, check_ori=co,
                                                    prev_xy=prev[p, :n])
            _check("pair %d ori %d" % (p, co), int(nm[p]), m12[p, :n], pd[p, :n], want)
            assert want[0] > 0


@pytest.mark.parametrize("cam,seed", [("euroc", 0), ("euroc", 1), ("tum1", 0)])
def test_distorted_bounds(orbref, cuda, cam, seed):
    """Cameras with distortion: mvKeysUn are the undistorted keypoints (fractional; EuRoC's barrel puts
    edge keypoints at x < 0) and the grid spans the undistorted corners, not 0..cols x 0..rows.  With
    EuRoC's bounds the answer differs from the undistorted-camera grid's (keypoints outside 0..cols
    join the grid, cells change), so the bounds are exercised, not just passed through."""
    import torch
    import orbx
    import orbx_synth
    cam_p, cols, rows = CAMS[cam]
    frames = np.stack([orbx_synth.gen_image(100 + seed, cols, rows),
                       np.roll(orbx_synth.gen_image(100 + seed, cols, rows), (2, 3), axis=(0, 1))])
    _, _, _, klist, dlist = _extract(frames, 1000, cuda)
    bounds = image_bounds(cols, rows, cam_p)
    assert min(abs(bounds[0]), abs(bounds[1] - cols), abs(bounds[2]), abs(bounds[3] - rows)) > 1, bounds
    kun = []
    for k in klist:
        u = k.copy()
        xy = undistort(_xy(k), cam_p)
        u["x"], u["y"] = xy[:, 0], xy[:, 1]
        kun.append(u)
    n1 = len(kun[0])
    cap = max(len(k) for k in kun)
    m = orbx.ORBmatcher(0.9, True)
    prev = _xy(kun[0])
    want = orbref.search_for_initialization(kun[0], dlist[0], kun[1], dlist[1], cols, rows, prev_xy=prev,
                                            bounds=bounds)
    plain = orbref.search_for_initialization(kun[0], dlist[0], kun[1], dlist[1], cols, rows, prev_xy=prev)
    assert want[0] > 50
    if cam == "euroc":
        assert not np.array_equal(want[1], plain[1]), "the bounds did not change the grid's answer"
    got_prev = prev.copy()
    n, m12 = m.SearchForInitialization((kun[0], dlist[0]), (kun[1], dlist[1]), got_prev, 100, bounds=bounds)
    _check("host", n, m12, got_prev, want)
    # the device batch path with the same mvKeysUn
    kp = np.zeros((2, cap, 7), np.int32)
    ds = np.zeros((2, cap, 32), np.uint8)
    for f in range(2):
        kp[f, :len(kun[f])] = kun[f].view(np.int32).reshape(-1, 7)
        ds[f, :len(kun[f])] = dlist[f]
    tk, td = torch.from_numpy(kp).to(cuda), torch.from_numpy(ds).to(cuda)
    tc = torch.tensor([len(kun[0]), len(kun[1])], dtype=torch.int32, device=cuda)
    pv = torch.zeros((1, cap, 2), dtype=torch.float32, device=cuda)
    pv[0, :n1] = torch.from_numpy(prev).to(cuda)
    pa = torch.tensor([0], dtype=torch.int32, device=cuda)
    pb = torch.tensor([1], dtype=torch.int32, device=cuda)
    dm12, dnm = m.search_for_initialization_batch(tk, td, tc, pa, pb, rows, cols, 100, bounds=bounds, prev_matched=pv)
    torch.cuda.synchronize()
    _check("device", int(dnm.item()), dm12.cpu().numpy()[0, :n1], pv.cpu().numpy()[0, :n1], want)


def test_host_edge_cases(orbref, cuda):
    import orbx
    m = orbx.ORBmatcher(0.9, True)
    k = np.zeros(3, orbx.KEYPOINT_DTYPE)
    k["x"], k["y"] = [10, 20, 30], [10, 20, 30]
    d = np.zeros((3, 32), np.uint8)
    # F2 without keypoints: every window is empty, vbPrevMatched untouched
    prev = _xy(k)
    n, m12 = m.SearchForInitialization((k, d), (k[:0], d[:0], (640, 480)), prev, 100)
    assert n == 0 and list(m12) == [-1, -1, -1] and np.array_equal(prev, _xy(k))
    # keypoints not in extractor order (a level-1 keypoint before a level-0 one) are rejected
    bad = k.copy()
    bad["octave"] = [0, 1, 0]
    with pytest.raises(orbx.OrbxError) as e:
        m.SearchForInitialization((bad, d), (k, d, (640, 480)), _xy(k), 100)
    assert e.value.code == orbx.EINVAL
    # more keypoints than the greedy pass's LDS holds (device-memory form), all in one grid cell with equal
    # descriptors: every query sees the same 3 candidates at distance 0
    big = np.zeros(5000, orbx.KEYPOINT_DTYPE)
    big["x"], big["y"], big["size"], big["class_id"] = 11.0, 12.0, 31.0, -1
    bd = np.zeros((5000, 32), np.uint8)
    got_prev = _xy(big)
    n, m12 = m.SearchForInitialization((big, bd), (k, d, (640, 480)), got_prev, 100)
    want = orbref.search_for_initialization(big, bd, k, d, 640, 480, prev_xy=_xy(big))
    _check("host 5000 x 3", n, m12, got_prev, want)
    # past the int16 match vectors: EINVAL
    with pytest.raises(orbx.OrbxError) as e:
        huge = np.zeros(40000, orbx.KEYPOINT_DTYPE)
        m.SearchForInitialization((huge, np.zeros((40000, 32), np.uint8)), (k, d, (640, 480)), _xy(huge), 100)
    assert e.value.code == orbx.EINVAL


def _synthetic_level0(n, seed, shift=(0.0, 0.0), base=None, W=1241, H=376):
    """n level-0 keypoints (random positions, angles) with random descriptors; with `base`, the same points
    moved by `shift` plus noise and the descriptors with a few flipped bits, so most have a true match."""
    import orbx
    rng = np.random.default_rng(seed)
    k = np.zeros(n, orbx.KEYPOINT_DTYPE)
    if base is None:
        k["x"] = rng.uniform(20, W - 20, n).astype(np.float32)
        k["y"] = rng.uniform(20, H - 20, n).astype(np.float32)
        k["angle"] = rng.uniform(0, 360, n).astype(np.float32)
        d = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    else:
        bk, bd = base
        k["x"] = (bk["x"] + shift[0] + rng.normal(0, 0.7, n)).astype(np.float32)
        k["y"] = (bk["y"] + shift[1] + rng.normal(0, 0.7, n)).astype(np.float32)
        k["angle"] = ((bk["angle"] + rng.normal(3, 2, n)) % 360).astype(np.float32)
        d = bd.copy()
        for _ in range(3):   # ~3 flipped bits per descriptor
            idx = rng.integers(0, 256, n)
            d[np.arange(n), idx // 8] ^= (1 << (idx % 8)).astype(np.uint8)
    k["size"], k["response"], k["octave"], k["class_id"] = 31.0, 1.0, 0, -1
    return k, d


def test_more_level0_keypoints_than_the_common_launch_holds(orbref, cuda):
    """The greedy pass keeps up to 1792 level-0 keypoints per frame in LDS in its common launch (two
    workgroups per CU); a pair with more goes to a launch sized for the LDS maximum (~3,800), and past that to
    a launch whose arrays live in device memory.  One device call with a 6000-, a 2400- and a 500-keypoint
    pair runs all of them; the host entry with 2400 and 6000 runs the last two."""
    import torch
    import orbx
    W_, H_ = 1920, 1080
    ka, da = _synthetic_level0(2400, 1, W=W_, H=H_)
    kb, db = _synthetic_level0(2400, 2, shift=(6.0, -2.0), base=(ka, da), W=W_, H=H_)
    kc, dc = _synthetic_level0(500, 3, W=W_, H=H_)
    kd, dd = _synthetic_level0(500, 4, shift=(-9.0, 4.0), base=(kc, dc), W=W_, H=H_)
    ke, de = _synthetic_level0(6000, 5, W=W_, H=H_)
    kf, df = _synthetic_level0(6000, 6, shift=(3.0, 5.0), base=(ke, de), W=W_, H=H_)
    frames = [(ka, da), (kb, db), (kc, dc), (kd, dd), (ke, de), (kf, df)]
    cap = 6000
    kp = np.zeros((6, cap, 7), np.int32)
    ds = np.zeros((6, cap, 32), np.uint8)
    for f, (k, d) in enumerate(frames):
        kp[f, :len(k)] = k.view(np.int32).reshape(-1, 7)
        ds[f, :len(k)] = d
    tk, td = torch.from_numpy(kp).to(cuda), torch.from_numpy(ds).to(cuda)
    tc = torch.tensor([len(k) for k, _ in frames], dtype=torch.int32, device=cuda)
    pa = torch.tensor([0, 2, 4], dtype=torch.int32, device=cuda)
    pb = torch.tensor([1, 3, 5], dtype=torch.int32, device=cuda)
    m = orbx.ORBmatcher(0.9, True)
    prev = np.zeros((3, cap, 2), np.float32)
    prev[0, :2400] = _xy(ka)
    prev[1, :500] = _xy(kc)
    prev[2, :6000] = _xy(ke)
    pv = torch.from_numpy(prev).to(cuda)
    dm12, dnm = m.search_for_initialization_batch(tk, td, tc, pa, pb, H_, W_, 100, bounds=(0.0, W_, 0.0, H_),
                                                  prev_matched=pv)
    torch.cuda.synchronize()
    dm12, dnm, pv = dm12.cpu().numpy(), dnm.cpu().numpy(), pv.cpu().numpy()
    for p, (a, b) in enumerate([(0, 1), (2, 3), (4, 5)]):
        n = len(frames[a][0])
        want = orbref.search_for_initialization(frames[a][0], frames[a][1], frames[b][0], frames[b][1], W_, H_,
                                                prev_xy=prev[p, :n])
        assert want[0] > n // 4, "pair %d: only %d oracle matches" % (p, want[0])
        _check("device pair %d" % p, int(dnm[p]), dm12[p, :n], pv[p, :n], want)
    for (k1, d1), (k2, d2) in (((ka, da), (kb, db)), ((ke, de), (kf, df))):
        got_prev = _xy(k1)
        n, m12 = m.SearchForInitialization((k1, d1), (k2, d2, (W_, H_)), got_prev, 100)
        want = orbref.search_for_initialization(k1, d1, k2, d2, W_, H_, prev_xy=_xy(k1))
        _check("host %d" % len(k1), n, m12, got_prev, want)
