"""Frame::ComputeStereoMatches (src/Frame.cc:630-872), SURVEY.md §8a row a15.

CPU: the C oracle (oracle/orbref.c) against an independent numpy restatement
written from the reference text, plus hand-built known answers (integer-shift
pairs recover the shift exactly; the 2.1 x median cut).
GPU: liborbx's host path (two extractor handles, orbx_compute_stereo_matches)
and the batched device path (orbx_stereo_batch_device) against the oracle.
Bar: mvuRight / mvDepth bit-exact (float32 equality), n_good equal.
"""
import numpy as np
import pytest

EUROC_BF, EUROC_FX = 47.90639384423901, 435.2046959714599   # Examples/Stereo/EuRoC.yaml:8,25
F32 = np.float32


def _cround(x):
    """C round(): half away from zero (x >= 0 here); numpy's round is half-to-even."""
    f = float(x)
    t = np.floor(f)
    return t + 1.0 if f - t >= 0.5 else t


def _reflect(p, n):
    while p < 0 or p >= n:
        p = -p if p < 0 else 2 * n - 2 - p
    return p


def py_stereo(p, left, right, rows, cols, bf, fx, orbref):
    """Second restatement of src/Frame.cc:630-872 (numpy, float32 scalars)."""
    t = orbref.tables(p)
    S = [F32(t.scale[l]) for l in range(p.nlevels)]
    IS = [F32(t.inv_scale[l]) for l in range(p.nlevels)]
    kL, kR = left.keypoints, right.keypoints
    dL, dR = left.descriptors, right.descriptors
    n = len(kL)
    uR_out = np.full(n, -1, np.float32)
    dp_out = np.full(n, -1, np.float32)
    rowidx = [[] for _ in range(rows)]
    for iR in range(len(kR)):
        y = F32(kR["y"][iR])
        r = F32(2.0) * S[kR["octave"][iR]]
        for yi in range(int(np.floor(F32(y - r))), int(np.ceil(F32(y + r))) + 1):
            if 0 <= yi < rows:
                rowidx[yi].append(iR)
    mb = F32(F32(bf) / F32(fx))
    maxD = F32(F32(bf) / mb)
    minD = F32(0)
    ham = lambda a, b: int(np.unpackbits(np.bitwise_xor(a, b)).sum())
    pairs = []
    for iL in range(n):
        lv = int(kL["octave"][iL])
        vL, uL = F32(kL["y"][iL]), F32(kL["x"][iL])
        cand = rowidx[int(vL)]
        if not cand:
            continue
        minU, maxU = F32(uL - maxD), F32(uL - minD)
        if maxU < 0:
            continue
        best, bi = 100, 0
        for iR in cand:
            o = int(kR["octave"][iR])
            if o < lv - 1 or o > lv + 1:
                continue
            u = F32(kR["x"][iR])
            if minU <= u <= maxU:
                d = ham(dL[iL], dR[iR])
                if d < best:
                    best, bi = d, iR
        if best >= 75:
            continue
        sf = IS[lv]
        sul = _cround(F32(kL["x"][iL] * sf))
        svl = _cround(F32(kL["y"][iL] * sf))
        sur = _cround(F32(F32(kR["x"][bi]) * sf))
        if sur < 0 or sur + 11 >= right.pyramid[lv].shape[1]:
            continue
        IL, IR = left.pyramid[lv].astype(np.int64), right.pyramid[lv].astype(np.int64)
        H, W = IL.shape
        vy, ux, ur = int(svl), int(sul), int(sur)
        ys = [_reflect(vy + k, H) for k in range(-5, 6)]
        wl = IL[np.ix_(ys, [_reflect(ux + k, W) for k in range(-5, 6)])]
        wl = wl - wl[5, 5]
        dists = []
        for inc in range(-5, 6):
            wr = IR[np.ix_(ys, [_reflect(ur + inc + k, W) for k in range(-5, 6)])]
            wr = wr - wr[5, 5]
            dists.append(int(np.abs(wl - wr).sum()))
        binc = int(np.argmin(dists)) - 5           # first minimum
        if binc in (-5, 5):
            continue
        d1, d2, d3 = (F32(dists[5 + binc + k]) for k in (-1, 0, 1))
        delta = F32(F32(d1 - d3) / F32(F32(2.0) * F32(F32(d1 + d3) - F32(F32(2.0) * d2))))
        if delta < -1 or delta > 1:
            continue
        buR = F32(S[lv] * F32(F32(F32(sur) + F32(binc)) + delta))
        disp = F32(uL - buR)
        if disp >= minD and disp < maxD:
            if disp <= 0:
                disp = F32(0.01)
                buR = F32(float(uL) - 0.01)
            dp_out[iL] = F32(F32(bf) / disp)
            uR_out[iL] = buR
            pairs.append((min(dists), iL))
    pairs.sort()
    good = len(pairs)
    if pairs:
        th = F32(F32(F32(1.5) * F32(1.4)) * F32(pairs[len(pairs) // 2][0]))
        for d, i in reversed(pairs):
            if F32(d) < th:
                break
            uR_out[i] = -1
            dp_out[i] = -1
            good -= 1
    return uR_out, dp_out, good


def _pair(seed, W, H):
    import orbx_synth
    return orbx_synth.stereo_pair(seed, W, H)


@pytest.mark.parametrize("seed", [3, 11])
def test_oracle_matches_python_restatement(orbref, seed):
    L, R = _pair(seed, 320, 240)
    p = orbref.make_params(300, 1.2, 8, 20, 7)
    a, b = orbref.extract(L, p), orbref.extract(R, p)
    ur, dp, sad, good = orbref.compute_stereo_matches(p, a, b, 240, 320, EUROC_BF, EUROC_FX)
    pur, pdp, pgood = py_stereo(p, a, b, 240, 320, EUROC_BF, EUROC_FX, orbref)
    assert good == pgood and good > 20
    assert np.array_equal(ur, pur) and np.array_equal(dp, pdp)


def _shifted(d, noise):
    import orbx_synth
    big = orbx_synth.gen_image(21, 400 + d, 300)
    L, R = big[:, :400].copy(), big[:, d:].copy()     # a scene point at L x appears at R x - d
    if noise:
        rng = np.random.default_rng(5)
        R = np.clip(R.astype(np.int32) + rng.integers(-noise, noise + 1, R.shape), 0, 255).astype(np.uint8)
    return L, R


def test_integer_shift_is_recovered(orbref):
    d = 9
    L, R = _shifted(d, 2)
    p = orbref.make_params(400, 1.2, 8, 20, 7)
    a, b = orbref.extract(L, p), orbref.extract(R, p)
    ur, dp, sad, good = orbref.compute_stereo_matches(p, a, b, 300, 400, EUROC_BF, EUROC_FX)
    lv0 = (a.keypoints["octave"] == 0) & (ur >= 0)
    assert lv0.sum() > 50
    disp = a.keypoints["x"][lv0] - ur[lv0]
    assert np.all(np.abs(disp - d) < 1.0)
    assert np.allclose(dp[lv0], np.float32(EUROC_BF) / disp, rtol=1e-6)


def test_noise_free_shift_has_zero_sad_at_level0(orbref):
    # noise-free integer shift: a level-0 window and its shifted twin are identical, so the
    # accepted level-0 SAD is exactly 0 at the true shift (11x11 windows, src/Frame.cc:771-812)
    d = 9
    L, R = _shifted(d, 0)
    p = orbref.make_params(400, 1.2, 8, 20, 7)
    a, b = orbref.extract(L, p), orbref.extract(R, p)
    ur, dp, sad, good = orbref.compute_stereo_matches(p, a, b, 300, 400, EUROC_BF, EUROC_FX)
    lv0 = (a.keypoints["octave"] == 0) & (sad >= 0)
    zero = lv0 & (sad == 0)
    assert lv0.sum() > 50 and zero.sum() >= 0.95 * lv0.sum()   # the rest: a wrong coarse match
    kept = zero & (ur >= 0)
    assert kept.sum() > 50
    assert np.all(np.abs(a.keypoints["x"][kept] - ur[kept] - d) < 1.0)


def test_median_cut_threshold(orbref):
    # every accepted pair has SAD < 2.1 x median or is cut: check on the synthetic EuRoC pair
    L, R = _pair(3, 752, 480)
    p = orbref.make_params(1000, 1.2, 8, 20, 7)
    a, b = orbref.extract(L, p), orbref.extract(R, p)
    ur, dp, sad, good = orbref.compute_stereo_matches(p, a, b, 480, 752, EUROC_BF, EUROC_FX)
    acc = np.sort(sad[sad >= 0])
    th = np.float32(np.float32(1.5) * np.float32(1.4)) * np.float32(acc[len(acc) // 2])
    kept = (sad >= 0) & (sad.astype(np.float32) < th)
    assert good == kept.sum() and np.array_equal(ur >= 0, kept)
    assert good < len(acc)          # the synthetic pair has outliers the cut removes


def test_no_right_keypoints(orbref):
    L, _ = _pair(3, 320, 240)
    R = np.full_like(L, 128)
    p = orbref.make_params(300, 1.2, 8, 20, 7)
    a, b = orbref.extract(L, p), orbref.extract(R, p)
    assert len(b.keypoints) == 0
    ur, dp, sad, good = orbref.compute_stereo_matches(p, a, b, 240, 320, EUROC_BF, EUROC_FX)
    assert good == 0 and np.all(ur == -1) and np.all(dp == -1)


# ---------------------------------------------------------------------------- GPU


STEREO_CONFIGS = [
    # (W, H, nfeatures, seed)
    (752, 480, 1000, 3),      # config 3: EuRoC MH01 geometry, 1000 feat/image
    (752, 480, 1200, 5),      # the reference EuRoC stereo YAML's 1200 (Examples/Stereo/EuRoC.yaml:88)
    (320, 240, 300, 7),
    (1241, 376, 2000, 9),     # KITTI-shaped stereo
]


@pytest.mark.gpu
@pytest.mark.parametrize("W,H,nfeat,seed", STEREO_CONFIGS)
def test_gpu_host_stereo_parity(orbref, cuda, W, H, nfeat, seed):
    import orbx
    L, R = _pair(seed, W, H)
    exl = orbx.ORBextractor(nfeat, 1.2, 8, 20, 7)
    exr = orbx.ORBextractor(nfeat, 1.2, 8, 20, 7)
    kl, dl = exl(L)
    kr, dr = exr(R)
    ur, dp, good = orbx.compute_stereo_matches(exl, exr, kl, dl, kr, dr, EUROC_BF, EUROC_FX)
    p = orbref.make_params(nfeat, 1.2, 8, 20, 7)
    a, b = orbref.extract(L, p), orbref.extract(R, p)
    assert np.array_equal(kl, a.keypoints) and np.array_equal(kr, b.keypoints)
    wur, wdp, _, wgood = orbref.compute_stereo_matches(p, a, b, H, W, EUROC_BF, EUROC_FX)
    assert good == wgood and good > 0
    bad = np.nonzero(ur != wur)[0]
    assert bad.size == 0, "uRight differs at %s: gpu %s oracle %s" % (bad[:5], ur[bad[:5]], wur[bad[:5]])
    assert np.array_equal(dp, wdp)


@pytest.mark.gpu
def test_gpu_batch_stereo_parity(orbref, cuda):
    import torch
    import orbx
    W, H, nfeat = 752, 480, 1000
    pairs = [_pair(s, W, H) for s in (3, 4, 5)]
    frames = np.stack([im for pr in pairs for im in pr])   # L0 R0 L1 R1 L2 R2
    ex = orbx.ORBextractor(nfeat, 1.2, 8, 20, 7)
    imgs = torch.from_numpy(frames).to(cuda)
    cap = ex.capacity(H, W)
    B = len(frames)
    kps = torch.empty((B, cap, 7), dtype=torch.int32, device=cuda)
    desc = torch.empty((B, cap, 32), dtype=torch.uint8, device=cuda)
    counts = torch.empty((B,), dtype=torch.int32, device=cuda)
    ex.extract_batch_device(imgs, kps, desc, counts)
    li = torch.tensor([0, 2, 4], dtype=torch.int32, device=cuda)
    ri = torch.tensor([1, 3, 5], dtype=torch.int32, device=cuda)
    ur, dp, ng = ex.stereo_batch_device(kps, desc, counts, li, ri, EUROC_BF, EUROC_FX)
    ex.sync(torch.cuda.current_stream())
    p = orbref.make_params(nfeat, 1.2, 8, 20, 7)
    c = counts.cpu().numpy()
    for k, (L, R) in enumerate(pairs):
        a, b = orbref.extract(L, p), orbref.extract(R, p)
        wur, wdp, _, wgood = orbref.compute_stereo_matches(p, a, b, H, W, EUROC_BF, EUROC_FX)
        n = c[2 * k]
        assert n == len(a.keypoints)
        assert int(ng[k].item()) == wgood
        assert np.array_equal(ur[k, :n].cpu().numpy(), wur)
        assert np.array_equal(dp[k, :n].cpu().numpy(), wdp)


@pytest.mark.gpu
def test_gpu_stereo_edge_cases(orbref, cuda):
    import orbx
    L, R = _pair(3, 320, 240)
    exl = orbx.ORBextractor(300, 1.2, 8, 20, 7)
    exr = orbx.ORBextractor(300, 1.2, 8, 20, 7)
    kl, dl = exl(L)
    kr, dr = exr(np.full_like(R, 128))     # no right keypoints
    assert len(kr) == 0
    ur, dp, good = orbx.compute_stereo_matches(exl, exr, kl, dl, kr, dr, EUROC_BF, EUROC_FX)
    assert good == 0 and np.all(ur == -1) and np.all(dp == -1)
    # no left keypoints: the Frame constructor returns before ComputeStereoMatches
    ur, dp, good = orbx.compute_stereo_matches(exl, exr, kl[:0], None, kr, dr, EUROC_BF, EUROC_FX)
    assert good == 0 and len(ur) == 0
    # geometry mismatch between the two handles is refused
    exo = orbx.ORBextractor(300, 1.2, 8, 20, 7)
    import orbx_synth
    exo(orbx_synth.gen_image(9, 400, 300))
    with pytest.raises(orbx.OrbxError):
        orbx.compute_stereo_matches(exl, exo, kl, dl, kl, dl, EUROC_BF, EUROC_FX)


# ------------------------------------------- orbm_stereo_band (the coarse stage alone)


def py_band(kL, dL, kR, dR, rows, scale, minD, maxD):
    """src/Frame.cc:645-757 restated with Python lists: vRowIndices, then the first strict minimum."""
    S = [F32(s) for s in scale]
    rowidx = [[] for _ in range(rows)]
    for iR in range(len(kR)):
        y, r = F32(kR["y"][iR]), F32(2.0) * S[kR["octave"][iR]]
        for yi in range(int(np.floor(F32(y - r))), int(np.ceil(F32(y + r))) + 1):
            if 0 <= yi < rows:
                rowidx[yi].append(iR)
    ham = lambda a, b: int(np.unpackbits(np.bitwise_xor(a, b)).sum())
    bi, bd = np.full(len(kL), -1), np.full(len(kL), 100)
    for iL in range(len(kL)):
        vL, uL, lv = F32(kL["y"][iL]), F32(kL["x"][iL]), int(kL["octave"][iL])
        if vL < 0 or int(vL) >= rows:
            continue
        minU, maxU = F32(uL - F32(maxD)), F32(uL - F32(minD))
        if maxU < 0:
            continue
        best, idx = 100, -1
        for iR in rowidx[int(vL)]:
            o = int(kR["octave"][iR])
            if lv - 1 <= o <= lv + 1 and minU <= F32(kR["x"][iR]) <= maxU:
                d = ham(dL[iL], dR[iR])
                if d < best:
                    best, idx = d, iR
        bi[iL], bd[iL] = idx, best
    return bi, bd


def band_case(seed, nl, nr, rows=240, cols=320, nlevels=8):
    """Keypoints on and beyond the image rows, descriptors from 6 prototypes (many equal distances)."""
    from orbref import KEYPOINT_DTYPE
    rng = np.random.default_rng(seed)
    proto = rng.integers(0, 256, (6, 32), dtype=np.uint8)

    def side(n):
        k = np.zeros(n, KEYPOINT_DTYPE)
        k["x"] = rng.uniform(-2, cols, n)
        k["y"] = rng.uniform(-3, rows + 3, n)
        k["octave"] = rng.integers(0, nlevels, n)
        bits = np.unpackbits(proto[rng.integers(0, 6, n)], axis=1) ^ (rng.random((n, 256)) < 0.03)
        return k, np.packbits(bits, axis=1)
    (kl, dl), (kr, dr) = side(nl), side(nr)
    m = min(nl, nr) // 8
    kr["y"][:m] = kl["y"][:m]                        # shared rows
    dr[m: 2 * m] = dr[:m]                            # duplicate descriptors: ties broken by index
    return kl, dl, kr, dr, [1.2 ** l for l in range(nlevels)]


@pytest.mark.parametrize("seed", [0, 1])
def test_band_oracle_matches_restatement(orbref, seed):
    kl, dl, kr, dr, sc = band_case(seed, 400, 500)
    maxD = EUROC_BF / (EUROC_BF / EUROC_FX)
    got = orbref.stereo_band(kl, dl, kr, dr, 240, sc, 0.0, maxD)
    want = py_band(kl, dl, kr, dr, 240, sc, 0.0, maxD)
    assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1])
    assert (got[0] >= 0).sum() > 100 and (got[0] == -1).sum() > 10
    # a narrow disparity range prunes candidates
    narrow = orbref.stereo_band(kl, dl, kr, dr, 240, sc, 5.0, 40.0)
    assert np.array_equal(narrow[1], py_band(kl, dl, kr, dr, 240, sc, 5.0, 40.0)[1])
    assert (narrow[0] >= 0).sum() < (got[0] >= 0).sum()


def test_band_agrees_with_full_stereo(orbref):
    """Every pair the full ComputeStereoMatches keeps went through a coarse best below thOrbDist."""
    L, R = _pair(3, 320, 240)
    p = orbref.make_params(300, 1.2, 8, 20, 7)
    a, b = orbref.extract(L, p), orbref.extract(R, p)
    t = orbref.tables(p)
    sc = [t.scale[l] for l in range(8)]
    mb = np.float32(np.float32(EUROC_BF) / np.float32(EUROC_FX))
    maxD = float(np.float32(np.float32(EUROC_BF) / mb))
    bi, bd = orbref.stereo_band(a.keypoints, a.descriptors, b.keypoints, b.descriptors, 240, sc, 0.0, maxD)
    ur, _, _, good = orbref.compute_stereo_matches(p, a, b, 240, 320, EUROC_BF, EUROC_FX)
    assert good > 20 and np.all(bd[ur >= 0] < 75) and np.all(bi[ur >= 0] >= 0)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [2, 3])
def test_gpu_stereo_band(orbref, cuda, seed):
    import orbx
    kl, dl, kr, dr, sc = band_case(seed, 3000, 2500, rows=480, cols=752)
    for lo, hi in ((0.0, 110.0), (3.0, 30.0)):
        got = orbx.stereo_band(kl, dl, kr, dr, 480, sc, lo, hi)
        want = orbref.stereo_band(kl, dl, kr, dr, 480, sc, lo, hi)
        assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1])
    # empty sides
    bi, bd = orbx.stereo_band(kl, dl, kr[:0], dr[:0], 480, sc, 0.0, 110.0)
    assert np.all(bi == -1) and np.all(bd == 100)
    assert len(orbx.stereo_band(kl[:0], dl[:0], kr, dr, 480, sc, 0.0, 110.0)[0]) == 0
    bad = kr.copy()
    bad["octave"][0] = 8
    with pytest.raises(orbx.OrbxError):
        orbx.stereo_band(kl, dl, bad, dr, 480, sc, 0.0, 110.0)


@pytest.mark.gpu
def test_gpu_stereo_band_batch(orbref, cuda):
    import torch
    import orbx
    W, H, nfeat = 752, 480, 1000
    pairs = [_pair(s, W, H) for s in (3, 4)]
    frames = np.stack([im for pr in pairs for im in pr])
    ex = orbx.ORBextractor(nfeat, 1.2, 8, 20, 7)
    cap = ex.capacity(H, W)
    kps = torch.empty((4, cap, 7), dtype=torch.int32, device=cuda)
    desc = torch.empty((4, cap, 32), dtype=torch.uint8, device=cuda)
    counts = torch.empty((4,), dtype=torch.int32, device=cuda)
    ex.extract_batch_device(torch.from_numpy(frames).to(cuda), kps, desc, counts)
    p = orbref.make_params(nfeat, 1.2, 8, 20, 7)
    t = orbref.tables(p)
    sc = [t.scale[l] for l in range(8)]
    bi, bd = orbx.stereo_band_batch_device(kps, desc, counts, [0, 2], [1, 3], H, sc, 0.0, 110.0)
    torch.cuda.synchronize()
    c = counts.cpu().numpy()
    for k, (L, R) in enumerate(pairs):
        a, b = orbref.extract(L, p), orbref.extract(R, p)
        wi, wd = orbref.stereo_band(a.keypoints, a.descriptors, b.keypoints, b.descriptors, H, sc, 0.0, 110.0)
        n = c[2 * k]
        assert n == len(a.keypoints)
        assert np.array_equal(bi[k, :n].cpu().numpy(), wi) and np.array_equal(bd[k, :n].cpu().numpy(), wd)


@pytest.mark.gpu
def test_gpu_batch_stereo_cross_stream_then_next_batch(orbref, cuda):
    """Stereo on stream B (behind a long kernel) reads the handle's pyramids; the next batch on stream A
    rewrites them.  The extractor orders the next batch after the stereo search (orbx_stereo_batch_device
    marks itself as the handle's last work), so stereo still sees the first batch's pyramids."""
    import torch
    import orbx
    W, H, nfeat = 752, 480, 1000
    pairs = [_pair(s, W, H) for s in (3, 4)]
    frames = np.stack([im for pr in pairs for im in pr])
    other = np.stack([_pair(s, W, H)[k] for s in (8, 9) for k in (0, 1)])
    ex = orbx.ORBextractor(nfeat, 1.2, 8, 20, 7)
    A = torch.cuda.current_stream()
    Bs = torch.cuda.Stream(device=cuda)
    imgs = torch.from_numpy(frames).to(cuda)
    imgs2 = torch.from_numpy(other).to(cuda)
    cap = ex.capacity(H, W)
    bufs = [(torch.empty((4, cap, 7), dtype=torch.int32, device=cuda), torch.empty((4, cap, 32), dtype=torch.uint8,
             device=cuda), torch.empty((4,), dtype=torch.int32, device=cuda)) for _ in range(2)]
    li = torch.tensor([0, 2], dtype=torch.int32, device=cuda)
    ri = torch.tensor([1, 3], dtype=torch.int32, device=cuda)
    torch.cuda.synchronize()
    ex.extract_batch_device(imgs, *bufs[0], stream=A)
    with torch.cuda.stream(Bs):
        torch.cuda._sleep(200_000_000)   # ~0.1 s: the stereo search is still queued when batch 2 is issued
        ur, dp, ng = ex.stereo_batch_device(*bufs[0], li, ri, EUROC_BF, EUROC_FX, stream=Bs)
    ex.extract_batch_device(imgs2, *bufs[1], stream=A)
    torch.cuda.synchronize()
    p = orbref.make_params(nfeat, 1.2, 8, 20, 7)
    for k, (L, R) in enumerate(pairs):
        a, b = orbref.extract(L, p), orbref.extract(R, p)
        wur, wdp, _, wgood = orbref.compute_stereo_matches(p, a, b, H, W, EUROC_BF, EUROC_FX)
        n = len(a.keypoints)
        assert int(ng[k].item()) == wgood and wgood > 0
        assert np.array_equal(ur[k, :n].cpu().numpy(), wur)
        assert np.array_equal(dp[k, :n].cpu().numpy(), wdp)
    klist = orbx.keypoints_from_device(bufs[1][0], bufs[1][2])
    for f in range(4):
        ref = orbref.extract(other[f], p, want_pyramid=False)
        for fld in ("x", "y", "octave", "response"):
            assert np.array_equal(klist[f][fld], ref.keypoints[fld]), (f, fld)
