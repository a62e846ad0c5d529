"""GPU (gfx950) vs CPU oracle parity through the C ABI (liborbx.so).

Bar: bit-exact for pyramid bytes, FAST candidates, keypoint x/y/size/response/
octave/class_id, keypoint order and BRIEF bits; |angle difference| <= 1e-4
degrees (the north-star tolerance; expected to be exact).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ANGLE_TOL = 1e-4


def _extractor(nfeat, scale=1.2, nlevels=8, ini=20, mn=7):
    import orbx
    return orbx.ORBextractor(nfeat, scale, nlevels, ini, mn)


def _run_batch(ex, frames, cuda):
    import torch
    import orbx
    imgs = torch.from_numpy(np.ascontiguousarray(frames)).to(cuda)
    B, H, W = imgs.shape
    cap = ex.capacity(H, W)
    kps = torch.empty((B, cap, 7), dtype=torch.int32, device=cuda)
    desc = torch.empty((B, cap, 32), dtype=torch.uint8, device=cuda)
    counts = torch.empty((B,), dtype=torch.int32, device=cuda)
    ex.extract_batch_device(imgs, kps, desc, counts)
    ex.sync(torch.cuda.current_stream())
    klist = orbx.keypoints_from_device(kps, counts)
    d = desc.cpu().numpy()
    c = counts.cpu().numpy()
    return imgs, kps, desc, counts, klist, [d[f, :c[f]] for f in range(B)]


def assert_same_keypoints(got, want, got_desc, want_desc, tag=""):
    assert len(got) == len(want), "%s: %d keypoints vs oracle %d" % (tag, len(got), len(want))
    for field in ("x", "y", "size", "response", "octave", "class_id"):
        bad = np.nonzero(got[field] != want[field])[0]
        assert bad.size == 0, "%s: field %s differs at %s (gpu %s, oracle %s)" % (
            tag, field, bad[:5], got[field][bad[:5]], want[field][bad[:5]])
    da = np.abs(got["angle"].astype(np.float64) - want["angle"].astype(np.float64))
    assert da.max(initial=0.0) <= ANGLE_TOL, "%s: angle max diff %g at %d" % (tag, da.max(), int(da.argmax()))
    bad = np.nonzero((got_desc != want_desc).any(axis=1))[0]
    assert bad.size == 0, "%s: %d descriptors differ, first %s" % (tag, bad.size, bad[:5])


CONFIGS = [
    # (name, W, H, nfeatures, frames)
    ("tum640", 640, 480, 1000, "gen"),
    ("kitti", 1241, 376, 2000, "kitti"),
    ("euroc", 752, 480, 1000, "gen"),
    ("small", 320, 240, 300, "gen"),
    ("kitti_init2x", 1241, 376, 4000, "kitti"),
    ("hd1080", 1920, 1080, 4000, "gen"),   # config 5; quadtree levels 0 and 2+ overflow their registers
    # uniform noise: ~35% of level-0 pixels are FAST corners at minThFAST, so cells outgrow the
    # 376-entry candidate list and take the whole-window NMS path (csrc/orbx_extract.hip, K2)
    ("noise640", 640, 480, 1000, "noise"),
]


def _frames(kind, W, H, n, seed0=1):
    import orbx_synth
    if kind == "kitti":
        return orbx_synth.kitti_sequence(n, start=seed0 * 7)
    if kind == "noise":
        return np.random.default_rng(seed0).integers(0, 256, (n, H, W), dtype=np.uint8)
    return np.stack([orbx_synth.gen_image(seed0 + i, W, H) for i in range(n)])


@pytest.mark.parametrize("name,W,H,nfeat,kind", CONFIGS)
def test_extract_parity(orbref, cuda, name, W, H, nfeat, kind):
    frames = _frames(kind, W, H, 2)
    ex = _extractor(nfeat)
    p = orbref.make_params(nfeat, 1.2, 8, 20, 7)
    sizes = orbref.level_sizes(p, W, H)
    _, _, _, _, klist, dlist = _run_batch(ex, frames, cuda)
    for f in range(len(frames)):
        ref = orbref.extract(frames[f], p)
        # stage 1: pyramid bytes
        pyr = ex.debug_pyramid(f, sizes)
        for l, (a, b) in enumerate(zip(pyr, ref.pyramid)):
            bad = np.argwhere(a != b)
            assert bad.size == 0, "%s f%d pyramid level %d differs at %s" % (name, f, l, bad[:3])
        # stage 2: FAST candidates per level, reference order
        for l in range(8):
            want = orbref.level_candidates(ref.pyramid[l])
            got = ex.debug_candidates(f, l)
            assert len(got) == len(want), "%s f%d level %d: %d candidates vs %d" % (name, f, l, len(got), len(want))
            assert np.array_equal(got, want), "%s f%d level %d candidates differ" % (name, f, l)
        # stage 3+4: final keypoints and descriptors
        assert len(ref.keypoints) >= 0.5 * nfeat,"%s: oracle kept only %d keypoints" % (name, len(ref.keypoints))
        assert_same_keypoints(klist[f], ref.keypoints, dlist[f], ref.descriptors, "%s f%d" % (name, f))


@pytest.mark.parametrize("W,H", [(642, 480), (643, 481), (1243, 377)])
@pytest.mark.parametrize("batch", [2, 10])
def test_extract_parity_row_alignments(orbref, cuda, W, H, batch):
    """Frames whose rows start at every byte alignment mod 4 (widths 642 / 643 / 1243 besides the suite's 640 and
    1241): describe's per-row-shift horizontal pass, FAST's unaligned ROI loads and the level-1 pyramid's
    unaligned source rows, for the small-batch (2 frames: one keypoint and one cell per wave, fused pyramid) and
    the large-batch (10 frames: four keypoints and three cells per wave, one launch per level) kernels."""
    frames = _frames("gen", W, H, batch, seed0=31)
    ex = _extractor(1000)
    p = orbref.make_params(1000, 1.2, 8, 20, 7)
    _, _, _, _, klist, dlist = _run_batch(ex, frames, cuda)
    for f in range(batch):
        ref = orbref.extract(frames[f], p)
        assert len(ref.keypoints) >= 500
        assert_same_keypoints(klist[f], ref.keypoints, dlist[f], ref.descriptors, "%dx%d b%d f%d" % (W, H, batch, f))


def test_host_api_matches_batch(orbref, cuda):
    import orbx_synth
    img = orbx_synth.gen_image(11, 640, 480)
    ex = _extractor(1000)
    kps, desc = ex(img)
    p = orbref.make_params(1000, 1.2, 8, 20, 7)
    ref = orbref.extract(img, p)
    assert_same_keypoints(kps, ref.keypoints, desc, ref.descriptors, "host api")
    pyr = ex.mvImagePyramid
    for l in range(8):
        assert np.array_equal(pyr[l], ref.pyramid[l])
    assert np.allclose(ex.GetScaleFactors(), orbref.tables(p).scale[:8])


def test_empty_and_flat_images(orbref, cuda):
    ex = _extractor(500)
    kps, desc = ex(np.zeros((0, 0), np.uint8))
    assert len(kps) == 0 and desc is None
    flat = np.full((240, 320), 77, np.uint8)
    kps, desc = ex(flat)
    ref = orbref.extract(flat, orbref.make_params(500, 1.2, 8, 20, 7))
    assert len(kps) == len(ref.keypoints) == 0
    # half flat / half textured: some cells fall back to minThFAST, some find nothing
    import orbx_synth
    img = orbx_synth.gen_image(5, 320, 240)
    img[:, :160] = 90
    img[:120, :160] += (np.arange(160) % 2 * 9).astype(np.uint8)[None, :]
    kps, desc = ex(img)
    ref = orbref.extract(img, orbref.make_params(500, 1.2, 8, 20, 7))
    assert_same_keypoints(kps, ref.keypoints, desc, ref.descriptors, "half flat")


def test_other_params(orbref, cuda):
    import orbx_synth
    img = orbx_synth.gen_image(21, 752, 480)
    for nfeat, scale, nl, ini, mn in [(1200, 1.2, 8, 20, 7), (500, 1.3, 6, 25, 10), (150, 1.2, 4, 12, 5)]:
        ex = _extractor(nfeat, scale, nl, ini, mn)
        kps, desc = ex(img)
        ref = orbref.extract(img, orbref.make_params(nfeat, scale, nl, ini, mn))
        assert_same_keypoints(kps, ref.keypoints, desc, ref.descriptors, "params %s" % ((nfeat, scale, nl),))


def test_host_graph_recapture_and_direct_launches(orbref, cuda):
    """The host path replays a captured hipGraph per handle (orbx_api.hip orbx_extract).  Alternating image
    sizes on one handle re-captures it (buffers and launch shapes change), a strided image goes through the
    same staging, and ORBX_NO_GRAPH=1 (direct launches) gives identical results."""
    import os
    import orbx_synth
    ex = _extractor(1000)
    p = orbref.make_params(1000, 1.2, 8, 20, 7)
    imgs = [orbx_synth.gen_image(31, 640, 480), orbx_synth.gen_image(32, 320, 240),
            orbx_synth.gen_image(33, 752, 480)]
    refs = [orbref.extract(im, p, want_pyramid=False) for im in imgs]
    for rnd in range(2):
        for i in (0, 1, 2, 0):
            kps, desc = ex(imgs[i])
            assert_same_keypoints(kps, refs[i].keypoints, desc, refs[i].descriptors, "graph rnd%d img%d" % (rnd, i))
    wide = np.zeros((480, 700), np.uint8)
    wide[:, 30:670] = imgs[0]
    view = wide[:, 30:670]   # step 700, not contiguous
    kps, desc = ex(view)
    assert_same_keypoints(kps, refs[0].keypoints, desc, refs[0].descriptors, "strided")
    os.environ["ORBX_NO_GRAPH"] = "1"
    try:
        for i in (2, 0):
            kps, desc = ex(imgs[i])
            assert_same_keypoints(kps, refs[i].keypoints, desc, refs[i].descriptors, "direct img%d" % i)
    finally:
        del os.environ["ORBX_NO_GRAPH"]


def test_pyramid_without_byte_window(orbref, cuda):
    """Scale factors above ~2.3 put a 4-column group's taps more than 8 bytes apart, so the pyramid kernel
    takes its per-byte path instead of the byte window (LevelGeom::pyr_win)."""
    import orbx_synth
    img = orbx_synth.gen_image(41, 640, 480)
    for scale, nl in [(2.5, 2), (2.0, 3)]:
        ex = _extractor(600, scale, nl, 20, 7)
        kps, desc = ex(img)
        ref = orbref.extract(img, orbref.make_params(600, scale, nl, 20, 7))
        assert_same_keypoints(kps, ref.keypoints, desc, ref.descriptors, "scale %.1f" % scale)
        for l in range(nl):
            assert np.array_equal(ex.mvImagePyramid[l], ref.pyramid[l]), "scale %.1f level %d" % (scale, l)


def test_search_for_initialization(orbref, cuda):
    import torch
    import orbx
    frames = _frames("kitti", 1241, 376, 4)
    ex = _extractor(2000)
    imgs, kps, desc, counts, klist, dlist = _run_batch(ex, frames, cuda)
    pa = torch.tensor([0, 1, 2, 0], dtype=torch.int32, device=cuda)
    pb = torch.tensor([1, 2, 3, 3], dtype=torch.int32, device=cuda)
    m = orbx.ORBmatcher(0.9, True)
    m12, nm = m.search_for_initialization_batch(kps, desc, counts, pa, pb, 376, 1241, 100)
    torch.cuda.synchronize()
    m12 = m12.cpu().numpy()
    nm = nm.cpu().numpy()
    for p, (a, b) in enumerate(zip(pa.tolist(), pb.tolist())):
        want_n, want_m, _ = orbref.search_for_initialization(klist[a], dlist[a], klist[b], dlist[b], 1241, 376,
                                                             window=100, nnratio=0.9, check_ori=True)
        got = m12[p, :len(klist[a])]
        assert nm[p] == want_n, "pair %d: %d matches vs oracle %d" % (p, nm[p], want_n)
        assert np.array_equal(got, want_m), "pair %d: match vectors differ at %s" % (p, np.nonzero(got != want_m)[0][:5])
    assert nm[0] > 50


@pytest.mark.parametrize("seed,noise,nproto", [(1, 0.02, 40), (2, 0.06, 25), (3, 0.10, 12), (4, 0.04, 4)])
def test_search_for_initialization_contended(orbref, cuda, seed, noise, nproto):
    """Adversarial SearchForInitialization: descriptors are noisy copies of a few
    prototypes, so windows hold many candidates within TH_LOW of each other.  This
    drives evictions, ratio-test near-ties, targets re-matched inside one 64-step
    chunk, and steps whose top-4 cannot settle them (the full-window scan)."""
    import torch
    import orbx
    rng = np.random.default_rng(seed)
    W, H, n = 1241, 376, 600
    cap = 640
    proto = rng.integers(0, 256, (nproto, 32), dtype=np.uint8)
    kl, dl = [], []
    for f in range(2):
        k = np.zeros(n, orbref.KEYPOINT_DTYPE)
        k["x"] = rng.uniform(20, W - 20, n).astype(np.float32)
        k["y"] = rng.uniform(20, H - 20, n).astype(np.float32)
        k["size"] = 31
        k["angle"] = rng.uniform(0, 360, n).astype(np.float32)
        k["response"] = rng.integers(1, 80, n).astype(np.float32)
        k["class_id"] = -1
        bits = (rng.random((n, 256)) < noise).astype(np.uint8)
        d = proto[rng.integers(0, nproto, n)] ^ np.packbits(bits, axis=1, bitorder="little")
        kl.append(k)
        dl.append(d)
    kps = np.zeros((2, cap, 7), np.int32)
    desc = np.zeros((2, cap, 32), np.uint8)
    for f in range(2):
        kps[f, :n] = kl[f].view(np.int32).reshape(n, 7)
        desc[f, :n] = dl[f]
    tk, td = torch.from_numpy(kps).to(cuda), torch.from_numpy(desc).to(cuda)
    tc = torch.tensor([n, n], dtype=torch.int32, device=cuda)
    pa = torch.tensor([0, 1], dtype=torch.int32, device=cuda)
    pb = torch.tensor([1, 0], dtype=torch.int32, device=cuda)
    for check_ori in (True, False):
        m = orbx.ORBmatcher(0.9, check_ori)
        m12, nm = m.search_for_initialization_batch(tk, td, tc, pa, pb, H, W, 100)
        torch.cuda.synchronize()
        m12, nm = m12.cpu().numpy(), nm.cpu().numpy()
        for p, (a, b) in enumerate([(0, 1), (1, 0)]):
            want_n, want_m, _ = orbref.search_for_initialization(kl[a], dl[a], kl[b], dl[b], W, H, window=100,
                                                                 nnratio=0.9, check_ori=check_ori)
            assert nm[p] == want_n, "pair %d ori %d: %d matches vs oracle %d" % (p, check_ori, nm[p], want_n)
            assert np.array_equal(m12[p, :n], want_m), "pair %d ori %d differ at %s" % (
                p, check_ori, np.nonzero(m12[p, :n] != want_m)[0][:5])
            assert want_n > 0


@pytest.mark.parametrize("nq,nt", [(1000, 777), (257, 5000), (10000, 1024), (300, 2056)])
def test_allpairs(orbref, cuda, nq, nt):
    import torch
    import orbx
    import orbx_synth
    q = orbx_synth.random_descriptors(nq, 55)
    t = orbx_synth.random_descriptors(nt, 56)
    t[:min(nq, nt) // 10] = q[:min(nq, nt) // 10] ^ (np.random.default_rng(1).random((min(nq, nt) // 10, 32)) < 0.03)
    dq, dt = torch.from_numpy(q).to(cuda), torch.from_numpy(t).to(cuda)
    bi, b1, b2 = orbx.allpairs(dq, dt, orbx.TOP2)
    full = orbx.allpairs(dq, dt, orbx.FULL_U16)
    torch.cuda.synchronize()
    # reference: popcount of xor
    x = np.unpackbits(q[:, None, :] ^ t[None, :, :], axis=2).sum(axis=2) if nq * nt <= 4_000_000 else None
    sel = np.arange(0, nq, max(1, nq // 300))
    if x is not None:
        assert np.array_equal(full.cpu().numpy().astype(np.int64), x)
    else:   # sampled rows of the large matrix
        xs = np.unpackbits(q[sel, None, :] ^ t[None, :, :], axis=2).sum(axis=2)
        assert np.array_equal(full.cpu().numpy()[sel].astype(np.int64), xs)
    wi, w1, w2 = orbref.allpairs_top2(q[sel], t)
    assert np.array_equal(bi.cpu().numpy()[sel], wi)
    assert np.array_equal(b1.cpu().numpy()[sel], w1)
    assert np.array_equal(b2.cpu().numpy()[sel], w2)


def test_extract_then_match_same_stream_without_host_sync(orbref, cuda):
    """Regression: extract and match queued back to back on one stream (the bench
    pattern) must give the same matches as with a host sync in between."""
    import torch
    import orbx
    frames = _frames("kitti", 1241, 376, 3)
    ex = _extractor(2000)
    imgs = torch.from_numpy(frames).to(cuda)
    cap = ex.capacity(376, 1241)
    m = orbx.ORBmatcher(0.9, True)
    pa = torch.tensor([0, 1], dtype=torch.int32, device=cuda)
    pb = torch.tensor([1, 2], dtype=torch.int32, device=cuda)
    outs = []
    for s in (torch.cuda.current_stream(), torch.cuda.Stream()):
        with torch.cuda.stream(s):
            kps = torch.empty((3, cap, 7), dtype=torch.int32, device=cuda)
            desc = torch.empty((3, cap, 32), dtype=torch.uint8, device=cuda)
            counts = torch.empty((3,), dtype=torch.int32, device=cuda)
            ex.extract_batch_device(imgs, kps, desc, counts, s)
            m12, nm = m.search_for_initialization_batch(kps, desc, counts, pa, pb, 376, 1241, 100, stream=s)
            s.synchronize()
            outs.append((m12.cpu().numpy(), nm.cpu().numpy()))
    klist = orbx.keypoints_from_device(kps, counts)
    d = desc.cpu().numpy()
    c = counts.cpu().numpy()
    want_n, want_m, _ = orbref.search_for_initialization(klist[0], d[0, :c[0]], klist[1], d[1, :c[1]], 1241, 376)
    for m12, nm in outs:
        assert nm[0] == want_n and want_n > 50
        assert np.array_equal(m12[0, :len(want_m)], want_m)


def test_cpp_mirror_example(orbref, cuda, tmp_path):
    """The C++ ORBextractor mirror (orb-slam-_amd/host/ORBextractor.hpp) end to end."""
    import os
    import subprocess
    import orbx_synth
    from orbref import KEYPOINT_DTYPE
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "orb-slam-_amd", "build", "extract_example")
    img = orbx_synth.gen_image(31, 752, 480)
    src = tmp_path / "in.raw"
    out = tmp_path / "out.bin"
    img.tofile(src)
    subprocess.check_call([exe, str(src), "480", "752", "1000", str(out)], timeout=120)
    raw = out.read_bytes()
    n = int(np.frombuffer(raw[:4], np.int32)[0])
    kps = np.frombuffer(raw[4:4 + 28 * n], KEYPOINT_DTYPE)
    desc = np.frombuffer(raw[4 + 28 * n:], np.uint8).reshape(n, 32)
    ref = orbref.extract(img, orbref.make_params(1000, 1.2, 8, 20, 7))
    assert_same_keypoints(kps, ref.keypoints, desc, ref.descriptors, "c++ mirror")


def test_allpairs_config5_full_size(orbref, cuda):
    """Config 5 at its stated size: 10,000 x 10,000 brute-force 256-bit Hamming.  TOP2 (best index,
    best and second distance, first-min tie rule) on EVERY query against the oracle's scalar loop
    (10^8 pairs), through both the device and the host entry points; the FULL_U16 matrix on 500
    sampled rows (10,000 columns each) against numpy popcount, plus a checksum of every row's sum."""
    import torch
    import orbx
    import orbx_synth
    n = 10000
    q = orbx_synth.random_descriptors(n, 501)
    t = orbx_synth.random_descriptors(n, 502)
    rng = np.random.default_rng(5)
    near = rng.choice(n, n // 10, replace=False)   # 10% of targets are noisy copies of queries: real minima
    t[near] = q[near] ^ np.packbits(rng.random((n // 10, 256)) < 0.05, axis=1)
    t[7] = t[3]                                    # exact duplicate targets: first-min tie rule
    wi, w1, w2 = orbref.allpairs_top2(q, t)
    dq, dt = torch.from_numpy(q).to(cuda), torch.from_numpy(t).to(cuda)
    bi, b1, b2 = orbx.allpairs(dq, dt, orbx.TOP2)
    torch.cuda.synchronize()
    assert np.array_equal(bi.cpu().numpy(), wi)
    assert np.array_equal(b1.cpu().numpy(), w1)
    assert np.array_equal(b2.cpu().numpy(), w2)
    hi, h1, h2 = orbx.allpairs_host(q, t)
    assert np.array_equal(hi, wi) and np.array_equal(h1, w1) and np.array_equal(h2, w2)
    full = orbx.allpairs(dq, dt, orbx.FULL_U16)
    rows = full.sum(dim=1, dtype=torch.int64).cpu().numpy()
    torch.cuda.synchronize()
    sel = np.sort(rng.choice(n, 500, replace=False))
    got = full[torch.from_numpy(sel).to(cuda)].cpu().numpy().view(np.uint16).astype(np.int64)
    pop = np.array([bin(i).count("1") for i in range(256)], np.uint8)
    for c in range(0, len(sel), 100):   # popcount LUT in 100-row chunks (160 MB of xor at a time)
        want = pop[q[sel[c:c + 100], None, :] ^ t[None, :, :]].sum(axis=2, dtype=np.int64)
        assert np.array_equal(got[c:c + 100], want)
    # every row: sum of its distances = sum over targets of popcount(q ^ t), computed bit-plane-wise
    qb = np.unpackbits(q, axis=1).astype(np.int64)               # (n, 256)
    tb = np.unpackbits(t, axis=1).astype(np.int64).sum(axis=0)   # ones per bit position over targets
    want_rows = (qb * (n - tb) + (1 - qb) * tb).sum(axis=1)
    assert np.array_equal(rows, want_rows)
    assert (wi >= 0).all() and w1[near].max() <= 40


def test_stage_times_cover_host_calls(orbref, cuda):
    """orbx_set_timing then host-path extracts (orbx_extract, which otherwise replays a captured graph):
    stage_times sums their stage events, and the timed calls still give the oracle's result."""
    import orbx_synth
    ex = _extractor(1000)
    img = orbx_synth.gen_image(12, 640, 480)
    ex(img)   # the graph path, untimed
    ex.set_timing(True)
    ref = orbref.extract(img, orbref.make_params(1000, 1.2, 8, 20, 7), want_pyramid=False)
    for _ in range(3):
        kps, desc = ex(img)
        assert_same_keypoints(kps, ref.keypoints, desc, ref.descriptors, "timed host call")
    ms = ex.stage_times()
    assert ms.shape == (4,) and (ms > 0).all() and ms.sum() < 1000, ms
    ex.set_timing(False)
    kps, desc = ex(img)   # back on the graph
    assert_same_keypoints(kps, ref.keypoints, desc, ref.descriptors, "untimed again")


def test_size_switch_while_a_batch_is_queued(orbref, cuda):
    """A batch at one size queued behind a long kernel on a side stream, then capacity() and a host-path
    extract at another size on the same handle, then a second batch at the first size on the default stream.
    The geometry tables of each size are separate device blocks (a switch never rewrites tables queued
    kernels read), and a call on another stream waits for the handle's last call (the workspace is shared),
    so every result equals the oracle's."""
    import torch
    import orbx
    import orbx_synth
    ex = _extractor(2000)
    kitti = orbx_synth.kitti_sequence(4, start=3)
    B, H, W = kitti.shape
    imgs = torch.from_numpy(np.ascontiguousarray(kitti)).to(cuda)
    cap = ex.capacity(H, W)
    side = torch.cuda.Stream(device=cuda)
    outs = []
    for _ in range(2):
        outs.append((torch.empty((B, cap, 7), dtype=torch.int32, device=cuda),
                     torch.empty((B, cap, 32), dtype=torch.uint8, device=cuda),
                     torch.empty((B,), dtype=torch.int32, device=cuda)))
    torch.cuda.synchronize()
    with torch.cuda.stream(side):
        torch.cuda._sleep(200_000_000)   # ~0.1 s: the batch is still queued when the host calls run
        ex.extract_batch_device(imgs, *outs[0], stream=side)
    small = orbx_synth.gen_image(5, 640, 480)
    assert ex.capacity(480, 640) > 0
    kps_s, desc_s = ex(small)
    ex.extract_batch_device(imgs, *outs[1])   # back to the first size, on the default stream
    torch.cuda.synchronize()
    p = orbref.make_params(2000, 1.2, 8, 20, 7)
    ref_s = orbref.extract(small, p, want_pyramid=False)
    assert_same_keypoints(kps_s, ref_s.keypoints, desc_s, ref_s.descriptors, "host call at 640x480")
    refs = [orbref.extract(kitti[f], p, want_pyramid=False) for f in range(B)]
    for r, (kps, desc, counts) in enumerate(outs):
        klist = orbx.keypoints_from_device(kps, counts)
        d = desc.cpu().numpy()
        for f in range(B):
            n = len(refs[f].keypoints)
            assert_same_keypoints(klist[f], refs[f].keypoints, d[f, :n], refs[f].descriptors, "batch %d frame %d" % (r, f))


def test_stage_times_cover_stage_split_calls(orbref, cuda):
    """Stage-split extraction (orbx_extract_stage_device) on a timed handle: each stage is timed on its
    own stream and stage_times() includes it."""
    import torch
    import orbx
    import orbx_synth
    ex = _extractor(2000)
    kitti = orbx_synth.kitti_sequence(2, start=7)
    B, H, W = kitti.shape
    imgs = torch.from_numpy(np.ascontiguousarray(kitti)).to(cuda)
    cap = ex.capacity(H, W)
    kps = torch.empty((B, cap, 7), dtype=torch.int32, device=cuda)
    desc = torch.empty((B, cap, 32), dtype=torch.uint8, device=cuda)
    counts = torch.empty((B,), dtype=torch.int32, device=cuda)
    ex.set_timing(True)
    for stage in range(4):
        ex.extract_stage_device(stage, imgs, kps, desc, counts)
    ex.sync(torch.cuda.current_stream())
    ms = ex.stage_times()
    assert ms.shape == (4,) and (ms > 0).all() and ms.sum() < 1000, ms
    ex.set_timing(False)
    klist = orbx.keypoints_from_device(kps, counts)
    d = desc.cpu().numpy()
    p = orbref.make_params(2000, 1.2, 8, 20, 7)
    for f in range(B):
        ref = orbref.extract(kitti[f], p, want_pyramid=False)
        n = len(ref.keypoints)
        assert_same_keypoints(klist[f], ref.keypoints, d[f, :n], ref.descriptors, "stage-split frame %d" % f)


@pytest.mark.parametrize("kind,W,H,nfeat", [("noise", 640, 480, 1000), ("kitti", 1241, 376, 2000)])
def test_candidates_multi_cell_waves(orbref, cuda, kind, W, H, nfeat):
    """Batches above kLatencyMaxBatch run kCellsPerWave (3) FAST cells per wave: the wave's buffered run from
    its first cell's slot base, cells written at their own base after a buffer overflow (kCellDirect; uniform
    noise overflows it), and the run decoding of orbx_debug_candidates.  Candidates per level, reference order."""
    frames = _frames(kind, W, H, 10, seed0=3)
    if kind == "noise":   # mixed batch: noise frames overflow the wave buffers, textured ones do not
        import orbx_synth
        frames[5:] = np.stack([orbx_synth.gen_image(50 + i, W, H) for i in range(5)])
    ex = _extractor(nfeat)
    p = orbref.make_params(nfeat, 1.2, 8, 20, 7)
    _, _, _, _, klist, dlist = _run_batch(ex, frames, cuda)
    for f in (0, 4, 5, 9):
        ref = orbref.extract(frames[f], p)
        for l in range(8):
            want = orbref.level_candidates(ref.pyramid[l])
            got = ex.debug_candidates(f, l)
            assert len(got) == len(want), "%s f%d level %d: %d candidates vs %d" % (kind, f, l, len(got), len(want))
            assert np.array_equal(got, want), "%s f%d level %d candidates differ" % (kind, f, l)
        assert_same_keypoints(klist[f], ref.keypoints, dlist[f], ref.descriptors, "%s f%d" % (kind, f))


def test_pyramid_per_level_launches_small_batch(orbref, cuda):
    """ORBX_PYR_FUSED=0 (read when a handle first sees an image size): small batches take the per-level pyramid
    launches of large batches instead of the fused groups (k_pyramid_fused).  Both settings are the oracle's
    bytes; this is the library's only runtime kernel switch besides ORBX_NO_GRAPH."""
    import os
    import orbx_synth
    img = orbx_synth.gen_image(61, 640, 480)
    p = orbref.make_params(1000, 1.2, 8, 20, 7)
    ref = orbref.extract(img, p)
    for setting in ("0", None):
        if setting is None:
            os.environ.pop("ORBX_PYR_FUSED", None)
        else:
            os.environ["ORBX_PYR_FUSED"] = setting
        try:
            ex = _extractor(1000)
            kps, desc = ex(img)
        finally:
            os.environ.pop("ORBX_PYR_FUSED", None)
        assert_same_keypoints(kps, ref.keypoints, desc, ref.descriptors, "ORBX_PYR_FUSED=%s" % setting)
        for l in range(8):
            assert np.array_equal(ex.mvImagePyramid[l], ref.pyramid[l]), "ORBX_PYR_FUSED=%s level %d" % (setting, l)
    # a 4-frame batch (still a small batch) the same way
    os.environ["ORBX_PYR_FUSED"] = "0"
    try:
        ex = _extractor(1000)
        frames = _frames("gen", 640, 480, 4, seed0=70)
        _, _, _, _, klist, dlist = _run_batch(ex, frames, cuda)
    finally:
        os.environ.pop("ORBX_PYR_FUSED", None)
    for f in range(4):
        r = orbref.extract(frames[f], p, want_pyramid=False)
        assert_same_keypoints(klist[f], r.keypoints, dlist[f], r.descriptors, "per-level batch f%d" % f)
