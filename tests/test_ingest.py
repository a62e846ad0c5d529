"""Image ingest, SURVEY.md §8f row 4:
  cv::remap(im, imRect, M1, M2, INTER_LINEAR), CV_32F maps, BORDER_CONSTANT 0   Examples/Stereo/stereo_euroc.cc:136-137
  cvtColor {RGB,BGR,RGBA,BGRA}2GRAY                                             src/Tracking.cc:185-210
  imDepth.convertTo(CV_32F, mDepthMapFactor)                                     src/Tracking.cc:234-235

OpenCV is absent, so the oracle restates OpenCV 3.x's fixed-point remap and
RGB2Gray<uchar> paths (parity unpinned against real OpenCV).  CPU: the C oracle against a numpy
restatement and known answers (identity maps copy exactly, half-pixel shifts average with
rounding up, pure primaries give the integer coefficients); maps hold integer, tie (k + 1/64),
out-of-range, NaN and huge coordinates.  GPU: liborbx batch path against the oracle, then
ingest -> extract against the oracle chain.
"""
import numpy as np
import pytest


def np_round_x86(v):
    """cvRound on x86: ties to even, NaN / out of range -> INT_MIN."""
    v = np.asarray(v, np.float32)
    ok = (v >= np.float32(-2147483648.0)) & (v < np.float32(2147483648.0))
    r = np.where(ok, np.rint(np.where(ok, v, 0)).astype(np.int64), -2 ** 31)
    return r.astype(np.int64)


def np_ingest(src, rgb=False, map_x=None, map_y=None):
    src = np.asarray(src, np.uint8)
    if src.ndim == 2:
        src = src[..., None]
    rows, cols, ch = src.shape
    if map_x is not None:
        sx32 = np_round_x86(np.asarray(map_x, np.float32) * np.float32(32))
        sy32 = np_round_x86(np.asarray(map_y, np.float32) * np.float32(32))
        fx, fy = sx32 & 31, sy32 & 31
        sx = np.clip(sx32 >> 5, -32768, 32767)
        sy = np.clip(sy32 >> 5, -32768, 32767)
        w = [(32 - fx) * (32 - fy) * 32, fx * (32 - fy) * 32, (32 - fx) * fy * 32, fx * fy * 32]

        def tap(yy, xx):
            ok = (xx >= 0) & (xx < cols) & (yy >= 0) & (yy < rows)
            v = src[np.clip(yy, 0, rows - 1), np.clip(xx, 0, cols - 1)].astype(np.int64)
            return np.where(ok[..., None], v, 0)

        acc = (tap(sy, sx) * w[0][..., None] + tap(sy, sx + 1) * w[1][..., None] +
               tap(sy + 1, sx) * w[2][..., None] + tap(sy + 1, sx + 1) * w[3][..., None])
        val = np.clip((acc + (1 << 14)) >> 15, 0, 255)
    else:
        val = src.astype(np.int64)
    if ch == 1:
        return val[..., 0].astype(np.uint8)
    w0, w2 = (4899, 1868) if rgb else (1868, 4899)
    return ((val[..., 0] * w0 + val[..., 1] * 9617 + val[..., 2] * w2 + (1 << 13)) >> 14).astype(np.uint8)


def rect_maps(rows, cols, seed, drows=None, dcols=None, adversarial=True):
    """initUndistortRectifyMap-like maps: a small rotation and radial-tangential distortion, plus
    adversarial entries."""
    rng = np.random.default_rng(seed)
    drows, dcols = drows or rows, dcols or cols
    fx = fy = 0.9 * cols
    cx, cy = cols / 2 + rng.normal(0, 5), rows / 2 + rng.normal(0, 5)
    k1, k2, p1, p2 = rng.normal(0, 0.05), rng.normal(0, 0.01), rng.normal(0, 1e-3), rng.normal(0, 1e-3)
    a = rng.normal(0, 0.01, 3)
    R = np.array([[1, -a[2], a[1]], [a[2], 1, -a[0]], [-a[1], a[0], 1]])
    v, u = np.mgrid[0:drows, 0:dcols].astype(np.float64)
    X = np.stack([(u - cx) / fx, (v - cy) / fy, np.ones_like(u)], -1) @ R.T
    x, y = X[..., 0] / X[..., 2], X[..., 1] / X[..., 2]
    r2 = x * x + y * y
    rad = 1 + k1 * r2 + k2 * r2 * r2
    xd = x * rad + 2 * p1 * x * y + p2 * (r2 + 2 * x * x)
    yd = y * rad + p1 * (r2 + 2 * y * y) + 2 * p2 * x * y
    mx = (xd * fx + cx).astype(np.float32)
    my = (yd * fy + cy).astype(np.float32)
    if adversarial:
        n = mx.size
        idx = rng.choice(n, n // 20, replace=False)
        k = len(idx) // 6
        flat_x, flat_y = mx.reshape(-1), my.reshape(-1)
        flat_x[idx[:k]] = np.round(flat_x[idx[:k]])                               # integer coordinates
        flat_x[idx[k:2 * k]] = np.floor(flat_x[idx[k:2 * k]]) + np.float32(1 / 64)   # x*32 ties
        flat_y[idx[k:2 * k]] = np.floor(flat_y[idx[k:2 * k]]) + np.float32(3 / 64)
        flat_x[idx[2 * k:3 * k]] = rng.uniform(-3, 0.5, k)                         # left border
        flat_y[idx[3 * k:4 * k]] = rows - 1 + rng.uniform(-0.5, 2, k)              # bottom border
        flat_x[idx[4 * k]] = np.nan
        flat_y[idx[4 * k + 1]] = np.float32(3e9)
        flat_x[idx[4 * k + 2]] = np.float32(-1e6)
    return mx, my


def textured(rows, cols, ch, seed):
    import orbx_synth
    g = orbx_synth.gen_image(seed, cols, rows)
    if ch == 1:
        return g
    rng = np.random.default_rng(seed)
    out = np.stack([np.clip(g.astype(int) + rng.integers(-40, 40), 0, 255) for _ in range(ch)], -1).astype(np.uint8)
    return out


@pytest.mark.parametrize("ch", [1, 3, 4])
@pytest.mark.parametrize("rgb", [False, True])
@pytest.mark.parametrize("remap", [False, True])
def test_oracle_matches_restatement(orbref, ch, rgb, remap):
    src = textured(120, 160, ch, 3)
    mx, my = rect_maps(120, 160, 4, 110, 150) if remap else (None, None)
    assert np.array_equal(orbref.ingest(src, rgb, mx, my), np_ingest(src, rgb, mx, my))


def test_known_answers(orbref):
    red = np.zeros((2, 2, 3), np.uint8)
    red[..., 0] = 255
    assert orbref.ingest(red, rgb=True)[0, 0] == (255 * 4899 + 8192) >> 14 == 76
    assert orbref.ingest(red, rgb=False)[0, 0] == (255 * 1868 + 8192) >> 14 == 29
    white = np.full((2, 2, 4), 255, np.uint8)
    assert orbref.ingest(white)[0, 0] == 255                                     # coefficients sum to 2^14
    img = np.random.default_rng(0).integers(0, 256, (50, 70), dtype=np.uint8)
    v, u = np.mgrid[0:50, 0:70].astype(np.float32)
    assert np.array_equal(orbref.ingest(img, map_x=u, map_y=v), img)              # identity map copies
    half = orbref.ingest(img, map_x=u + np.float32(0.5), map_y=v)
    want = (img[:, :-1].astype(int) + img[:, 1:] + 1) >> 1
    assert np.array_equal(half[:, :-1], want)
    assert np.array_equal(half[:, -1], (img[:, -1].astype(int) + 1) >> 1)         # right neighbour is border 0
    out = orbref.ingest(img, map_x=u - 100, map_y=v)
    assert not out.any()


def test_depth_convert(orbref):
    d = np.random.default_rng(1).integers(0, 65535, (40, 60), dtype=np.uint16)
    f = np.float32(1.0 / 5000.0)
    assert np.array_equal(orbref.depth_convert(d, f), d.astype(np.float32) * f)


# ---------------------------------------------------------------------------- GPU

@pytest.mark.gpu
@pytest.mark.parametrize("ch,rgb", [(1, False), (3, False), (3, True), (4, True)])
def test_gpu_ingest_batch(orbref, cuda, ch, rgb):
    """Four frames, two map pairs (L / R alternate), against the oracle per frame."""
    import torch
    import orbx
    rows, cols = 120, 162                                                          # cols % 4 != 0: ragged tail
    frames = [textured(rows, cols, ch, 10 + f) for f in range(4)]
    maps = [rect_maps(rows, cols, 20 + i, 112, 150) for i in range(2)]
    src = torch.from_numpy(np.stack(frames)).to(cuda)
    mx = torch.from_numpy(np.stack([m[0] for m in maps])).to(cuda)
    my = torch.from_numpy(np.stack([m[1] for m in maps])).to(cuda)
    out = orbx.ingest_batch_device(src, rgb, mx, my)
    plain = orbx.ingest_batch_device(src, rgb)
    torch.cuda.synchronize()
    for f in range(4):
        want = orbref.ingest(frames[f], rgb, *maps[f % 2])
        assert np.array_equal(out[f].cpu().numpy(), want)
        assert np.array_equal(plain[f].cpu().numpy(), orbref.ingest(frames[f], rgb))


@pytest.mark.gpu
def test_gpu_ingest_then_extract(orbref, cuda):
    """Colour stereo frames -> remap + gray -> extract, on the device, against the oracle chain."""
    import torch
    import orbx
    rows, cols = 480, 752
    frames = [textured(rows, cols, 3, 30 + f) for f in range(2)]
    maps = [rect_maps(rows, cols, 40 + i, adversarial=False) for i in range(2)]
    src = torch.from_numpy(np.stack(frames)).to(cuda)
    mx = torch.from_numpy(np.stack([m[0] for m in maps])).to(cuda)
    my = torch.from_numpy(np.stack([m[1] for m in maps])).to(cuda)
    gray = orbx.ingest_batch_device(src, False, mx, my)
    ex = orbx.ORBextractor(1000, 1.2, 8, 20, 7)
    cap = ex.capacity(rows, cols)
    kps = torch.empty((2, cap, 7), dtype=torch.int32, device=cuda)
    desc = torch.empty((2, cap, 32), dtype=torch.uint8, device=cuda)
    counts = torch.empty((2,), dtype=torch.int32, device=cuda)
    ex.extract_batch_device(gray, kps, desc, counts)
    torch.cuda.synchronize()
    p = orbref.make_params(1000, 1.2, 8, 20, 7)
    got = orbx.keypoints_from_device(kps, counts)
    for f in range(2):
        g = orbref.ingest(frames[f], False, *maps[f])
        assert np.array_equal(gray[f].cpu().numpy(), g)
        ref = orbref.extract(g, p, want_pyramid=False)
        n = int(counts[f])
        assert n == len(ref.keypoints) and n > 500
        assert np.array_equal(desc[f, :n].cpu().numpy(), ref.descriptors)
        for k in ("x", "y", "octave", "response"):
            assert np.array_equal(got[f][k], ref.keypoints[k])


@pytest.mark.gpu
def test_gpu_depth(orbref, cuda):
    import torch
    import orbx
    d = np.random.default_rng(2).integers(0, 65535, (3, 48, 64), dtype=np.uint16)
    f = 1.0 / 5000.0
    out = orbx.depth_batch_device(torch.from_numpy(d.view(np.int16)).to(cuda), f)
    torch.cuda.synchronize()
    for b in range(3):
        assert np.array_equal(out[b].cpu().numpy(), orbref.depth_convert(d[b], f))
