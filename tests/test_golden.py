"""Committed golden fixtures (tests/golden/*.npz, made by tests/golden/make_golden.py)
against the CPU oracle (CPU) and the gfx950 path (GPU)."""
import hashlib
import os
import sys

import numpy as np
import pytest

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
sys.path.insert(0, HERE)


def _load(name):
    import make_golden
    d = dict(np.load(os.path.join(HERE, name + ".npz"), allow_pickle=False))
    imgs = d["images"] if "images" in d else make_golden.FIXTURES[name][0]()
    assert hashlib.sha256(imgs.tobytes()).hexdigest() == str(d["image_sha256"]), "input generator drifted"
    nf, sc, nl, ini, mn = d["params"]
    return d, imgs, (int(nf), float(sc), int(nl), int(ini), int(mn))


NAMES = ["small_320x240_300", "tum_640x480_1000", "kitti_1241x376_2000", "euroc_752x480_1000_stereo",
         "hd_1920x1080_4000"]
EUROC_BF, EUROC_FX = 47.90639384423901, 435.2046959714599   # Examples/Stereo/EuRoC.yaml:8,25


@pytest.mark.parametrize("name", NAMES)
def test_oracle_reproduces_golden(orbref, name):
    d, imgs, prm = _load(name)
    p = orbref.make_params(*prm)
    res = [orbref.extract(im, p, want_pyramid="u_right" in d) for im in imgs]
    for f, r in enumerate(res):
        assert np.array_equal(r.keypoints.view(np.uint8).reshape(-1, 28), d["kps%d" % f])
        assert np.array_equal(r.descriptors, d["desc%d" % f])
        assert np.array_equal(r.level_counts, d["levels%d" % f])
    H, W = imgs.shape[1:]
    if "nmatches" in d:
        nm, m12, _ = orbref.search_for_initialization(res[0].keypoints, res[0].descriptors, res[1].keypoints,
                                                      res[1].descriptors, W, H)
        assert nm == int(d["nmatches"]) and np.array_equal(m12, d["matches12"])
    if "u_right" in d:
        ur, dp, _, good = orbref.compute_stereo_matches(p, res[0], res[1], H, W, EUROC_BF, EUROC_FX)
        assert good == int(d["n_good"]) and np.array_equal(ur, d["u_right"]) and np.array_equal(dp, d["depth"])


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_gpu_reproduces_golden(cuda, name):
    import torch
    import orbx
    d, imgs, prm = _load(name)
    ex = orbx.ORBextractor(*prm)
    B, H, W = imgs.shape
    cap = ex.capacity(H, W)
    t = torch.from_numpy(np.ascontiguousarray(imgs)).to(cuda)
    kps = torch.empty((B, cap, 7), dtype=torch.int32, device=cuda)
    desc = torch.empty((B, cap, 32), dtype=torch.uint8, device=cuda)
    counts = torch.empty((B,), dtype=torch.int32, device=cuda)
    s = torch.cuda.current_stream()
    ex.extract_batch_device(t, kps, desc, counts, s)
    pa = torch.tensor([0], dtype=torch.int32, device=cuda)
    pb = torch.tensor([1], dtype=torch.int32, device=cuda)
    if "nmatches" in d:
        m12, nm = orbx.ORBmatcher(0.9, True).search_for_initialization_batch(kps, desc, counts, pa, pb, H, W, 100,
                                                                             stream=s)
    if "u_right" in d:
        ur, dp, ng = ex.stereo_batch_device(kps, desc, counts, pa, pb, EUROC_BF, EUROC_FX, stream=s)
    ex.sync(s)
    c = counts.cpu().numpy()
    k = kps.cpu().numpy()
    dd = desc.cpu().numpy()
    for f in range(B):
        assert np.array_equal(k[f, :c[f]].view(np.uint8).reshape(-1, 28), d["kps%d" % f])
        assert np.array_equal(dd[f, :c[f]], d["desc%d" % f])
    if "nmatches" in d:
        assert int(nm.item()) == int(d["nmatches"])
        assert np.array_equal(m12.cpu().numpy()[0, :len(d["matches12"])], d["matches12"])
    if "u_right" in d:
        n = int(c[0])
        assert int(ng[0].item()) == int(d["n_good"])
        assert np.array_equal(ur[0, :n].cpu().numpy(), d["u_right"])
        assert np.array_equal(dp[0, :n].cpu().numpy(), d["depth"])
