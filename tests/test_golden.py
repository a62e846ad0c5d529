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


NAMES = ["small_320x240_300", "tum_640x480_1000"]


@pytest.mark.parametrize("name", NAMES)
def test_oracle_reproduces_golden(orbref, name):
    d, imgs, prm = _load(name)
    p = orbref.make_params(*prm)
    res = [orbref.extract(im, p, want_pyramid=False) for im in imgs]
    for f, r in enumerate(res):
        assert np.array_equal(r.keypoints.view(np.uint8).reshape(-1, 28), d["kps%d" % f])
        assert np.array_equal(r.descriptors, d["desc%d" % f])
        assert np.array_equal(r.level_counts, d["levels%d" % f])
    H, W = imgs.shape[1:]
    nm, m12, _ = orbref.search_for_initialization(res[0].keypoints, res[0].descriptors, res[1].keypoints,
                                                  res[1].descriptors, W, H)
    assert nm == int(d["nmatches"]) and np.array_equal(m12, d["matches12"])


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_gpu_reproduces_golden(cuda, name):
    import torch
    import orbx
    d, imgs, prm = _load(name)
    ex = orbx.ORBextractor(*prm)
    H, W = imgs.shape[1:]
    cap = ex.capacity(H, W)
    t = torch.from_numpy(np.ascontiguousarray(imgs)).to(cuda)
    kps = torch.empty((2, cap, 7), dtype=torch.int32, device=cuda)
    desc = torch.empty((2, cap, 32), dtype=torch.uint8, device=cuda)
    counts = torch.empty((2,), dtype=torch.int32, device=cuda)
    s = torch.cuda.current_stream()
    ex.extract_batch_device(t, kps, desc, counts, s)
    m12, nm = orbx.ORBmatcher(0.9, True).search_for_initialization_batch(
        kps, desc, counts, torch.tensor([0], dtype=torch.int32, device=cuda),
        torch.tensor([1], dtype=torch.int32, device=cuda), H, W, 100, stream=s)
    ex.sync(s)
    c = counts.cpu().numpy()
    k = kps.cpu().numpy()
    dd = desc.cpu().numpy()
    for f in range(2):
        assert np.array_equal(k[f, :c[f]].view(np.uint8).reshape(-1, 28), d["kps%d" % f])
        assert np.array_equal(dd[f, :c[f]], d["desc%d" % f])
    assert int(nm.item()) == int(d["nmatches"])
    assert np.array_equal(m12.cpu().numpy()[0, :len(d["matches12"])], d["matches12"])
