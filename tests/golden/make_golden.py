"""Regenerate the committed golden fixtures from the CPU oracle.

    python tests/golden/make_golden.py

Each fixture holds the input images (or their sha256 when they are regenerated
from a seed) and the oracle's ORBextractor output per frame (keypoints as the
28-byte cv::KeyPoint layout, 32-byte descriptors, per-level counts), plus, per
fixture kind, one SearchForInitialization result over frames 0 -> 1 ("si",
ORBmatcher(0.9, true), r = 100, src/ORBmatcher.cc:417-588) and/or
Frame::ComputeStereoMatches of frame 0 (left) against frame 1 (right)
("stereo", src/Frame.cc:630-872, EuRoC's bf / fx).  The BASELINE configs are
covered at their own geometry: config 1 (TUM 640x480 / 1000), config 2 (KITTI
1241x376 / 2000 + SearchForInitialization), config 3 (EuRoC 752x480 / 1000
stereo) and config 5 (1920x1080 / 4000).  The reference itself cannot
run here (no OpenCV), so these pin the oracle against regressions and the GPU
path against the same bytes; see DESIGN.md "Oracle" for what is and is not
pinned against the reference.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "orb-slam-_amd")]

import orbref  # noqa: E402
import orbx_synth  # noqa: E402

EUROC_BF, EUROC_FX = 47.90639384423901, 435.2046959714599   # Examples/Stereo/EuRoC.yaml:8,25

FIXTURES = {
    # name: (image factory, nfeatures, scale, nlevels, ini, min)
    "small_320x240_300": (lambda: np.stack([orbx_synth.gen_image(7, 320, 240), orbx_synth.gen_image(8, 320, 240)]),
                          300, 1.2, 8, 20, 7),
    "tum_640x480_1000": (lambda: orbx_synth.kitti_sequence(2, start=40, width=640, height=480), 1000, 1.2, 8, 20, 7),
    "kitti_1241x376_2000": (lambda: orbx_synth.kitti_sequence(2, start=11), 2000, 1.2, 8, 20, 7),
    "euroc_752x480_1000_stereo": (lambda: np.stack(orbx_synth.stereo_pair(21, 752, 480)), 1000, 1.2, 8, 20, 7),
    "hd_1920x1080_4000": (lambda: orbx_synth.gen_image(31, 1920, 1080)[None], 4000, 1.2, 8, 20, 7),
}
# what each fixture checks beyond the per-frame extraction
KINDS = {"small_320x240_300": ("si",), "tum_640x480_1000": ("si",), "kitti_1241x376_2000": ("si",),
         "euroc_752x480_1000_stereo": ("stereo",), "hd_1920x1080_4000": ()}


def make(name):
    fac, nf, sc, nl, ini, mn = FIXTURES[name]
    imgs = fac()
    p = orbref.make_params(nf, sc, nl, ini, mn)
    kinds = KINDS[name]
    res = [orbref.extract(im, p, want_pyramid="stereo" in kinds) for im in imgs]
    H, W = imgs.shape[1:]
    import hashlib
    out = {"params": np.array([nf, sc, nl, ini, mn], np.float64),
           "image_sha256": np.array(hashlib.sha256(imgs.tobytes()).hexdigest())}
    if "si" in kinds:
        nm, m12, _ = orbref.search_for_initialization(res[0].keypoints, res[0].descriptors, res[1].keypoints,
                                                      res[1].descriptors, W, H, window=100, nnratio=0.9,
                                                      check_ori=True)
        out["nmatches"], out["matches12"] = np.int32(nm), m12
    if "stereo" in kinds:
        ur, dp, _, good = orbref.compute_stereo_matches(p, res[0], res[1], H, W, EUROC_BF, EUROC_FX)
        out["u_right"], out["depth"], out["n_good"] = ur, dp, np.int32(good)
    if imgs.nbytes <= 200_000:     # small inputs are stored; larger ones are regenerated from their seed
        out["images"] = imgs
    for f, r in enumerate(res):
        out["kps%d" % f] = r.keypoints.view(np.uint8).reshape(-1, 28)
        out["desc%d" % f] = r.descriptors
        out["levels%d" % f] = r.level_counts
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
    print(name, [len(r.keypoints) for r in res], "matches", out.get("nmatches"), "stereo", out.get("n_good"))


if __name__ == "__main__":
    for n in sys.argv[1:] or FIXTURES:
        make(n)
