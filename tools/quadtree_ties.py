"""Measure how often DistributeOctTree's heap-address tie-break (the reference, src/ORBextractor.cc:815)
changes the kept keypoints relative to the canonical creation order that oracle/orbref.c and the GPU
kernel K3 implement.

    python tools/quadtree_ties.py [--frames N] [--out profiles/r02/quadtree_ties.json]

Per config sequence and per (frame, level): the oracle's FAST
candidates of that level go through
  * orbref.distribute               canonical: size ties by creation order,
  * orbref.distribute_faithful(0)   std::list nodes + sort of (size, ExtractorNode*) under glibc malloc,
  * orbref.distribute_faithful(0)   again, right after (the reference against itself: the heap moved),
  * orbref.distribute_faithful(1)   the faithful code with the canonical tie-break (must equal canonical).
Reported: levels / frames whose kept keypoint SET differs, whose ORDER differs (the output order is
the keypoint index order of ORBextractor::operator()), and the fraction of kept keypoints that differ.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "orb-slam-_amd"), os.path.join(ROOT, "oracle")]

import orbref  # noqa: E402
import orbx_synth  # noqa: E402

CONFIGS = [
    # name, W, H, nfeatures, frame source
    ("config1_tum_640x480_1000", 640, 480, 1000, "gen"),
    ("config2_kitti_1241x376_2000", 1241, 376, 2000, "kitti"),
    ("config3_euroc_752x480_1000", 752, 480, 1000, "gen"),
    ("config5_1920x1080_4000", 1920, 1080, 4000, "gen"),
]


def frames_for(kind, W, H, n):
    if kind == "kitti":
        return orbx_synth.kitti_sequence(n, start=0)
    return np.stack([orbx_synth.gen_image(300 + i, W, H) for i in range(n)])


def compare(a, b):
    # kept keypoints that the other order does not keep (the counts may differ by up to 3)
    sa, sb = set(a.tolist()), set(b.tolist())
    return (not np.array_equal(a, b)), (sa != sb), max(len(sa - sb), len(sb - sa))


def measure(name, W, H, nfeat, kind, nframes):
    p = orbref.make_params(nfeat, 1.2, 8, 20, 7)
    t = orbref.tables(p)
    st = {k: 0 for k in ("levels", "kept", "order_diff_levels", "set_diff_levels", "kp_diff", "frames_order_diff",
                         "frames_set_diff", "self_order_diff_levels", "self_set_diff_levels", "self_kp_diff",
                         "canonical_mode_mismatch_levels")}
    for f in frames_for(kind, W, H, nframes):
        r = orbref.extract(f, p)
        fo = fs = False
        for l in range(8):
            lev = r.pyramid[l]
            h, w = lev.shape
            c = orbref.level_candidates(lev)
            N = t.nfeat_level[l]
            can = orbref.distribute(c, w, h, N)
            fa = orbref.distribute_faithful(c, w, h, N, 0)
            fa2 = orbref.distribute_faithful(c, w, h, N, 0)
            fc = orbref.distribute_faithful(c, w, h, N, 1)
            od, sd, kd = compare(can, fa)
            sod, ssd, skd = compare(fa, fa2)
            st["levels"] += 1
            st["kept"] += len(can)
            st["order_diff_levels"] += od
            st["set_diff_levels"] += sd
            st["kp_diff"] += kd
            st["self_order_diff_levels"] += sod
            st["self_set_diff_levels"] += ssd
            st["self_kp_diff"] += skd
            st["canonical_mode_mismatch_levels"] += int(not np.array_equal(can, fc))
            fo |= od
            fs |= sd
        st["frames_order_diff"] += fo
        st["frames_set_diff"] += fs
    st["frames"] = nframes
    st["kp_diff_frac"] = st["kp_diff"] / max(st["kept"], 1)
    st["self_kp_diff_frac"] = st["self_kp_diff"] / max(st["kept"], 1)
    return st


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=16)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r02", "quadtree_ties.json"))
    a = ap.parse_args()
    res = {"what": __doc__.strip().splitlines()[0], "allocator": "glibc malloc (this process)", "configs": {}}
    for name, W, H, nf, kind in CONFIGS:
        t0 = time.time()
        n = a.frames if W * H < 1_000_000 else max(4, a.frames // 4)
        res["configs"][name] = measure(name, W, H, nf, kind, n)
        res["configs"][name]["seconds"] = round(time.time() - t0, 1)
        print(name, json.dumps(res["configs"][name]), flush=True)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
