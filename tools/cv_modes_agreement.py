#!/usr/bin/env python3
"""How far SURVEY Appendix A's alternative OpenCV builds move the extractor's output.

The reference links whatever OpenCV 2.4 / 3.x its user has (CMakeLists.txt:31-37).  The oracle and the GPU pin
OpenCV 3.x's generic scalar paths (cv::setUseOptimized(false)); a stock x86 build takes SIMD paths instead for
the pyramid's vertical resize pass (A.2, src/ORBextractor.cc:1361) and, up to 3.4.1, the blur's column pass
(A.3, :1301-1306), and 3.4.6+ / 4.x blur with a different fixed-point kernel.  BRIEF's cos / sin (A.5, :146-148)
come from glibc.  For each BASELINE config this runs the CPU oracle (test infrastructure) on the same frames
under every mode and counts, against the canonical modes:
  pyramid bytes (levels 1..), FAST candidates (per level, as (x, y) sets), kept keypoints ((octave, x, y) sets),
  descriptors of the keypoints kept in both (bits and rows that change), and angles.
Writes profiles/r06/cv_modes_agreement.json and prints a markdown table.
  python tools/cv_modes_agreement.py [--frames 16]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "orb-slam-_amd")]
import orbref  # noqa: E402
import orbx_synth  # noqa: E402

CONFIGS = [
    # (tag, W, H, nfeatures, frame source)
    ("1: TUM 640x480, 1000", 640, 480, 1000, "gen"),
    ("2: KITTI 1241x376, 2000", 1241, 376, 2000, "kitti"),
    ("3: EuRoC 752x480, 1000", 752, 480, 1000, "gen"),
    ("5: 1920x1080, 4000", 1920, 1080, 4000, "gen"),
]
R, B, T = orbref, orbref, orbref
MODES = [
    ("resize SSE2 (A.2)", (R.RESIZE_SSE2, B.BLUR_SCALAR, T.TRIG_GLIBC)),
    ("blur SSE2 float column, <= 3.4.1 (A.3)", (R.RESIZE_SCALAR, B.BLUR_SSE2, T.TRIG_GLIBC)),
    ("blur bit-exact ED kernel, >= 3.4.6 / 4.x (A.3)", (R.RESIZE_SCALAR, B.BLUR_BITEXACT, T.TRIG_GLIBC)),
    ("trig correctly rounded (A.5)", (R.RESIZE_SCALAR, B.BLUR_SCALAR, T.TRIG_CR)),
    ("stock x86 <= 3.4.1 build (resize + blur SSE2)", (R.RESIZE_SSE2, B.BLUR_SSE2, T.TRIG_GLIBC)),
    ("stock x86 >= 3.4.6 build (resize SSE2 + bit-exact blur)", (R.RESIZE_SSE2, B.BLUR_BITEXACT, T.TRIG_GLIBC)),
]


def frames_for(src, W, H, n, seed0):
    if src == "kitti":
        return orbx_synth.kitti_sequence(n, start=seed0)
    return np.stack([orbx_synth.gen_image(seed0 + i, W, H) for i in range(n)])


def kp_keys(kps):
    return {(int(o), int(round(float(x) * 1e3)), int(round(float(y) * 1e3))): i
            for i, (x, y, o) in enumerate(zip(kps["x"], kps["y"], kps["octave"]))}


def compare(frames, p, modes):
    st = {"frames": len(frames), "pyr_bytes": 0, "pyr_bytes_diff": 0, "cand": 0, "cand_diff": 0, "kept": 0,
          "kept_diff": 0, "common": 0, "desc_rows_diff": 0, "desc_bits_diff": 0, "angle_diff": 0}
    for img in frames:
        a = orbref.extract(img, p, want_pyramid=True)
        b = orbref.extract(img, p, want_pyramid=True, modes=modes)
        for l in range(1, len(a.pyramid)):
            st["pyr_bytes"] += a.pyramid[l].size
            st["pyr_bytes_diff"] += int((a.pyramid[l] != b.pyramid[l]).sum())
        for l in range(len(a.pyramid)):
            if modes[0] == orbref.RESIZE_SCALAR and l > 0:
                ca = cb = None   # same pyramid: same candidates
                st["cand"] += int(a.cand_counts[l])
                continue
            ca = {(int(x), int(y)) for x, y, _ in orbref.level_candidates(a.pyramid[l])}
            cb = {(int(x), int(y)) for x, y, _ in orbref.level_candidates(b.pyramid[l])}
            st["cand"] += len(ca)
            st["cand_diff"] += len(ca ^ cb)
        ka, kb = kp_keys(a.keypoints), kp_keys(b.keypoints)
        st["kept"] += len(ka)
        st["kept_diff"] += len(set(ka) ^ set(kb))
        for k, i in ka.items():
            j = kb.get(k)
            if j is None:
                continue
            st["common"] += 1
            bits = int(np.unpackbits(a.descriptors[i] ^ b.descriptors[j]).sum())
            st["desc_bits_diff"] += bits
            st["desc_rows_diff"] += int(bits > 0)
            st["angle_diff"] += int(a.keypoints["angle"][i] != b.keypoints["angle"][j])
    st["pyr_frac"] = st["pyr_bytes_diff"] / max(st["pyr_bytes"], 1)
    st["cand_frac"] = st["cand_diff"] / max(st["cand"], 1)
    st["kept_frac"] = st["kept_diff"] / max(st["kept"], 1)
    st["desc_rows_frac"] = st["desc_rows_diff"] / max(st["common"], 1)
    st["desc_bits_frac"] = st["desc_bits_diff"] / max(256 * st["common"], 1)
    return st


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=16)
    ap.add_argument("--frames-1080", type=int, default=4)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r06", "cv_modes_agreement.json"))
    args = ap.parse_args()
    orbref.build()
    t0 = time.time()
    res = {"what": __doc__.strip().splitlines()[0], "blur_kernels": {
        "scalar/sse2 (<= 3.4.1)": orbref.blur_kernel(orbref.BLUR_SCALAR).tolist(),
        "bit-exact ED (>= 3.4.6 / 4.x)": orbref.blur_kernel(orbref.BLUR_BITEXACT).tolist()}, "configs": {}}
    for tag, W, H, nf, src in CONFIGS:
        n = args.frames_1080 if W >= 1920 else args.frames
        frames = frames_for(src, W, H, n, 100)
        p = orbref.make_params(nf, 1.2, 8, 20, 7)
        res["configs"][tag] = {name: compare(frames, p, m) for name, m in MODES}
        print(tag, "done", round(time.time() - t0, 1), "s", file=sys.stderr, flush=True)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    json.dump(res, open(args.out, "w"), indent=1)
    print("| Config | Mode | pyramid bytes | FAST candidates | kept keypoints | descriptors changed (rows / bits) | angles |")
    print("|---|---|---|---|---|---|---|")
    for tag, d in res["configs"].items():
        for name, s in d.items():
            print("| %s | %s | %.3f%% | %.3f%% | %.3f%% | %.2f%% / %.4f%% | %d |" % (
                tag, name, 100 * s["pyr_frac"], 100 * s["cand_frac"], 100 * s["kept_frac"], 100 * s["desc_rows_frac"],
                100 * s["desc_bits_frac"], s["angle_diff"]))


if __name__ == "__main__":
    main()
