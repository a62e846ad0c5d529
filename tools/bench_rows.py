#!/usr/bin/env python3
"""Measurements of the SURVEY.md §8f rows (the callers and data formats either side of the
headline path), each on a device-resident batch with HIP events on the launch stream, next to
the CPU oracle on a bounded sample:

  ingest        EuRoC 752x480 BGR stereo frames: remap (2 map pairs) + cvtColor -> gray (I1)
  voc           DBoW2 transform of KITTI frames (k=10, L=4 vocabulary trained here; ORBvoc.txt absent)
  bow_kf_f      SearchByBoW(KF, F) on consecutive KITTI frames over those FeatureVectors
  proj_local    SearchByProjection(F, local MapPoints, th=1)   (Tracking::SearchLocalPoints)
  last_frame    SearchByProjection(F, LastFrame, th=7, mono)    (TrackWithMotionModel)
  keyframe      SearchByProjection(F, KF, sFound, 10, 100)     (Relocalization)
  sim3          SearchByProjection(KF, Scw, points, matched, 10) (LoopClosing::ComputeSim3)
  fuse          Fuse(KF, MapPoints, 3)                          (LocalMapping::SearchInNeighbors)
  fuse_sim3     Fuse(KF, Scw, points, 4, replace)              (LoopClosing::SearchAndFuse)

  python tools/bench_rows.py [--batch 64] [--steps 20] [--cpu-seconds 2]

Prints one JSON object: per row the device ms per launch, units/s, and the oracle's rate.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "orb-slam-_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import orbx  # noqa: E402
import orbx_synth  # noqa: E402

HBM_PEAK_GBS = 8000.0
KITTI_K = (718.856, 718.856, 607.1928, 185.2157)   # Examples/Stereo/KITTI00-02.yaml
KITTI_BF = 386.1448
LEVELSUP = 2   # FeatureVector nodes at depth L - levelsup = 2, as ORBvoc (L 6) with levelsup 4


def dev_time(fn, steps, warmup, stream):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(steps):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / steps * 1e-3


def cpu_rate(fn, budget, n_items):
    t0 = time.perf_counter()
    k = 0
    while True:
        fn(k)
        k += 1
        if time.perf_counter() - t0 >= budget:
            break
    return k * n_items / (time.perf_counter() - t0), k


def row_ingest(args, s, dev):
    import orbref
    W, H, B = 752, 480, args.batch
    rng = np.random.default_rng(0)
    pairs = [orbx_synth.stereo_pair(200 + i, W, H) for i in range(B // 2)]
    gray = np.stack([im for pr in pairs for im in pr])
    bgr = np.clip(gray[..., None].astype(int) + rng.integers(-30, 30, (1, 1, 3)), 0, 255).astype(np.uint8)
    v, u = np.mgrid[0:H, 0:W].astype(np.float32)
    maps = []
    for i in range(2):   # small rotation + radial distortion, like initUndistortRectifyMap
        r2 = ((u - W / 2) ** 2 + (v - H / 2) ** 2) / (W * W / 4)
        k = 1 + (0.02 if i else -0.015) * r2
        maps.append(((u - W / 2) * k + W / 2 + 0.3 * i, (v - H / 2) * k + H / 2 - 0.2 * i))
    src = torch.from_numpy(bgr).to(dev)
    mx = torch.from_numpy(np.stack([m[0] for m in maps]).astype(np.float32)).to(dev)
    my = torch.from_numpy(np.stack([m[1] for m in maps]).astype(np.float32)).to(dev)
    out = torch.empty((B, H, W), dtype=torch.uint8, device=dev)
    t = dev_time(lambda: orbx.ingest_batch_device(src, False, mx, my, out, s), args.steps, args.warmup, s)
    torch.cuda.synchronize()
    ok = all(np.array_equal(out[f].cpu().numpy(), orbref.ingest(bgr[f], False, *maps[f % 2])) for f in (0, 1))
    alg = B * W * H * (3 + 1)   # source + gray out per frame (the maps are L2/MALL-resident across the batch)
    rate, k = cpu_rate(lambda i: orbref.ingest(bgr[i % B], False, *maps[i % 2]), args.cpu_seconds, 1)
    return {"unit": "frames/s", "value": round(B / t, 1), "ms_per_launch": round(t * 1e3, 4), "batch": B,
            "parity_sampled": ok, "roofline": {"bound": "hbm", "achieved": round(alg / t / 1e9, 1),
                                               "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                               "frac": round(alg / t / 1e9 / HBM_PEAK_GBS, 4),
                                               "alg_bytes_per_launch": alg},
            "cpu_baseline": {"value": round(rate, 1), "unit": "frames/s", "cores": 1, "kind": "port",
                             "sample": "oracle orbref_ingest, %d frames" % k}}


def kitti_batch(args, s, dev):
    B = args.batch
    frames = orbx_synth.kitti_sequence(B, start=40)
    ex = orbx.ORBextractor(2000, 1.2, 8, 20, 7)
    imgs = torch.from_numpy(frames).to(dev)
    cap = ex.capacity(376, 1241)
    kps = torch.empty((B, cap, 7), dtype=torch.int32, device=dev)
    desc = torch.empty((B, cap, 32), dtype=torch.uint8, device=dev)
    counts = torch.empty((B,), dtype=torch.int32, device=dev)
    ex.extract_batch_device(imgs, kps, desc, counts, s)
    ex.sync(s)
    host = orbx.keypoints_from_device(kps, counts)
    hdesc = [desc[f, :int(counts[f])].cpu().numpy() for f in range(B)]
    return frames, kps, desc, counts, host, hdesc, cap


def row_voc_bow(args, s, dev, kb):
    import orbref
    frames, kps, desc, counts, host, hdesc, cap = kb
    B = args.batch
    v = orbx_synth.Vocabulary.train(hdesc[:8], 10, 4, 0)
    gv = orbx.ORBVocabulary.from_arrays(v.k, v.L, v.parent, v.is_leaf, v.desc, v.weight)
    res = {}
    t = dev_time(lambda: res.__setitem__("r", gv.transform_batch_device(desc, counts, LEVELSUP, s)),
                 args.steps, args.warmup, s)
    bw, bv, bn, fn, fp, fi, fnn = res["r"]
    nd = int(counts.sum())
    rate, k = cpu_rate(lambda i: orbref.voc_transform(v, hdesc[i % B], LEVELSUP), args.cpu_seconds,
                       float(np.mean([len(d) for d in hdesc])))
    out = {"voc": {"unit": "descriptors/s", "value": round(nd / t, 1), "ms_per_launch": round(t * 1e3, 4),
                   "batch": B, "vocabulary": "k=10 L=4, %d nodes (trained here)" % v.nnodes,
                   "cpu_baseline": {"value": round(rate, 1), "unit": "descriptors/s", "cores": 1, "kind": "port",
                                    "sample": "oracle orbref_voc_transform, %d frames" % k}}}
    torch.cuda.synchronize()
    fvs = []
    for f in range(B):
        nn = int(fnn[f])
        fvs.append((fn[f, :nn].cpu().numpy(), fp[f, :nn + 1].cpu().numpy(), fi[f, :int(fp[f, nn])].cpu().numpy()))
    rng = np.random.default_rng(0)
    mps = [(rng.random(len(host[f])) < 0.7).astype(np.uint8) for f in range(B)]
    s1 = [{"kps": kps[f, :len(host[f])], "desc": desc[f, :len(host[f])], "has_mp": mps[f], "fv": fvs[f]}
          for f in range(B - 1)]
    s2 = [{"kps": kps[f + 1, :len(host[f + 1])], "desc": desc[f + 1, :len(host[f + 1])], "fv": fvs[f + 1]}
          for f in range(B - 1)]
    bb = orbx.BowBatch(orbx.BOW_KF_F, s1, s2)
    t = dev_time(lambda: bb.run(0.7, True, s), args.steps, args.warmup, s)
    wn, _ = orbref.search_by_bow_kf_f(host[0], hdesc[0], mps[0], fvs[0], host[1], hdesc[1], fvs[1], 0.7, True)
    rate, k = cpu_rate(lambda i: orbref.search_by_bow_kf_f(host[i % (B - 1)], hdesc[i % (B - 1)], mps[i % (B - 1)],
                                                          fvs[i % (B - 1)], host[i % (B - 1) + 1],
                                                          hdesc[i % (B - 1) + 1], fvs[i % (B - 1) + 1], 0.7, True),
                       args.cpu_seconds, 1)
    out["bow_kf_f"] = {"unit": "frame pairs/s", "value": round((B - 1) / t, 1), "ms_per_launch": round(t * 1e3, 4),
                       "pairs": B - 1, "matches_pair0": int(bb.nmatches[0]), "parity_pair0": int(bb.nmatches[0]) == wn,
                       "cpu_baseline": {"value": round(rate, 1), "unit": "frame pairs/s", "cores": 1, "kind": "port",
                                        "sample": "oracle orbref_search_by_bow_kf_f, %d pairs" % k}}
    return out


def _pose_params(th, **kw):
    sc = [np.float32(1.2) ** i for i in range(8)]
    pp = orbx.pose_params(KITTI_K, (0.0, 1241.0, 0.0, 376.0), sc, bf=KITTI_BF, th=th)
    for k, v in kw.items():
        setattr(pp, k, v)
    return pp


def row_pose(args, s, dev, kb):
    import orbref
    frames, kps, desc, counts, host, hdesc, cap = kb
    B, NMP = args.batch, args.mappoints
    scenes = [orbx_synth.pose_scene(300 + f, host[f], hdesc[f], NMP, KITTI_K, KITTI_BF) for f in range(B)]
    rng = np.random.default_rng(1)
    ur = torch.zeros((B, cap), dtype=torch.float32, device=dev)
    cl = torch.zeros((B, cap), dtype=torch.uint8, device=dev)
    claimed = []
    for f, (Tcw, pts, pdesc, u) in enumerate(scenes):
        ur[f, :len(u)] = torch.from_numpy(u)
        c = (rng.random(len(u)) < 0.1).astype(np.uint8)
        claimed.append(c)
        cl[f, :len(c)] = torch.from_numpy(c)
    pts = torch.from_numpy(np.stack([sc[1] for sc in scenes]).view(np.int32).reshape(B, NMP, 12)).to(dev)
    pdesc = torch.from_numpy(np.stack([sc[2] for sc in scenes])).to(dev)
    npts = torch.full((B,), NMP, dtype=torch.int32, device=dev)
    out = {}
    cases = [("last_frame", orbx.PROJ_LAST_FRAME, _pose_params(7.0, mono=1)),
             ("keyframe", orbx.PROJ_KEYFRAME, _pose_params(10.0, orb_dist=100)),
             ("sim3", orbx.PROJ_SIM3, _pose_params(10.0)),
             ("fuse", orbx.FUSE, _pose_params(3.0)),
             ("fuse_sim3", orbx.FUSE_SIM3, _pose_params(4.0))]
    for name, mode, pp in cases:
        sim3 = mode in (orbx.PROJ_SIM3, orbx.FUSE_SIM3)
        poses = []
        for Tcw, *_ in scenes:
            P = (Tcw * np.float32(1.7)).astype(np.float32) if sim3 else Tcw
            poses.append(np.concatenate([P.ravel(), Tcw.ravel()]))
        pose = torch.from_numpy(np.stack(poses).astype(np.float32)).to(dev)
        mt = orbx.ORBmatcher(0.9, True)
        res = {}
        t = dev_time(lambda: res.__setitem__("r", mt.project_search_batch_device(
            mode, kps, desc, ur, cl, counts, pose, pts, pdesc, npts, pp, stream=s)),
            args.steps, args.warmup, s)
        torch.cuda.synchronize()
        match, nm = res["r"]
        wn, wm = orbref.project_search(mode, host[0], hdesc[0], scenes[0][3], claimed[0], poses[0], scenes[0][1],
                                       scenes[0][2], orbref.PoseParams.from_buffer_copy(pp))
        ok = int(nm[0]) == wn and np.array_equal(match[0, :len(wm)].cpu().numpy(), wm)
        rate, k = cpu_rate(lambda i: orbref.project_search(mode, host[i % B], hdesc[i % B], scenes[i % B][3],
                                                           claimed[i % B], poses[i % B], scenes[i % B][1],
                                                           scenes[i % B][2], orbref.PoseParams.from_buffer_copy(pp)),
                           args.cpu_seconds, NMP)
        out[name] = {"unit": "MapPoints/s", "value": round(B * NMP / t, 1), "ms_per_launch": round(t * 1e3, 4),
                     "frames": B, "mappoints_per_frame": NMP, "matches_frame0": int(nm[0]), "parity_frame0": ok,
                     "cpu_baseline": {"value": round(rate, 1), "unit": "MapPoints/s", "cores": 1, "kind": "port",
                                      "sample": "oracle orbref_project_search, %d frames" % k}}
    # SearchByProjection(F, local MapPoints): what isInFrustum leaves in each MapPoint
    lp = []
    for f, (Tcw, P, pd, u) in enumerate(scenes):
        q = np.zeros(NMP, orbx.PROJ_POINT_DTYPE)
        r2 = np.random.default_rng(f)
        tgt = r2.integers(0, len(host[f]), NMP)
        q["proj_x"] = host[f]["x"][tgt] + r2.normal(0, 2, NMP)
        q["proj_y"] = host[f]["y"][tgt] + r2.normal(0, 2, NMP)
        q["proj_xr"] = np.where(u[tgt] > 0, u[tgt] + r2.normal(0, 2, NMP), 0)
        q["view_cos"] = r2.uniform(0.99, 1.0, NMP)
        q["level"] = host[f]["octave"][tgt]
        q["flags"] = P["flags"]
        lp.append(q)
    lpts = torch.from_numpy(np.stack(lp).view(np.int32).reshape(B, NMP, 6)).to(dev)
    grid = (0.0, 0.0, np.float32(64) / np.float32(1241), np.float32(48) / np.float32(376))
    sc = np.array([np.float32(1.2) ** i for i in range(8)], np.float32)
    prm = orbx.proj_params(grid, sc, 1.0, 0.8)
    import ctypes
    match = torch.empty((B, cap), dtype=torch.int32, device=dev)
    nm = torch.empty((B,), dtype=torch.int32, device=dev)
    P_ = lambda t_: ctypes.c_void_p(t_.data_ptr())
    call = lambda: orbx.lib.orbm_search_by_projection_device(
        P_(kps), P_(desc), P_(ur), P_(cl), P_(counts), B, cap, P_(lpts), P_(pdesc), P_(npts), NMP, ctypes.byref(prm),
        P_(match), P_(nm), ctypes.c_void_p(s.cuda_stream))
    t = dev_time(call, args.steps, args.warmup, s)
    torch.cuda.synchronize()
    wn, wm = orbref.search_by_projection(host[0], hdesc[0], scenes[0][3], claimed[0], grid, sc, lp[0], scenes[0][2],
                                         1.0, 0.8)
    ok = int(nm[0]) == wn and np.array_equal(match[0, :len(wm)].cpu().numpy(), wm)
    rate, k = cpu_rate(lambda i: orbref.search_by_projection(host[i % B], hdesc[i % B], scenes[i % B][3],
                                                             claimed[i % B], grid, sc, lp[i % B], scenes[i % B][2],
                                                             1.0, 0.8), args.cpu_seconds, NMP)
    out["proj_local"] = {"unit": "MapPoints/s", "value": round(B * NMP / t, 1), "ms_per_launch": round(t * 1e3, 4),
                         "frames": B, "mappoints_per_frame": NMP, "matches_frame0": int(nm[0]), "parity_frame0": ok,
                         "cpu_baseline": {"value": round(rate, 1), "unit": "MapPoints/s", "cores": 1, "kind": "port",
                                          "sample": "oracle orbref_search_by_projection, %d frames" % k}}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--mappoints", type=int, default=1500)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--cpu-seconds", type=float, default=2.0)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(s)
    rows = {"ingest": row_ingest(args, s, dev)}
    print("ingest done", file=sys.stderr, flush=True)
    kb = kitti_batch(args, s, dev)
    rows.update(row_voc_bow(args, s, dev, kb))
    print("voc/bow done", file=sys.stderr, flush=True)
    rows.update(row_pose(args, s, dev, kb))
    print(json.dumps({"bench": "section 8f rows", "n_gpus": 1, "data": "synthetic", "rows": rows}), flush=True)


if __name__ == "__main__":
    main()
