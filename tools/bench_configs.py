#!/usr/bin/env python3
"""Secondary benchmarks: the BASELINE.json configs other than the headline (bench.py = config 2/4).

  python tools/bench_configs.py --config 1     TUM 640x480, 1000 feat: host-API latency per frame
                                               (PCIe included) next to the CPU oracle
  python tools/bench_configs.py --config 3     EuRoC 752x480 stereo pair, 1000 feat/image: extract
                                               both + Frame::ComputeStereoMatches on device
  python tools/bench_configs.py --config 5     1920x1080, 4000 feat extraction + 10k x 10k 256-bit
                                               Hamming (TOP2 and FULL_U16); --gpus N under
                                               torch.distributed.run shards the targets

Each prints one JSON line (rank 0).  Inputs are synthetic (orbx_synth) and, except for
config 1's host path, already resident in HBM when the timed region starts.
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
import torch.distributed as dist  # noqa: E402

import orbx  # noqa: E402
import orbx_dist  # noqa: E402
import orbx_synth  # noqa: E402

HBM_PEAK_GBS = 8000.0
EUROC_BF, EUROC_FX = 47.90639384423901, 435.2046959714599   # Examples/Stereo/EuRoC.yaml:8,25


def timed(fn, steps, warmup, stream):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(steps):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps, e0.elapsed_time(e1) / steps * 1e-3


def cpu_loop(fn, budget_s):
    t0 = time.perf_counter()
    n = 0
    while True:
        fn(n)
        n += 1
        if time.perf_counter() - t0 >= budget_s:
            break
    return n, time.perf_counter() - t0


def config1(args):
    import orbref
    W, H, NF = 640, 480, 1000
    frames = np.stack([orbx_synth.gen_image(1 + i, W, H) for i in range(16)])
    ex = orbx.ORBextractor(NF, 1.2, 8, 20, 7)
    for i in range(3):
        ex(frames[i])
    t0 = time.perf_counter()
    for k in range(args.steps):
        ex(frames[k % 16])
    dt = (time.perf_counter() - t0) / args.steps
    p = orbref.make_params(NF, 1.2, 8, 20, 7)
    n, ct = cpu_loop(lambda i: orbref.extract(frames[i % 16], p, want_pyramid=False), args.cpu_seconds)
    return {"config": "config1_tum_640x480_1000feat_host_api", "metric": "ms per frame, ORBextractor::operator() "
            "host path (H2D image, D2H keypoints+descriptors)", "value": round(dt * 1e3, 4), "unit": "ms/frame",
            "higher_is_better": False, "frames_per_s": round(1.0 / dt, 1),
            "cpu_baseline": {"value": round(ct / n * 1e3, 3), "unit": "ms/frame", "cores": 1, "kind": "port",
                             "sample": "oracle/orbref scalar C, %d frames, %.1f s" % (n, ct)}}


def config3(args):
    import orbref
    W, H, NF, B = 752, 480, args.feat or 1000, args.batch or 96
    dev = torch.device("cuda", 0)
    pairs = [orbx_synth.stereo_pair(100 + i, W, H) for i in range(B)]
    frames = torch.from_numpy(np.stack([im for pr in pairs for im in pr])).to(dev)   # L0 R0 L1 R1 ...
    ex = orbx.ORBextractor(NF, 1.2, 8, 20, 7)
    cap = ex.capacity(H, W)
    kps = torch.empty((2 * B, cap, 7), dtype=torch.int32, device=dev)
    desc = torch.empty((2 * B, cap, 32), dtype=torch.uint8, device=dev)
    counts = torch.empty((2 * B,), dtype=torch.int32, device=dev)
    li = torch.arange(0, 2 * B, 2, dtype=torch.int32, device=dev)
    ri = li + 1
    ur = torch.empty((B, cap), dtype=torch.float32, device=dev)
    dp = torch.empty_like(ur)
    ng = torch.empty((B,), dtype=torch.int32, device=dev)
    s = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(s)
    st = {}

    def step():
        ex.extract_batch_device(frames, kps, desc, counts, s)
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(s)
        ex.stereo_batch_device(kps, desc, counts, li, ri, EUROC_BF, EUROC_FX, ur, dp, ng, s)
        e1.record(s)
        st.setdefault("ev", []).append((e0, e1))

    wall, dev_t = timed(step, args.steps, args.warmup, s)
    ex.sync(s)
    stereo_ms = np.mean([a.elapsed_time(b) for a, b in st["ev"][args.warmup:]])
    nkl = counts[0::2].float().mean().item()
    p = orbref.make_params(NF, 1.2, 8, 20, 7)

    def cpu_pair(i):
        L, R = pairs[i % B]
        a, b = orbref.extract(L, p), orbref.extract(R, p)
        orbref.compute_stereo_matches(p, a, b, H, W, EUROC_BF, EUROC_FX)

    n, ct = cpu_loop(cpu_pair, args.cpu_seconds)
    value = B / wall
    # stereo kernel algorithmic bytes per pair: both keypoint sets + descriptors in, the
    # 11x11 left and 11x21 right windows of every left keypoint, uRight/depth out
    alg = (2 * nkl * (28 + 32) + nkl * (121 + 231) + nkl * 8)
    return {"config": "config3_euroc_752x480_stereo_%dfeat" % NF,
            "metric": "stereo frames/s (extract L+R + ComputeStereoMatches)", "value": round(value, 1),
            "unit": "stereo pairs/s", "higher_is_better": True, "n_gpus": 1, "pairs_per_step": B,
            "ms_per_step": round(wall * 1e3, 4), "stereo_kernels_ms_per_step": round(float(stereo_ms), 4),
            "keypoints_left": round(nkl, 1), "stereo_matches_per_pair": round(ng.float().mean().item(), 1),
            "stereo_roofline": {"bound": "hbm", "achieved": round(alg * B / (stereo_ms * 1e-3) / 1e9, 2),
                                "peak": HBM_PEAK_GBS, "unit": "GB/s"},
            "cpu_baseline": {"value": round(n / ct, 2), "unit": "stereo pairs/s", "cores": 1, "kind": "port",
                             "sample": "oracle/orbref scalar C: extract L, extract R, ComputeStereoMatches; "
                                       "%d pairs in %.1f s" % (n, ct)},
            "speedup_vs_cpu": round(value / (n / ct), 1)}


def config5(args, world, rank, local):
    import orbref
    dev = torch.device("cuda", local)
    W, H, NF, B = 1920, 1080, 4000, args.batch or 128
    out = {"config": "config5_1920x1080_4000feat + 10k x 10k Hamming", "n_gpus": world}
    # extraction (frames sharded like config 4: every rank its own batch)
    frames = torch.from_numpy(np.stack([orbx_synth.gen_image(5 + 97 * rank + i, W, H) for i in range(B)])).to(dev)
    ex = orbx.ORBextractor(NF, 1.2, 8, 20, 7, device=local)
    cap = ex.capacity(H, W)
    kps = torch.empty((B, cap, 7), dtype=torch.int32, device=dev)
    desc = torch.empty((B, cap, 32), dtype=torch.uint8, device=dev)
    counts = torch.empty((B,), dtype=torch.int32, device=dev)
    s = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(s)
    wall, _ = timed(lambda: ex.extract_batch_device(frames, kps, desc, counts, s), args.steps, args.warmup, s)
    ex.sync(s)
    out["extract_frames_per_s"] = round(world * B / wall, 1)
    out["keypoints_per_frame"] = round(counts.float().mean().item(), 1)
    # 10k x 10k all-pairs: seeded uniform descriptors, 10% of queries with a planted target at distance 5..20
    rng = np.random.default_rng(55)
    nq = nt = 10000
    Q = rng.integers(0, 256, (nq, 32), dtype=np.uint8)
    T = rng.integers(0, 256, (nt, 32), dtype=np.uint8)
    plant = rng.choice(nq, nq // 10, replace=False)
    for i in plant:
        j = int(rng.integers(0, nt))
        bits = np.unpackbits(Q[i])
        flip = rng.choice(256, int(rng.integers(5, 21)), replace=False)
        bits[flip] ^= 1
        T[j] = np.packbits(bits)
    q, t = torch.from_numpy(Q).to(dev), torch.from_numpy(T).to(dev)
    if world > 1:
        dist.barrier()
    res = {}

    def top2():
        res["r"] = orbx_dist.sharded_top2(q, t, rank, world, lambda a, b: orbx.allpairs(a, b, orbx.TOP2, s))

    wall2, _ = timed(top2, args.steps, args.warmup, s)
    if world > 1:
        tt = torch.tensor([wall2], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        wall2 = float(tt.item())
    out["top2_pairs_per_s"] = round(nq * nt / wall2, 1)
    out["top2_ms"] = round(wall2 * 1e3, 4)
    if rank == 0:
        bi, b1, b2 = (x.cpu().numpy() for x in res["r"])
        sub = np.arange(0, nq, 97)
        wbi, wb1, wb2 = orbref.allpairs_top2(Q[sub], T)
        out["top2_parity_sampled"] = bool(np.array_equal(bi[sub], wbi) and np.array_equal(b1[sub], wb1) and
                                          np.array_equal(b2[sub], wb2))
        wall3, dev3 = timed(lambda: orbx.allpairs(q, t, orbx.FULL_U16, s), args.steps, args.warmup, s)
        alg = 2 * 32 * (nq + nt) + 2 * nq * nt
        out["full_u16_ms"] = round(dev3 * 1e3, 4)
        out["full_u16_roofline"] = {"bound": "hbm", "achieved": round(alg / dev3 / 1e9, 1), "peak": HBM_PEAK_GBS,
                                    "unit": "GB/s", "frac": round(alg / dev3 / 1e9 / HBM_PEAK_GBS, 4),
                                    "alg_bytes": alg}
        p = orbref.make_params(NF, 1.2, 8, 20, 7)
        img = frames[0].cpu().numpy()
        n, ct = cpu_loop(lambda i: orbref.extract(img, p, want_pyramid=False), args.cpu_seconds / 2)
        sub2 = np.arange(0, nq, 10)
        c0 = time.perf_counter()
        orbref.allpairs_top2(Q[sub2], T)
        ctp = time.perf_counter() - c0
        out["cpu_baseline"] = {"extract_frames_per_s": round(n / ct, 3),
                               "top2_pairs_per_s": round(len(sub2) * nt / ctp, 1), "cores": 1, "kind": "port",
                               "sample": "oracle/orbref scalar C: %d 1080p extractions; top-2 of %d queries x %d "
                                         "targets" % (n, len(sub2), nt)}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, required=True, choices=[1, 3, 5])
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--feat", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=8.0)
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    if args.config == 1:
        out = config1(args)
    elif args.config == 3:
        out = config3(args)
    else:
        out = config5(args, world, rank, local)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
