"""Pipeline schedules for config 2 (KITTI, 384-frame batches, extract + SearchForInitialization), device-resident:

  default  bench.py's: P streams, batch k on stream k % P, each stream in order (extract -> match)
  split    two streams: V runs the VALU-bound stages (FAST, describe) back to back, alternating batches
           (FAST(i), describe(i-1), FAST(i+1), ...); L runs the latency-bound ones (quadtree, match, pyramid)
           of the neighbouring batches beside them; events order each batch's stages
           (orbx_extract_stage_device).  P workspaces rotate.

Prints frames/s of each schedule (alternating runs) and checks that both give the same keypoints,
descriptors and matches for the last batch."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "orb-slam-_amd")]
import torch  # noqa: E402
import orbx  # noqa: E402
import orbx_synth  # noqa: E402

H, W = 376, 1241
ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=384)
ap.add_argument("--steps", type=int, default=100)
ap.add_argument("--warmup", type=int, default=10)
ap.add_argument("--P", type=int, default=3)
ap.add_argument("--rounds", type=int, default=2)
ap.add_argument("--lstreams", type=int, default=1, help="split: 1 = quadtree, match and pyramid on one stream; "
                "2 = match on a stream of its own")
ap.add_argument("--lprio", type=int, default=0, help="split: priority of the latency-bound streams L, L2 "
                "(-1 = high: the dispatcher places their workgroups first as CU space frees)")
args = ap.parse_args()
dev = torch.device("cuda", 0)
B, P, nb = args.batch, args.P, 4
frames = torch.from_numpy(orbx_synth.kitti_sequence(B * nb)).to(dev)
exs = [orbx.ORBextractor(2000, 1.2, 8, 20, 7) for _ in range(P)]
cap = exs[0].capacity(H, W)
kps = [torch.empty((B, cap, 7), dtype=torch.int32, device=dev) for _ in range(P)]
desc = [torch.empty((B, cap, 32), dtype=torch.uint8, device=dev) for _ in range(P)]
cnt = [torch.empty((B,), dtype=torch.int32, device=dev) for _ in range(P)]
m12 = [torch.empty((B - 1, cap), dtype=torch.int32, device=dev) for _ in range(P)]
nm = [torch.empty((B - 1,), dtype=torch.int32, device=dev) for _ in range(P)]
pa = torch.arange(0, B - 1, dtype=torch.int32, device=dev)
pb = torch.arange(1, B, dtype=torch.int32, device=dev)
matcher = orbx.ORBmatcher(0.9, True)
streams = [torch.cuda.Stream(device=dev) for _ in range(P)]
V = streams[0]
if args.lprio:
    L = torch.cuda.Stream(device=dev, priority=args.lprio)
    L2 = torch.cuda.Stream(device=dev, priority=args.lprio) if args.lstreams > 1 else L
else:
    L = streams[1]
    L2 = streams[2] if args.lstreams > 1 and P > 2 else L


def imgs(i):
    b = (i % nb) * B
    return frames[b:b + B]


def run_default(n0, n):
    for i in range(n0, n0 + n):
        j = i % P
        exs[j].extract_batch_device(imgs(i), kps[j], desc[j], cnt[j], streams[j])
        matcher.search_for_initialization_batch(kps[j], desc[j], cnt[j], pa, pb, H, W, 100, m12[j], nm[j], streams[j])


def run_split(n0, n):
    ev = {}

    def rec(name, i, s):
        e = torch.cuda.Event()
        e.record(s)
        ev[(name, i)] = e

    def stage(st, i, s):
        j = i % P
        exs[j].extract_stage_device(st, imgs(i), kps[j], desc[j], cnt[j], s)

    def match(i, s):
        j = i % P
        matcher.search_for_initialization_batch(kps[j], desc[j], cnt[j], pa, pb, H, W, 100, m12[j], nm[j], s)

    # the previous call's work is complete (caller synchronises), so every slot is free
    stage(0, n0, L)
    rec("pyr", n0, L)
    last = n0 + n - 1
    for i in range(n0, n0 + n + 1):
        # L: quadtree(i-1), match(i-2), pyramid(i+1)
        if i - 1 >= n0:
            L.wait_event(ev[("fast", i - 1)])
            stage(2, i - 1, L)
            rec("qt", i - 1, L)
        if i - 2 >= n0:
            L2.wait_event(ev[("desc", i - 2)])
            match(i - 2, L2)
            rec("match", i - 2, L2)
        if i + 1 <= last:
            if i + 1 - P >= n0:   # slot (i+1) % P: its previous batch's describe and match are done
                L.wait_event(ev[("desc", i + 1 - P)])
                L.wait_event(ev[("match", i + 1 - P)])
            stage(0, i + 1, L)
            rec("pyr", i + 1, L)
        # V: FAST(i), describe(i-1)
        if i <= last:
            V.wait_event(ev[("pyr", i)])
            stage(1, i, V)
            rec("fast", i, V)
        if i - 1 >= n0:
            V.wait_event(ev[("qt", i - 1)])
            stage(3, i - 1, V)
            rec("desc", i - 1, V)
    L2.wait_event(ev[("desc", last)])
    match(last, L2)


def timed(fn):
    torch.cuda.synchronize()
    fn(0, args.warmup)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn(args.warmup, args.steps)
    torch.cuda.synchronize()
    return B * args.steps / (time.perf_counter() - t0)


res = {"default": [], "split": []}
for r in range(args.rounds):
    for name, fn in (("default", run_default), ("split", run_split)):
        res[name].append(timed(fn))
        print("%-8s round %d: %.1f frames/s" % (name, r, res[name][-1]), flush=True)
# parity: the last batch of each schedule, same frames
last = args.warmup + args.steps - 1
j = last % P
run_default(last, 1)
torch.cuda.synchronize()
ref = (kps[j].clone(), desc[j].clone(), cnt[j].clone(), m12[j].clone(), nm[j].clone())
run_split(last, 1)
torch.cuda.synchronize()
same = all(torch.equal(a, b) for a, b in zip(ref, (kps[j], desc[j], cnt[j], m12[j], nm[j])))
for e in exs:
    e.sync(V)
print("split == default on the last batch: %s" % same)
print("best: default %.1f, split %.1f frames/s" % (max(res["default"]), max(res["split"])))
