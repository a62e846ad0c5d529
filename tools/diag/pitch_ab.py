"""Extraction of 384 KITTI frames with the input at its own width as pitch (1241: unaligned rows) or padded to a
4-byte-aligned pitch (--pad 1248), same pixels.  Prints the extraction time per batch and checks that both
pitches give the same keypoints and descriptors.  Per-kernel times: run under rocprofv3 --kernel-trace --stats,
once per --pad value."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "orb-slam-_amd")]
import torch  # noqa: E402
import orbx  # noqa: E402
import orbx_synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--pad", type=int, default=0, help="row pitch (0: the width)")
ap.add_argument("--batch", type=int, default=384)
ap.add_argument("--steps", type=int, default=30)
args = ap.parse_args()
H, W, B = 376, 1241, args.batch
dev = torch.device("cuda", 0)
src = torch.from_numpy(orbx_synth.kitti_sequence(B)).to(dev)
if args.pad:
    buf = torch.zeros((B, H, args.pad), dtype=torch.uint8, device=dev)
    buf[:, :, :W] = src
    imgs = buf[:, :, :W]
else:
    imgs = src
ex = orbx.ORBextractor(2000, 1.2, 8, 20, 7)
cap = ex.capacity(H, W)
kps = torch.zeros((B, cap, 7), dtype=torch.int32, device=dev)
desc = torch.zeros((B, cap, 32), dtype=torch.uint8, device=dev)
cnt = torch.zeros((B,), dtype=torch.int32, device=dev)
s = torch.cuda.Stream(device=dev)
for _ in range(3):
    ex.extract_batch_device(imgs, kps, desc, cnt, s)
ex.sync(s)
t0 = time.perf_counter()
for _ in range(args.steps):
    ex.extract_batch_device(imgs, kps, desc, cnt, s)
ex.sync(s)
dt = (time.perf_counter() - t0) / args.steps
print("pitch %d: %.3f ms per %d-frame batch" % (imgs.stride(1), dt * 1e3, B), flush=True)
if args.pad:   # parity with the contiguous input
    k2 = torch.zeros_like(kps)
    d2 = torch.zeros_like(desc)
    c2 = torch.zeros_like(cnt)
    ex.extract_batch_device(src, k2, d2, c2, s)
    ex.sync(s)
    same = torch.equal(cnt, c2) and all(torch.equal(kps[f, :cnt[f]], k2[f, :cnt[f]]) and
                                        torch.equal(desc[f, :cnt[f]], d2[f, :cnt[f]]) for f in range(B))
    print("padded == contiguous: %s" % same)
    sys.exit(0 if same else 1)
