import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "orb-slam-_amd"), os.path.join(ROOT, "oracle")]
import numpy as np, torch
import orbx, orbx_dist, orbx_synth, orbref
dev = torch.device("cuda", 0)
B, nb = 64, 8
seq = orbx_synth.kitti_sequence(B * nb)
frames = torch.from_numpy(seq).to(dev)
ex = orbx.ORBextractor(2000, 1.2, 8, 20, 7)
cap = ex.capacity(376, 1241)
pay = orbx_dist.Payload(B, cap, dev)
m = orbx.ORBmatcher(0.9, True)
pa = torch.arange(0, B - 1, dtype=torch.int32, device=dev)
pb = torch.arange(1, B, dtype=torch.int32, device=dev)
m12 = torch.empty((B - 1, cap), dtype=torch.int32, device=dev)
nm = torch.empty((B - 1,), dtype=torch.int32, device=dev)
s = torch.cuda.current_stream()
for k in range(12):
    base = (k % nb) * B
    ex.extract_batch_device(frames[base:base + B], pay.kps, pay.desc, pay.counts, s)
    m.search_for_initialization_batch(pay.kps, pay.desc, pay.counts, pa, pb, 376, 1241, 100, m12, nm, s)
    torch.cuda.synchronize()
    n = nm.cpu().numpy()
    print("step", k, "base", base, "nm min/mean/max", n.min(), n.mean(), n.max(), "counts", pay.counts.cpu().numpy()[:4], flush=True)
# oracle check of batch 6 pair 0
klist = orbx.keypoints_from_device(pay.kps, pay.counts)
d = pay.desc.cpu().numpy(); c = pay.counts.cpu().numpy()
want_n, want_m, _ = orbref.search_for_initialization(klist[0], d[0, :c[0]], klist[1], d[1, :c[1]], 1241, 376)
print("oracle on last batch pair0:", want_n, "gpu:", nm.cpu().numpy()[0])
p = orbref.make_params(2000, 1.2, 8, 20, 7)
r0 = orbref.extract(seq[(11 % nb) * B], p, want_pyramid=False)
print("oracle kps", len(r0.keypoints), "gpu", c[0], "same x:", np.array_equal(r0.keypoints["x"], klist[0]["x"]))
