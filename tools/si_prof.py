"""Phase cycle counts of k_si_greedy (build liborbx with -DORBX_SI_PROF first)."""
import sys, os
if os.environ.get("ORBX_LIB") is None and os.path.exists(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "orb-slam-_amd", "build_prof_si", "liborbx.so")):
    os.environ["ORBX_LIB"] = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "orb-slam-_amd", "build_prof_si", "liborbx.so")
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "orb-slam-_amd"))
import numpy as np, torch
import orbx, orbx_synth
B = 16
ex = orbx.ORBextractor(2000, 1.2, 8, 20, 7)
imgs = torch.from_numpy(orbx_synth.kitti_sequence(B)).cuda()
cap = ex.capacity(376, 1241)
kps = torch.empty((B, cap, 7), dtype=torch.int32, device="cuda")
desc = torch.empty((B, cap, 32), dtype=torch.uint8, device="cuda")
counts = torch.empty((B,), dtype=torch.int32, device="cuda")
s = torch.cuda.current_stream()
ex.extract_batch_device(imgs, kps, desc, counts, s)
pa = torch.arange(0, B - 1, dtype=torch.int32, device="cuda")
pb = pa + 1
m = orbx.ORBmatcher(0.9, True)
for it in range(3):
    m12, nm = m.search_for_initialization_batch(kps, desc, counts, pa, pb, 376, 1241, 100, stream=s)
ex.sync(s)
t = m12.view(B - 1, cap)[:, cap - 4:].cpu().numpy()
c = m12.view(B - 1, cap)[:, cap - 6:cap - 4].cpu().numpy()
print("chunks, full-window scans per pair:", c[:6].tolist(), "mean", c.mean(axis=0).tolist())
print("staging cycles, loop cycles, post cycles, n10 (per pair):")
print(t[:6])
print("loop cycles per step: %.0f" % (t[:, 1] / t[:, 3]).mean())
