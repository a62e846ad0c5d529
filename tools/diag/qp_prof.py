"""k_qt_paths phase profile: per level, average cycles per workgroup of each phase (instrumented build
orb-slam-_amd/build_prof/liborbx.so, -DORBX_QT_PROF), KITTI 192-frame batch, one stream."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["ORBX_LIB"] = os.path.join(ROOT, "orb-slam-_amd", sys.argv[1] if len(sys.argv) > 1 else "build_prof", "liborbx.so")
sys.path[:0] = [os.path.join(ROOT, "orb-slam-_amd")]
import numpy as np, torch, orbx, orbx_synth
dev = torch.device("cuda", 0)
B = 192
frames = torch.from_numpy(orbx_synth.kitti_sequence(B)).to(dev)
ex = orbx.ORBextractor(2000, 1.2, 8, 20, 7)
cap = ex.capacity(376, 1241)
kps = torch.empty((B, cap, 7), dtype=torch.int32, device=dev)
desc = torch.empty((B, cap, 32), dtype=torch.uint8, device=dev)
cnt = torch.empty((B,), dtype=torch.int32, device=dev)
fn = orbx.lib.orbx_debug_qt_prof
fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = np.zeros((16, 16), np.uint64)
for it in range(4):
    ex.extract_batch_device(frames, kps, desc, cnt)
    torch.cuda.synchronize()
    if it == 0:
        fn(buf.ctypes.data, 1)
fn(buf.ctypes.data, 0)
names = ["counts", "gather", "keys", "binscan", "rank", "stats", "nodes", "list", "#wg", "p2.tail", "#p2rnd",
         "retain", "p2.A", "p2.C", "p2.D", "p2.init"]
print("level  " + " ".join("%8s" % n for n in names) + "     total")
for l in range(8):
    wg = max(int(buf[l, 8]), 1)
    tot = sum(buf[l, k] for k in (0, 1, 2, 3, 4, 5, 6, 7, 9, 11, 12, 13, 14, 15)) / wg
    print("%5d  " % l + " ".join("%8.0f" % (buf[l, k] / wg) for k in range(16)) + "  %8.0f" % tot)
