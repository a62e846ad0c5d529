"""FAST phase profile: cycles per cell of each phase, summed over all waves (instrumented build:
orb-slam-_amd/build_fprof/liborbx.so compiled with -DORBX_FAST_PROF, tools/diag/build_alt.sh), KITTI
384-frame batch, one stream.  Phases: staging commit (waits for the prefetched ROI loads), map clear,
pass 1 (compass), pass 2 (strength), NMS, output, and loop/setup overhead."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["ORBX_LIB"] = os.path.join(ROOT, "orb-slam-_amd", sys.argv[1] if len(sys.argv) > 1 else "build_fprof",
                                      "liborbx.so")
sys.path[:0] = [os.path.join(ROOT, "orb-slam-_amd")]
import numpy as np, torch, orbx, orbx_synth
dev = torch.device("cuda", 0)
B = 384
frames = torch.from_numpy(orbx_synth.kitti_sequence(B)).to(dev)
ex = orbx.ORBextractor(2000, 1.2, 8, 20, 7)
cap = ex.capacity(376, 1241)
kps = torch.empty((B, cap, 7), dtype=torch.int32, device=dev)
desc = torch.empty((B, cap, 32), dtype=torch.uint8, device=dev)
cnt = torch.empty((B,), dtype=torch.int32, device=dev)
fn = orbx.lib.orbx_debug_fast_prof
fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = np.zeros(8, np.uint64)
for it in range(4):
    ex.extract_batch_device(frames, kps, desc, cnt)
    torch.cuda.synchronize()
    if it == 0:
        fn(buf.ctypes.data, 1)
fn(buf.ctypes.data, 0)
cells = max(int(buf[6]), 1)
names = ["commit", "mapclr", "pass1", "pass2", "nms", "output", "loop"]
idx = [0, 1, 2, 3, 4, 5, 7]
tot = sum(int(buf[k]) for k in idx)
print("cells %d" % cells)
for n, k in zip(names, idx):
    print("%-8s %8.0f cycles/cell  %5.1f%%" % (n, buf[k] / cells, 100.0 * buf[k] / tot))
