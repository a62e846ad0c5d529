"""Single-frame host path (config 1: TUM 640x480, 1000 features) latency: wall time per orbx_extract call and,
under rocprofv3 --kernel-trace, the kernels of the calls.  python tools/diag/host_latency.py [calls]"""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "orb-slam-_amd")]
import numpy as np
import orbx, orbx_synth
n = int(sys.argv[1]) if len(sys.argv) > 1 else 400
frames = np.stack([orbx_synth.gen_image(1 + i, 640, 480) for i in range(16)])
ex = orbx.ORBextractor(1000, 1.2, 8, 20, 7)
for i in range(20):
    ex(frames[i % 16])
t = []
for k in range(n):
    t0 = time.perf_counter()
    ex(frames[k % 16])
    t.append(time.perf_counter() - t0)
t = np.array(t) * 1e3
print("ms per call: mean %.4f  median %.4f  p10 %.4f  p90 %.4f" % (t.mean(), np.median(t), np.percentile(t, 10),
                                                                   np.percentile(t, 90)))
