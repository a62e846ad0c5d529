"""Which host entry points wait for work on the legacy default (null) stream?"""
import sys, time, os
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "orb-slam-_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import numpy as np, torch, orbx, orbx_synth, test_proj

q = orbx_synth.random_descriptors(300, 1)
t = orbx_synth.random_descriptors(400, 2)
kps, desc, ur, cl, grid, pts, pdesc = test_proj.scene(2)
ex = orbx.ORBextractor(500, 1.2, 8, 20, 7)
img = orbx_synth.gen_image(9, 640, 480)
calls = {
    "allpairs_host": lambda: orbx.allpairs_host(q, t),
    "search_by_projection": lambda: orbx.ORBmatcher(0.8).SearchByProjection(kps, desc, ur, cl, grid, test_proj.SCALE, pts, pdesc, 3.0),
    "extract": lambda: ex(img),
}
for k, f in calls.items():
    f()
torch.cuda.synchronize()
s0 = torch.cuda.Stream()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
with torch.cuda.stream(s0):
    torch.cuda._sleep(1000); a.record(s0); torch.cuda._sleep(2_000_000); b.record(s0)
s0.synchronize()
per_ms = 2_000_000 / a.elapsed_time(b)
print("cycles per ms", per_ms)
for k, f in list(calls.items()) * 8:
    for where in ("default", "side"):
        s = torch.cuda.default_stream() if where == "default" else torch.cuda.Stream()
        with torch.cuda.stream(s):
            torch.cuda._sleep(int(per_ms * 500))
        t0 = time.perf_counter()
        f()
        dt = time.perf_counter() - t0
        s.synchronize()
        print("%-22s %-8s %.1f ms" % (k, where, dt * 1e3), flush=True)
