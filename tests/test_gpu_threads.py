"""The host entry points under concurrency, as ORB-SLAM2 runs them.

The reference extracts the left and right images on two threads (src/Frame.cc:94-103) while
LocalMapping (SearchForTriangulation, Fuse: src/LocalMapping.cc:215, 268, 489) and LoopClosing
(SearchByBoW, SearchByProjection(Sim3): src/LoopClosing.cc:265, 375) call ORBmatcher from their own
threads next to Tracking's searches.  ctypes releases the GIL around each C call, so the Python
threads below overlap inside liborbx.  Every result must stay bit-exact against the oracle, and a
host call must not wait for work queued on other streams (no device-wide synchronisation, no legacy
null stream, no per-call hipFree).
"""
import threading
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ITERS = 6


def _oracle_jobs(orbref):
    """Inputs and oracle answers for every job, computed before any thread starts."""
    import orbx_synth
    import test_bow
    import test_proj
    jobs = {}
    p = orbref.make_params(1000, 1.2, 8, 20, 7)
    left = [orbx_synth.gen_image(200 + i, 752, 480) for i in range(3)]
    right = [np.ascontiguousarray(np.roll(im, -7, axis=1)) for im in left]
    jobs["left"] = [(im, orbref.extract(im, p, want_pyramid=False)) for im in left]
    jobs["right"] = [(im, orbref.extract(im, p, want_pyramid=False)) for im in right]
    # SearchForInitialization between consecutive left frames, vbPrevMatched carried over
    r = [x[1] for x in jobs["left"]]
    prev0 = np.stack([r[0].keypoints["x"], r[0].keypoints["y"]], axis=1).astype(np.float32)
    w1 = orbref.search_for_initialization(r[0].keypoints, r[0].descriptors, r[1].keypoints, r[1].descriptors, 752, 480,
                                          prev_xy=prev0)
    w2 = orbref.search_for_initialization(r[0].keypoints, r[0].descriptors, r[2].keypoints, r[2].descriptors, 752, 480,
                                          prev_xy=w1[2])
    jobs["si"] = (r, prev0, w1, w2)
    # SearchByBoW(KF, KF) and SearchForTriangulation (LocalMapping / LoopClosing)
    s = test_bow._kitti_sides(orbref)
    a, b = s[0], s[1]
    wbow = orbref.search_by_bow_kf_kf(a["kps"], a["desc"], a["has_mp"], a["fv"], b["kps"], b["desc"], b["has_mp"],
                                      b["fv"], 0.75, True)
    mp1 = (a["has_mp"] == 0).astype(np.uint8)
    mp2 = (b["has_mp"] == 0).astype(np.uint8)
    F = test_bow._translation_F(-3, -1)
    wtri = orbref.search_for_triangulation(a["kps"], a["desc"], mp1, a["u_right"], a["fv"], b["kps"], b["desc"], mp2,
                                           b["u_right"], b["fv"], F, 600.0, 180.0, test_bow.SCALE, test_bow.SIGMA2,
                                           False, True)
    jobs["bow"] = (a, b, mp1, mp2, F, wbow, wtri)
    # SearchByProjection(Frame, local MapPoints) (Tracking) and brute-force top-2
    sc = test_proj.scene(1)
    kps, desc, ur, cl, grid, pts, pdesc = sc
    jobs["proj"] = (sc, orbref.search_by_projection(kps, desc, ur, cl, grid, test_proj.SCALE, pts, pdesc, 3.0, 0.8))
    q = orbx_synth.random_descriptors(1500, 5)
    t = orbx_synth.random_descriptors(2500, 6)
    jobs["top2"] = (q, t, orbref.allpairs_top2(q, t))
    return jobs


def _run_threads(fns):
    errors = []

    def wrap(fn):
        try:
            fn()
        except BaseException as e:   # noqa: BLE001 -- reported below
            errors.append((fn.__name__, repr(e)))

    th = [threading.Thread(target=wrap, args=(f,)) for f in fns]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in th), "a host-call thread hung"
    assert not errors, errors


def test_extractors_and_matchers_on_concurrent_threads(orbref, cuda):
    import orbx
    import test_bow
    import test_proj
    from test_gpu_parity import assert_same_keypoints
    jobs = _oracle_jobs(orbref)

    def extractor(side):
        def run():
            ex = orbx.ORBextractor(1000, 1.2, 8, 20, 7)
            for it in range(ITERS):
                for im, ref in jobs[side]:
                    k, d = ex(im)
                    assert_same_keypoints(k, ref.keypoints, d, ref.descriptors, "%s it%d" % (side, it))
            ex.close()
        run.__name__ = "extract_" + side
        return run

    def initializer():
        r, prev0, w1, w2 = jobs["si"]
        m = orbx.ORBmatcher(0.9, True)
        for _ in range(ITERS):
            prev = prev0.copy()
            for f, want in ((1, w1), (2, w2)):
                n, m12 = m.SearchForInitialization((r[0].keypoints, r[0].descriptors),
                                                   (r[f].keypoints, r[f].descriptors, (752, 480)), prev, 100)
                assert n == want[0] and np.array_equal(m12, want[1]) and np.array_equal(prev, want[2])

    def local_mapping():
        a, b, mp1, mp2, F, wbow, wtri = jobs["bow"]
        for _ in range(ITERS):
            n, mm = orbx.ORBmatcher(0.75, True).SearchByBoW_KF_KF((a["kps"], a["desc"], a["fv"], a["has_mp"]),
                                                                  (b["kps"], b["desc"], b["fv"], b["has_mp"]))
            assert n == wbow[0] and np.array_equal(mm, wbow[1])
            n, mm = orbx.ORBmatcher(0.6, True).SearchForTriangulation(
                (a["kps"], a["desc"], a["fv"], mp1, a["u_right"]), (b["kps"], b["desc"], b["fv"], mp2, b["u_right"]),
                F, 600.0, 180.0, test_bow.SCALE, test_bow.SIGMA2, False)
            assert n == wtri[0] and np.array_equal(mm, wtri[1])

    def tracking():
        (kps, desc, ur, cl, grid, pts, pdesc), want = jobs["proj"]
        q, t, (wi, w1, w2) = jobs["top2"]
        for _ in range(ITERS):
            n, m = orbx.ORBmatcher(0.8).SearchByProjection(kps, desc, ur, cl, grid, test_proj.SCALE, pts, pdesc, 3.0)
            assert n == want[0] and np.array_equal(m, want[1])
            bi, b1, b2 = orbx.allpairs_host(q, t)
            assert np.array_equal(bi, wi) and np.array_equal(b1, w1) and np.array_equal(b2, w2)

    _run_threads([extractor("left"), extractor("right"), initializer, local_mapping, tracking])


def _spin_cycles_per_ms(cuda):
    import torch
    s = torch.cuda.Stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(s):
        torch.cuda._sleep(1000)   # warm the kernel up
        a.record(s)
        torch.cuda._sleep(2_000_000)
        b.record(s)
    s.synchronize()
    return 2_000_000 / max(a.elapsed_time(b), 1e-3)


@pytest.mark.parametrize("where", ["side_stream", "default_stream"])
def test_host_calls_do_not_wait_for_other_streams(orbref, cuda, where):
    """A long kernel sits on another stream (a fresh torch side stream each round, or the legacy default
    stream); every host matcher / extractor call must return while it is still running.  Besides the
    absence of device-wide synchronisation this needs the library's streams on hardware queues of their
    own: HIP maps streams round-robin onto GPU_MAX_HW_QUEUES queues (4 here) and a shared queue runs in
    order, so liborbx creates its host-path streams at high priority, which HIP keeps apart from the
    application's default-priority streams.  (With default-priority streams about one call in six
    waited behind the sleeping kernel at 4 queues, none at 16.)"""
    import torch
    import orbx
    import orbx_synth
    import test_proj
    if not hasattr(torch.cuda, "_sleep"):
        pytest.skip("torch.cuda._sleep unavailable")
    q = orbx_synth.random_descriptors(300, 1)
    t = orbx_synth.random_descriptors(400, 2)
    kps, desc, ur, cl, grid, pts, pdesc = test_proj.scene(2)
    ex = orbx.ORBextractor(500, 1.2, 8, 20, 7)
    img = orbx_synth.gen_image(9, 640, 480)
    calls = [lambda: orbx.allpairs_host(q, t),
             lambda: orbx.ORBmatcher(0.8).SearchByProjection(kps, desc, ur, cl, grid, test_proj.SCALE, pts, pdesc,
                                                             3.0),
             lambda: ex(img)]
    for c in calls:   # warm every path (pool contexts, handle workspace, code objects) before timing
        c()
    per_ms = _spin_cycles_per_ms(cuda)
    slow = []
    for rnd in range(4):
        for k, c in enumerate(calls):
            s = torch.cuda.Stream() if where == "side_stream" else torch.cuda.default_stream()
            done = torch.cuda.Event()
            with torch.cuda.stream(s):
                torch.cuda._sleep(int(per_ms * 300))   # ~0.3 s
                done.record(s)
            t0 = time.perf_counter()
            c()
            dt = time.perf_counter() - t0
            running = not done.query()
            s.synchronize()
            if not running or dt > 0.15:
                slow.append((rnd, k, round(dt, 3), running))
    assert not slow, "host calls waited for the %s kernel: %s" % (where, slow)


@pytest.mark.parametrize("where", ["side_stream", "default_stream"])
def test_growing_host_calls_do_not_wait_for_other_streams(orbref, cuda, where):
    """Cold variant: every timed call needs a larger pinned staging buffer or device workspace than any call
    before it (host matcher contexts and extractor handles only grow: an outgrown buffer is retired, not
    freed, since hipFree / hipHostFree wait for the whole device).  Only the kernels are warmed, on small
    inputs; each timed call must still return while the sleeping kernel on the other stream runs, and give
    the oracle's result."""
    import torch
    import orbx
    import orbx_synth
    from test_gpu_parity import assert_same_keypoints
    if not hasattr(torch.cuda, "_sleep"):
        pytest.skip("torch.cuda._sleep unavailable")
    ex = orbx.ORBextractor(1000, 1.2, 8, 20, 7)
    ex(orbx_synth.gen_image(3, 320, 240))   # code objects; a small workspace
    orbx.allpairs_host(orbx_synth.random_descriptors(8, 1), orbx_synth.random_descriptors(8, 2))
    per_ms = _spin_cycles_per_ms(cuda)
    p = orbref.make_params(1000, 1.2, 8, 20, 7)
    sizes = [(400, 300), (640, 480), (752, 480), (1241, 376), (1280, 720), (1920, 1080)]
    nq = [600, 2000, 6000, 12000, 30000, 60000]
    slow = []
    for k, ((w, h), n) in enumerate(zip(sizes, nq)):
        img = orbx_synth.gen_image(40 + k, w, h)
        q = orbx_synth.random_descriptors(n, 10 + k)
        t = orbx_synth.random_descriptors(n // 2, 20 + k)
        for j, call in enumerate((lambda: ex(img), lambda: orbx.allpairs_host(q, t))):
            s = torch.cuda.Stream() if where == "side_stream" else torch.cuda.default_stream()
            done = torch.cuda.Event()
            with torch.cuda.stream(s):
                torch.cuda._sleep(int(per_ms * 400))   # ~0.4 s
                done.record(s)
            t0 = time.perf_counter()
            out = call()
            dt = time.perf_counter() - t0
            running = not done.query()
            s.synchronize()
            if not running:
                slow.append((k, j, round(dt, 3)))
            if j == 0:
                ref = orbref.extract(img, p, want_pyramid=False)
                assert_same_keypoints(out[0], ref.keypoints, out[1], ref.descriptors, "%dx%d" % (w, h))
            elif k < 2:
                wi, w1, w2 = orbref.allpairs_top2(q[:200], t)
                assert np.array_equal(out[0][:200], wi) and np.array_equal(out[1][:200], w1)
    assert not slow, "growing host calls waited for the %s kernel: %s" % (where, slow)
