"""Multi-rank path (config 4) on CPU with gloo, world_size 2 and 4: frame
sharding covers every frame exactly once, and the rank-0 gather returns every
rank's padded {keypoints, descriptors, counts} payload intact."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, B, cap, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "orb-slam-_amd"))
    import orbx_dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        pay = orbx_dist.Payload(B, cap, torch.device("cpu"))
        g = torch.Generator().manual_seed(100 + rank)
        pay.kps.copy_(torch.randint(-2**30, 2**30, pay.kps.shape, generator=g, dtype=torch.int32))
        pay.desc.copy_(torch.randint(0, 256, pay.desc.shape, generator=g, dtype=torch.int32).to(torch.uint8))
        pay.counts.copy_(torch.arange(B, dtype=torch.int32) + 10 * rank)
        out = orbx_dist.Gatherer(pay, world, rank).gather()
        if rank == 0:
            ok = len(out) == world
            for r, buf in enumerate(out):
                kps, desc, counts = orbx_dist.Payload.unpack(buf, B, cap)
                g2 = torch.Generator().manual_seed(100 + r)
                ek = torch.randint(-2**30, 2**30, kps.shape, generator=g2, dtype=torch.int32)
                ed = torch.randint(0, 256, desc.shape, generator=g2, dtype=torch.int32).to(torch.uint8)
                ok &= torch.equal(kps, ek) and torch.equal(desc, ed)
                ok &= torch.equal(counts, torch.arange(B, dtype=torch.int32) + 10 * r)
            q.put(bool(ok))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_gather_to_rank0(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, 3, 17, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs)
    assert q.get(timeout=5) is True


def test_shard_range_covers_frames():
    import orbx_dist
    for n in (1, 7, 64, 1024):
        for world in (1, 2, 3, 8):
            seen = []
            for r in range(world):
                a, b = orbx_dist.shard_range(n, r, world)
                seen.extend(range(a, b))
            assert seen == list(range(n))


def _np_top2(q, t):
    x = np.unpackbits(q[:, None, :] ^ t[None, :, :], axis=2).sum(axis=2).astype(np.int32)
    bi = np.argmin(x, axis=1).astype(np.int32)                # first minimum
    b1 = x[np.arange(len(q)), bi]
    xs = x.copy()
    xs[np.arange(len(q)), bi] = 1 << 20
    b2 = xs.min(axis=1) if t.shape[0] > 1 else np.full(len(q), 256, np.int32)
    return bi, b1, np.minimum(b2, 256).astype(np.int32)


def _top2_worker(rank, world, port, nq, nt, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "orb-slam-_amd"))
    import orbx_dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(55)
        Q = rng.integers(0, 256, (nq, 32), dtype=np.uint8)
        T = rng.integers(0, 256, (nt, 32), dtype=np.uint8)
        T[::7] = T[0]                       # duplicated targets: ties across slices
        fn = lambda qq, tt: tuple(torch.from_numpy(a) for a in _np_top2(qq.numpy(), tt.numpy()))
        out = orbx_dist.sharded_top2(torch.from_numpy(Q), torch.from_numpy(T), rank, world, fn)
        if rank == 0:
            want = _np_top2(Q, T)
            q.put(all(np.array_equal(o.numpy(), w) for o, w in zip(out, want)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,nt", [(2, 300), (4, 301), (4, 3)])
def test_sharded_allpairs_top2(world, nt):
    """Config 5 on G ranks: target slices + rank-0 merge == the single-device first-min top-2."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_top2_worker, args=(r, world, port, 50, nt, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs)
    assert q.get(timeout=5) is True


# ---- config 4 with real extractor-format payloads ------------------------------------------
_OR_W, _OR_H, _OR_N, _OR_B = 320, 240, 300, 2   # frames per batch


def _oracle_payload(orbref, frames, cap):
    """The bytes orbx_extract_batch_device leaves in a Payload for `frames`, from the CPU oracle."""
    p = orbref.make_params(_OR_N, 1.2, 8, 20, 7)
    kps = np.zeros((len(frames), cap, 7), np.int32)
    desc = np.zeros((len(frames), cap, 32), np.uint8)
    counts = np.zeros(len(frames), np.int32)
    for f, img in enumerate(frames):
        r = orbref.extract(img, p, want_pyramid=False)
        n = len(r.keypoints)
        kps[f, :n] = np.ascontiguousarray(r.keypoints).view(np.int32).reshape(n, 7)
        desc[f, :n] = r.descriptors
        counts[f] = n
    return np.concatenate([kps.view(np.uint8).ravel(), desc.ravel(), counts.view(np.uint8)])


def _oracle_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "orb-slam-_amd"), os.path.join(root, "oracle")]
    import orbref
    import orbx_dist
    import orbx_synth
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cap = _OR_N + 64
        nfr = 2 * _OR_B * world                        # two batches per rank, contiguous shards
        a, b = orbx_dist.shard_range(nfr, rank, world)
        seq = [orbx_synth.gen_image(900 + i, _OR_W, _OR_H) for i in range(nfr)]
        hb = orbx_dist.HandBack(_OR_B, cap, torch.device("cpu"), world, rank)
        for k in range(2):                             # batch k fills payload k % 2 while k - 1 is in flight
            pl = hb.next_payload()
            mine = _oracle_payload(orbref, seq[a + k * _OR_B:a + (k + 1) * _OR_B], cap)
            pl.buf.copy_(torch.from_numpy(mine))
            hb.send()
        hb.drain()
        if rank == 0:
            ok = True
            for r in range(world):
                ra, _ = orbx_dist.shard_range(nfr, r, world)
                for k in range(2):
                    want = _oracle_payload(orbref, seq[ra + k * _OR_B:ra + (k + 1) * _OR_B], cap)
                    got = hb.payloads[k].buf if r == 0 else hb.gatherers[k].recv[r - 1]
                    kps, desc, counts = orbx_dist.Payload.unpack(got, _OR_B, cap)
                    ok &= bool(np.array_equal(got.numpy(), want)) and int(counts.min()) > 100
            q.put(ok)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_hand_back_of_oracle_payloads(world):
    """Each rank extracts its shard of a frame sequence into the extractor's payload layout (the CPU
    oracle stands in for the device here) and hands two batches back through the double-buffered
    HandBack; rank 0 must hold every rank's payloads byte for byte."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_oracle_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
    assert all(p.exitcode == 0 for p in procs)
    assert q.get(timeout=5) is True


# ---- bench.py's exact hand-back sequencing ------------------------------------------------
_BP_P, _BP_B, _BP_CAP = 3, 2, 5   # pipeline slots, frames per batch, keypoints per frame


def _bench_payload(rank, k):
    """Deterministic payload bytes of rank `rank`'s global step k."""
    kb = _BP_B * _BP_CAP * 28
    db = _BP_B * _BP_CAP * 32
    n = kb + db + _BP_B * 4
    v = (np.arange(n, dtype=np.int64) * 131 + rank * 7919 + k * 104729) % 251
    return torch.from_numpy(v.astype(np.uint8))


def _bench_pattern_worker(rank, world, port, steps, q):
    """Drives HandBack exactly as bench.py's step() does: step k runs on slot k % P, takes the slot's
    next payload (which orders it after that payload's previous send), fills it and sends it.  Rank 0
    checks every peer's every batch as soon as its receive is known complete (the slot's payload comes
    round again two slot-steps later, i.e. global step k - 2P), and the rest after drain()."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "orb-slam-_amd"))
    import orbx_dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        P = _BP_P
        hands = [orbx_dist.HandBack(_BP_B, _BP_CAP, torch.device("cpu"), world, rank) for _ in range(P)]
        seen, bad = set(), []

        def check(recv, kstep):
            for r in range(1, world):
                if not torch.equal(recv[r - 1], _bench_payload(r, kstep)):
                    bad.append((r, kstep))
                seen.add((r, kstep))

        for k in range(steps):
            j = k % P
            hb = hands[j]
            i = hb.k % 2
            pl = hb.next_payload()
            if rank == 0 and hb.k >= 2:
                check(hb.gatherers[i].recv, k - 2 * P)
            pl.buf.copy_(_bench_payload(rank, k))
            hb.send()
        for hb in hands:
            hb.drain()
        if rank == 0:
            for j, hb in enumerate(hands):
                for s in (hb.k - 2, hb.k - 1):
                    if s >= 0:
                        check(hb.gatherers[s % 2].recv, s * P + j)
            want = {(r, k) for r in range(1, world) for k in range(steps)}
            q.put((not bad) and seen == want)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,steps", [(2, 13), (4, 20)])
def test_hand_back_in_bench_sequence(world, steps):
    """bench.py's multi-GPU pattern on gloo: P = 3 pipeline slots, each its own double-buffered HandBack,
    sends interleaved across slots over many steps (a step count that is not a multiple of P); rank 0
    receives every rank's every batch byte for byte, each in its slot's order."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_pattern_worker, args=(r, world, port, steps, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs)
    assert q.get(timeout=5) is True
