"""BASELINE config 4 on the GPU box: the frame-sharded replay (orbx_dist.py) with two ranks
sharing cuda:0 over gloo (the box has one GPU; RCCL needs one GPU per rank).  Each rank owns a contiguous
shard of a KITTI 1241x376 / 2000-feature sequence (orbx_dist.shard_range), runs orbx_extract_batch_device +
orbm_search_init_batch_device on its batches on its own stream, and hands every batch back to rank 0 through
the double-buffered HandBack, device payloads staged through pinned host buffers for gloo.  Rank 0 checks
every frame's keypoints and descriptors and every consecutive pair's matches against the CPU oracle: the pairs
inside a batch from the ranks' own match results, the pairs that straddle two batches or two shards by
matching the handed-back payloads on rank 0's device (the one-frame halo of §8e).

The reference's only concurrency on this path is the left / right extraction threads
(/root/reference/src/Frame.cc:94-103); the sharding itself has no reference counterpart to compare with."""
import os
import socket
import traceback

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

W, H, NFEAT = 1241, 376, 2000
B, NB = 3, 2          # frames per batch, batches per rank


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, nfr, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "orb-slam-_amd"), os.path.join(root, "oracle"), os.path.join(root, "tests")]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    errs = []
    try:
        import orbx
        import orbx_dist
        import orbx_synth
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        a, b = orbx_dist.shard_range(nfr, rank, world)
        assert b - a == B * NB
        frames = torch.from_numpy(orbx_synth.kitti_sequence(b - a, start=a)).to(dev)
        ex = orbx.ORBextractor(NFEAT, 1.2, 8, 20, 7, device=0)
        cap = ex.capacity(H, W)
        m = orbx.ORBmatcher(0.9, True)
        s = torch.cuda.Stream(device=dev)
        hb = orbx_dist.HandBack(B, cap, dev, world, rank, host_stage=True)
        pa = torch.arange(0, B - 1, dtype=torch.int32, device=dev)
        pb = torch.arange(1, B, dtype=torch.int32, device=dev)
        mine = []   # (matches12, nmatches) of the in-batch pairs, per batch
        with torch.cuda.stream(s):
            for k in range(NB):
                pl = hb.next_payload()
                ex.extract_batch_device(frames[k * B:(k + 1) * B], pl.kps, pl.desc, pl.counts, s)
                m12, nm = m.search_for_initialization_batch(pl.kps, pl.desc, pl.counts, pa, pb, H, W, 100, stream=s)
                mine.append((m12, nm))
                hb.send()
            hb.drain()
        ex.sync(s)
        # the in-batch match results go to rank 0 as well (host tensors over gloo)
        res = torch.cat([torch.cat([m12.flatten(), nm]) for m12, nm in mine]).cpu()
        if rank != 0:
            dist.send(res, 0)
        else:
            import orbref
            from test_gpu_parity import assert_same_keypoints
            allres = [res] + [torch.empty_like(res) for _ in range(world - 1)]
            for r in range(1, world):
                dist.recv(allres[r], r)
            p = orbref.make_params(NFEAT, 1.2, 8, 20, 7)
            seq = orbx_synth.kitti_sequence(nfr)
            refs = [orbref.extract(seq[i], p, want_pyramid=False) for i in range(nfr)]
            # every frame's payload, in sequence order (rank r's batch k holds frames a_r + kB .. a_r + kB + B - 1)
            kps_all = torch.empty((nfr, cap, 7), dtype=torch.int32)
            desc_all = torch.empty((nfr, cap, 32), dtype=torch.uint8)
            cnt_all = torch.empty((nfr,), dtype=torch.int32)
            for r in range(world):
                ra, _ = orbx_dist.shard_range(nfr, r, world)
                for k in range(NB):
                    buf = hb.payloads[k % 2].buf.cpu() if r == 0 else hb.gatherers[k % 2].recv[r - 1]
                    kk, dd, cc = orbx_dist.Payload.unpack(buf, B, cap)
                    i0 = ra + k * B
                    kps_all[i0:i0 + B], desc_all[i0:i0 + B], cnt_all[i0:i0 + B] = kk, dd, cc
            klist = orbx.keypoints_from_device(kps_all, cnt_all)
            for i in range(nfr):
                n = len(refs[i].keypoints)
                try:
                    assert n > 1500
                    assert_same_keypoints(klist[i], refs[i].keypoints, desc_all[i, :n].numpy(), refs[i].descriptors,
                                          "frame %d" % i)
                except AssertionError as e:
                    errs.append(str(e))
            want = {}
            for i in range(1, nfr):
                nmw, mw, _ = orbref.search_for_initialization(refs[i - 1].keypoints, refs[i - 1].descriptors,
                                                              refs[i].keypoints, refs[i].descriptors, W, H)
                want[i] = (nmw, mw)
            checked = set()
            per = NB * ((B - 1) * cap + (B - 1))
            for r in range(world):
                ra, _ = orbx_dist.shard_range(nfr, r, world)
                rr = allres[r]
                assert rr.numel() == per
                for k in range(NB):
                    o = k * ((B - 1) * cap + (B - 1))
                    m12 = rr[o:o + (B - 1) * cap].view(B - 1, cap).numpy()
                    nm = rr[o + (B - 1) * cap:o + (B - 1) * cap + B - 1].numpy()
                    for j in range(B - 1):
                        i = ra + k * B + j + 1
                        nmw, mw = want[i]
                        if int(nm[j]) != nmw or not np.array_equal(m12[j, :len(mw)], mw):
                            errs.append("pair (%d, %d) on rank %d: %d matches vs oracle %d" % (i - 1, i, r, nm[j], nmw))
                        checked.add(i)
            # the straddling pairs: on rank 0's device, from the handed-back payloads
            edge = [i for i in range(1, nfr) if i not in checked]
            assert edge == [i for i in range(B, nfr, B)], edge
            ea = torch.tensor([i - 1 for i in edge], dtype=torch.int32, device=dev)
            eb = torch.tensor(edge, dtype=torch.int32, device=dev)
            m12, nm = m.search_for_initialization_batch(kps_all.to(dev), desc_all.to(dev), cnt_all.to(dev), ea, eb,
                                                        H, W, 100)
            m12, nm = m12.cpu().numpy(), nm.cpu().numpy()
            for j, i in enumerate(edge):
                nmw, mw = want[i]
                if int(nm[j]) != nmw or not np.array_equal(m12[j, :len(mw)], mw):
                    errs.append("straddling pair (%d, %d): %d matches vs oracle %d" % (i - 1, i, nm[j], nmw))
                checked.add(i)
            assert checked == set(range(1, nfr))
            q.put(errs)
    except Exception:
        q.put(["rank %d: %s" % (rank, traceback.format_exc())])
    finally:
        dist.destroy_process_group()


def test_sharded_replay_two_ranks_on_one_gpu(cuda):
    world = 2
    nfr = world * NB * B
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, nfr, q)) for r in range(world)]
    for p in procs:
        p.start()
    errs = []
    try:
        errs = q.get(timeout=100)
    finally:
        for p in procs:
            p.join(30)
            if p.exitcode is None:
                p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert errs == [], errs[:5]
