"""Frame-sharded multi-GPU replay (BASELINE.json config 4).

Frames are independent (ORBextractor::operator() depends only on the image),
so frame i goes to rank i mod G ... here: rank r owns a contiguous block of
frames, which also keeps the SearchForInitialization pairs (t-1, t) local.
The only collective is the hand-back of every rank's keypoints/descriptors to
rank 0, where the unchanged Tracking/Optimizer would consume them.

Payload per rank = one flat uint8 buffer holding, for B frames with per-frame
capacity `cap`:  kps  [B, cap, 7] int32 (cv::KeyPoint, 28 B)
                 desc [B, cap, 32] uint8
                 counts [B] int32
so the extractor writes straight into the buffer that is sent (no pack copy).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_range(n_frames: int, rank: int, world: int):
    """Contiguous block of frames owned by `rank`."""
    per = (n_frames + world - 1) // world
    a = min(n_frames, rank * per)
    return a, min(n_frames, a + per)


class Payload:
    def __init__(self, batch: int, cap: int, device):
        self.batch, self.cap = batch, cap
        self.kps_bytes = batch * cap * 28
        self.desc_bytes = batch * cap * 32
        self.nbytes = self.kps_bytes + self.desc_bytes + batch * 4
        self.buf = torch.zeros(self.nbytes, dtype=torch.uint8, device=device)
        self.kps = self.buf[:self.kps_bytes].view(torch.int32).view(batch, cap, 7)
        self.desc = self.buf[self.kps_bytes:self.kps_bytes + self.desc_bytes].view(batch, cap, 32)
        self.counts = self.buf[self.kps_bytes + self.desc_bytes:].view(torch.int32)

    @staticmethod
    def unpack(buf: torch.Tensor, batch: int, cap: int):
        kb, db = batch * cap * 28, batch * cap * 32
        kps = buf[:kb].view(torch.int32).view(batch, cap, 7)
        desc = buf[kb:kb + db].view(batch, cap, 32)
        counts = buf[kb + db:kb + db + batch * 4].view(torch.int32)
        return kps, desc, counts


class Gatherer:
    """Collects every rank's payload on rank 0 (RCCL over xGMI for backend 'nccl').

    Uses point-to-point sends to rank 0: each peer pushes over its own xGMI
    link, which is what a rank-0 collection needs on a point-to-point fabric
    (a ring all-gather would push (G-1)x the bytes through every link).

    host_stage: the process group's backend cannot move device tensors (gloo between ranks that share
    one GPU, the -m gpu test of the sharded replay): a peer copies its device payload into a pinned host
    buffer (ordered after the work queued on the current stream) and sends that; rank 0 receives into
    host buffers."""

    def __init__(self, payload: Payload, world: int, rank: int, host_stage: bool = False):
        self.world, self.rank = world, rank
        self.payload = payload
        self.host_stage = bool(host_stage) and payload.buf.is_cuda
        self.recv = None
        self.stage = None
        if world > 1 and self.host_stage and rank != 0:
            self.stage = torch.empty(payload.nbytes, dtype=torch.uint8, pin_memory=True)
        if rank == 0 and world > 1:
            dev = torch.device("cpu") if self.host_stage else payload.buf.device
            self.recv = [torch.empty(payload.nbytes, dtype=torch.uint8, device=dev) for _ in range(world - 1)]

    def gather_async(self):
        """Queue the hand-back and return its work handles without waiting.  The sends read the
        payload after the work already queued on the current stream (the extraction that filled
        it); call finish() on the stream that next writes this payload, before writing it."""
        if self.world == 1:
            return []
        if self.rank == 0:
            ops = [dist.P2POp(dist.irecv, self.recv[r - 1], r) for r in range(1, self.world)]
        else:
            src = self.payload.buf
            if self.stage is not None:
                self.stage.copy_(src)   # waits for the current stream's work, then the D2H copy
                src = self.stage
            ops = [dist.P2POp(dist.isend, src, 0)]
        return list(dist.batch_isend_irecv(ops))

    @staticmethod
    def finish(works):
        """Order the current stream after the hand-back (NCCL: a stream wait, the host does not block)."""
        for w in works:
            w.wait()

    def gather(self):
        self.finish(self.gather_async())
        if self.world == 1:
            return [self.payload.buf]
        return [self.payload.buf] + self.recv if self.rank == 0 else None


class HandBack:
    """Double-buffered payloads for one pipeline slot: batch k of the slot fills payload k % 2 while
    payload (k - 1) % 2 may still be on its way to rank 0.  A payload's send is waited for (a stream
    wait, not a host wait) only when the slot is about to overwrite it, so the hand-back of batch k
    overlaps the extraction of batch k + 1 on the same stream instead of sitting in its way."""

    def __init__(self, batch: int, cap: int, device, world: int, rank: int, depth: int = 2, host_stage: bool = False):
        self.payloads = [Payload(batch, cap, device) for _ in range(depth)]
        self.gatherers = [Gatherer(p, world, rank, host_stage) for p in self.payloads]
        self.pending = [[] for _ in range(depth)]
        self.k = 0

    def next_payload(self) -> Payload:
        """The payload the slot's next batch writes; orders the current stream after its last send."""
        i = self.k % len(self.payloads)
        Gatherer.finish(self.pending[i])
        self.pending[i] = []
        return self.payloads[i]

    def send(self):
        """Hand the payload returned by next_payload() back to rank 0 (asynchronously)."""
        i = self.k % len(self.payloads)
        self.pending[i] = self.gatherers[i].gather_async()
        self.k += 1

    def drain(self):
        for i in range(len(self.pending)):
            Gatherer.finish(self.pending[i])
            self.pending[i] = []


# ---- config 5: 10k x 10k brute-force Hamming sharded over ranks ----------------
#
# Targets are split into contiguous slices (shard_range); every rank computes the
# (first-min index, best, second) triple of all queries against its slice, and
# rank 0 merges the slices in rank order.  Merging in target order with a strict
# `<` keeps the reference's first-min tie rule (src/ORBmatcher.cc:214-224): a
# later slice only wins with a strictly smaller distance.

def merge_top2(parts):
    """parts: list (rank order) of (best_idx, best, second) int32 tensors, best_idx
    already global (-1 for an empty slice).  Returns the merged triple."""
    bi, b1, b2 = (p.clone() for p in parts[0])
    for yi, y1, y2 in parts[1:]:
        win = y1 < b1
        nb2 = torch.where(win, torch.minimum(b1, y2), torch.minimum(b2, y1))
        b1 = torch.where(win, y1, b1)
        bi = torch.where(win, yi, bi)
        b2 = nb2
    return bi, b1, b2


def sharded_top2(q, t, rank: int, world: int, top2_fn):
    """This rank's slice of the all-pairs TOP2 search, gathered and merged on rank 0.

    top2_fn(q, t_slice) -> (idx, best, second) is the device search (orbx.allpairs on
    an MI355X).  Returns the merged triple on rank 0, None elsewhere."""
    a, b = shard_range(t.shape[0], rank, world)
    if b > a:
        bi, b1, b2 = top2_fn(q, t[a:b])
        bi = torch.where(bi >= 0, bi + a, bi)
    else:
        nq = q.shape[0]
        bi = torch.full((nq,), -1, dtype=torch.int32, device=q.device)
        b1 = torch.full((nq,), 256, dtype=torch.int32, device=q.device)
        b2 = b1.clone()
    mine = torch.stack([bi.to(torch.int32), b1.to(torch.int32), b2.to(torch.int32)])
    if world == 1:
        return bi, b1, b2
    if rank == 0:
        recv = [torch.empty_like(mine) for _ in range(world - 1)]
        ops = [dist.P2POp(dist.irecv, recv[r - 1], r) for r in range(1, world)]
    else:
        ops = [dist.P2POp(dist.isend, mine, 0)]
    for w in dist.batch_isend_irecv(ops):
        w.wait()
    if rank != 0:
        return None
    return merge_top2([(m[0], m[1], m[2]) for m in [mine] + recv])
