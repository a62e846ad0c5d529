"""orbx_extract_stage_device: the batch extraction issued stage by stage across two streams (events between
the stages) gives exactly orbx_extract_batch_device's output, and stages that do not match the workspace
are refused."""
import numpy as np
import pytest


@pytest.mark.gpu
def test_stage_split_matches_batch_call(cuda):
    import torch
    import orbx
    import orbx_synth
    H, W, B = 376, 1241, 8
    frames = torch.from_numpy(orbx_synth.kitti_sequence(B)).cuda()
    ex = orbx.ORBextractor(2000, 1.2, 8, 20, 7)
    cap = ex.capacity(H, W)
    out = []
    for split in (False, True):
        kps = torch.zeros((B, cap, 7), dtype=torch.int32, device="cuda")
        desc = torch.zeros((B, cap, 32), dtype=torch.uint8, device="cuda")
        cnt = torch.zeros((B,), dtype=torch.int32, device="cuda")
        if not split:
            s = torch.cuda.Stream()
            ex.extract_batch_device(frames, kps, desc, cnt, s)
            ex.sync(s)
        else:
            a, b = torch.cuda.Stream(), torch.cuda.Stream()
            for st in range(4):   # alternate the streams, each stage after the previous one
                s = a if st % 2 == 0 else b
                if st:
                    s.wait_event(ev)
                ex.extract_stage_device(st, frames, kps, desc, cnt, s)
                ev = torch.cuda.Event()
                ev.record(s)
            ex.sync(b)
        out.append((kps.cpu().numpy(), desc.cpu().numpy(), cnt.cpu().numpy()))
    (k0, d0, c0), (k1, d1, c1) = out
    assert np.array_equal(c0, c1) and c0.min() > 0
    for f in range(B):
        n = c0[f]
        assert np.array_equal(k0[f, :n], k1[f, :n]) and np.array_equal(d0[f, :n], d1[f, :n])


@pytest.mark.gpu
def test_stage_outside_the_workspace_is_refused(cuda):
    import torch
    import orbx
    import orbx_synth
    ex = orbx.ORBextractor(1000, 1.2, 8, 20, 7)
    frames = torch.from_numpy(orbx_synth.kitti_sequence(2)).cuda()
    cap = ex.capacity(376, 1241)
    kps = torch.empty((4, cap, 7), dtype=torch.int32, device="cuda")
    desc = torch.empty((4, cap, 32), dtype=torch.uint8, device="cuda")
    cnt = torch.empty((4,), dtype=torch.int32, device="cuda")
    s = torch.cuda.Stream()
    ex.extract_stage_device(0, frames, kps[:2], desc[:2], cnt[:2], s)
    with pytest.raises(orbx.OrbxError):   # a larger batch than stage 0 sized the workspace for
        ex.extract_stage_device(1, torch.cat([frames, frames]), kps, desc, cnt, s)
    with pytest.raises(orbx.OrbxError):   # another image size
        ex.extract_stage_device(1, frames[:, :300, :1000].contiguous(), kps[:2], desc[:2], cnt[:2], s)
    with pytest.raises(orbx.OrbxError):   # no such stage
        ex.extract_stage_device(4, frames, kps[:2], desc[:2], cnt[:2], s)
    ex.sync(s)
