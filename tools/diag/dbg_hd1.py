"""Batch-1 1920x1080 extraction status (debug)."""
import os
import sys
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "..", "orb-slam-_amd")]
import numpy as np
import torch
import orbx
import orbx_synth
for B in (1, 2):
    img = np.stack([orbx_synth.gen_image(31 + i, 1920, 1080) for i in range(B)])
    ex = orbx.ORBextractor(4000, 1.2, 8, 20, 7)
    cap = ex.capacity(1080, 1920)
    t = torch.from_numpy(img).cuda()
    kps = torch.empty((B, cap, 7), dtype=torch.int32, device="cuda")
    desc = torch.empty((B, cap, 32), dtype=torch.uint8, device="cuda")
    cnt = torch.empty((B,), dtype=torch.int32, device="cuda")
    rc = orbx.lib.orbx_extract_batch_device(ex._h, orbx._ptr(t), B, 1080, 1920, t.stride(1), t.stride(0),
                                            orbx._ptr(kps), orbx._ptr(desc), orbx._ptr(cnt), cap,
                                            orbx._stream(None))
    print("B", B, "cap", cap, "rc", rc, "last hip error", torch.cuda.synchronize() or "ok", cnt.cpu().numpy())
