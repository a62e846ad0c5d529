#!/usr/bin/env python3
"""Cost of the vocabulary transform's per-frame sort past the LDS limit (k_voc_vectors<true> runs its
bitonic network in global memory for more than 8,192 descriptors).  One frame of n descriptors per batch, the
device batch entry point, HIP events around 20 calls after 3 warmups; a 10-level-deep k = 10 vocabulary trained
with orbx_synth's DBoW2 recipe (ORBvoc.txt is absent).  Prints one JSON line per n.
  python tools/diag/voc_large_n.py            (on the GPU box)"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "orb-slam-_amd")]
import orbx  # noqa: E402
import orbx_synth  # noqa: E402


def main():
    rng = np.random.default_rng(1)
    base = rng.integers(0, 256, (200, 32), dtype=np.uint8)
    imgs = []
    for _ in range(6):
        src = rng.integers(0, 200, 400)
        imgs.append(np.packbits(np.unpackbits(base[src], axis=1) ^ (rng.random((400, 256)) < 0.08), axis=1))
    v = orbx_synth.Vocabulary.train(imgs, 10, 3, 0)
    voc = orbx.ORBVocabulary.from_arrays(v.k, v.L, v.parent, v.is_leaf, v.desc, v.weight, v.scoring, v.weighting)
    dev = torch.device("cuda", 0)
    allb = np.concatenate(imgs)
    for n in (2000, 4096, 8192, 8193, 16384, 32768, 65536):
        src = rng.integers(0, len(allb), n)
        q = np.packbits(np.unpackbits(allb[src], axis=1) ^ (rng.random((n, 256)) < 0.03), axis=1)
        d = torch.from_numpy(q.reshape(1, n, 32)).to(dev)
        c = torch.tensor([n], dtype=torch.int32, device=dev)
        for _ in range(3):
            voc.transform_batch_device(d, c, 4)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            voc.transform_batch_device(d, c, 4)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 20
        print(json.dumps({"descriptors": n, "ms_per_frame": round(ms, 4), "us_per_1k_desc": round(1e3 * ms / n * 1e3, 2),
                          "sort": "LDS" if n <= 8192 else "global"}), flush=True)


if __name__ == "__main__":
    main()
