"""Content hash of the sources the GPU kernels are built from (orb-slam-_amd/csrc/*, include/orbx.h).

The committed counter files (profiles/pmc_traffic.json, profiles/sq_counters.json) carry the hash of the
tree they were measured on; bench.py reports their figures only when it equals the hash of the tree it is
timing (the GPU box has no .git, so a content hash stands in for the commit)."""
import glob
import hashlib
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kernel_sources_sha256(root=ROOT):
    h = hashlib.sha256()
    files = sorted(glob.glob(os.path.join(root, "orb-slam-_amd", "csrc", "*")) + [os.path.join(root, "include", "orbx.h")])
    for fn in files:
        if os.path.isfile(fn):
            h.update(os.path.relpath(fn, root).encode())
            h.update(open(fn, "rb").read())
    return h.hexdigest()


def bench_default_batch(root=ROOT):
    """bench.py's DEFAULT_BATCH (frames per GPU per step), read from its source so the counter tools
    record the same step as the bench without importing torch."""
    m = re.search(r"^DEFAULT_BATCH = (\d+)", open(os.path.join(root, "bench.py")).read(), re.M)
    return int(m.group(1))


if __name__ == "__main__":
    print(kernel_sources_sha256())
