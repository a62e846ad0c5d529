"""The built device code (liborbx.so's gfx950 code objects) uses no flat memory instructions: every kernel reaches
global memory through global/buffer instructions and LDS through DS ones.  A flat access (a pointer whose address
space the compiler cannot see: one that may point to LDS or global memory, or an integer cast back to a pointer)
counts against both wait counters and forces full waits; round 5 found and removed them in FAST's output,
describe's IC_Angle loads, SearchForInitialization's window scan, the BoW views and ingest.
CPU-only: extracts the code objects with llvm-objcopy / clang-offload-bundler and disassembles them."""
import os, shutil, subprocess, tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "orb-slam-_amd", "liborbx.so")
LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _tools():
    t = {n: os.path.join(LLVM, n) for n in ("llvm-objcopy", "clang-offload-bundler", "llvm-objdump")}
    return t if all(os.path.exists(p) for p in t.values()) else None


@pytest.mark.skipif(not os.path.exists(LIB) or _tools() is None, reason="liborbx.so or the LLVM tools are absent")
def test_no_flat_memory_instructions():
    t = _tools()
    d = tempfile.mkdtemp()
    try:
        fb = os.path.join(d, "fatbin")
        subprocess.run([t["llvm-objcopy"], "--dump-section", ".hip_fatbin=" + fb, LIB], check=True)
        data = open(fb, "rb").read()
        starts = [i for i in range(len(data)) if data.startswith(MAGIC, i)]
        assert starts, "no offload bundles in liborbx.so"
        kernels, flat = 0, []
        for n, a in enumerate(starts):
            b = starts[n + 1] if n + 1 < len(starts) else len(data)
            chunk = os.path.join(d, "b%d" % n)
            with open(chunk, "wb") as f:
                f.write(data[a:b])
            co = os.path.join(d, "b%d.co" % n)
            r = subprocess.run([t["clang-offload-bundler"], "--type=o", "--input=" + chunk, "--output=" + co,
                                "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--unbundle"], capture_output=True)
            if r.returncode != 0 or not os.path.exists(co) or os.path.getsize(co) == 0:
                continue
            dis = subprocess.run([t["llvm-objdump"], "-d", "--mcpu=gfx950", co], capture_output=True,
                                 text=True, check=True).stdout
            kernels += dis.count("s_endpgm")
            flat += [l.strip() for l in dis.splitlines() if l.strip().startswith(("flat_load", "flat_store", "flat_atomic"))]
        assert kernels > 20, "only %d kernels disassembled" % kernels
        assert not flat, "%d flat memory instructions, first: %s" % (len(flat), flat[:3])
    finally:
        shutil.rmtree(d, ignore_errors=True)
