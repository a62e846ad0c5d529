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


def _disassembly():
    """The gfx950 disassembly of every code object in liborbx.so (one string per offload bundle)."""
    t = _tools()
    d = tempfile.mkdtemp()
    out = []
    try:
        fb = os.path.join(d, "fatbin")
        subprocess.run([t["llvm-objcopy"], "--dump-section", ".hip_fatbin=" + fb, LIB], check=True)
        data = open(fb, "rb").read()
        starts = [i for i in range(len(data)) if data.startswith(MAGIC, i)]
        assert starts, "no offload bundles in liborbx.so"
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
            out.append(subprocess.run([t["llvm-objdump"], "-d", "--mcpu=gfx950", co], capture_output=True,
                                      text=True, check=True).stdout)
        return out
    finally:
        shutil.rmtree(d, ignore_errors=True)


@pytest.mark.skipif(not os.path.exists(LIB) or _tools() is None, reason="liborbx.so or the LLVM tools are absent")
def test_hot_kernels_do_not_spill():
    """The extraction kernels (pyramid, FAST, the LDS quadtree forms, describe) hold their state in registers and
    LDS: no scratch (private memory) instruction, which would be per-lane HBM traffic.  Round 5 removed the last
    spills, in k_quadtree<256,4> and <512,16>, by giving the dynamic LDS a constant base (orbx_extract.hip
    dyn_lds)."""
    import re
    spills = {}
    for dis in _disassembly():
        fn = None
        for line in dis.splitlines():
            m = re.match(r"^[0-9a-f]+ <(\S+)>:", line)
            if m:
                fn = m.group(1)
            elif "scratch_" in line and fn:
                spills[fn] = spills.get(fn, 0) + 1
    # (the quadtree's kWide forms, for images wider or taller than 4096 px, are not held to this: a runtime
    # x / y split of the packed coordinates costs <256,4> a spilled register)
    hot = ("k_pyramid_level", "k_fast_cells", "k_describe", "k_quadtreeILi512ELi16ELb0ELb0E",
           "k_quadtreeILi512ELi8ELb0ELb0E", "k_quadtreeILi256ELi4ELb0ELb0E")
    bad = {f: n for f, n in spills.items() if any(h in f for h in hot)}
    assert not bad, "scratch instructions in %s" % bad


@pytest.mark.skipif(not os.path.exists(LIB) or _tools() is None, reason="liborbx.so or the LLVM tools are absent")
def test_no_flat_memory_instructions():
    kernels, flat = 0, []
    for dis in _disassembly():
        kernels += dis.count("s_endpgm")
        flat += [l.strip() for l in dis.splitlines() if l.strip().startswith(("flat_load", "flat_store", "flat_atomic"))]
    assert kernels > 20, "only %d kernels disassembled" % kernels
    assert not flat, "%d flat memory instructions, first: %s" % (len(flat), flat[:3])
