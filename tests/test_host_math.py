"""Host-side checks of the product's arithmetic building blocks (no GPU).

* the glibc cosf/sinf restatement in csrc/orbx_math.hpp (used by the gfx950
  BRIEF kernel) equals the host libm on EVERY float in [0, 2*pi]
  (BRIEF angles are fastAtan2 outputs in [0, 360) deg);
* the rBRIEF pattern table equals bit_pattern_31_ of the reference.
"""
import hashlib
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "orb-slam-_amd", "csrc")

SWEEP = r"""
#include <cmath>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>
#include "orbx_math.hpp"
#include "../../oracle/orbref.h"
int main() {
    const float twopi = 6.2831855f;
    uint32_t hi; std::memcpy(&hi, &twopi, 4); hi += 1;
    const int T = 8;
    std::vector<long> bad(T, 0), badat(T, 0);
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t) th.emplace_back([&, t] {
        for (uint32_t u = t; u < hi; u += T) {
            float f; std::memcpy(&f, &u, 4);
            const float c = cosf(f), s = sinf(f);
            if (orbx::f32_bits(c) != orbx::f32_bits(orbx::glibc_sincosf(f, 1)) ||
                orbx::f32_bits(s) != orbx::f32_bits(orbx::glibc_sincosf(f, 0))) { if (!bad[t]) badat[t] = u; bad[t]++; }
        }
    });
    for (auto& x : th) x.join();
    long tot = 0; for (long b : bad) tot += b;
    long atan_bad = 0;
    for (int y = -300; y <= 300; y += 3) for (int x = -300; x <= 300; x += 7) {
        const float a = orbx::fast_atan2_deg((float)y * 37.f, (float)x * 41.f);
        const float b = orbref_fast_atan2((float)y * 37.f, (float)x * 41.f);
        if (orbx::f32_bits(a) != orbx::f32_bits(b)) atan_bad++;
    }
    std::printf("%u %ld %ld\n", hi, tot, atan_bad);
    return 0;
}
"""


@pytest.fixture(scope="module")
def sweep_bin(tmp_path_factory, orbref):
    d = tmp_path_factory.mktemp("sweep")
    src = os.path.join(CSRC, "_sweep_test.cpp")
    with open(src, "w") as f:
        f.write(SWEEP)
    exe = str(d / "sweep")
    try:
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-march=x86-64-v3", "-pthread",
                               "-I", CSRC, src, os.path.join(ROOT, "oracle", "orbref.c"), "-o", exe, "-lm"])
    finally:
        os.remove(src)
    return exe


def test_glibc_sincosf_restatement_exhaustive(sweep_bin):
    out = subprocess.run([sweep_bin], capture_output=True, text=True, timeout=600).stdout.split()
    n, bad, atan_bad = int(out[0]), int(out[1]), int(out[2])
    assert n > 1_000_000_000
    assert bad == 0, "%d floats in [0, 2pi] where the restated cosf/sinf differ from libm" % bad
    assert atan_bad == 0


def _pattern_values():
    txt = "".join(l for l in open(os.path.join(CSRC, "orb_pattern.inc")) if not l.lstrip().startswith(("/*", "*")))
    return [int(x) for x in txt.replace("\n", "").split(",") if x.strip()]


def test_pattern_table():
    v = _pattern_values()
    assert len(v) == 1024 and min(v) == -13 and max(v) == 12
    assert hashlib.sha256(",".join(map(str, v)).encode()).hexdigest() == \
        "88df8ca875cc8db56799edd57bb914edad8acb2d48c202b7a464a575b55dbdb8"
    ref = "/root/reference/src/ORBextractor.cc"
    if os.path.exists(ref):   # CPU container only: compare with the reference's table text
        src = open(ref, encoding="utf-8").read()
        body = src[src.index("bit_pattern_31_[256*4]"):]
        body = re.sub(r"/\*.*?\*/", "", body[body.index("{") + 1:body.index("};")], flags=re.S)
        assert [int(x) for x in re.findall(r"-?\d+", body)] == v
