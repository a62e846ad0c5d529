"""orbm_best2_csr, the shared best / second loop of the ORBmatcher searches:
per query, the candidates of its list in the caller's visiting order; first-min ties (strict <,
e.g. SearchByBoW src/ORBmatcher.cc:214-224) or last-min ties (SearchForTriangulation's
dist > bestDist skip, :806-823); the multiset second distance.
CPU: the C oracle against a pure-Python loop, lists full of equal distances, empty lists.
GPU: liborbx host path against the oracle.
"""
import numpy as np
import pytest


def py_best2(q, t, ptr, idx, tie_last):
    bi, b1, b2 = [], [], []
    for i in range(len(q)):
        best, second, bidx = 256, 256, -1
        for c in range(ptr[i], ptr[i + 1]):
            j = idx[c]
            d = int(np.unpackbits(q[i] ^ t[j]).sum())
            if d < best:
                second, best, bidx = best, d, j
            else:
                if tie_last and d == best:
                    bidx = j
                if d < second:
                    second = d
        bi.append(bidx)
        b1.append(best)
        b2.append(second)
    return np.array(bi), np.array(b1), np.array(b2)


def case(seed, nq=300, nt=500):
    rng = np.random.default_rng(seed)
    proto = rng.integers(0, 256, (8, 32), dtype=np.uint8)            # few prototypes: many equal distances
    flip = lambda a, p: np.packbits(np.unpackbits(a, axis=1) ^ (rng.random((len(a), 256)) < p), axis=1)
    q = flip(proto[rng.integers(0, 8, nq)], 0.02)
    t = flip(proto[rng.integers(0, 8, nt)], 0.02)
    t[rng.integers(0, nt, nt // 4)] = t[rng.integers(0, nt, nt // 4)]   # exact duplicates
    lens = rng.integers(0, 40, nq)
    lens[::17] = 0                                                     # empty lists
    ptr = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    idx = rng.integers(0, nt, ptr[-1]).astype(np.int32)
    return q, t, ptr, idx


@pytest.mark.parametrize("seed", [0, 1])
@pytest.mark.parametrize("tie_last", [False, True])
def test_oracle_matches_restatement(orbref, seed, tie_last):
    q, t, ptr, idx = case(seed)
    got = orbref.best2_csr(q, t, ptr, idx, tie_last)
    want = py_best2(q, t, ptr, idx, tie_last)
    for a, b in zip(got, want):
        assert np.array_equal(a, b)
    assert (got[0] == -1).sum() >= len(q) // 17                       # empty lists: -1 / 256 / 256
    if tie_last:
        first = orbref.best2_csr(q, t, ptr, idx, False)
        assert (first[0] != got[0]).any() and np.array_equal(first[1], got[1])


@pytest.mark.gpu
@pytest.mark.parametrize("tie_mode", [0, 1])
def test_gpu_best2_csr(orbref, cuda, tie_mode):
    import orbx
    for seed in (2, 3):
        q, t, ptr, idx = case(seed, nq=2000, nt=3000)
        got = orbx.best2_csr(q, t, ptr, idx, tie_mode)
        want = orbref.best2_csr(q, t, ptr, idx, bool(tie_mode))
        for a, b in zip(got, want):
            assert np.array_equal(a, b)


@pytest.mark.gpu
def test_gpu_best2_csr_rejects_bad_index(cuda):
    import orbx
    q, t, ptr, idx = case(4, nq=10, nt=20)
    idx = idx.copy()
    idx[0] = 20
    with pytest.raises(orbx.OrbxError):
        orbx.best2_csr(q, t, ptr, idx)


@pytest.mark.gpu
def test_gpu_allpairs_host(orbref, cuda):
    """orbm_allpairs (host arrays): TOP2 against the oracle, FULL_U16 against numpy popcounts."""
    import orbx
    q, t, _, _ = case(5, nq=700, nt=900)
    bi, b1, b2 = orbx.allpairs_host(q, t, orbx.TOP2)
    wi, w1, w2 = orbref.allpairs_top2(q, t)
    assert np.array_equal(bi, wi) and np.array_equal(b1, w1) and np.array_equal(b2, w2)
    full = orbx.allpairs_host(q[:50], t, orbx.FULL_U16)
    want = np.unpackbits(q[:50, None, :] ^ t[None, :, :], axis=2).sum(axis=2)
    assert np.array_equal(full.astype(np.int64), want)
    bi, b1, b2 = orbx.allpairs_host(q[:5], t[:0], orbx.TOP2)
    assert np.all(bi == -1) and np.all(b1 == 256) and np.all(b2 == 256)
