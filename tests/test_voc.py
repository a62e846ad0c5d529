"""DBoW2 vocabulary transform, SURVEY.md §8f row 2:
  TemplatedVocabulary::transform(features, BowVector, FeatureVector, levelsup)
  Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1125-1259, BowVector.cpp, FeatureVector.cpp

ORBvoc.txt is absent: vocabularies are trained here with DBoW2's recipe
(orbx_synth.Vocabulary), balanced and unbalanced, with stopped (zero-weight) words.
CPU: the C oracle against a pure-Python restatement of the reference text.
GPU: liborbx (host path, text loader, batched device path) against the oracle:
word ids, node ids and feature lists identical, BowVector weights equal as doubles.
"""
import math

import numpy as np
import pytest

SCORINGS = [0, 1, 5]          # L1_NORM, L2_NORM, DOT_PRODUCT
WEIGHTINGS = [0, 1, 2, 3]     # TF_IDF, TF, IDF, BINARY


def py_transform(voc, desc, levelsup):
    """Pure-Python restatement of TemplatedVocabulary::transform (TemplatedVocabulary.h:1125-1259)."""
    ch = [[] for _ in range(voc.nnodes)]
    for i in range(1, voc.nnodes):
        ch[voc.parent[i]].append(i)
    word = {}
    for i in range(1, voc.nnodes):
        if voc.is_leaf[i]:
            word[i] = len(word)
    nid_level = voc.L - levelsup
    bow, fv = {}, {}
    for f, d in enumerate(desc):
        final_id, level, nid = 0, 0, 0
        while True:
            level += 1
            nodes = ch[final_id]
            final_id = nodes[0]
            best = int(np.unpackbits(d ^ voc.desc[final_id]).sum())
            for nd in nodes[1:]:
                dd = int(np.unpackbits(d ^ voc.desc[nd]).sum())
                if dd < best:
                    best, final_id = dd, nd
            if level == nid_level:
                nid = final_id
            if not ch[final_id]:
                break
        if nid_level <= 0:
            nid = 0
        elif level < nid_level:
            nid = final_id
        w = float(voc.weight[final_id])
        wid = word.get(final_id, 0)
        if w > 0:
            if voc.weighting in (0, 1):
                bow[wid] = bow[wid] + w if wid in bow else w
            elif wid not in bow:
                bow[wid] = w
            fv.setdefault(nid, []).append(f)
    must = voc.scoring != 5
    if voc.weighting in (0, 1) and bow and not must:
        nd = float(len(bow))
        bow = {k: v / nd for k, v in bow.items()}
    if must:
        if voc.scoring == 1:
            norm = math.sqrt(sum(v * v for _, v in sorted(bow.items())))
        else:
            norm = 0.0
            for _, v in sorted(bow.items()):
                norm += abs(v)
        if norm > 0.0:
            bow = {k: v / norm for k, v in bow.items()}
    words = sorted(bow)
    nodes = sorted(fv)
    ptr = np.concatenate([[0], np.cumsum([len(fv[n]) for n in nodes])]).astype(np.int32)
    idx = np.array([f for n in nodes for f in fv[n]], np.int32)
    return (np.array(words, np.int32), np.array([bow[w] for w in words], np.float64),
            (np.array(nodes, np.int32), ptr, idx))


def _vocab(seed, k, L, nimg, nper, scoring=0, weighting=0):
    import orbx_synth
    rng = np.random.default_rng(seed)
    base = rng.integers(0, 256, (60, 32), dtype=np.uint8)
    imgs = []
    for _ in range(nimg):   # clustered descriptors: near-copies of 60 prototypes
        src = rng.integers(0, 60, nper)
        bits = np.unpackbits(base[src], axis=1) ^ (rng.random((nper, 256)) < 0.08)
        imgs.append(np.packbits(bits, axis=1))
    v = orbx_synth.Vocabulary.train(imgs, k, L, seed)
    v.scoring, v.weighting = scoring, weighting
    leaves = np.nonzero(v.is_leaf)[0]
    v.weight[leaves[::7]] = 0.0                                     # stopped words (stopWords)
    return v, imgs


def _same(a, b):
    assert np.array_equal(a[0], b[0]), "word ids"
    assert np.array_equal(a[1], b[1]), "weights (max diff %g)" % np.abs(a[1] - b[1]).max(initial=0)
    for x, y in zip(a[2], b[2]):
        assert np.array_equal(x, y), "feature vector"


@pytest.mark.parametrize("scoring", SCORINGS)
@pytest.mark.parametrize("weighting", WEIGHTINGS)
def test_oracle_matches_restatement(orbref, scoring, weighting):
    v, imgs = _vocab(1, 6, 4, 8, 80, scoring, weighting)
    assert v.is_leaf.sum() > 30
    assert (v.weight[v.is_leaf == 1] == 0).any()                    # stopped words exist
    depths = []
    for i in range(1, v.nnodes):
        d, p = 1, v.parent[i]
        while p != 0:
            d, p = d + 1, v.parent[p]
        if v.is_leaf[i]:
            depths.append(d)
    assert min(depths) < max(depths)                                # unbalanced tree
    q = np.concatenate(imgs[:2])
    for levelsup in (0, 1, 2, 4):
        _same(orbref.voc_transform(v, q, levelsup), py_transform(v, q, levelsup))


def test_oracle_feature_vector_matches_synth_generator(orbref):
    v, imgs = _vocab(2, 10, 3, 6, 300)
    v.weight[v.is_leaf == 1] = 1.0                                  # no stopped words
    q = imgs[0]
    _, _, fv = orbref.voc_transform(v, q, 1)
    for x, y in zip(fv, v.feature_vector(q, 1)):
        assert np.array_equal(x, y)


# ---------------------------------------------------------------------------- GPU

@pytest.mark.gpu
@pytest.mark.parametrize("scoring,weighting", [(0, 0), (1, 0), (5, 0), (0, 2), (5, 1), (1, 3)])
def test_gpu_transform_host(orbref, cuda, scoring, weighting):
    import orbx
    v, imgs = _vocab(3, 6, 4, 8, 120, scoring, weighting)
    gv = orbx.ORBVocabulary.from_arrays(v.k, v.L, v.parent, v.is_leaf, v.desc, v.weight, scoring, weighting)
    q = np.concatenate(imgs[:3])
    for levelsup in (0, 1, 2, 4):
        _same(gv.transform(q, levelsup), orbref.voc_transform(v, q, levelsup))
    assert len(gv.transform(q[:0], 2)[0]) == 0


@pytest.mark.gpu
def test_gpu_text_loader_round_trip(orbref, cuda, tmp_path):
    import orbx
    v, imgs = _vocab(4, 8, 3, 6, 200, 0, 0)
    path = tmp_path / "voc.txt"
    v.save_text(str(path))
    with open(path, "a") as f:
        f.write("\n")                                               # trailing newline: skipped
    gv = orbx.ORBVocabulary.loadFromTextFile(path)
    assert (gv.k, gv.L, gv.nnodes, gv.nwords) == (8, 3, v.nnodes, int(v.is_leaf.sum()))
    q = np.concatenate(imgs[:2])
    _same(gv.transform(q, 1), orbref.voc_transform(v, q, 1))


@pytest.mark.gpu
def test_gpu_transform_batch_then_search_by_bow(orbref, cuda):
    """Extract -> transform -> SearchByBoW fully on the device, against the oracle chain."""
    import torch
    import orbx
    import orbx_synth
    frames = orbx_synth.kitti_sequence(4, start=60)
    p = orbref.make_params(2000, 1.2, 8, 20, 7)
    refs = [orbref.extract(f, p, want_pyramid=False) for f in frames]
    v = orbx_synth.Vocabulary.train([r.descriptors for r in refs], 10, 3, 0)
    gv = orbx.ORBVocabulary.from_arrays(v.k, v.L, v.parent, v.is_leaf, v.desc, v.weight)
    ex = orbx.ORBextractor(2000, 1.2, 8, 20, 7)
    imgs = torch.from_numpy(frames).to(cuda)
    cap = ex.capacity(376, 1241)
    kps = torch.empty((4, cap, 7), dtype=torch.int32, device=cuda)
    desc = torch.empty((4, cap, 32), dtype=torch.uint8, device=cuda)
    counts = torch.empty((4,), dtype=torch.int32, device=cuda)
    ex.extract_batch_device(imgs, kps, desc, counts)
    bw, bv, bn, fn, fp, fi, fnn = gv.transform_batch_device(desc, counts, 1)
    torch.cuda.synchronize()
    want = [orbref.voc_transform(v, r.descriptors, 1) for r in refs]
    for f in range(4):
        nb, nn = int(bn[f]), int(fnn[f])
        got = (bw[f, :nb].cpu().numpy(), bv[f, :nb].cpu().numpy(),
               (fn[f, :nn].cpu().numpy(), fp[f, :nn + 1].cpu().numpy(), fi[f, :int(fp[f, nn])].cpu().numpy()))
        _same(got, want[f])
    # SearchByBoW(KF = frame 0, F = frame 1) on the device FeatureVectors
    rng = np.random.default_rng(0)
    mp = (rng.random(cap) < 0.7).astype(np.uint8)
    n0, n1 = int(counts[0]), int(counts[1])
    s1 = {"kps": kps[0, :n0], "desc": desc[0, :n0], "has_mp": mp[:n0],
          "fv": (fn[0, :int(fnn[0])].cpu().numpy(), fp[0, :int(fnn[0]) + 1].cpu().numpy(),
                 fi[0, :int(fp[0, int(fnn[0])])].cpu().numpy())}
    s2 = {"kps": kps[1, :n1], "desc": desc[1, :n1],
          "fv": (fn[1, :int(fnn[1])].cpu().numpy(), fp[1, :int(fnn[1]) + 1].cpu().numpy(),
                 fi[1, :int(fp[1, int(fnn[1])])].cpu().numpy())}
    bb = orbx.BowBatch(orbx.BOW_KF_F, [s1], [s2])
    match, nm = bb.run(0.7, True)
    torch.cuda.synchronize()
    wn, wm = orbref.search_by_bow_kf_f(refs[0].keypoints, refs[0].descriptors, mp[:n0], want[0][2],
                                       refs[1].keypoints, refs[1].descriptors, want[1][2], 0.7, True)
    assert int(nm[0]) == wn and wn > 50
    assert np.array_equal(match[0, :n1].cpu().numpy(), wm)
