"""Seeded synthetic grayscale inputs for the ORB front-end.

There are no images or datasets in the reference and no network,
so every config runs on textures made here:

* ``gen_image(seed, W, H)``: blocky texture — random axis-aligned rectangles of
  uniform intensity (400 per 640x480 of area), an additive uniform +-12 noise
  field and a smooth gradient.  Gives several FAST-20 corners per 30-px cell,
  like the real KITTI/TUM frames the reference YAMLs target.
* ``kitti_sequence(n)``: config 2/4 — 1241x376 crops translating 3 px/frame
  across one seeded 4096x1024 texture (seed 2), so consecutive frames overlap
  and SearchForInitialization finds matches.
* ``stereo_pair``: config 3 — right view = left view warped by a piecewise
  constant disparity field, plus noise.
"""
from __future__ import annotations

import numpy as np

__all__ = ["gen_image", "kitti_sequence", "stereo_pair", "random_descriptors"]


def gen_image(seed: int, width: int, height: int, rect_density: float = 400.0 / (640 * 480)) -> np.ndarray:
    rng = np.random.default_rng(seed)
    img = np.full((height, width), 128, dtype=np.int32)
    nrect = max(1, int(round(rect_density * width * height)))
    x0 = rng.integers(-16, width, size=nrect)
    y0 = rng.integers(-16, height, size=nrect)
    rw = rng.integers(6, max(8, width // 10), size=nrect)
    rh = rng.integers(6, max(8, height // 8), size=nrect)
    val = rng.integers(0, 256, size=nrect)
    for i in range(nrect):
        xa, ya = max(0, x0[i]), max(0, y0[i])
        xb, yb = min(width, x0[i] + rw[i]), min(height, y0[i] + rh[i])
        if xb > xa and yb > ya:
            img[ya:yb, xa:xb] = val[i]
    img += rng.integers(-12, 13, size=(height, width), dtype=np.int32)
    gx = np.linspace(0.0, 24.0, width, dtype=np.float64)[None, :]
    gy = np.linspace(0.0, 16.0, height, dtype=np.float64)[:, None]
    img = img + np.round(gx + gy).astype(np.int32) - 20
    return np.clip(img, 0, 255).astype(np.uint8)


_TEXTURE_CACHE: dict = {}


def kitti_sequence(n: int, start: int = 0, width: int = 1241, height: int = 376, step_px: int = 3,
                   seed: int = 2) -> np.ndarray:
    """Frames ``start .. start+n-1`` of the config-2 replay sequence, shape (n, H, W)."""
    key = (seed, width, height)
    tex = _TEXTURE_CACHE.get(key)
    if tex is None:
        tex = gen_image(seed, 4096, 1024)
        _TEXTURE_CACHE[key] = tex
    out = np.empty((n, height, width), dtype=np.uint8)
    span_x = tex.shape[1] - width
    span_y = tex.shape[0] - height
    for k in range(n):
        t = start + k
        # triangle wave so arbitrarily long sequences stay inside the texture
        px = (t * step_px) % (2 * span_x)
        px = px if px <= span_x else 2 * span_x - px
        py = (t * 1) % (2 * span_y)
        py = py if py <= span_y else 2 * span_y - py
        out[k] = tex[py:py + height, px:px + width]
    return out


def stereo_pair(seed: int = 3, width: int = 752, height: int = 480):
    left = gen_image(seed, width, height)
    rng = np.random.default_rng(seed + 1000)
    right = np.empty_like(left)
    nb = 8
    bounds = np.linspace(0, height, nb + 1).astype(int)
    for b in range(nb):
        d = int(rng.integers(2, 41))
        ya, yb = bounds[b], bounds[b + 1]
        right[ya:yb, :width - d] = left[ya:yb, d:]
        right[ya:yb, width - d:] = left[ya:yb, width - 1:width][:, [0] * d]
    noise = rng.integers(-4, 5, size=right.shape)
    right = np.clip(right.astype(np.int32) + noise, 0, 255).astype(np.uint8)
    return left, right


def random_descriptors(n: int, seed: int) -> np.ndarray:
    rng = np.random.default_rng(seed)
    return rng.integers(0, 256, size=(n, 32), dtype=np.uint8)


# ---- vocabulary-node candidate sets (SearchByBoW / SearchForTriangulation inputs) ----
#
# ORBvoc.txt is not in the reference and there is no network, so the
# FeatureVectors are made by a small vocabulary trained here with DBoW2's recipe:
# hierarchical k-medians in Hamming space with bit-majority centres (FORB::meanValue,
# Thirdparty/DBoW2/DBoW2/FORB.cpp), nodes numbered breadth-first from root 0, and
# TemplatedVocabulary::transform's descent (first child at the strictly smallest
# distance) recording the ancestor `levelsup` levels above the leaf
# (TemplatedVocabulary.h:1127-1259).

def _ham_matrix(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    x = np.bitwise_xor(a[:, None, :], b[None, :, :])
    return np.unpackbits(x, axis=2).sum(axis=2).astype(np.int32)


class Vocabulary:
    """A DBoW2-style vocabulary tree: k-ary, depth <= L, nodes numbered like
    TemplatedVocabulary::HKmeansStep (the children of a node are consecutive ids,
    parents before children), leaf weights idf = ln(N / n_i) over the training images
    (setNodeWeights, TF_IDF).  Clusters of one descriptor become leaves early, so
    the tree is unbalanced like real vocabularies."""

    def __init__(self, k, L, parent, is_leaf, desc, weight, scoring=0, weighting=0):
        self.k, self.L = k, L
        self.parent = np.asarray(parent, np.int32)      # [nnodes]; parent[0] unused
        self.is_leaf = np.asarray(is_leaf, np.uint8)
        self.desc = np.asarray(desc, np.uint8)          # [nnodes, 32]
        self.weight = np.asarray(weight, np.float64)
        self.scoring, self.weighting = scoring, weighting

    @property
    def nnodes(self):
        return len(self.parent)

    @staticmethod
    def train(images_descs, k: int = 10, L: int = 3, seed: int = 0, iters: int = 3) -> "Vocabulary":
        """images_descs: list of [n_i, 32] uint8 arrays (one per training image)."""
        rng = np.random.default_rng(seed)
        allx = np.concatenate(images_descs)
        parent, desc = [0], [np.zeros(32, np.uint8)]
        children = {0: []}

        def step(pid, d, level):
            if len(d) <= k:
                cent = [x for x in d]
            else:
                c = d[rng.choice(len(d), k, replace=False)]
                for _ in range(iters):
                    lab = np.argmin(_ham_matrix(d, c), axis=1)
                    for j in range(k):
                        m = d[lab == j]
                        if len(m):
                            c[j] = np.packbits(np.unpackbits(m, axis=1).mean(axis=0) > 0.5)
                cent = list(c)
            lab = np.argmin(_ham_matrix(d, np.stack(cent)), axis=1)
            ids = []
            for j in range(len(cent)):
                parent.append(pid)
                desc.append(cent[j])
                ids.append(len(parent) - 1)
                children[ids[-1]] = []
            children[pid] = ids
            if level < L:
                for j, cid in enumerate(ids):
                    sub = d[lab == j]
                    if len(sub) > 1:
                        step(cid, sub, level + 1)

        step(0, allx, 1)
        n = len(parent)
        is_leaf = np.array([1 if (i > 0 and not children[i]) else 0 for i in range(n)], np.uint8)
        voc = Vocabulary(k, L, parent, is_leaf, np.stack(desc), np.zeros(n))
        # idf of each leaf: ln(N / n_i), n_i = training images holding the word
        N = len(images_descs)
        seen = np.zeros(n, np.int64)
        for d in images_descs:
            words = np.unique(voc.leaf_of(d))
            seen[words] += 1
        w = np.zeros(n)
        mask = (is_leaf == 1) & (seen > 0)
        w[mask] = np.log(N / seen[mask])
        voc.weight = w
        return voc

    def _children(self):
        ch = [[] for _ in range(self.nnodes)]
        for i in range(1, self.nnodes):
            ch[self.parent[i]].append(i)
        return ch

    def leaf_of(self, descs):
        ch = self._children()
        out = np.zeros(len(descs), np.int64)
        for f, d in enumerate(np.asarray(descs, np.uint8)):
            node = 0
            while ch[node]:
                dist = np.unpackbits(np.bitwise_xor(self.desc[ch[node]], d), axis=1).sum(axis=1)
                node = ch[node][int(np.argmin(dist))]
            out[f] = node
        return out

    def feature_vector(self, descs: np.ndarray, levelsup: int = 1):
        """FeatureVector as CSR (node ids ascending, ptr, feature indices in insertion order);
        features are grouped by their ancestor at depth L - levelsup (the leaf if shallower)."""
        ch = self._children()
        descs = np.asarray(descs, np.uint8)
        target = self.L - levelsup
        rec = np.zeros(len(descs), np.int64)
        for f, d in enumerate(descs):
            node, level, nid = 0, 0, 0
            while ch[node]:
                level += 1
                dist = np.unpackbits(np.bitwise_xor(self.desc[ch[node]], d), axis=1).sum(axis=1)
                node = ch[node][int(np.argmin(dist))]
                if level == target:
                    nid = node
            if target > 0 and level < target:
                nid = node
            rec[f] = nid if target > 0 else 0
        ids = np.unique(rec)
        order = np.argsort(rec, kind="stable")
        ptr = np.concatenate([[0], np.cumsum([(rec == i).sum() for i in ids])]).astype(np.int32)
        return ids.astype(np.int32), ptr, order.astype(np.int32)

    def save_text(self, path: str):
        """DBoW2 text format (TemplatedVocabulary::saveToTextFile / loadFromTextFile)."""
        with open(path, "w") as f:
            f.write("%d %d %d %d\n" % (self.k, self.L, self.scoring, self.weighting))
            for i in range(1, self.nnodes):
                f.write("%d %d %s %r\n" % (self.parent[i], self.is_leaf[i], " ".join(str(int(x)) for x in self.desc[i]),
                                          float(self.weight[i])))


# ---- MapPoints for the projection searches (SearchByProjection / Fuse inputs) ----

MAP_POINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("nx", "<f4"), ("ny", "<f4"), ("nz", "<f4"),
                            ("max_dist", "<f4"), ("min_dist", "<f4"), ("angle", "<f4"), ("octave", "<i4"),
                            ("flags", "<i4"), ("pad", "<i4")])


def _rotation(w: np.ndarray) -> np.ndarray:
    th = float(np.linalg.norm(w))
    if th < 1e-12:
        return np.eye(3)
    k = w / th
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K


def pose_scene(seed: int, kps: np.ndarray, desc: np.ndarray, n_mp: int, K=(718.856, 718.856, 607.19, 185.22),
               bf: float = 386.14, scale_factor: float = 1.2, nlevels: int = 8):
    """MapPoints seen by a frame with keypoints `kps` (a structured KEYPOINT array, e.g. an extraction
    result) and descriptors `desc`: each MapPoint re-projects near a keypoint (1.5 px noise) at a
    per-keypoint depth, with a distance range whose predicted level is the keypoint's octave (or the
    next), a normal towards the camera, the keypoint's angle (20% random) and a descriptor 8% away
    from the keypoint's.  Returns (pose 3x4 float32 Tcw, map points, their descriptors, uRight)."""
    rng = np.random.default_rng(seed)
    n = len(kps)
    depth = rng.uniform(2.0, 40.0, n)
    uright = np.where(rng.random(n) < 0.4, kps["x"] - bf / depth, -1).astype(np.float32)
    R = _rotation(rng.normal(0, 0.1, 3))
    t = rng.normal(0, 0.5, 3)
    tgt = rng.integers(0, n, n_mp)
    u = kps["x"][tgt] + rng.normal(0, 1.5, n_mp)
    v = kps["y"][tgt] + rng.normal(0, 1.5, n_mp)
    d = depth[tgt] * (1 + rng.normal(0, 0.01, n_mp))
    Xc = np.stack([(u - K[2]) / K[0] * d, (v - K[3]) / K[1] * d, d], 1)
    Xw = (Xc - t) @ R
    Ow = -R.T @ t
    dist = np.linalg.norm(Xw - Ow, axis=1)
    lvl = np.clip(kps["octave"][tgt] + rng.integers(0, 2, n_mp), 0, nlevels - 1)
    max_dist = dist * scale_factor ** (lvl - rng.uniform(0.05, 0.95, n_mp))
    pts = np.zeros(n_mp, MAP_POINT_DTYPE)
    pts["x"], pts["y"], pts["z"] = Xw[:, 0], Xw[:, 1], Xw[:, 2]
    nrm = (Xw - Ow) / dist[:, None] + rng.normal(0, 0.2, (n_mp, 3))
    nrm /= np.linalg.norm(nrm, axis=1)[:, None]
    pts["nx"], pts["ny"], pts["nz"] = nrm[:, 0], nrm[:, 1], nrm[:, 2]
    pts["max_dist"] = max_dist
    pts["min_dist"] = max_dist / scale_factor ** (nlevels - 1)
    ang = (kps["angle"][tgt] + rng.normal(0, 3, n_mp)) % 360
    pts["angle"] = np.where(rng.random(n_mp) < 0.2, rng.uniform(0, 360, n_mp), ang)
    pts["octave"] = lvl
    pts["flags"] = (rng.random(n_mp) < 0.95).astype(np.int32) | ((rng.random(n_mp) < 0.8).astype(np.int32) << 1)
    bits = np.unpackbits(desc[tgt], axis=1) ^ (rng.random((n_mp, 256)) < 0.08)
    pdesc = np.packbits(bits, axis=1)
    Tcw = np.hstack([R, t[:, None]]).astype(np.float32)
    return Tcw, pts, pdesc, uright
