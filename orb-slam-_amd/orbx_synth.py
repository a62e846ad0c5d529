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
    def __init__(self, k: int, L: int, centers: np.ndarray):
        self.k, self.L = k, L
        self.centers = centers            # [n_nodes, 32]; row 0 (root) unused

    @staticmethod
    def train(descs: np.ndarray, k: int = 10, L: int = 3, seed: int = 0, iters: int = 3) -> "Vocabulary":
        rng = np.random.default_rng(seed)
        n_nodes = sum(k ** d for d in range(L + 1))
        centers = np.zeros((n_nodes, 32), np.uint8)
        groups = {0: np.asarray(descs, np.uint8)}
        first = 1
        for depth in range(1, L + 1):
            ngroups = {}
            for parent in range(first - k ** (depth - 1), first):
                d = groups.get(parent)
                child0 = first + (parent - (first - k ** (depth - 1))) * k
                if d is None or len(d) == 0:
                    centers[child0:child0 + k] = rng.integers(0, 256, (k, 32), dtype=np.uint8)
                    continue
                c = d[rng.choice(len(d), k, replace=len(d) < k)]
                for _ in range(iters):
                    lab = np.argmin(_ham_matrix(d, c), axis=1)
                    for j in range(k):
                        m = d[lab == j]
                        if len(m):
                            bits = np.unpackbits(m, axis=1).mean(axis=0) > 0.5   # bit majority
                            c[j] = np.packbits(bits)
                lab = np.argmin(_ham_matrix(d, c), axis=1)
                centers[child0:child0 + k] = c
                for j in range(k):
                    ngroups[child0 + j] = d[lab == j]
            groups = ngroups
            first += k ** depth
        return Vocabulary(k, L, centers)

    def feature_vector(self, descs: np.ndarray, levelsup: int = 1):
        """FeatureVector as CSR (node ids ascending, ptr, feature indices in insertion order)."""
        descs = np.asarray(descs, np.uint8)
        n = len(descs)
        node = np.zeros(n, np.int64)
        target_depth = self.L - levelsup
        rec = np.zeros(n, np.int64)
        first_child = np.full(n, 1, np.int64)   # root's first child
        level_first = 1
        for depth in range(1, self.L + 1):
            kids = first_child[:, None] + np.arange(self.k)[None, :]
            dist = np.unpackbits(np.bitwise_xor(descs[:, None, :], self.centers[kids]), axis=2).sum(axis=2)
            node = kids[np.arange(n), np.argmin(dist, axis=1)]   # first strict minimum
            if depth == target_depth:
                rec = node.copy()
            next_first = level_first + self.k ** depth
            first_child = next_first + (node - level_first) * self.k
            level_first = next_first
        if target_depth <= 0:
            rec = np.zeros(n, np.int64)
        ids = np.unique(rec)
        order = np.argsort(rec, kind="stable")
        counts = np.array([(rec == i).sum() for i in ids], np.int64)
        ptr = np.concatenate([[0], np.cumsum(counts)]).astype(np.int32)
        return ids.astype(np.int32), ptr, order.astype(np.int32)
