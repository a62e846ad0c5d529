"""Pose-projection searches, SURVEY.md §8f row 3 (the overloads after SearchByProjection(F, vpMapPoints)):
  SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, th, bMono)   src/ORBmatcher.cc:1396-1538
  SearchByProjection(Frame& CurrentFrame, KeyFrame*, sAlreadyFound, th, ORBdist)  src/ORBmatcher.cc:1540-1667
  SearchByProjection(KeyFrame*, Scw, vpPoints, vpMatched, th)                   src/ORBmatcher.cc:290-403
  Fuse(KeyFrame*, vpMapPoints, th)                                               src/ORBmatcher.cc:893-1043
  Fuse(KeyFrame*, Scw, vpPoints, th, vpReplacePoint)                             src/ORBmatcher.cc:1045-1168
over Frame::GetFeaturesInArea (src/Frame.cc:410-495) / KeyFrame::GetFeaturesInArea (src/KeyFrame.cc:569-608)
and MapPoint::PredictScale (src/MapPoint.cc:385-417).

CPU: the C oracle against a pure-Python restatement written from the reference text (float32
arithmetic, the GCC -march=native FMAs of the reference's own expressions, cv::Mat products as
OpenCV 3.x's small-matrix gemm), on scenes where many MapPoints compete for the same features
so that the in-call claims and the rotation histogram decide the result; plus known-answer cases.
GPU: liborbx host and batched device paths against the oracle, outputs identical.
Parity against the reference binary: unpinned (OpenCV absent).
"""
import math
from fractions import Fraction

import numpy as np
import pytest

F32 = np.float32
SCALE = np.array([F32(1.2) ** i for i in range(8)], np.float32)
K = (500.0, 500.0, 320.0, 240.0)
BOUNDS = (0.0, 640.0, 0.0, 480.0)
BF = 60.0
MODES = ["last_frame", "keyframe", "sim3", "fuse", "fuse_sim3"]
MODE_ID = {m: i for i, m in enumerate(MODES)}
INT_MIN = -2 ** 31


# ------------------------------------------------------------------ float helpers
def fmaf(a, b, c):
    """Correctly rounded float32 fma."""
    if not (math.isfinite(float(a)) and math.isfinite(float(b)) and math.isfinite(float(c))):
        return F32(float(a) * float(b) + float(c))
    x = Fraction(float(a)) * Fraction(float(b)) + Fraction(float(c))
    r = float(x)
    f = F32(r)
    if float(f) != r and math.isfinite(r):
        lo, hi = (f, np.nextafter(f, F32(np.inf))) if float(f) < r else (np.nextafter(f, F32(-np.inf)), f)
        mid = (Fraction(float(lo)) + Fraction(float(hi))) / 2
        if Fraction(r) == mid and x != mid:
            f = hi if x > mid else lo
    return F32(f)


def x86_int(v):
    v = float(v)
    return int(v) if (-2147483648.0 <= v < 2147483648.0) else INT_MIN


def roundf(v):
    v = float(v)
    return math.floor(v + 0.5) if v >= 0 else -math.floor(-v + 0.5)


def mat3_row(r, x, y, z):
    """One row of a cv::Mat 3x3 * 3x1 product (OpenCV 3.x gemm small-matrix path)."""
    return F32(F32(F32(r[0] * x) + F32(r[1] * y)) + F32(r[2] * z))


# ------------------------------------------------------------------ reference restatement
class Cam:
    """Rcw / tcw / Ow of the call, from mTcw or a Sim3 Scw (:298-303)."""

    def __init__(self, pose, sim3):
        S = np.asarray(pose, np.float32).reshape(-1)
        if sim3:
            d = 0.0
            for k in range(3):
                d += float(S[k]) * float(S[k])                       # sRcw.row(0).dot(sRcw.row(0))
            scw = F32(math.sqrt(d))
            s = F32(1.0 / float(scw))                                # sRcw/scw == convertTo(alpha = 1./scw)
            self.R = [[F32(F32(S[4 * r + k] * s) + F32(0)) for k in range(3)] for r in range(3)]
            self.t = [F32(F32(S[4 * r + 3] * s) + F32(0)) for r in range(3)]
        else:
            self.R = [[S[4 * r + k] for k in range(3)] for r in range(3)]
            self.t = [S[4 * r + 3] for r in range(3)]
        self.Ow = [-mat3_row([self.R[0][r], self.R[1][r], self.R[2][r]], *self.t) for r in range(3)]

    def to_cam(self, X):
        return [F32(mat3_row(self.R[r], *X) + self.t[r]) for r in range(3)]


class View:
    """A Frame / KeyFrame: mvKeysUn, mDescriptors, mvuRight and its 64x48 grid (AssignFeaturesToGrid)."""

    def __init__(self, kps, desc, uright, P):
        self.kps, self.desc, self.ur, self.P = kps, desc, uright, P
        self.grid = {}
        for i in range(len(kps)):                                    # PosInGrid (src/Frame.cc:504-518)
            px = roundf(F32(F32(kps["x"][i] - F32(P.min_x)) * F32(P.grid_w_inv)))
            py = roundf(F32(F32(kps["y"][i] - F32(P.min_y)) * F32(P.grid_h_inv)))
            if 0 <= px < 64 and 0 <= py < 48:
                self.grid.setdefault((px, py), []).append(i)

    def area(self, x, y, r, minLevel=-1, maxLevel=-1, frame=True):
        """Frame::GetFeaturesInArea (frame=True) / KeyFrame::GetFeaturesInArea."""
        P = self.P
        mnx, mny, wi, hi = F32(P.min_x), F32(P.min_y), F32(P.grid_w_inv), F32(P.grid_h_inv)
        out = []
        nMinCellX = max(0, x86_int(np.floor(F32(F32(F32(x - mnx) - r) * wi))))
        if nMinCellX >= 64:
            return out
        nMaxCellX = min(63, x86_int(np.ceil(F32(F32(F32(x - mnx) + r) * wi))))
        if nMaxCellX < 0:
            return out
        nMinCellY = max(0, x86_int(np.floor(F32(F32(F32(y - mny) - r) * hi))))
        if nMinCellY >= 48:
            return out
        nMaxCellY = min(47, x86_int(np.ceil(F32(F32(F32(y - mny) + r) * hi))))
        if nMaxCellY < 0:
            return out
        bCheckLevels = frame and (minLevel > 0 or maxLevel >= 0)
        for ix in range(nMinCellX, nMaxCellX + 1):
            for iy in range(nMinCellY, nMaxCellY + 1):
                for j in self.grid.get((ix, iy), []):
                    o = int(self.kps["octave"][j])
                    if bCheckLevels:
                        if o < minLevel:
                            continue
                        if maxLevel >= 0 and o > maxLevel:
                            continue
                    distx = F32(self.kps["x"][j] - x)
                    disty = F32(self.kps["y"][j] - y)
                    if abs(distx) < r and abs(disty) < r:
                        out.append(j)
        return out

    def dist(self, d, j):
        return int(np.unpackbits(d ^ self.desc[j]).sum())


def predict_scale(max_dist, dist, P):
    ratio = F32(F32(max_dist) / F32(dist))
    lr = math.log(float(ratio)) if ratio > 0 else -math.inf
    q = lr / float(F32(P.log_scale))
    n = x86_int(math.ceil(q)) if math.isfinite(q) else INT_MIN
    return 0 if n < 0 else (P.nlevels - 1 if n >= P.nlevels else n)


def rot_bin(a1, a2):
    rot = F32(F32(a1) - F32(a2))
    if rot < 0.0:
        rot = F32(rot + F32(360.0))
    b = roundf(F32(rot * F32(F32(1.0) / F32(30))))
    return 0 if b == 30 else b


def three_maxima(hist):
    max1 = max2 = max3 = 0
    i1 = i2 = i3 = -1
    for i, s in enumerate(hist):
        if s > max1:
            max3, max2, max1, i3, i2, i1 = max2, max1, s, i2, i1, i
        elif s > max2:
            max3, max2, i3, i2 = max2, s, i2, i
        elif s > max3:
            max3, i3 = s, i
    if F32(max2) < F32(0.1) * F32(max1):
        i2 = i3 = -1
    elif F32(max3) < F32(0.1) * F32(max1):
        i3 = -1
    return i1, i2, i3


def apply_rotation(rotHist, out, nmatches):
    keep = three_maxima([len(h) for h in rotHist])
    for i in range(30):
        if i not in keep:
            for j in rotHist[i]:
                out[j] = -2
                nmatches -= 1
    return nmatches


def py_last_frame(view, taken, pose, pts, pdesc, P, th, mono, check_ori):
    """SearchByProjection(CurrentFrame, LastFrame, th, bMono), src/ORBmatcher.cc:1396-1538."""
    cam = Cam(pose[:12], False)
    L = np.asarray(pose, np.float32).reshape(-1)[12:24]
    tlc2 = F32(mat3_row(L[8:11], *cam.Ow) + L[11])                # tlc = Rlw*twc+tlw
    bForward = tlc2 > P.b and not mono
    bBackward = -tlc2 > P.b and not mono
    out, taken, nmatches = [-1] * len(view.kps), list(taken), 0
    rotHist = [[] for _ in range(30)]
    for i, M in enumerate(pts):
        if not (M["flags"] & 1):
            continue
        xc, yc, zc = cam.to_cam((M["x"], M["y"], M["z"]))
        invzc = F32(1.0 / float(zc)) if zc != 0 else F32(math.copysign(math.inf, float(zc)))
        if invzc < 0:
            continue
        u = fmaf(F32(F32(P.fx) * xc), invzc, F32(P.cx))
        v = fmaf(F32(F32(P.fy) * yc), invzc, F32(P.cy))
        if u < F32(P.min_x) or u > F32(P.max_x) or v < F32(P.min_y) or v > F32(P.max_y):
            continue
        nLastOctave = int(M["octave"])
        radius = F32(F32(th) * SCALE16(P)[nLastOctave])
        if bForward:
            vIndices2 = view.area(u, v, radius, nLastOctave)
        elif bBackward:
            vIndices2 = view.area(u, v, radius, 0, nLastOctave)
        else:
            vIndices2 = view.area(u, v, radius, nLastOctave - 1, nLastOctave + 1)
        bestDist, bestIdx2 = 256, -1
        for i2 in vIndices2:
            if taken[i2]:
                continue
            if view.ur[i2] > 0:
                ur = fmaf(F32(-P.bf), invzc, u)
                er = abs(F32(ur - view.ur[i2]))
                if er > radius:
                    continue
            dist = view.dist(pdesc[i], i2)
            if dist < bestDist:
                bestDist, bestIdx2 = dist, i2
        if bestDist <= 100:
            out[bestIdx2] = i
            taken[bestIdx2] = bool(M["flags"] & 2)
            nmatches += 1
            if check_ori:
                rotHist[rot_bin(M["angle"], view.kps["angle"][bestIdx2])].append(bestIdx2)
    if check_ori:
        nmatches = apply_rotation(rotHist, out, nmatches)
    return nmatches, out


def SCALE16(P):
    return np.array(P.scale[:], np.float32)


def _dist_ok(cam, M, P):
    """The distance-invariance part shared by four overloads: returns (PO, dist3D) or None."""
    X = (M["x"], M["y"], M["z"])
    PO = [F32(X[k] - cam.Ow[k]) for k in range(3)]
    s = 0.0
    for k in range(3):
        s += float(PO[k]) * float(PO[k])
    dist = F32(math.sqrt(s))                                          # cv::norm(PO)
    maxDistance = F32(F32(1.2) * M["max_dist"])
    minDistance = F32(F32(0.8) * M["min_dist"])
    if dist < minDistance or dist > maxDistance:
        return None
    return PO, dist


def _view_angle_ok(PO, dist, M):
    dot = 0.0
    for k, nk in enumerate(("nx", "ny", "nz")):
        dot += float(PO[k]) * float(M[nk])                           # PO.dot(Pn)
    return not (dot < 0.5 * float(dist))


def py_keyframe(view, taken, pose, pts, pdesc, P, th, ORBdist, check_ori):
    """SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist), src/ORBmatcher.cc:1540-1667."""
    cam = Cam(pose[:12], False)
    out, taken, nmatches = [-1] * len(view.kps), list(taken), 0
    rotHist = [[] for _ in range(30)]
    for i, M in enumerate(pts):
        if not (M["flags"] & 1):
            continue
        xc, yc, zc = cam.to_cam((M["x"], M["y"], M["z"]))
        invzc = F32(1.0 / float(zc)) if zc != 0 else F32(math.copysign(math.inf, float(zc)))
        u = fmaf(F32(F32(P.fx) * xc), invzc, F32(P.cx))
        v = fmaf(F32(F32(P.fy) * yc), invzc, F32(P.cy))
        if u < F32(P.min_x) or u > F32(P.max_x) or v < F32(P.min_y) or v > F32(P.max_y):
            continue
        r = _dist_ok(cam, M, P)
        if r is None:
            continue
        nPredictedLevel = predict_scale(M["max_dist"], r[1], P)
        radius = F32(F32(th) * SCALE16(P)[nPredictedLevel])
        vIndices2 = view.area(u, v, radius, nPredictedLevel - 1, nPredictedLevel + 1)
        bestDist, bestIdx2 = 256, -1
        for i2 in vIndices2:
            if taken[i2]:
                continue
            dist = view.dist(pdesc[i], i2)
            if dist < bestDist:
                bestDist, bestIdx2 = dist, i2
        if bestDist <= ORBdist and bestIdx2 >= 0:
            out[bestIdx2] = i
            taken[bestIdx2] = True
            nmatches += 1
            if check_ori:
                rotHist[rot_bin(M["angle"], view.kps["angle"][bestIdx2])].append(bestIdx2)
    if check_ori:
        nmatches = apply_rotation(rotHist, out, nmatches)
    return nmatches, out


def _kf_project(cam, M, P, double_inv):
    xc, yc, zc = cam.to_cam((M["x"], M["y"], M["z"]))
    if zc < 0.0:
        return None
    if zc == 0:
        invz = F32(math.copysign(math.inf, float(zc)))
    elif double_inv:
        invz = F32(1.0 / float(zc))
    else:
        invz = F32(F32(1.0) / zc)
    x, y = F32(xc * invz), F32(yc * invz)
    u = fmaf(F32(P.fx), x, F32(P.cx))
    v = fmaf(F32(P.fy), y, F32(P.cy))
    if not (u >= F32(P.min_x) and u < F32(P.max_x) and v >= F32(P.min_y) and v < F32(P.max_y)):   # IsInImage
        return None
    return u, v, invz


def py_sim3(view, taken, Scw, pts, pdesc, P, th):
    """SearchByProjection(pKF, Scw, vpPoints, vpMatched, th), src/ORBmatcher.cc:290-403."""
    cam = Cam(Scw, True)
    out, vpMatched, nmatches = [-1] * len(view.kps), list(taken), 0
    for iMP, M in enumerate(pts):
        if not (M["flags"] & 1):
            continue
        p = _kf_project(cam, M, P, False)
        if p is None:
            continue
        u, v, _ = p
        r = _dist_ok(cam, M, P)
        if r is None or not _view_angle_ok(r[0], r[1], M):
            continue
        nPredictedLevel = predict_scale(M["max_dist"], r[1], P)
        radius = F32(F32(int(th)) * SCALE16(P)[nPredictedLevel])
        bestDist, bestIdx = 256, -1
        for idx in view.area(u, v, radius, frame=False):
            if vpMatched[idx]:
                continue
            kpLevel = int(view.kps["octave"][idx])
            if kpLevel < nPredictedLevel - 1 or kpLevel > nPredictedLevel:
                continue
            dist = view.dist(pdesc[iMP], idx)
            if dist < bestDist:
                bestDist, bestIdx = dist, idx
        if bestDist <= 50:
            vpMatched[bestIdx] = True
            out[bestIdx] = iMP
            nmatches += 1
    return nmatches, out


def py_fuse(view, pose, pts, pdesc, P, th, sim3):
    """Fuse(pKF, vpMapPoints, th) :893-1043 (sim3=False) / Fuse(pKF, Scw, vpPoints, th, ...) :1045-1168.
    Returns (nFused, the feature each MapPoint fuses into or -1)."""
    cam = Cam(pose[:12], sim3)
    out, nFused = [-1] * len(pts), 0
    inv_sigma2 = np.array(P.inv_sigma2[:], np.float32)
    for i, M in enumerate(pts):
        if not (M["flags"] & 1):
            continue
        p = _kf_project(cam, M, P, sim3)
        if p is None:
            continue
        u, v, invz = p
        ur = fmaf(F32(-P.bf), invz, u)
        r = _dist_ok(cam, M, P)
        if r is None or not _view_angle_ok(r[0], r[1], M):
            continue
        nPredictedLevel = predict_scale(M["max_dist"], r[1], P)
        radius = F32(F32(th) * SCALE16(P)[nPredictedLevel])
        bestDist, bestIdx = 256, -1
        for idx in view.area(u, v, radius, frame=False):
            kpLevel = int(view.kps["octave"][idx])
            if kpLevel < nPredictedLevel - 1 or kpLevel > nPredictedLevel:
                continue
            if not sim3:
                kpx, kpy = view.kps["x"][idx], view.kps["y"][idx]
                ex, ey = F32(u - kpx), F32(v - kpy)
                if view.ur[idx] >= 0:
                    er = F32(ur - view.ur[idx])
                    e2 = fmaf(er, er, fmaf(ex, ex, F32(ey * ey)))
                    if float(F32(e2 * inv_sigma2[kpLevel])) > 7.8:
                        continue
                else:
                    e2 = fmaf(ex, ex, F32(ey * ey))
                    if float(F32(e2 * inv_sigma2[kpLevel])) > 5.99:
                        continue
            dist = view.dist(pdesc[i], idx)
            if dist < bestDist:
                bestDist, bestIdx = dist, idx
        if bestDist <= 50:
            out[i] = bestIdx
            nFused += 1
    return nFused, out


# ------------------------------------------------------------------ scenes
def rodrigues(w):
    th = np.linalg.norm(w)
    if th < 1e-12:
        return np.eye(3)
    k = w / th
    Kx = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + math.sin(th) * Kx + (1 - math.cos(th)) * Kx @ Kx


def params(P_over=None, **kw):
    import orbref
    pp = orbref.PoseParams()
    pp.fx, pp.fy, pp.cx, pp.cy = K
    pp.bf, pp.b = BF, float(F32(BF) / F32(K[0]))
    pp.min_x, pp.max_x, pp.min_y, pp.max_y = BOUNDS
    pp.grid_w_inv = float(F32(64) / F32(BOUNDS[1] - BOUNDS[0]))
    pp.grid_h_inv = float(F32(48) / F32(BOUNDS[3] - BOUNDS[2]))
    pp.log_scale = float(F32(math.log(float(F32(1.2)))))
    pp.nlevels = 8
    sc = np.zeros(16, np.float32)
    sc[:8] = SCALE
    pp.scale[:] = [float(x) for x in sc]
    s2 = np.zeros(16, np.float32)
    s2[:8] = F32(1) / (SCALE * SCALE)
    pp.inv_sigma2[:] = [float(x) for x in s2]
    pp.th, pp.mono, pp.orb_dist, pp.check_ori = 1.0, 0, 100, 1
    for k, v in kw.items():
        setattr(pp, k, v)
    return pp


def scene(seed, n_kp=500, n_mp=700, sim3_scale=1.0, last_dz=0.0):
    """Keypoints on a 6-px lattice with clustered descriptors and per-keypoint depths; MapPoints
    back-projected from noisy copies of keypoints (several per keypoint), with distance ranges,
    normals and angles that mostly pass and sometimes fail each test."""
    import orbref
    rng = np.random.default_rng(seed)
    W, H = BOUNDS[1], BOUNDS[3]
    kps = np.zeros(n_kp, orbref.KEYPOINT_DTYPE)
    kps["x"] = (rng.integers(2, int(W) // 6 - 1, n_kp) * 6 + rng.random(n_kp)).astype(np.float32)
    kps["y"] = (rng.integers(2, int(H) // 6 - 1, n_kp) * 6 + rng.random(n_kp)).astype(np.float32)
    kps["octave"] = rng.integers(0, 8, n_kp)
    kps["angle"] = rng.uniform(0, 360, n_kp).astype(np.float32)
    proto = rng.integers(0, 256, (40, 32), dtype=np.uint8)
    owner = rng.integers(0, 40, n_kp)
    flip = lambda src, p: np.packbits(np.unpackbits(src, axis=-1) ^ (rng.random(src.shape[:-1] + (256,)) < p),
                                      axis=-1)
    desc = flip(proto[owner], 0.05)
    depth = rng.uniform(2.0, 30.0, n_kp)
    uright = np.where(rng.random(n_kp) < 0.4, kps["x"] - BF / depth, -1).astype(np.float32)
    claimed = (rng.random(n_kp) < 0.1).astype(np.uint8)
    R = rodrigues(rng.normal(0, 0.15, 3))
    t = rng.normal(0, 0.5, 3)
    Tcw = np.hstack([R, t[:, None]]).astype(np.float32)
    tgt = rng.integers(0, n_kp, n_mp)
    u = kps["x"][tgt] + rng.normal(0, 1.5, n_mp)
    v = kps["y"][tgt] + rng.normal(0, 1.5, n_mp)
    d = depth[tgt] * (1 + rng.normal(0, 0.01, n_mp))
    d = np.where(rng.random(n_mp) < 0.03, -d, d)                      # behind the camera
    Xc = np.stack([(u - K[2]) / K[0] * d, (v - K[3]) / K[1] * d, d], 1)
    Xw = (Xc - t) @ R                                                  # R^T (Xc - t)
    Ow = -R.T @ t
    dist = np.linalg.norm(Xw - Ow, axis=1)
    lvl = np.clip(kps["octave"][tgt] + rng.integers(0, 2, n_mp), 0, 7)
    max_dist = dist * 1.2 ** (lvl - rng.uniform(0.05, 0.95, n_mp))
    max_dist = np.where(rng.random(n_mp) < 0.05, dist * 0.5, max_dist)
    pts = np.zeros(n_mp, orbref.MAP_POINT_DTYPE)
    pts["x"], pts["y"], pts["z"] = Xw[:, 0], Xw[:, 1], Xw[:, 2]
    nrm = (Xw - Ow) / dist[:, None] + rng.normal(0, 0.2, (n_mp, 3))
    nrm = np.where((rng.random(n_mp) < 0.05)[:, None], -nrm, nrm)
    nrm /= np.linalg.norm(nrm, axis=1)[:, None]
    pts["nx"], pts["ny"], pts["nz"] = nrm[:, 0], nrm[:, 1], nrm[:, 2]
    pts["max_dist"] = max_dist
    pts["min_dist"] = max_dist / SCALE[7]
    ang = (kps["angle"][tgt] + rng.normal(0, 3, n_mp)) % 360
    pts["angle"] = np.where(rng.random(n_mp) < 0.2, rng.uniform(0, 360, n_mp), ang)
    pts["octave"] = lvl
    pts["flags"] = (rng.random(n_mp) < 0.9).astype(np.int32) | ((rng.random(n_mp) < 0.8).astype(np.int32) << 1)
    pdesc = flip(proto[owner[tgt]], 0.08)
    Tlw = Tcw.copy()
    Tlw[2, 3] += last_dz                                               # tlc_z = last_dz: forward / backward
    pose = np.concatenate([Tcw.ravel(), Tlw.ravel()]).astype(np.float32)
    Scw = (Tcw * F32(sim3_scale)).astype(np.float32)
    return kps, desc, uright, claimed, pose, Scw, pts, pdesc


CASES = {   # mode -> (kwargs of params, scene kwargs)
    "last_frame": [dict(th=7.0, mono=1), dict(th=15.0, mono=0)],
    "keyframe": [dict(th=10.0, orb_dist=100), dict(th=3.0, orb_dist=64)],
    "sim3": [dict(th=10.0)],
    "fuse": [dict(th=3.0)],
    "fuse_sim3": [dict(th=4.0)],
}


def run_py(mode, sc, pp):
    import orbref
    kps, desc, ur, cl, pose, Scw, pts, pdesc = sc
    view = View(kps, desc, ur, pp)
    if mode == "last_frame":
        return py_last_frame(view, cl.astype(bool), pose, pts, pdesc, pp, pp.th, pp.mono, pp.check_ori)
    if mode == "keyframe":
        return py_keyframe(view, cl.astype(bool), pose, pts, pdesc, pp, pp.th, pp.orb_dist, pp.check_ori)
    if mode == "sim3":
        return py_sim3(view, cl.astype(bool), Scw, pts, pdesc, pp, pp.th)
    return py_fuse(view, Scw if mode == "fuse_sim3" else pose, pts, pdesc, pp, pp.th, mode == "fuse_sim3")


def run_oracle(mode, sc, pp):
    import orbref
    kps, desc, ur, cl, pose, Scw, pts, pdesc = sc
    ps = Scw.ravel() if mode in ("sim3", "fuse_sim3") else pose
    return orbref.project_search(MODE_ID[mode], kps, desc, ur, cl, ps, pts, pdesc, pp)


def all_cases():
    out = []
    for mode, plist in CASES.items():
        for ci, kw in enumerate(plist):
            for seed in (0, 1):
                out.append((mode, ci, seed))
    return out


def case(mode, ci, seed):
    kw = CASES[mode][ci]
    scene_kw = {}
    if mode == "last_frame" and ci == 1:
        scene_kw["last_dz"] = 0.5 if seed == 0 else -0.5             # bForward, then bBackward
    if mode in ("sim3", "fuse_sim3"):
        scene_kw["sim3_scale"] = 1.7
    return scene(seed + 10 * ci, **scene_kw), params(**kw)


@pytest.mark.parametrize("mode,ci,seed", all_cases())
def test_oracle_matches_restatement(orbref, mode, ci, seed):
    sc, pp = case(mode, ci, seed)
    n, m = run_oracle(mode, sc, pp)
    pn, pm = run_py(mode, sc, pp)
    assert n == pn and list(m) == pm
    assert n > 30
    if mode in ("last_frame", "keyframe"):
        assert (m == -2).any()                                        # the rotation filter removed some


def test_last_frame_forward_backward_windows(orbref):
    """bForward restricts candidates to octave >= nLastOctave, bBackward to <= it: the three
    windows give different results on one scene."""
    res = []
    for dz in (0.0, 0.5, -0.5):
        sc = scene(3, last_dz=dz)
        res.append(run_oracle("last_frame", sc, params(th=15.0, mono=0)))
    assert res[0][0] != res[1][0] and res[0][0] != res[2][0]


def _tiny(orbref, xs, octs=None, angles=None):
    kps = np.zeros(len(xs), orbref.KEYPOINT_DTYPE)
    kps["x"] = [x for x, _ in xs]
    kps["y"] = [y for _, y in xs]
    if octs is not None:
        kps["octave"] = octs
    if angles is not None:
        kps["angle"] = angles
    return kps


def _point_at(orbref, u, v, d, Tcw=None):
    P = np.zeros(1, orbref.MAP_POINT_DTYPE)
    P["x"], P["y"], P["z"] = (u - K[2]) / K[0] * d, (v - K[3]) / K[1] * d, d
    P["nz"] = -1.0                                                     # irrelevant unless a test needs it
    P["max_dist"], P["min_dist"] = d * 1.1, d * 0.5                    # predicted level 1
    P["flags"] = 3
    return P


def test_last_frame_claims(orbref):
    """Two MapPoints with the same descriptor: with Observations() > 0 the first one takes the
    feature and the second falls back to the next; with 0 the second overwrites the first."""
    kps = _tiny(orbref, [(100, 100), (103, 100)])
    desc = np.zeros((2, 32), np.uint8)
    desc[1, 0] = 0x0F
    pts = np.concatenate([_point_at(orbref, 100, 100, 10), _point_at(orbref, 100, 100, 10)])
    pd = np.zeros((2, 32), np.uint8)
    pose = np.concatenate([np.hstack([np.eye(3), np.zeros((3, 1))]).ravel()] * 2).astype(np.float32)
    ur = np.full(2, -1, np.float32)
    pp = params(th=7.0, mono=1, check_ori=0)
    n, m = orbref.project_search(0, kps, desc, ur, np.zeros(2, np.uint8), pose, pts, pd, pp)
    assert n == 2 and list(m) == [0, 1]
    pts["flags"][0] = 1
    n, m = orbref.project_search(0, kps, desc, ur, np.zeros(2, np.uint8), pose, pts, pd, pp)
    assert n == 2 and list(m) == [1, -1]


def test_fuse_reprojection_threshold(orbref):
    """Monocular Fuse keeps a feature whose squared reprojection error * invSigma2 is <= 5.99
    (2 px at level 0) and rejects 2.5 px; a stereo feature is held to 7.8 with the right error."""
    pose = np.hstack([np.eye(3), np.zeros((3, 1))]).astype(np.float32).ravel()
    pp = params(th=3.0)
    for off, want in ((2.0, 0), (2.5, -1)):
        kps = _tiny(orbref, [(200 + off, 150)])
        P = _point_at(orbref, 200, 150, 5)
        P["max_dist"], P["min_dist"] = 5.0 * 1.1, 2.0                  # level 1: window 3*1.2, levels 0..1
        P["nx"], P["ny"], P["nz"] = 0, 0, 1
        n, m = orbref.project_search(3, kps, np.zeros((1, 32), np.uint8), np.full(1, -1, np.float32), None, pose, P,
                                     np.zeros((1, 32), np.uint8), pp)
        assert list(m) == [want] and n == (want == 0)


# ---------------------------------------------------------------------------- GPU

@pytest.mark.gpu
@pytest.mark.parametrize("mode,ci,seed", all_cases())
def test_gpu_project_search_host(orbref, cuda, mode, ci, seed):
    import orbx
    sc, pp = case(mode, ci, seed)
    kps, desc, ur, cl, pose, Scw, pts, pdesc = sc
    ps = Scw.ravel() if mode in ("sim3", "fuse_sim3") else pose
    gp = orbx.PoseParams.from_buffer_copy(pp)
    mt = orbx.ORBmatcher(0.9, bool(pp.check_ori))
    n, m = mt.project_search(MODE_ID[mode], kps, desc, ur, cl, ps, pts, pdesc, gp)
    wn, wm = run_oracle(mode, sc, pp)
    assert n == wn and np.array_equal(m, wm)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", MODES)
def test_gpu_project_search_batch(orbref, cuda, mode):
    """Four frames with their own poses in one device call."""
    import ctypes
    import torch
    import orbx
    ci = 1 if mode in ("last_frame", "keyframe") else 0
    cases = [case(mode, ci, s) for s in range(4)]
    scenes = [c[0] for c in cases]
    pp = cases[0][1]
    B = len(scenes)
    cap = max(len(s[0]) for s in scenes)
    pcap = max(len(s[6]) for s in scenes)
    kps = np.zeros((B, cap), orbx.KEYPOINT_DTYPE)
    desc = np.zeros((B, cap, 32), np.uint8)
    ur = np.zeros((B, cap), np.float32)
    cl = np.zeros((B, cap), np.uint8)
    pose = np.zeros((B, 24), np.float32)
    pts = np.zeros((B, pcap), orbx.MAP_POINT_DTYPE)
    pdesc = np.zeros((B, pcap, 32), np.uint8)
    counts = np.array([len(s[0]) for s in scenes], np.int32)
    npts = np.array([len(s[6]) for s in scenes], np.int32)
    for b, (k, d, u, c, po, Sc, p, pd) in enumerate(scenes):
        kps[b, :len(k)], desc[b, :len(k)], ur[b, :len(k)], cl[b, :len(k)] = k, d, u, c
        pose[b] = np.concatenate([Sc.ravel(), np.zeros(12, np.float32)]) if mode in ("sim3", "fuse_sim3") else po
        pts[b, :len(p)], pdesc[b, :len(p)] = p, pd
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(cuda)
    dk, dd, du, dc = T(kps.view(np.int32).reshape(B, cap, 7)), T(desc), T(ur), T(cl)
    dpo, dp, dpd, dn, dnp = T(pose), T(pts.view(np.int32).reshape(B, pcap, 12)), T(pdesc), T(counts), T(npts)
    nout = cap if MODE_ID[mode] <= 2 else pcap
    match = torch.empty((B, nout), dtype=torch.int32, device=cuda)
    nm = torch.empty((B,), dtype=torch.int32, device=cuda)
    gp = orbx.PoseParams.from_buffer_copy(pp)
    P = lambda t: ctypes.c_void_p(t.data_ptr())
    rc = orbx.lib.orbm_project_search_device(MODE_ID[mode], P(dk), P(dd), P(du), P(dc), P(dn), B, cap, P(dpo), P(dp),
                                             P(dpd), P(dnp), pcap, ctypes.byref(gp), P(match), P(nm),
                                             ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc == 0
    torch.cuda.synchronize()
    for b, sc in enumerate(scenes):
        wn, wm = run_oracle(mode, sc, pp)
        assert int(nm[b]) == wn
        assert np.array_equal(match[b, :len(wm)].cpu().numpy(), wm)


def _chain(orbref):
    """Fourteen MapPoints at one 3D point with one descriptor; twelve features around its projection at
    growing Hamming distance: each MapPoint (Observations() > 0) takes the next feature."""
    kps = _tiny(orbref, [(100.0 + i, 100.0) for i in range(12)])
    desc = np.zeros((12, 32), np.uint8)
    for i in range(12):
        desc[i, :i] = 0xFF
    pts = np.concatenate([_point_at(orbref, 105.5, 100, 10)] * 14)
    pose = np.concatenate([np.hstack([np.eye(3), np.zeros((3, 1))]).ravel()] * 2).astype(np.float32)
    return kps, desc, np.full(12, -1, np.float32), np.zeros(12, np.uint8), pose, pts, np.zeros((14, 32), np.uint8)


def test_claim_chain(orbref):
    kps, desc, ur, cl, pose, pts, pd = _chain(orbref)
    pp = params(th=7.0, mono=1, check_ori=0)
    n, m = orbref.project_search(0, kps, desc, ur, cl, pose, pts, pd, pp)
    assert n == 12 and list(m) == list(range(12))
    pn, pm = run_py("last_frame", (kps, desc, ur, cl, pose, pose[:12].reshape(3, 4), pts, pd), pp)
    assert pn == n and pm == list(m)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [0, 1])
def test_gpu_claim_chain(orbref, cuda, mode):
    """The replay runs out of its candidate list and scans the window again."""
    import orbx
    kps, desc, ur, cl, pose, pts, pd = _chain(orbref)
    pp = params(th=7.0, mono=1, check_ori=0, orb_dist=100)
    n, m = orbx.ORBmatcher(0.9, False).project_search(mode, kps, desc, ur, cl, pose, pts, pd,
                                                        orbx.PoseParams.from_buffer_copy(pp))
    wn, wm = orbref.project_search(mode, kps, desc, ur, cl, pose, pts, pd, pp)
    assert n == wn == 12 and np.array_equal(m, wm)
