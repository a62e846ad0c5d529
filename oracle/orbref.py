"""ctypes binding of the CPU parity oracle (TEST INFRASTRUCTURE ONLY).

Loaded by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg to
check (never to produce) the MI355X results.  See orbref.h for what it
restates and its parity status.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# ORBREF_LIB: another build of orbref.c (bench.py's -march=native CPU-baseline copy)
_LIB_PATH = os.environ.get("ORBREF_LIB") or os.path.join(_HERE, "_build", "liborbref.so")
_FAITHFUL_PATH = os.path.join(_HERE, "_build", "liborbref_faithful.so")

KEYPOINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                           ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
assert KEYPOINT_DTYPE.itemsize == 28

MAX_LEVELS = 16


class Params(C.Structure):
    _fields_ = [("nfeatures", C.c_int), ("scale_factor", C.c_float), ("nlevels", C.c_int),
                ("ini_th_fast", C.c_int), ("min_th_fast", C.c_int)]


class Tables(C.Structure):
    _fields_ = [("nlevels", C.c_int), ("nfeatures", C.c_int),
                ("scale", C.c_float * MAX_LEVELS), ("inv_scale", C.c_float * MAX_LEVELS),
                ("sigma2", C.c_float * MAX_LEVELS), ("inv_sigma2", C.c_float * MAX_LEVELS),
                ("nfeat_level", C.c_int * MAX_LEVELS), ("umax", C.c_int * 16)]


class CvModes(C.Structure):
    """SURVEY Appendix A's OpenCV build modes (orbref.h orbref_cv_modes)."""
    _fields_ = [("resize", C.c_int), ("blur", C.c_int), ("trig", C.c_int)]


RESIZE_SCALAR, RESIZE_SSE2 = 0, 1
BLUR_SCALAR, BLUR_SSE2, BLUR_BITEXACT = 0, 1, 2
TRIG_GLIBC, TRIG_CR = 0, 1


class ProjPoint(C.Structure):
    _fields_ = [("proj_x", C.c_float), ("proj_y", C.c_float), ("proj_xr", C.c_float), ("view_cos", C.c_float),
                ("level", C.c_int32), ("flags", C.c_int32)]


PROJ_DTYPE = np.dtype([("proj_x", "<f4"), ("proj_y", "<f4"), ("proj_xr", "<f4"), ("view_cos", "<f4"),
                       ("level", "<i4"), ("flags", "<i4")])


PROJ_LAST_FRAME, PROJ_KEYFRAME, PROJ_SIM3, FUSE, FUSE_SIM3 = 0, 1, 2, 3, 4

MAP_POINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("nx", "<f4"), ("ny", "<f4"), ("nz", "<f4"),
                            ("max_dist", "<f4"), ("min_dist", "<f4"), ("angle", "<f4"), ("octave", "<i4"),
                            ("flags", "<i4"), ("pad", "<i4")])
assert MAP_POINT_DTYPE.itemsize == 48


class PoseParams(C.Structure):
    _fields_ = [("fx", C.c_float), ("fy", C.c_float), ("cx", C.c_float), ("cy", C.c_float), ("bf", C.c_float),
                ("b", C.c_float), ("min_x", C.c_float), ("max_x", C.c_float), ("min_y", C.c_float),
                ("max_y", C.c_float), ("grid_w_inv", C.c_float), ("grid_h_inv", C.c_float),
                ("log_scale", C.c_float), ("nlevels", C.c_int32), ("th", C.c_float), ("mono", C.c_int32),
                ("orb_dist", C.c_int32), ("check_ori", C.c_int32), ("scale", C.c_float * 16),
                ("inv_sigma2", C.c_float * 16)]


class FeatVec(C.Structure):
    _fields_ = [("node", C.POINTER(C.c_int)), ("ptr", C.POINTER(C.c_int)), ("idx", C.POINTER(C.c_int)),
                ("nnodes", C.c_int)]


def build(force: bool = False) -> str:
    if os.environ.get("ORBREF_LIB"):
        return _LIB_PATH
    if force or not os.path.exists(_LIB_PATH) or not os.path.exists(_FAITHFUL_PATH):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    return _LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(_LIB_PATH)
        P = C.POINTER
        u8p, i32p, f32p = P(C.c_uint8), P(C.c_int), P(C.c_float)
        L.orbref_make_tables.argtypes = [P(Params), P(Tables)]
        L.orbref_resize_linear.argtypes = [u8p, C.c_int, C.c_int, C.c_size_t, u8p, C.c_int, C.c_int, C.c_size_t]
        L.orbref_fast.argtypes = [u8p, C.c_size_t, C.c_int, C.c_int, C.c_int, i32p, C.c_int]
        L.orbref_level_candidates.argtypes = [u8p, C.c_size_t, C.c_int, C.c_int, C.c_int, C.c_int, i32p, C.c_int]
        L.orbref_level_cells.argtypes = [C.c_int, C.c_int]
        L.orbref_distribute.argtypes = [i32p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, i32p, C.c_int]
        L.orbref_fast_atan2.argtypes = [C.c_float, C.c_float]
        L.orbref_fast_atan2.restype = C.c_float
        L.orbref_ic_angle.argtypes = [u8p, C.c_size_t, C.c_int, C.c_int, i32p]
        L.orbref_ic_angle.restype = C.c_float
        L.orbref_gaussian_blur7.argtypes = [u8p, C.c_int, C.c_int, C.c_size_t, u8p, C.c_size_t]
        L.orbref_brief.argtypes = [u8p, C.c_size_t, C.c_float, C.c_float, C.c_float, u8p]
        L.orbref_extract.argtypes = [P(Params), u8p, C.c_int, C.c_int, C.c_size_t, C.c_void_p, C.c_int,
                                     u8p, i32p, u8p, i32p, i32p]
        L.orbref_extract_mode.argtypes = [P(Params), P(CvModes), u8p, C.c_int, C.c_int, C.c_size_t, C.c_void_p,
                                          C.c_int, u8p, i32p, u8p, i32p, i32p]
        L.orbref_resize_simd_end.argtypes = [C.c_int]
        L.orbref_resize_linear_mode.argtypes = [u8p, C.c_int, C.c_int, C.c_size_t, u8p, C.c_int, C.c_int, C.c_size_t,
                                                C.c_int]
        L.orbref_blur_kernel.argtypes = [C.c_int, i32p]
        L.orbref_blur_kernel.restype = None
        L.orbref_gaussian_blur7_mode.argtypes = [u8p, C.c_int, C.c_int, C.c_size_t, u8p, C.c_size_t, C.c_int]
        L.orbref_brief_mode.argtypes = [u8p, C.c_size_t, C.c_float, C.c_float, C.c_float, u8p, C.c_int]
        L.orbref_descriptor_distance.argtypes = [u8p, u8p]
        L.orbref_search_for_initialization.argtypes = [C.c_void_p, u8p, C.c_int, C.c_void_p, u8p, C.c_int,
                                                       C.c_float, C.c_float, C.c_float, C.c_float, f32p, i32p,
                                                       C.c_int, C.c_float, C.c_int]
        L.orbref_compute_stereo_matches.argtypes = [P(Params), C.c_int, C.c_int, u8p, u8p, C.c_void_p, u8p,
                                                     C.c_int, C.c_void_p, u8p, C.c_int, C.c_float, C.c_float,
                                                     f32p, f32p, i32p]
        FV = P(FeatVec)
        L.orbref_search_by_bow_kf_f.argtypes = [C.c_void_p, u8p, u8p, C.c_int, FV, C.c_void_p, u8p, C.c_int, FV,
                                                C.c_float, C.c_int, i32p]
        L.orbref_search_by_bow_kf_kf.argtypes = [C.c_void_p, u8p, u8p, C.c_int, FV, C.c_void_p, u8p, u8p, C.c_int,
                                                 FV, C.c_float, C.c_int, i32p]
        L.orbref_search_for_triangulation.argtypes = [C.c_void_p, u8p, u8p, f32p, C.c_int, FV, C.c_void_p, u8p, u8p,
                                                      f32p, C.c_int, FV, f32p, C.c_float, C.c_float, f32p, f32p,
                                                      C.c_int, C.c_int, i32p]
        f64p = P(C.c_double)
        L.orbref_voc_transform.argtypes = [C.c_int, i32p, u8p, u8p, f64p, C.c_int, C.c_int, C.c_int, u8p, C.c_int,
                                           C.c_int, i32p, f64p, i32p, i32p, i32p, i32p, i32p]
        L.orbref_search_by_projection.argtypes = [C.c_void_p, u8p, f32p, u8p, C.c_int, C.c_float, C.c_float,
                                                  C.c_float, C.c_float, f32p, C.c_void_p, u8p, C.c_int, C.c_float,
                                                  C.c_float, i32p]
        L.orbref_project_search.argtypes = [C.c_int, C.c_void_p, u8p, f32p, u8p, C.c_int, f32p, C.c_void_p, u8p,
                                            C.c_int, P(PoseParams), i32p]
        L.orbref_ingest.argtypes = [u8p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_size_t, f32p, f32p, C.c_int, C.c_int,
                                    u8p, C.c_size_t]
        L.orbref_ingest.restype = None
        L.orbref_depth_convert.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_size_t, C.c_float, f32p,
                                           C.c_size_t]
        L.orbref_depth_convert.restype = None
        L.orbref_best2_csr.argtypes = [u8p, C.c_int, u8p, i32p, i32p, C.c_int, i32p, i32p, i32p]
        L.orbref_best2_csr.restype = None
        L.orbref_stereo_band.argtypes = [C.c_void_p, u8p, C.c_int, C.c_void_p, u8p, C.c_int, C.c_int, f32p,
                                         C.c_float, C.c_float, i32p, i32p]
        L.orbref_allpairs_top2.argtypes = [u8p, C.c_int, u8p, C.c_int, i32p, i32p, i32p]
        _lib = L
    return _lib


def _u8(a):
    return a.ctypes.data_as(C.POINTER(C.c_uint8))


def _i32(a):
    return a.ctypes.data_as(C.POINTER(C.c_int))


def _f32(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def make_params(nfeatures=1000, scale_factor=1.2, nlevels=8, ini_th_fast=20, min_th_fast=7) -> Params:
    return Params(nfeatures, scale_factor, nlevels, ini_th_fast, min_th_fast)


def tables(p: Params) -> Tables:
    t = Tables()
    rc = lib().orbref_make_tables(C.byref(p), C.byref(t))
    if rc != 0:
        raise ValueError("bad params")
    return t


def level_sizes(p: Params, cols: int, rows: int):
    t = tables(p)
    out = []
    for l in range(p.nlevels):
        s = np.float32(t.inv_scale[l])
        w = int(np.rint(np.float32(cols) * s))
        h = int(np.rint(np.float32(rows) * s))
        out.append((w, h))
    return out


def resize_linear(src: np.ndarray, dw: int, dh: int, mode: int = RESIZE_SCALAR) -> np.ndarray:
    src = np.ascontiguousarray(src, dtype=np.uint8)
    dst = np.empty((dh, dw), np.uint8)
    lib().orbref_resize_linear_mode(_u8(src), src.shape[1], src.shape[0], src.strides[0], _u8(dst), dw, dh, dw, mode)
    return dst


def resize_simd_end(width: int) -> int:
    return lib().orbref_resize_simd_end(width)


def blur_kernel(mode: int = BLUR_SCALAR) -> np.ndarray:
    k = np.zeros(7, np.int32)
    lib().orbref_blur_kernel(mode, _i32(k))
    return k


def fast(roi: np.ndarray, threshold: int) -> np.ndarray:
    roi = np.ascontiguousarray(roi, dtype=np.uint8)
    cap = roi.size
    out = np.empty((cap, 3), np.int32)
    n = lib().orbref_fast(_u8(roi), roi.strides[0], roi.shape[0], roi.shape[1], threshold, _i32(out), cap)
    assert n >= 0
    return out[:n].copy()


def level_candidates(level: np.ndarray, ini_th=20, min_th=7) -> np.ndarray:
    level = np.ascontiguousarray(level, dtype=np.uint8)
    cap = level.size // 2 + 16
    out = np.empty((cap, 3), np.int32)
    n = lib().orbref_level_candidates(_u8(level), level.strides[0], level.shape[1], level.shape[0],
                                      ini_th, min_th, _i32(out), cap)
    assert n >= 0
    return out[:n].copy()


def level_cells(w: int, h: int) -> int:
    return lib().orbref_level_cells(w, h)


def distribute(cands: np.ndarray, w: int, h: int, N: int) -> np.ndarray:
    cands = np.ascontiguousarray(cands, dtype=np.int32)
    cap = len(cands) + 8
    out = np.empty(cap, np.int32)
    n = lib().orbref_distribute(_i32(cands), len(cands), 16, w - 16, 16, h - 16, N, _i32(out), cap)
    assert n >= 0
    return out[:n].copy()


_faithful = None


def distribute_faithful(cands: np.ndarray, w: int, h: int, N: int, tie_mode: int = 0) -> np.ndarray:
    """DistributeOctTree with the reference's std::list nodes and (size, ExtractorNode*) sort
    (oracle/orbref_faithful.cpp): size ties broken by heap address, as in the reference process
    (tie_mode 0), or by creation order (tie_mode 1, which must equal distribute())."""
    global _faithful
    if _faithful is None:
        build()
        _faithful = C.CDLL(_FAITHFUL_PATH)
        i32p = C.POINTER(C.c_int)
        _faithful.orbref_distribute_faithful.argtypes = [i32p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                                         C.c_int, i32p, C.c_int]
    cands = np.ascontiguousarray(cands, dtype=np.int32)
    cap = len(cands) + 8
    out = np.empty(cap, np.int32)
    n = _faithful.orbref_distribute_faithful(_i32(cands), len(cands), 16, w - 16, 16, h - 16, N, tie_mode, _i32(out),
                                             cap)
    assert n >= 0
    return out[:n].copy()


def fast_atan2(y: float, x: float) -> float:
    return lib().orbref_fast_atan2(y, x)


def ic_angle(img: np.ndarray, cx: int, cy: int, umax) -> float:
    img = np.ascontiguousarray(img, dtype=np.uint8)
    um = np.ascontiguousarray(np.asarray(list(umax), np.int32))
    return lib().orbref_ic_angle(_u8(img), img.strides[0], cx, cy, _i32(um))


def gaussian_blur7(img: np.ndarray, mode: int = BLUR_SCALAR) -> np.ndarray:
    img = np.ascontiguousarray(img, dtype=np.uint8)
    dst = np.empty_like(img)
    lib().orbref_gaussian_blur7_mode(_u8(img), img.shape[1], img.shape[0], img.strides[0], _u8(dst), dst.strides[0],
                                     mode)
    return dst


def brief(blur: np.ndarray, x: float, y: float, angle: float, trig: int = TRIG_GLIBC) -> np.ndarray:
    blur = np.ascontiguousarray(blur, dtype=np.uint8)
    d = np.zeros(32, np.uint8)
    lib().orbref_brief_mode(_u8(blur), blur.strides[0], x, y, angle, _u8(d), trig)
    return d


class ExtractResult:
    def __init__(self, kps, desc, pyramid_levels, level_counts, cand_counts):
        self.keypoints = kps
        self.descriptors = desc
        self.pyramid = pyramid_levels
        self.level_counts = level_counts
        self.cand_counts = cand_counts


def extract(img: np.ndarray, p: Params, want_pyramid: bool = True, modes=None) -> ExtractResult:
    """ORBextractor::operator() restated; modes = (resize, blur, trig) OpenCV build modes (None: canonical)."""
    img = np.ascontiguousarray(img, dtype=np.uint8)
    rows, cols = img.shape
    sizes = level_sizes(p, cols, rows)
    cap = p.nfeatures + 64 * p.nlevels + 64
    kps = np.zeros(cap, KEYPOINT_DTYPE)
    desc = np.zeros((cap, 32), np.uint8)
    n = C.c_int(0)
    pyr = np.zeros(sum(w * h for w, h in sizes), np.uint8) if want_pyramid else None
    lc = np.zeros(MAX_LEVELS, np.int32)
    cc = np.zeros(MAX_LEVELS, np.int32)
    m = None if modes is None else C.byref(CvModes(*modes))
    rc = lib().orbref_extract_mode(C.byref(p), m, _u8(img), rows, cols, img.strides[0], kps.ctypes.data, cap,
                                   _u8(desc), C.byref(n), _u8(pyr) if pyr is not None else None, _i32(lc), _i32(cc))
    if rc != 0:
        raise RuntimeError("orbref_extract failed: %d" % rc)
    levels = None
    if pyr is not None:
        levels, o = [], 0
        for w, h in sizes:
            levels.append(pyr[o:o + w * h].reshape(h, w))
            o += w * h
    k = n.value
    return ExtractResult(kps[:k].copy(), desc[:k].copy(), levels, lc[:p.nlevels].copy(), cc[:p.nlevels].copy())


def descriptor_distance(a: np.ndarray, b: np.ndarray) -> int:
    a = np.ascontiguousarray(a, np.uint8)
    b = np.ascontiguousarray(b, np.uint8)
    return lib().orbref_descriptor_distance(_u8(a), _u8(b))


def search_for_initialization(kps1, desc1, kps2, desc2, cols, rows, window=100, nnratio=0.9, check_ori=True,
                              prev_xy=None, bounds=None):
    """ORBmatcher::SearchForInitialization (src/ORBmatcher.cc:417-588).  bounds = (mnMinX, mnMaxX, mnMinY,
    mnMaxY) (default 0..cols x 0..rows); prev_xy = vbPrevMatched (n1, 2) (default F1's keypoints).
    Returns (nmatches, vnMatches12, updated vbPrevMatched)."""
    kps1 = np.ascontiguousarray(kps1, KEYPOINT_DTYPE)
    kps2 = np.ascontiguousarray(kps2, KEYPOINT_DTYPE)
    desc1 = np.ascontiguousarray(desc1, np.uint8)
    desc2 = np.ascontiguousarray(desc2, np.uint8)
    n1, n2 = len(kps1), len(kps2)
    if prev_xy is None:
        prev_xy = np.stack([kps1["x"], kps1["y"]], axis=1).astype(np.float32)
    prev_xy = np.ascontiguousarray(prev_xy, np.float32).copy()
    m12 = np.full(max(n1, 1), -1, np.int32)
    if bounds is None:
        bounds = (0.0, float(cols), 0.0, float(rows))
    nm = lib().orbref_search_for_initialization(kps1.ctypes.data, _u8(desc1), n1, kps2.ctypes.data, _u8(desc2),
                                                n2, *[float(np.float32(b)) for b in bounds], _f32(prev_xy),
                                                _i32(m12), window, nnratio, 1 if check_ori else 0)
    return nm, m12[:n1].copy(), prev_xy


def compute_stereo_matches(p: Params, left: ExtractResult, right: ExtractResult, rows: int, cols: int,
                           bf: float, fx: float):
    """Frame::ComputeStereoMatches on two oracle extractions (want_pyramid=True).
    Returns (uRight, depth, sad, ngood)."""
    pl = np.ascontiguousarray(np.concatenate([l.ravel() for l in left.pyramid]))
    pr = np.ascontiguousarray(np.concatenate([l.ravel() for l in right.pyramid]))
    kl = np.ascontiguousarray(left.keypoints, KEYPOINT_DTYPE)
    kr = np.ascontiguousarray(right.keypoints, KEYPOINT_DTYPE)
    dl = np.ascontiguousarray(left.descriptors, np.uint8)
    dr = np.ascontiguousarray(right.descriptors, np.uint8)
    n = len(kl)
    ur = np.empty(max(n, 1), np.float32)
    dp = np.empty(max(n, 1), np.float32)
    sd = np.empty(max(n, 1), np.int32)
    good = lib().orbref_compute_stereo_matches(C.byref(p), rows, cols, _u8(pl), _u8(pr), kl.ctypes.data, _u8(dl), n,
                                               kr.ctypes.data, _u8(dr), len(kr), bf, fx, _f32(ur), _f32(dp), _i32(sd))
    if good < 0:
        raise RuntimeError("orbref_compute_stereo_matches failed: %d" % good)
    return ur[:n].copy(), dp[:n].copy(), sd[:n].copy(), good


def _fv(fv):
    node, ptr, idx = (np.ascontiguousarray(a, np.int32) for a in fv)
    f = FeatVec(_i32(node), _i32(ptr), _i32(idx), len(node))
    f._keep = (node, ptr, idx)
    return f


def _kp(k):
    return np.ascontiguousarray(k, KEYPOINT_DTYPE)


def search_by_bow_kf_f(kkf, dkf, kf_has_mp, fvkf, kf, df, fvf, nnratio=0.7, check_ori=True):
    """SearchByBoW(KeyFrame*, Frame&): returns (nmatches, match_f[nF] = KF index or -1)."""
    kkf, kf = _kp(kkf), _kp(kf)
    dkf, df = np.ascontiguousarray(dkf, np.uint8), np.ascontiguousarray(df, np.uint8)
    mp = np.ascontiguousarray(kf_has_mp, np.uint8)
    out = np.empty(max(len(kf), 1), np.int32)
    a, b = _fv(fvkf), _fv(fvf)
    n = lib().orbref_search_by_bow_kf_f(kkf.ctypes.data, _u8(dkf), _u8(mp), len(kkf), C.byref(a), kf.ctypes.data,
                                        _u8(df), len(kf), C.byref(b), nnratio, 1 if check_ori else 0, _i32(out))
    return n, out[:len(kf)].copy()


def search_by_bow_kf_kf(k1, d1, mp1, fv1, k2, d2, mp2, fv2, nnratio=0.75, check_ori=True):
    """SearchByBoW(KeyFrame*, KeyFrame*): returns (nmatches, match12[n1] = idx2 or -1)."""
    k1, k2 = _kp(k1), _kp(k2)
    d1, d2 = np.ascontiguousarray(d1, np.uint8), np.ascontiguousarray(d2, np.uint8)
    m1, m2 = np.ascontiguousarray(mp1, np.uint8), np.ascontiguousarray(mp2, np.uint8)
    out = np.empty(max(len(k1), 1), np.int32)
    a, b = _fv(fv1), _fv(fv2)
    n = lib().orbref_search_by_bow_kf_kf(k1.ctypes.data, _u8(d1), _u8(m1), len(k1), C.byref(a), k2.ctypes.data,
                                         _u8(d2), _u8(m2), len(k2), C.byref(b), nnratio, 1 if check_ori else 0,
                                         _i32(out))
    return n, out[:len(k1)].copy()


def search_for_triangulation(k1, d1, mp1, ur1, fv1, k2, d2, mp2, ur2, fv2, F12, ex, ey, scale2, sigma2_2,
                             only_stereo=False, check_ori=True):
    """SearchForTriangulation: returns (nmatches, match12[n1] = idx2 or -1)."""
    k1, k2 = _kp(k1), _kp(k2)
    d1, d2 = np.ascontiguousarray(d1, np.uint8), np.ascontiguousarray(d2, np.uint8)
    m1, m2 = np.ascontiguousarray(mp1, np.uint8), np.ascontiguousarray(mp2, np.uint8)
    u1, u2 = np.ascontiguousarray(ur1, np.float32), np.ascontiguousarray(ur2, np.float32)
    F = np.ascontiguousarray(F12, np.float32).reshape(9)
    s2, g2 = np.ascontiguousarray(scale2, np.float32), np.ascontiguousarray(sigma2_2, np.float32)
    out = np.empty(max(len(k1), 1), np.int32)
    a, b = _fv(fv1), _fv(fv2)
    n = lib().orbref_search_for_triangulation(k1.ctypes.data, _u8(d1), _u8(m1), _f32(u1), len(k1), C.byref(a),
                                              k2.ctypes.data, _u8(d2), _u8(m2), _f32(u2), len(k2), C.byref(b),
                                              _f32(F), ex, ey, _f32(s2), _f32(g2), 1 if only_stereo else 0,
                                              1 if check_ori else 0, _i32(out))
    return n, out[:len(k1)].copy()


def voc_transform(voc, desc, levelsup=4):
    """DBoW2 transform with the oracle: voc has parent/is_leaf/desc/weight/L/scoring/weighting.
    Returns (bow_word, bow_weight, (fv_node, fv_ptr, fv_idx))."""
    desc = np.ascontiguousarray(desc, np.uint8)
    n = len(desc)
    par = np.ascontiguousarray(voc.parent, np.int32)
    leaf = np.ascontiguousarray(voc.is_leaf, np.uint8)
    vd = np.ascontiguousarray(voc.desc, np.uint8)
    w = np.ascontiguousarray(voc.weight, np.float64)
    bw = np.zeros(n + 1, np.int32)
    bv = np.zeros(n + 1, np.float64)
    fn = np.zeros(n + 1, np.int32)
    fp = np.zeros(n + 2, np.int32)
    fi = np.zeros(n + 1, np.int32)
    nb, nn = C.c_int(0), C.c_int(0)
    lib().orbref_voc_transform(len(par), _i32(par), _u8(leaf), _u8(vd), w.ctypes.data_as(C.POINTER(C.c_double)),
                               voc.L, voc.scoring, voc.weighting, _u8(desc), n, levelsup, _i32(bw),
                               bv.ctypes.data_as(C.POINTER(C.c_double)), C.byref(nb), _i32(fn), _i32(fp), _i32(fi),
                               C.byref(nn))
    k, m = nb.value, nn.value
    return bw[:k].copy(), bv[:k].copy(), (fn[:m].copy(), fp[:m + 1].copy(), fi[:fp[m]].copy())


def search_by_projection(kps, desc, uright, claimed, grid, scale, pts, pdesc, th=1.0, nnratio=0.8):
    """SearchByProjection(Frame&, vector<MapPoint*>, th).  grid = (min_x, min_y, w_inv, h_inv);
    pts: PROJ_DTYPE array.  Returns (nmatches, match[n])."""
    kps = np.ascontiguousarray(kps, KEYPOINT_DTYPE)
    desc = np.ascontiguousarray(desc, np.uint8)
    ur = np.ascontiguousarray(uright, np.float32)
    cl = np.ascontiguousarray(claimed, np.uint8)
    sc = np.ascontiguousarray(scale, np.float32)
    pts = np.ascontiguousarray(pts, PROJ_DTYPE)
    pd = np.ascontiguousarray(pdesc, np.uint8)
    n = len(kps)
    out = np.full(max(n, 1), -1, np.int32)
    nm = lib().orbref_search_by_projection(kps.ctypes.data, _u8(desc), _f32(ur), _u8(cl), n, grid[0], grid[1],
                                           grid[2], grid[3], _f32(sc), pts.ctypes.data, _u8(pd), len(pts), th,
                                           nnratio, _i32(out))
    return nm, out[:n].copy()


def project_search(mode, kps, desc, uright, claimed, pose, pts, pdesc, params: PoseParams):
    """The pose-projection searches (orbref.h ORBREF_PROJ_* / ORBREF_FUSE*).  pose: 24 floats
    (Tcw or Scw 3x4, then LastFrame Tcw).  Returns (n, match) with match[n] for the search
    modes and match[np] for the Fuse modes."""
    kps = np.ascontiguousarray(kps, KEYPOINT_DTYPE)
    desc = np.ascontiguousarray(desc, np.uint8)
    ur = np.ascontiguousarray(uright, np.float32)
    cl = np.ascontiguousarray(claimed if claimed is not None else np.zeros(len(kps), np.uint8), np.uint8)
    ps = np.zeros(24, np.float32)
    pose = np.asarray(pose, np.float32).ravel()
    ps[:len(pose)] = pose
    pts = np.ascontiguousarray(pts, MAP_POINT_DTYPE)
    pd = np.ascontiguousarray(pdesc, np.uint8)
    nout = len(kps) if mode <= PROJ_SIM3 else len(pts)
    out = np.full(max(nout, 1), -1, np.int32)
    nm = lib().orbref_project_search(mode, kps.ctypes.data, _u8(desc), _f32(ur), _u8(cl), len(kps), _f32(ps),
                                     pts.ctypes.data, _u8(pd), len(pts), C.byref(params), _i32(out))
    return nm, out[:nout].copy()


def ingest(src, rgb=False, map_x=None, map_y=None):
    """remap(INTER_LINEAR, BORDER_CONSTANT) then cvtColor to gray.  src: (H, W) or (H, W, C) uint8."""
    src = np.ascontiguousarray(src, np.uint8)
    rows, cols = src.shape[:2]
    ch = 1 if src.ndim == 2 else src.shape[2]
    if map_x is not None:
        mx = np.ascontiguousarray(map_x, np.float32)
        my = np.ascontiguousarray(map_y, np.float32)
        dr, dc = mx.shape
    else:
        mx = my = None
        dr, dc = rows, cols
    out = np.zeros((dr, dc), np.uint8)
    lib().orbref_ingest(_u8(src), rows, cols, ch, int(bool(rgb)), cols * ch, _f32(mx) if mx is not None else None,
                        _f32(my) if my is not None else None, dr, dc, _u8(out), dc)
    return out


def depth_convert(src, factor):
    src = np.ascontiguousarray(src)
    dt = 0 if src.dtype == np.uint16 else 1
    if dt == 1:
        src = src.astype(np.float32, copy=False)
    rows, cols = src.shape
    out = np.zeros((rows, cols), np.float32)
    lib().orbref_depth_convert(src.ctypes.data, dt, rows, cols, src.strides[0], factor, _f32(out), cols * 4)
    return out


def best2_csr(q, t, ptr, idx, tie_last=False):
    q = np.ascontiguousarray(q, np.uint8)
    t = np.ascontiguousarray(t if len(t) else np.zeros((1, 32), np.uint8), np.uint8)
    ptr = np.ascontiguousarray(ptr, np.int32)
    idx = np.ascontiguousarray(idx if len(idx) else np.zeros(1, np.int32), np.int32)
    nq = len(q)
    bi, b1, b2 = (np.zeros(max(nq, 1), np.int32) for _ in range(3))
    lib().orbref_best2_csr(_u8(q), nq, _u8(t), _i32(ptr), _i32(idx), int(bool(tie_last)), _i32(bi), _i32(b1), _i32(b2))
    return bi[:nq].copy(), b1[:nq].copy(), b2[:nq].copy()


def stereo_band(kl, dl, kr, dr, rows, scale, min_d, max_d):
    """The coarse stage of ComputeStereoMatches alone: (best_idx, best_dist) per left keypoint."""
    n, nr = len(kl), len(kr)
    kl, kr = _kp(kl if n else np.zeros(1, KEYPOINT_DTYPE)), _kp(kr if nr else np.zeros(1, KEYPOINT_DTYPE))
    dl = np.ascontiguousarray(dl if n else np.zeros((1, 32), np.uint8), np.uint8)
    dr = np.ascontiguousarray(dr if nr else np.zeros((1, 32), np.uint8), np.uint8)
    sc = np.ascontiguousarray(scale, np.float32)
    bi, bd = np.zeros(max(n, 1), np.int32), np.zeros(max(n, 1), np.int32)
    lib().orbref_stereo_band(kl.ctypes.data, _u8(dl), n, kr.ctypes.data, _u8(dr), nr, rows, _f32(sc), min_d, max_d,
                             _i32(bi), _i32(bd))
    return bi[:n].copy(), bd[:n].copy()


def allpairs_top2(q: np.ndarray, t: np.ndarray):
    q = np.ascontiguousarray(q, np.uint8)
    t = np.ascontiguousarray(t, np.uint8)
    bi = np.empty(len(q), np.int32)
    b1 = np.empty(len(q), np.int32)
    b2 = np.empty(len(q), np.int32)
    lib().orbref_allpairs_top2(_u8(q), len(q), _u8(t), len(t), _i32(bi), _i32(b1), _i32(b2))
    return bi, b1, b2
