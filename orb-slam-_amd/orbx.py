"""Python binding of liborbx (the MI355X ORB front-end C ABI, include/orbx.h).

Mirrors the reference's operator interface for the hot path:

* ``ORBextractor(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST)`` with
  ``__call__(image) -> (keypoints, descriptors)``, the getters
  ``GetLevels/GetScaleFactor/GetScaleFactors/...`` and ``mvImagePyramid``
  (include/ORBextractor.h:45-111).
* ``ORBmatcher.DescriptorDistance`` (include/ORBmatcher.h:44) plus the batched
  device searches.

Keypoints are numpy structured arrays laid out like cv::KeyPoint (28 bytes).
Device-batch entry points take torch tensors (torch is used only for device
memory and streams).  There is no CPU fallback: if liborbx.so is missing this
module raises on import.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liborbx.so")

KEYPOINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                           ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])

OK, EMPTY, EINVAL, ENOMEM, EDEVICE, ENOSPC = 0, 1, -22, -12, -5, -28
TOP2, FULL_U16 = 0, 1

EXPORTED = [
    "orbx_create", "orbx_destroy", "orbx_get_tables", "orbx_capacity", "orbx_extract", "orbx_get_level",
    "orbx_extract_batch_device", "orbx_sync", "orbx_set_timing", "orbx_get_stage_times",
    "orbx_debug_pyramid", "orbx_debug_candidates", "orbm_descriptor_distance", "orbm_allpairs_device",
    "orbm_search_init_batch_device", "orbx_compute_stereo_matches", "orbx_stereo_batch_device",
]


class OrbxError(RuntimeError):
    def __init__(self, fn, code):
        super().__init__("%s failed with status %d" % (fn, code))
        self.code = code


class _Params(C.Structure):
    _fields_ = [("nfeatures", C.c_int), ("scale_factor", C.c_float), ("nlevels", C.c_int),
                ("ini_th_fast", C.c_int), ("min_th_fast", C.c_int)]


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError("liborbx.so not built (run `make -C orb-slam-_amd` or __graft_entry__.build())")
    L = C.CDLL(LIB_PATH)
    P, vp = C.POINTER, C.c_void_p
    u8p, i32p, f32p = P(C.c_uint8), P(C.c_int), P(C.c_float)
    L.orbx_create.argtypes = [P(_Params), C.c_int, P(vp)]
    L.orbx_destroy.argtypes = [vp]
    L.orbx_destroy.restype = None
    L.orbx_get_tables.argtypes = [vp, i32p, f32p, f32p, f32p, f32p, f32p, i32p]
    L.orbx_capacity.argtypes = [vp, C.c_int, C.c_int]
    L.orbx_extract.argtypes = [vp, u8p, C.c_int, C.c_int, C.c_size_t, vp, C.c_int, u8p, i32p]
    L.orbx_get_level.argtypes = [vp, C.c_int, P(u8p), i32p, i32p, P(C.c_size_t)]
    L.orbx_extract_batch_device.argtypes = [vp, vp, C.c_int, C.c_int, C.c_int, C.c_size_t, C.c_size_t, vp, vp,
                                            vp, C.c_int, vp]
    L.orbx_sync.argtypes = [vp, vp]
    L.orbx_set_timing.argtypes = [vp, C.c_int]
    L.orbx_get_stage_times.argtypes = [vp, f32p, C.c_int]
    L.orbx_debug_pyramid.argtypes = [vp, C.c_int, u8p, C.c_size_t]
    L.orbx_debug_candidates.argtypes = [vp, C.c_int, C.c_int, i32p, C.c_int, i32p]
    L.orbm_descriptor_distance.argtypes = [u8p, u8p]
    L.orbm_allpairs_device.argtypes = [vp, C.c_int, vp, C.c_int, C.c_int, vp, vp, vp, vp, vp]
    L.orbm_search_init_batch_device.argtypes = [vp, vp, vp, C.c_int, C.c_int, vp, vp, C.c_int, C.c_int, C.c_int,
                                                C.c_int, C.c_float, C.c_int, vp, vp, vp]
    L.orbx_compute_stereo_matches.argtypes = [vp, vp, vp, u8p, C.c_int, vp, u8p, C.c_int, C.c_float, C.c_float,
                                              f32p, f32p, i32p]
    L.orbx_stereo_batch_device.argtypes = [vp, vp, vp, vp, C.c_int, vp, vp, C.c_int, C.c_float, C.c_float, vp, vp,
                                           vp, vp]
    return L


lib = _load()


def _check(fn, rc):
    if rc not in (OK, EMPTY):
        raise OrbxError(fn, rc)
    return rc


def _u8(a):
    return a.ctypes.data_as(C.POINTER(C.c_uint8))


def _ptr(t):
    return C.c_void_p(t.data_ptr()) if t is not None else None


def _stream(stream):
    if stream is None:
        import torch
        stream = torch.cuda.current_stream()
    return C.c_void_p(stream.cuda_stream)


class ORBextractor:
    """ORB_SLAM2::ORBextractor (include/ORBextractor.h:45-111) on an MI355X."""

    def __init__(self, nfeatures=1000, scaleFactor=1.2, nlevels=8, iniThFAST=20, minThFAST=7, device=0):
        self.params = _Params(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST)
        h = C.c_void_p()
        _check("orbx_create", lib.orbx_create(C.byref(self.params), device, C.byref(h)))
        self._h = h
        n = nlevels
        self._scale = np.zeros(n, np.float32)
        self._inv = np.zeros(n, np.float32)
        self._s2 = np.zeros(n, np.float32)
        self._is2 = np.zeros(n, np.float32)
        self._nfl = np.zeros(n, np.int32)
        f32 = lambda a: a.ctypes.data_as(C.POINTER(C.c_float))
        _check("orbx_get_tables", lib.orbx_get_tables(h, None, None, f32(self._scale), f32(self._inv), f32(self._s2),
                                                      f32(self._is2), self._nfl.ctypes.data_as(C.POINTER(C.c_int))))
        self._last_shape = None

    def close(self):
        if getattr(self, "_h", None):
            lib.orbx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # getters, include/ORBextractor.h:63-83
    def GetLevels(self):
        return self.params.nlevels

    def GetScaleFactor(self):
        return float(np.float32(self.params.scale_factor))

    def GetScaleFactors(self):
        return self._scale.copy()

    def GetInverseScaleFactors(self):
        return self._inv.copy()

    def GetScaleSigmaSquares(self):
        return self._s2.copy()

    def GetInverseScaleSigmaSquares(self):
        return self._is2.copy()

    def features_per_level(self):
        return self._nfl.copy()

    def capacity(self, rows, cols):
        c = lib.orbx_capacity(self._h, rows, cols)
        if c < 0:
            raise OrbxError("orbx_capacity", c)
        return c

    def __call__(self, image, mask=None):
        """operator()(image, mask, keypoints, descriptors); mask ignored like the reference."""
        img = np.ascontiguousarray(image, dtype=np.uint8)
        if img.size == 0:
            return np.zeros(0, KEYPOINT_DTYPE), None
        rows, cols = img.shape
        cap = self.capacity(rows, cols)
        kps = np.zeros(cap, KEYPOINT_DTYPE)
        desc = np.zeros((cap, 32), np.uint8)
        n = C.c_int(0)
        _check("orbx_extract", lib.orbx_extract(self._h, _u8(img), rows, cols, img.strides[0], kps.ctypes.data, cap,
                                                _u8(desc), C.byref(n)))
        self._last_shape = (rows, cols)
        k = n.value
        return kps[:k].copy(), (desc[:k].copy() if k else None)

    @property
    def mvImagePyramid(self):
        out = []
        for l in range(self.params.nlevels):
            p = C.POINTER(C.c_uint8)()
            r, c, s = C.c_int(), C.c_int(), C.c_size_t()
            _check("orbx_get_level", lib.orbx_get_level(self._h, l, C.byref(p), C.byref(r), C.byref(c), C.byref(s)))
            buf = np.ctypeslib.as_array(p, shape=(r.value * s.value,))
            out.append(buf.reshape(r.value, s.value)[:, :c.value].copy())
        return out

    # ---- device batch (config 2/4 replay) ----
    def extract_batch_device(self, imgs, kps, desc, counts, stream=None):
        """imgs: uint8 cuda tensor (B, H, W) (row pitch = stride(1)); kps: int32 (B, cap, 7);
        desc: uint8 (B, cap, 32); counts: int32 (B,).  Asynchronous on `stream`."""
        B, H, W = imgs.shape
        cap = kps.shape[1]
        rc = lib.orbx_extract_batch_device(self._h, _ptr(imgs), B, H, W, imgs.stride(1), imgs.stride(0), _ptr(kps),
                                           _ptr(desc), _ptr(counts), cap, _stream(stream))
        _check("orbx_extract_batch_device", rc)

    def stereo_batch_device(self, kps, desc, counts, left, right, bf, fx, u_right=None, depth=None, n_good=None,
                            stream=None):
        """Frame::ComputeStereoMatches on pairs (left[p], right[p]) of the last device batch.
        Returns (u_right (P, cap) f32, depth (P, cap) f32, n_good (P,) i32) cuda tensors."""
        import torch
        npairs, cap = left.shape[0], kps.shape[1]
        if u_right is None:
            u_right = torch.empty((npairs, cap), dtype=torch.float32, device=kps.device)
        if depth is None:
            depth = torch.empty((npairs, cap), dtype=torch.float32, device=kps.device)
        if n_good is None:
            n_good = torch.empty((npairs,), dtype=torch.int32, device=kps.device)
        rc = lib.orbx_stereo_batch_device(self._h, _ptr(kps), _ptr(desc), _ptr(counts), cap, _ptr(left), _ptr(right),
                                          npairs, bf, fx, _ptr(u_right), _ptr(depth), _ptr(n_good), _stream(stream))
        _check("orbx_stereo_batch_device", rc)
        return u_right, depth, n_good

    def sync(self, stream=None):
        _check("orbx_sync", lib.orbx_sync(self._h, _stream(stream)))

    def set_timing(self, enable=True):
        _check("orbx_set_timing", lib.orbx_set_timing(self._h, 1 if enable else 0))

    def stage_times(self):
        ms = np.zeros(4, np.float32)
        _check("orbx_get_stage_times", lib.orbx_get_stage_times(self._h, ms.ctypes.data_as(C.POINTER(C.c_float)), 4))
        return ms

    def debug_pyramid(self, frame, sizes):
        total = sum(w * h for w, h in sizes)
        buf = np.zeros(total, np.uint8)
        _check("orbx_debug_pyramid", lib.orbx_debug_pyramid(self._h, frame, _u8(buf), total))
        out, o = [], 0
        for w, h in sizes:
            out.append(buf[o:o + w * h].reshape(h, w))
            o += w * h
        return out

    def debug_candidates(self, frame, level, cap=1 << 20):
        out = np.zeros((cap, 3), np.int32)
        n = C.c_int(0)
        _check("orbx_debug_candidates", lib.orbx_debug_candidates(self._h, frame, level,
                                                                  out.ctypes.data_as(C.POINTER(C.c_int)), cap,
                                                                  C.byref(n)))
        return out[:n.value].copy()


def compute_stereo_matches(left, right, kps_l, desc_l, kps_r, desc_r, bf, fx):
    """Frame::ComputeStereoMatches (src/Frame.cc:630-872) for the host path: `left` / `right`
    are the two ORBextractor objects right after extracting the left / right image.
    Returns (mvuRight, mvDepth, n_good)."""
    kl = np.ascontiguousarray(kps_l, KEYPOINT_DTYPE)
    kr = np.ascontiguousarray(kps_r, KEYPOINT_DTYPE)
    nl, nr = len(kl), len(kr)
    dl = np.ascontiguousarray(desc_l if desc_l is not None else np.zeros((0, 32), np.uint8), np.uint8)
    dr = np.ascontiguousarray(desc_r if desc_r is not None else np.zeros((0, 32), np.uint8), np.uint8)
    ur = np.full(max(nl, 1), -1.0, np.float32)
    dp = np.full(max(nl, 1), -1.0, np.float32)
    ng = C.c_int(0)
    f32 = lambda a: a.ctypes.data_as(C.POINTER(C.c_float))
    _check("orbx_compute_stereo_matches",
           lib.orbx_compute_stereo_matches(left._h, right._h, kl.ctypes.data, _u8(dl), nl, kr.ctypes.data, _u8(dr), nr,
                                           bf, fx, f32(ur), f32(dp), C.byref(ng)))
    return ur[:nl].copy(), dp[:nl].copy(), ng.value


def keypoints_from_device(kps_i32, counts):
    """(B, cap, 7) int32 torch tensor + counts -> list of structured numpy arrays."""
    arr = kps_i32.cpu().numpy()
    cnt = counts.cpu().numpy()
    return [arr[f, :cnt[f]].copy().view(KEYPOINT_DTYPE).reshape(-1) for f in range(arr.shape[0])]


class ORBmatcher:
    """ORBmatcher Hamming searches (include/ORBmatcher.h:37-102)."""

    TH_HIGH, TH_LOW, HISTO_LENGTH = 100, 50, 30

    def __init__(self, nnratio=0.6, checkOri=True):
        self.mfNNratio = float(nnratio)
        self.mbCheckOrientation = bool(checkOri)

    @staticmethod
    def DescriptorDistance(a, b):
        a = np.ascontiguousarray(a, np.uint8)
        b = np.ascontiguousarray(b, np.uint8)
        return lib.orbm_descriptor_distance(_u8(a), _u8(b))

    def search_for_initialization_batch(self, kps, desc, counts, pair_a, pair_b, rows, cols, window=100,
                                        matches12=None, nmatches=None, stream=None):
        """SearchForInitialization over device frame pairs; returns (matches12, nmatches) tensors."""
        import torch
        npairs = pair_a.shape[0]
        cap = kps.shape[1]
        if matches12 is None:
            matches12 = torch.empty((npairs, cap), dtype=torch.int32, device=kps.device)
        if nmatches is None:
            nmatches = torch.empty((npairs,), dtype=torch.int32, device=kps.device)
        rc = lib.orbm_search_init_batch_device(_ptr(kps), _ptr(desc), _ptr(counts), kps.shape[0], cap, _ptr(pair_a),
                                               _ptr(pair_b),
                                               npairs, rows, cols, window, self.mfNNratio,
                                               1 if self.mbCheckOrientation else 0, _ptr(matches12), _ptr(nmatches),
                                               _stream(stream))
        _check("orbm_search_init_batch_device", rc)
        return matches12, nmatches


def allpairs(q, t, mode=TOP2, stream=None):
    """Config-5 brute force: q (nq,32), t (nt,32) uint8 cuda tensors."""
    import torch
    nq, nt = q.shape[0], t.shape[0]
    if mode == TOP2:
        bi = torch.empty(nq, dtype=torch.int32, device=q.device)
        b1 = torch.empty_like(bi)
        b2 = torch.empty_like(bi)
        _check("orbm_allpairs_device", lib.orbm_allpairs_device(_ptr(q), nq, _ptr(t), nt, TOP2, _ptr(bi), _ptr(b1),
                                                                _ptr(b2), None, _stream(stream)))
        return bi, b1, b2
    full = torch.empty((nq, nt), dtype=torch.int16, device=q.device)
    _check("orbm_allpairs_device", lib.orbm_allpairs_device(_ptr(q), nq, _ptr(t), nt, FULL_U16, None, None, None,
                                                            _ptr(full), _stream(stream)))
    return full
