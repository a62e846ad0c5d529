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
# ORBX_LIB: an instrumented build of the same library for profiling experiments (tools/diag)
LIB_PATH = os.environ.get("ORBX_LIB") or os.path.join(_HERE, "liborbx.so")

KEYPOINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                           ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])

OK, EMPTY, EINVAL, ENOMEM, EDEVICE, ENOSPC = 0, 1, -22, -12, -5, -28
ORBM_MAX_FEATURES = 16384   # include/orbx.h: keypoints per frame of the matcher searches
ORBV_MAX_FEATURES = 65536   # include/orbx.h: descriptors per frame of the vocabulary transform
TOP2, FULL_U16 = 0, 1
RESIZE_SCALAR, RESIZE_SSE2 = 0, 1              # orbx_set_cv_modes (include/orbx.h)
BLUR_SCALAR, BLUR_SSE2, BLUR_BITEXACT = 0, 1, 2

EXPORTED = [
    "orbx_create", "orbx_destroy", "orbx_get_tables", "orbx_capacity", "orbx_set_cv_modes", "orbx_extract", "orbx_get_level",
    "orbx_extract_batch_device", "orbx_extract_stage_device", "orbx_sync", "orbx_set_timing", "orbx_get_stage_times",
    "orbx_debug_pyramid", "orbx_debug_candidates", "orbx_debug_launches", "orbm_descriptor_distance", "orbm_allpairs_device", "orbm_allpairs",
    "orbm_search_init_batch_device", "orbm_search_for_initialization_device", "orbm_search_for_initialization",
    "orbx_compute_stereo_matches", "orbx_stereo_batch_device",
    "orbm_bow_search_device", "orbm_bow_search",
    "orbm_search_by_projection_device", "orbm_search_by_projection",
    "orbm_project_search_device", "orbm_project_search", "orbx_ingest_batch_device", "orbx_depth_batch_device",
    "orbm_best2_csr_device", "orbm_best2_csr", "orbm_stereo_band", "orbm_stereo_band_device",
    "orbv_load_text", "orbv_create", "orbv_destroy", "orbv_info", "orbv_transform", "orbv_transform_batch_device",
]
BOW_KF_F, BOW_KF_KF, TRIANGULATION = 0, 1, 2


class OrbxError(RuntimeError):
    def __init__(self, fn, code):
        super().__init__("%s failed with status %d" % (fn, code))
        self.code = code


class BowView(C.Structure):
    """orbm_bow_view: one side of a vocabulary-node search (host or device pointers)."""
    _fields_ = [("kps", C.c_void_p), ("desc", C.c_void_p), ("has_mp", C.c_void_p), ("u_right", C.c_void_p),
                ("fv_node", C.c_void_p), ("fv_ptr", C.c_void_p), ("fv_idx", C.c_void_p), ("n", C.c_int32),
                ("fv_nnodes", C.c_int32)]


class TriangParams(C.Structure):
    """orbm_triang_params (SearchForTriangulation geometry)."""
    _fields_ = [("F12", C.c_float * 9), ("ex", C.c_float), ("ey", C.c_float), ("scale2", C.c_float * 16),
                ("sigma2_2", C.c_float * 16), ("only_stereo", C.c_int32)]


PROJ_POINT_DTYPE = np.dtype([("proj_x", "<f4"), ("proj_y", "<f4"), ("proj_xr", "<f4"), ("view_cos", "<f4"),
                             ("level", "<i4"), ("flags", "<i4")])


class ProjParams(C.Structure):
    """orbm_proj_params (Frame grid bounds, th, nnratio, mvScaleFactors)."""
    _fields_ = [("min_x", C.c_float), ("min_y", C.c_float), ("grid_w_inv", C.c_float), ("grid_h_inv", C.c_float),
                ("th", C.c_float), ("nnratio", C.c_float), ("scale", C.c_float * 16)]


def proj_params(grid, scale, th=1.0, nnratio=0.8):
    pp = ProjParams()
    pp.min_x, pp.min_y, pp.grid_w_inv, pp.grid_h_inv = (float(g) for g in grid)
    pp.th, pp.nnratio = th, nnratio
    sc = np.zeros(16, np.float32)
    sc[:len(scale)] = scale
    pp.scale[:] = [float(x) for x in sc]
    return pp


PROJ_LAST_FRAME, PROJ_KEYFRAME, PROJ_SIM3, FUSE, FUSE_SIM3 = 0, 1, 2, 3, 4


class Grid(C.Structure):
    """orbm_grid: Frame's image bounds and grid cell inverses (src/Frame.cc:32-33, 127-128)."""
    _fields_ = [("min_x", C.c_float), ("min_y", C.c_float), ("grid_w_inv", C.c_float), ("grid_h_inv", C.c_float)]


def frame_grid(bounds):
    """bounds = (mnMinX, mnMaxX, mnMinY, mnMaxY) -> Grid, with the inverses computed in float like
    Frame's constructor: 64.f / (mnMaxX - mnMinX), 48.f / (mnMaxY - mnMinY)."""
    b = [np.float32(v) for v in bounds]
    g = Grid()
    g.min_x, g.min_y = float(b[0]), float(b[2])
    g.grid_w_inv = float(np.float32(64) / np.float32(b[1] - b[0]))
    g.grid_h_inv = float(np.float32(48) / np.float32(b[3] - b[2]))
    return g

MAP_POINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("nx", "<f4"), ("ny", "<f4"), ("nz", "<f4"),
                            ("max_dist", "<f4"), ("min_dist", "<f4"), ("angle", "<f4"), ("octave", "<i4"),
                            ("flags", "<i4"), ("pad", "<i4")])


class PoseParams(C.Structure):
    """orbm_pose_params (camera, image bounds, grid, scale pyramid, the search arguments)."""
    _fields_ = [("fx", C.c_float), ("fy", C.c_float), ("cx", C.c_float), ("cy", C.c_float), ("bf", C.c_float),
                ("b", C.c_float), ("min_x", C.c_float), ("max_x", C.c_float), ("min_y", C.c_float),
                ("max_y", C.c_float), ("grid_w_inv", C.c_float), ("grid_h_inv", C.c_float),
                ("log_scale", C.c_float), ("nlevels", C.c_int32), ("th", C.c_float), ("mono", C.c_int32),
                ("orb_dist", C.c_int32), ("check_ori", C.c_int32), ("scale", C.c_float * 16),
                ("inv_sigma2", C.c_float * 16)]


def pose_params(K, bounds, scale, inv_sigma2=None, log_scale=None, bf=0.0, th=1.0, mono=False, orb_dist=100,
                check_ori=True):
    """K = (fx, fy, cx, cy); bounds = (mnMinX, mnMaxX, mnMinY, mnMaxY); scale = mvScaleFactors.
    The grid cell sizes follow Frame's constructor (64 x 48 cells over the bounds);
    log_scale defaults to (float)log(scale[1]) like Frame::mfLogScaleFactor."""
    pp = PoseParams()
    pp.fx, pp.fy, pp.cx, pp.cy = (float(v) for v in K)
    pp.bf = float(bf)
    pp.b = float(np.float32(bf) / np.float32(K[0])) if K[0] else 0.0
    pp.min_x, pp.max_x, pp.min_y, pp.max_y = (float(v) for v in bounds)
    pp.grid_w_inv = float(np.float32(64) / np.float32(np.float32(bounds[1]) - np.float32(bounds[0])))
    pp.grid_h_inv = float(np.float32(48) / np.float32(np.float32(bounds[3]) - np.float32(bounds[2])))
    sc = np.zeros(16, np.float32)
    sc[:len(scale)] = scale
    pp.scale[:] = [float(x) for x in sc]
    pp.nlevels = len(scale)
    if inv_sigma2 is None:
        inv_sigma2 = np.float32(1) / (np.asarray(scale, np.float32) * np.asarray(scale, np.float32))
    s2 = np.zeros(16, np.float32)
    s2[:len(inv_sigma2)] = inv_sigma2
    pp.inv_sigma2[:] = [float(x) for x in s2]
    pp.log_scale = float(np.float32(np.log(np.float64(np.float32(scale[1]))))) if log_scale is None else log_scale
    pp.th, pp.mono, pp.orb_dist, pp.check_ori = float(th), int(bool(mono)), int(orb_dist), int(bool(check_ori))
    return pp


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
    L.orbx_set_cv_modes.argtypes = [vp, C.c_int, C.c_int]
    L.orbx_extract.argtypes = [vp, u8p, C.c_int, C.c_int, C.c_size_t, vp, C.c_int, u8p, i32p]
    L.orbx_get_level.argtypes = [vp, C.c_int, P(u8p), i32p, i32p, P(C.c_size_t)]
    L.orbx_extract_batch_device.argtypes = [vp, vp, C.c_int, C.c_int, C.c_int, C.c_size_t, C.c_size_t, vp, vp,
                                            vp, C.c_int, vp]
    L.orbx_extract_stage_device.argtypes = [vp, C.c_int, vp, C.c_int, C.c_int, C.c_int, C.c_size_t, C.c_size_t, vp,
                                            vp, vp, C.c_int, vp]
    L.orbx_sync.argtypes = [vp, vp]
    L.orbx_set_timing.argtypes = [vp, C.c_int]
    L.orbx_get_stage_times.argtypes = [vp, f32p, C.c_int]
    L.orbx_debug_pyramid.argtypes = [vp, C.c_int, u8p, C.c_size_t]
    L.orbx_debug_candidates.argtypes = [vp, C.c_int, C.c_int, i32p, C.c_int, i32p]
    L.orbx_debug_launches.argtypes = [vp, C.c_int, C.c_int, C.c_int, i32p, C.c_int]
    L.orbm_descriptor_distance.argtypes = [u8p, u8p]
    L.orbm_allpairs_device.argtypes = [vp, C.c_int, vp, C.c_int, C.c_int, vp, vp, vp, vp, vp]
    L.orbm_allpairs.argtypes = [C.c_int, u8p, C.c_int, u8p, C.c_int, C.c_int, vp, vp, vp, vp]
    L.orbm_search_init_batch_device.argtypes = [vp, vp, vp, C.c_int, C.c_int, vp, vp, C.c_int, C.c_int, C.c_int,
                                                C.c_int, C.c_float, C.c_int, vp, vp, vp]
    L.orbm_search_for_initialization_device.argtypes = [vp, vp, vp, C.c_int, C.c_int, vp, vp, C.c_int, vp,
                                                        C.c_int, C.c_float, C.c_int, vp, vp, vp, vp]
    L.orbm_search_for_initialization.argtypes = [C.c_int, vp, u8p, C.c_int, vp, u8p, C.c_int, vp, f32p, C.c_int,
                                                 C.c_float, C.c_int, i32p, i32p]
    L.orbx_compute_stereo_matches.argtypes = [vp, vp, vp, u8p, C.c_int, vp, u8p, C.c_int, C.c_float, C.c_float,
                                              f32p, f32p, i32p]
    L.orbx_stereo_batch_device.argtypes = [vp, vp, vp, vp, C.c_int, vp, vp, C.c_int, C.c_float, C.c_float, vp, vp,
                                           vp, vp]
    f64p = P(C.c_double)
    L.orbv_load_text.argtypes = [C.c_char_p, C.c_int, P(vp)]
    L.orbv_create.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, i32p, u8p, u8p, f64p, C.c_int, P(vp)]
    L.orbv_destroy.argtypes = [vp]
    L.orbv_destroy.restype = None
    L.orbv_info.argtypes = [vp, i32p, i32p, i32p, i32p, i32p, i32p]
    L.orbv_transform.argtypes = [vp, u8p, C.c_int, C.c_int, i32p, f64p, i32p, i32p, i32p, i32p, i32p]
    L.orbv_transform_batch_device.argtypes = [vp, vp, vp, C.c_int, C.c_int, C.c_int, vp, vp, vp, vp, vp, vp, vp, vp]
    L.orbm_search_by_projection_device.argtypes = [vp, vp, vp, vp, vp, C.c_int, C.c_int, vp, vp, vp, C.c_int,
                                                   P(ProjParams), vp, vp, vp]
    L.orbm_search_by_projection.argtypes = [C.c_int, vp, u8p, f32p, u8p, C.c_int, vp, u8p, C.c_int, P(ProjParams),
                                            i32p, i32p]
    L.orbm_project_search_device.argtypes = [C.c_int, vp, vp, vp, vp, vp, C.c_int, C.c_int, vp, vp, vp, vp, C.c_int,
                                             P(PoseParams), vp, vp, vp]
    L.orbm_project_search.argtypes = [C.c_int, C.c_int, vp, u8p, f32p, u8p, C.c_int, f32p, vp, u8p, C.c_int,
                                      P(PoseParams), i32p, i32p]
    L.orbx_ingest_batch_device.argtypes = [vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_size_t, C.c_size_t,
                                           vp, vp, C.c_int, C.c_int, C.c_int, vp, C.c_size_t, C.c_size_t, vp]
    L.orbx_depth_batch_device.argtypes = [vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_size_t, C.c_size_t, C.c_float,
                                          vp, C.c_size_t, C.c_size_t, vp]
    L.orbm_best2_csr_device.argtypes = [vp, C.c_int, vp, C.c_int, vp, vp, C.c_int, vp, vp, vp, vp]
    L.orbm_best2_csr.argtypes = [C.c_int, u8p, C.c_int, u8p, C.c_int, i32p, i32p, C.c_int, i32p, i32p, i32p]
    L.orbm_stereo_band.argtypes = [C.c_int, vp, u8p, C.c_int, vp, u8p, C.c_int, C.c_int, f32p, C.c_int, C.c_float,
                                   C.c_float, i32p, i32p]
    L.orbm_stereo_band_device.argtypes = [vp, vp, vp, C.c_int, vp, vp, C.c_int, C.c_int, f32p, C.c_int, C.c_float,
                                          C.c_float, vp, vp, vp]
    L.orbm_bow_search_device.argtypes = [C.c_int, vp, vp, vp, C.c_int, C.c_int, C.c_float, C.c_int, vp, C.c_int,
                                         vp, vp]
    L.orbm_bow_search.argtypes = [C.c_int, C.c_int, P(BowView), P(BowView), P(TriangParams), C.c_float, C.c_int,
                                  i32p, i32p]
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
        self._modes = (RESIZE_SCALAR, BLUR_SCALAR)

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

    def set_cv_modes(self, resize=None, blur=None):
        """The OpenCV build the extractor reproduces (include/orbx.h orbx_set_cv_modes):
        resize RESIZE_SCALAR / RESIZE_SSE2, blur BLUR_SCALAR / BLUR_SSE2 / BLUR_BITEXACT (None: keep)."""
        self._modes = (self._modes[0] if resize is None else int(resize), self._modes[1] if blur is None else int(blur))
        _check("orbx_set_cv_modes", lib.orbx_set_cv_modes(self._h, self._modes[0], self._modes[1]))

    def capacity(self, rows, cols):
        c = lib.orbx_capacity(self._h, rows, cols)
        if c < 0:
            raise OrbxError("orbx_capacity", c)
        return c

    def __call__(self, image, mask=None):
        """operator()(image, mask, keypoints, descriptors); mask ignored like the reference."""
        img = np.asarray(image)
        # a cv::Mat ROI keeps its parent's step: rows with unit-stride pixels pass through as they are
        if img.dtype != np.uint8 or img.ndim != 2 or img.strides[1] != 1 or img.strides[0] < img.shape[1]:
            img = np.ascontiguousarray(img, dtype=np.uint8)
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

    def extract_stage_device(self, stage, imgs, kps, desc, counts, stream=None):
        """One stage (0 pyramid, 1 FAST, 2 quadtree, 3 describe) of extract_batch_device, on `stream`; the caller
        orders a batch's stages across streams (orbx_extract_stage_device)."""
        B, H, W = imgs.shape
        cap = kps.shape[1]
        rc = lib.orbx_extract_stage_device(self._h, int(stage), _ptr(imgs), B, H, W, imgs.stride(1), imgs.stride(0),
                                           _ptr(kps), _ptr(desc), _ptr(counts), cap, _stream(stream))
        _check("orbx_extract_stage_device", rc)

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

    def debug_launches(self, rows, cols, batch):
        """Kernel launches per stage of one batched extract: {pyramid, fast, quadtree, describe}, and
        pyramid_sources, the bit mask of the levels the pyramid launches resize from."""
        c = np.zeros(5, np.int32)
        _check("orbx_debug_launches", lib.orbx_debug_launches(self._h, rows, cols, batch,
                                                              c.ctypes.data_as(C.POINTER(C.c_int)), 5))
        return dict(zip(("pyramid", "fast", "quadtree", "describe", "pyramid_sources"), (int(v) for v in c)))


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


def ingest_batch_device(src, rgb=False, map_x=None, map_y=None, out=None, stream=None):
    """Tracking::GrabImage* colour conversion after the examples' cv::remap rectification, on a device
    batch.  src: uint8 tensor (B, H, W) or (B, H, W, C); map_x / map_y: float32 (nmaps, H', W') or None.
    Returns the gray (B, H', W') uint8 tensor (the layout orbx_extract_batch_device reads)."""
    import torch
    B, rows, cols = src.shape[:3]
    ch = 1 if src.dim() == 3 else src.shape[3]
    if map_x is not None:
        nmaps, drows, dcols = map_x.shape
    else:
        nmaps, drows, dcols = 1, rows, cols
    if out is None:
        out = torch.empty((B, drows, dcols), dtype=torch.uint8, device=src.device)
    _check("orbx_ingest_batch_device",
           lib.orbx_ingest_batch_device(_ptr(src), B, rows, cols, ch, int(bool(rgb)), src.stride(1), src.stride(0),
                                        _ptr(map_x) if map_x is not None else None,
                                        _ptr(map_y) if map_y is not None else None, nmaps, drows, dcols, _ptr(out),
                                        out.stride(1), out.stride(0), _stream(stream)))
    return out


def depth_batch_device(src, factor, out=None, stream=None):
    """GrabImageRGBD's imDepth.convertTo(CV_32F, mDepthMapFactor), applied under the reference's own
    condition (factor != 1 or a non-float depth map); src: (B, H, W) uint16-as-int16 or float32 tensor."""
    import torch
    B, rows, cols = src.shape
    isf = src.dtype == torch.float32
    if isf and abs(factor - 1.0) <= 1e-5:
        return src
    if out is None:
        out = torch.empty((B, rows, cols), dtype=torch.float32, device=src.device)
    esz = src.element_size()
    _check("orbx_depth_batch_device",
           lib.orbx_depth_batch_device(_ptr(src), 1 if isf else 0, B, rows, cols, src.stride(1) * esz,
                                       src.stride(0) * esz, factor, _ptr(out), out.stride(1) * 4, out.stride(0) * 4,
                                       _stream(stream)))
    return out


TIE_FIRST, TIE_LAST = 0, 1


def best2_csr(q, t, cand_ptr, cand_idx, tie_mode=TIE_FIRST, device=0):
    """orbm_best2_csr on host arrays: per query (best target index, best distance, second distance)
    over its candidate list, in the list's order."""
    q = np.ascontiguousarray(q, np.uint8)
    nt = len(t)
    t = np.ascontiguousarray(t if nt else np.zeros((1, 32), np.uint8), np.uint8)
    ptr = np.ascontiguousarray(cand_ptr, np.int32)
    idx = np.ascontiguousarray(cand_idx if len(cand_idx) else np.zeros(1, np.int32), np.int32)
    nq = len(q)
    out = [np.zeros(max(nq, 1), np.int32) for _ in range(3)]
    i32 = lambda a: a.ctypes.data_as(C.POINTER(C.c_int))
    _check("orbm_best2_csr", lib.orbm_best2_csr(device, _u8(q), nq, _u8(t), nt, i32(ptr), i32(idx), tie_mode,
                                                i32(out[0]), i32(out[1]), i32(out[2])))
    return tuple(o[:nq].copy() for o in out)


def stereo_band(kps_l, desc_l, kps_r, desc_r, rows, scale, min_d, max_d, device=0):
    """orbm_stereo_band on host arrays, the coarse stage of ComputeStereoMatches (src/Frame.cc:645-757):
    per left keypoint (best right index or -1, best distance or 100)."""
    kl = np.ascontiguousarray(kps_l, KEYPOINT_DTYPE)
    kr = np.ascontiguousarray(kps_r, KEYPOINT_DTYPE)
    nl, nr = len(kl), len(kr)
    dl = np.ascontiguousarray(desc_l if nl else np.zeros((1, 32), np.uint8), np.uint8)
    dr = np.ascontiguousarray(desc_r if nr else np.zeros((1, 32), np.uint8), np.uint8)
    sc = np.ascontiguousarray(scale, np.float32)
    bi, bd = np.zeros(max(nl, 1), np.int32), np.zeros(max(nl, 1), np.int32)
    i32 = lambda a: a.ctypes.data_as(C.POINTER(C.c_int))
    _check("orbm_stereo_band",
           lib.orbm_stereo_band(device, kl.ctypes.data, _u8(dl), nl, kr.ctypes.data, _u8(dr), nr, rows,
                                sc.ctypes.data_as(C.POINTER(C.c_float)), len(sc), min_d, max_d, i32(bi), i32(bd)))
    return bi[:nl].copy(), bd[:nl].copy()


def stereo_band_batch_device(kps, desc, counts, left, right, rows, scale, min_d, max_d, stream=None):
    """orbm_stereo_band_device over pairs (left[p], right[p]) of a device batch (kps int32 (F, cap, 7),
    desc uint8 (F, cap, 32), counts int32 (F,)).  Returns (best_idx, best_dist), int32 (npairs, cap)."""
    import torch
    cap = kps.shape[1]
    left = torch.as_tensor(left, dtype=torch.int32, device=kps.device).contiguous()
    right = torch.as_tensor(right, dtype=torch.int32, device=kps.device).contiguous()
    npairs = left.numel()
    bi = torch.empty((npairs, cap), dtype=torch.int32, device=kps.device)
    bd = torch.empty((npairs, cap), dtype=torch.int32, device=kps.device)
    sc = np.ascontiguousarray(scale, np.float32)
    _check("orbm_stereo_band_device",
           lib.orbm_stereo_band_device(_ptr(kps), _ptr(desc), _ptr(counts), cap, _ptr(left), _ptr(right), npairs, rows,
                                       sc.ctypes.data_as(C.POINTER(C.c_float)), len(sc), min_d, max_d, _ptr(bi),
                                       _ptr(bd), _stream(stream)))
    return bi, bd


def keypoints_from_device(kps_i32, counts):
    """(B, cap, 7) int32 torch tensor + counts -> list of structured numpy arrays."""
    arr = kps_i32.cpu().numpy()
    cnt = counts.cpu().numpy()
    return [arr[f, :cnt[f]].copy().view(KEYPOINT_DTYPE).reshape(-1) for f in range(arr.shape[0])]


class ORBmatcher:
    """ORBmatcher Hamming searches (include/ORBmatcher.h:37-102).

    SearchByBoW(KF, F) / SearchByBoW(KF1, KF2) / SearchForTriangulation take the
    per-side arrays the reference reads from its KeyFrame/Frame objects:
    (keypoints, descriptors, FeatureVector CSR (node, ptr, idx), MapPoint flags
    and, for triangulation, mvuRight)."""

    TH_HIGH, TH_LOW, HISTO_LENGTH = 100, 50, 30

    def __init__(self, nnratio=0.6, checkOri=True):
        self.mfNNratio = float(nnratio)
        self.mbCheckOrientation = bool(checkOri)

    @staticmethod
    def DescriptorDistance(a, b):
        a = np.ascontiguousarray(a, np.uint8)
        b = np.ascontiguousarray(b, np.uint8)
        return lib.orbm_descriptor_distance(_u8(a), _u8(b))

    def SearchByBoW_KF_F(self, kf, f, device=0):
        """kf = (kps, desc, fv, has_mp), f = (kps, desc, fv).  Returns (nmatches, match_f)."""
        v1 = _host_view(kf[0], kf[1], kf[2], has_mp=kf[3])
        v2 = _host_view(f[0], f[1], f[2])
        return bow_search(BOW_KF_F, v1, v2, None, self.mfNNratio, self.mbCheckOrientation, device)

    def SearchByBoW_KF_KF(self, kf1, kf2, device=0):
        """kf = (kps, desc, fv, has_mp).  Returns (nmatches, match12)."""
        v1 = _host_view(kf1[0], kf1[1], kf1[2], has_mp=kf1[3])
        v2 = _host_view(kf2[0], kf2[1], kf2[2], has_mp=kf2[3])
        return bow_search(BOW_KF_KF, v1, v2, None, self.mfNNratio, self.mbCheckOrientation, device)

    def SearchForTriangulation(self, kf1, kf2, F12, ex, ey, scale2, sigma2_2, bOnlyStereo=False, device=0):
        """kf = (kps, desc, fv, has_mp, u_right).  Returns (nmatches, match12)."""
        v1 = _host_view(kf1[0], kf1[1], kf1[2], has_mp=kf1[3], u_right=kf1[4])
        v2 = _host_view(kf2[0], kf2[1], kf2[2], has_mp=kf2[3], u_right=kf2[4])
        tp = triang_params(F12, ex, ey, scale2, sigma2_2, bOnlyStereo)
        return bow_search(TRIANGULATION, v1, v2, tp, self.mfNNratio, self.mbCheckOrientation, device)

    def SearchByProjection(self, kps, desc, uright, claimed, grid, scale, pts, pdesc, th=1.0, device=0):
        """SearchByProjection(Frame& F, vector<MapPoint*>, th) (src/ORBmatcher.cc:45-129).
        kps = F.mvKeysUn, uright = F.mvuRight, claimed[i] = F.mvpMapPoints[i] && Observations() > 0,
        grid = (mnMinX, mnMinY, mfGridElementWidthInv, mfGridElementHeightInv), scale = mvScaleFactors,
        pts: PROJ_POINT_DTYPE per MapPoint, pdesc its descriptors.  Returns (nmatches, match[n])."""
        k = np.ascontiguousarray(kps, KEYPOINT_DTYPE)
        d = np.ascontiguousarray(desc, np.uint8)
        ur = np.ascontiguousarray(uright, np.float32)
        cl = np.ascontiguousarray(claimed, np.uint8)
        pp = np.ascontiguousarray(pts, PROJ_POINT_DTYPE)
        pd = np.ascontiguousarray(pdesc, np.uint8)
        n = len(k)
        out = np.full(max(n, 1), -1, np.int32)
        nm = C.c_int(0)
        prm = proj_params(grid, scale, th, self.mfNNratio)
        _check("orbm_search_by_projection",
               lib.orbm_search_by_projection(device, k.ctypes.data, _u8(d), ur.ctypes.data_as(C.POINTER(C.c_float)),
                                             _u8(cl), n, pp.ctypes.data, _u8(pd), len(pp), C.byref(prm),
                                             out.ctypes.data_as(C.POINTER(C.c_int)), C.byref(nm)))
        return nm.value, out[:n].copy()

    def project_search(self, mode, kps, desc, uright, claimed, pose, pts, pdesc, params, device=0):
        """The pose-projection searches (include/orbx.h ORBM_PROJ_* / ORBM_FUSE*) on host arrays.
        pose: Tcw (Scw for the Sim3 modes) 3x4 [+ LastFrame Tcw 3x4]; pts: MAP_POINT_DTYPE;
        params: PoseParams (check_ori is taken from this matcher).  Returns (n, match)."""
        k = np.ascontiguousarray(kps, KEYPOINT_DTYPE)
        d = np.ascontiguousarray(desc, np.uint8)
        ur = np.ascontiguousarray(uright, np.float32)
        cl = np.ascontiguousarray(claimed if claimed is not None else np.zeros(len(k), np.uint8), np.uint8)
        ps = np.zeros(24, np.float32)
        pz = np.asarray(pose, np.float32).ravel()
        ps[:len(pz)] = pz
        pp = np.ascontiguousarray(pts, MAP_POINT_DTYPE)
        pd = np.ascontiguousarray(pdesc, np.uint8)
        nout = len(k) if mode <= PROJ_SIM3 else len(pp)
        out = np.full(max(nout, 1), -1, np.int32)
        nm = C.c_int(0)
        prm = PoseParams.from_buffer_copy(params)
        prm.check_ori = int(self.mbCheckOrientation)
        f32 = lambda a: a.ctypes.data_as(C.POINTER(C.c_float))
        _check("orbm_project_search",
               lib.orbm_project_search(device, mode, k.ctypes.data, _u8(d), f32(ur), _u8(cl), len(k), f32(ps),
                                       pp.ctypes.data, _u8(pd), len(pp), C.byref(prm),
                                       out.ctypes.data_as(C.POINTER(C.c_int)), C.byref(nm)))
        return nm.value, out[:nout].copy()

    def project_search_batch_device(self, mode, kps, desc, uright, claimed, counts, pose, pts, pdesc, npts, params,
                                    match=None, nmatches=None, stream=None):
        """Batched device form of project_search: kps (B, cap, 7) int32, desc (B, cap, 32) uint8, uright
        (B, cap) float32, claimed (B, cap) uint8, counts (B,), pose (B, 24) float32, pts (B, pcap, 12)
        int32 view of MAP_POINT_DTYPE, pdesc (B, pcap, 32), npts (B,).  Returns (match, nmatches)."""
        import torch
        B, cap = kps.shape[0], kps.shape[1]
        pcap = pts.shape[1]
        nout = cap if mode <= PROJ_SIM3 else pcap
        if match is None:
            match = torch.empty((B, nout), dtype=torch.int32, device=kps.device)
        if nmatches is None:
            nmatches = torch.empty((B,), dtype=torch.int32, device=kps.device)
        prm = PoseParams.from_buffer_copy(params)
        prm.check_ori = int(self.mbCheckOrientation)
        _check("orbm_project_search_device",
               lib.orbm_project_search_device(mode, _ptr(kps), _ptr(desc), _ptr(uright), _ptr(claimed), _ptr(counts),
                                              B, cap, _ptr(pose), _ptr(pts), _ptr(pdesc), _ptr(npts), pcap,
                                              C.byref(prm), _ptr(match), _ptr(nmatches), _stream(stream)))
        return match, nmatches

    def SearchByProjectionLastFrame(self, cur, last_pts, last_pdesc, Tcw, Tlw, params, th, bMono, device=0):
        """SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, th, bMono) (src/ORBmatcher.cc:1396-1538).
        cur = (mvKeysUn, mDescriptors, mvuRight, taken) with taken[i] = mvpMapPoints[i] && Observations() > 0."""
        prm = PoseParams.from_buffer_copy(params)
        prm.th, prm.mono = float(th), int(bool(bMono))
        pose = np.concatenate([np.asarray(Tcw, np.float32).reshape(-1)[:12], np.asarray(Tlw, np.float32).reshape(-1)[:12]])
        return self.project_search(PROJ_LAST_FRAME, cur[0], cur[1], cur[2], cur[3], pose, last_pts, last_pdesc, prm,
                                   device)

    def SearchByProjectionKeyFrame(self, cur, kf_pts, kf_pdesc, Tcw, params, th, ORBdist, device=0):
        """SearchByProjection(Frame& CurrentFrame, KeyFrame*, sAlreadyFound, th, ORBdist) (:1540-1667).
        taken[i] = CurrentFrame.mvpMapPoints[i] != NULL."""
        prm = PoseParams.from_buffer_copy(params)
        prm.th, prm.orb_dist = float(th), int(ORBdist)
        return self.project_search(PROJ_KEYFRAME, cur[0], cur[1], cur[2], cur[3], Tcw, kf_pts, kf_pdesc, prm, device)

    def SearchByProjectionSim3(self, kf, pts, pdesc, Scw, params, th, device=0):
        """SearchByProjection(KeyFrame*, Scw, vpPoints, vpMatched, th) (:290-403); taken[i] = vpMatched[i]."""
        prm = PoseParams.from_buffer_copy(params)
        prm.th = float(int(th))
        return self.project_search(PROJ_SIM3, kf[0], kf[1], kf[2], kf[3], Scw, pts, pdesc, prm, device)

    def Fuse(self, kf, pts, pdesc, Tcw, params, th=3.0, device=0):
        """Fuse(KeyFrame*, vpMapPoints, th) (:893-1043): per MapPoint the KeyFrame feature it fuses into."""
        prm = PoseParams.from_buffer_copy(params)
        prm.th = float(th)
        return self.project_search(FUSE, kf[0], kf[1], kf[2], None, Tcw, pts, pdesc, prm, device)

    def FuseSim3(self, kf, pts, pdesc, Scw, params, th, device=0):
        """Fuse(KeyFrame*, Scw, vpPoints, th, vpReplacePoint) (:1045-1168)."""
        prm = PoseParams.from_buffer_copy(params)
        prm.th = float(th)
        return self.project_search(FUSE_SIM3, kf[0], kf[1], kf[2], None, Scw, pts, pdesc, prm, device)

    def search_for_initialization_batch(self, kps, desc, counts, pair_a, pair_b, rows, cols, window=100,
                                        matches12=None, nmatches=None, stream=None, bounds=None, prev_matched=None):
        """SearchForInitialization over device frame pairs; returns (matches12, nmatches) tensors.
        bounds = (mnMinX, mnMaxX, mnMinY, mnMaxY) (default 0..cols x 0..rows); prev_matched: float32
        (npairs, cap, 2) cuda tensor holding each pair's vbPrevMatched, updated in place (default: F1's
        keypoints, not written)."""
        import torch
        npairs = pair_a.shape[0]
        cap = kps.shape[1]
        if matches12 is None:
            matches12 = torch.empty((npairs, cap), dtype=torch.int32, device=kps.device)
        if nmatches is None:
            nmatches = torch.empty((npairs,), dtype=torch.int32, device=kps.device)
        ori = 1 if self.mbCheckOrientation else 0
        if bounds is None and prev_matched is None:
            rc = lib.orbm_search_init_batch_device(_ptr(kps), _ptr(desc), _ptr(counts), kps.shape[0], cap,
                                                   _ptr(pair_a), _ptr(pair_b), npairs, rows, cols, window,
                                                   self.mfNNratio, ori, _ptr(matches12), _ptr(nmatches),
                                                   _stream(stream))
            _check("orbm_search_init_batch_device", rc)
            return matches12, nmatches
        g = frame_grid(bounds if bounds is not None else (0.0, cols, 0.0, rows))
        if prev_matched is not None:
            assert prev_matched.dtype == torch.float32 and tuple(prev_matched.shape) == (npairs, cap, 2)
            assert prev_matched.is_contiguous()
        rc = lib.orbm_search_for_initialization_device(_ptr(kps), _ptr(desc), _ptr(counts), kps.shape[0], cap,
                                                       _ptr(pair_a), _ptr(pair_b), npairs, C.byref(g), window,
                                                       self.mfNNratio, ori, _ptr(prev_matched), _ptr(matches12),
                                                       _ptr(nmatches), _stream(stream))
        _check("orbm_search_for_initialization_device", rc)
        return matches12, nmatches

    def SearchForInitialization(self, F1, F2, vbPrevMatched, windowSize=100, bounds=None, device=0):
        """ORBmatcher::SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12, windowSize)
        (src/ORBmatcher.cc:417-588) on host arrays: F = (mvKeysUn, mDescriptors[, (cols, rows)]);
        bounds = (mnMinX, mnMaxX, mnMinY, mnMaxY) (default 0..cols x 0..rows from F2).  vbPrevMatched is
        a float32 (n1, 2) numpy array, updated in place like the reference's.  Returns (nmatches, vnMatches12)."""
        k1 = np.ascontiguousarray(F1[0], KEYPOINT_DTYPE)
        k2 = np.ascontiguousarray(F2[0], KEYPOINT_DTYPE)
        n1, n2 = len(k1), len(k2)
        d1 = np.ascontiguousarray(F1[1] if n1 else np.zeros((1, 32), np.uint8), np.uint8)
        d2 = np.ascontiguousarray(F2[1] if n2 else np.zeros((1, 32), np.uint8), np.uint8)
        if bounds is None:
            cols, rows = F2[2]
            bounds = (0.0, cols, 0.0, rows)
        assert isinstance(vbPrevMatched, np.ndarray) and vbPrevMatched.dtype == np.float32
        assert vbPrevMatched.shape == (n1, 2) and vbPrevMatched.flags.c_contiguous
        g = frame_grid(bounds)
        m12 = np.full(max(n1, 1), -1, np.int32)
        nm = C.c_int(0)
        pv = vbPrevMatched if n1 else np.zeros((1, 2), np.float32)
        _check("orbm_search_for_initialization",
               lib.orbm_search_for_initialization(device, k1.ctypes.data, _u8(d1), n1, k2.ctypes.data, _u8(d2), n2,
                                                  C.byref(g), pv.ctypes.data_as(C.POINTER(C.c_float)), windowSize,
                                                  self.mfNNratio, 1 if self.mbCheckOrientation else 0,
                                                  m12.ctypes.data_as(C.POINTER(C.c_int)), C.byref(nm)))
        return nm.value, m12[:n1].copy()


def _host_view(kps, desc, fv, has_mp=None, u_right=None):
    keep = [np.ascontiguousarray(kps, KEYPOINT_DTYPE), np.ascontiguousarray(desc, np.uint8)]
    node, ptr, idx = (np.ascontiguousarray(a, np.int32) for a in fv)
    keep += [node, ptr, idx]
    mp = ur = None
    if has_mp is not None:
        mp = np.ascontiguousarray(has_mp, np.uint8)
        keep.append(mp)
    if u_right is not None:
        ur = np.ascontiguousarray(u_right, np.float32)
        keep.append(ur)
    v = BowView(keep[0].ctypes.data, keep[1].ctypes.data, mp.ctypes.data if mp is not None else None,
                ur.ctypes.data if ur is not None else None, node.ctypes.data, ptr.ctypes.data, idx.ctypes.data,
                len(keep[0]), len(node))
    v._keep = keep
    return v


def triang_params(F12, ex, ey, scale2, sigma2_2, only_stereo=False):
    tp = TriangParams()
    tp.F12[:] = [float(x) for x in np.asarray(F12, np.float32).reshape(9)]
    tp.ex, tp.ey = ex, ey
    s2 = np.zeros(16, np.float32)
    g2 = np.zeros(16, np.float32)
    s2[:len(scale2)] = scale2
    g2[:len(sigma2_2)] = sigma2_2
    tp.scale2[:] = [float(x) for x in s2]
    tp.sigma2_2[:] = [float(x) for x in g2]
    tp.only_stereo = 1 if only_stereo else 0
    return tp


def bow_search(mode, view1, view2, tp=None, nnratio=0.6, check_ori=True, device=0):
    """Host path of the vocabulary-node searches; view1/view2 from _host_view.  Returns (nmatches, match)."""
    nout = view2.n if mode == BOW_KF_F else view1.n
    out = np.full(max(nout, 1), -1, np.int32)
    nm = C.c_int(0)
    _check("orbm_bow_search", lib.orbm_bow_search(device, mode, C.byref(view1), C.byref(view2),
                                                  C.byref(tp) if tp is not None else None, nnratio,
                                                  1 if check_ori else 0, out.ctypes.data_as(C.POINTER(C.c_int)),
                                                  C.byref(nm)))
    return nm.value, out[:nout].copy()


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


class ORBVocabulary:
    """DBoW2 TemplatedVocabulary<FORB> on the device (Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h):
    loadFromTextFile, transform(features, BowVector, FeatureVector, levelsup)."""

    def __init__(self, handle):
        self._h = handle
        k, L, sc, wt, nn, nw = (C.c_int() for _ in range(6))
        _check("orbv_info", lib.orbv_info(self._h, C.byref(k), C.byref(L), C.byref(sc), C.byref(wt), C.byref(nn),
                                          C.byref(nw)))
        self.k, self.L, self.scoring, self.weighting = k.value, L.value, sc.value, wt.value
        self.nnodes, self.nwords = nn.value, nw.value

    @staticmethod
    def loadFromTextFile(path, device=0):
        h = C.c_void_p()
        _check("orbv_load_text", lib.orbv_load_text(str(path).encode(), device, C.byref(h)))
        return ORBVocabulary(h)

    @staticmethod
    def from_arrays(k, L, parent, is_leaf, desc, weight, scoring=0, weighting=0, device=0):
        par = np.ascontiguousarray(parent, np.int32)
        leaf = np.ascontiguousarray(is_leaf, np.uint8)
        d = np.ascontiguousarray(desc, np.uint8)
        w = np.ascontiguousarray(weight, np.float64)
        h = C.c_void_p()
        _check("orbv_create", lib.orbv_create(k, L, scoring, weighting, len(par),
                                              par.ctypes.data_as(C.POINTER(C.c_int)), _u8(leaf), _u8(d),
                                              w.ctypes.data_as(C.POINTER(C.c_double)), device, C.byref(h)))
        return ORBVocabulary(h)

    def close(self):
        if getattr(self, "_h", None):
            lib.orbv_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def transform(self, desc, levelsup=4):
        """Returns (bow_word, bow_weight, (fv_node, fv_ptr, fv_idx))."""
        d = np.ascontiguousarray(desc if desc is not None else np.zeros((0, 32), np.uint8), np.uint8)
        n = len(d)
        bw = np.zeros(n + 1, np.int32)
        bv = np.zeros(n + 1, np.float64)
        fn = np.zeros(n + 1, np.int32)
        fp = np.zeros(n + 2, np.int32)
        fi = np.zeros(n + 1, np.int32)
        nb, nn = C.c_int(0), C.c_int(0)
        i32 = lambda a: a.ctypes.data_as(C.POINTER(C.c_int))
        _check("orbv_transform", lib.orbv_transform(self._h, _u8(d), n, levelsup, i32(bw),
                                                    bv.ctypes.data_as(C.POINTER(C.c_double)), C.byref(nb), i32(fn),
                                                    i32(fp), i32(fi), C.byref(nn)))
        k, m = nb.value, nn.value
        return bw[:k].copy(), bv[:k].copy(), (fn[:m].copy(), fp[:m + 1].copy(), fi[:fp[m]].copy())

    def transform_batch_device(self, desc, counts, levelsup=4, stream=None):
        """desc: (B, cap, 32) uint8 cuda tensor, counts (B,) int32.  Returns device tensors
        (bow_word, bow_weight, bow_n, fv_node, fv_ptr, fv_idx, fv_nnodes)."""
        import torch
        B, cap = desc.shape[0], desc.shape[1]
        dev = desc.device
        bw = torch.empty((B, cap), dtype=torch.int32, device=dev)
        bv = torch.empty((B, cap), dtype=torch.float64, device=dev)
        bn = torch.empty((B,), dtype=torch.int32, device=dev)
        fn = torch.empty((B, cap), dtype=torch.int32, device=dev)
        fp = torch.empty((B, cap + 1), dtype=torch.int32, device=dev)
        fi = torch.empty((B, cap), dtype=torch.int32, device=dev)
        fnn = torch.empty((B,), dtype=torch.int32, device=dev)
        _check("orbv_transform_batch_device",
               lib.orbv_transform_batch_device(self._h, _ptr(desc), _ptr(counts), B, cap, levelsup, _ptr(bw),
                                               _ptr(bv), _ptr(bn), _ptr(fn), _ptr(fp), _ptr(fi), _ptr(fnn),
                                               _stream(stream)))
        return bw, bv, bn, fn, fp, fi, fnn


class BowBatch:
    """Device-resident batch of vocabulary-node searches (orbm_bow_search_device).

    sides1 / sides2: lists (one entry per pair) of dicts with keys kps, desc, fv=(node, ptr,
    idx) and optionally has_mp, u_right -- host numpy arrays, uploaded once; or `kps`/`desc`
    may already be cuda tensors (e.g. a slice of an extract batch), used in place.
    tps: list of TriangParams for TRIANGULATION."""

    def __init__(self, mode, sides1, sides2, tps=None, device=0):
        import torch
        self.mode = mode
        self.dev = torch.device("cuda", device)
        self._keep = []
        v1 = [self._view(s) for s in sides1]
        v2 = [self._view(s) for s in sides2]
        self.npairs = len(v1)
        self.max_nodes1 = max([v.fv_nnodes for v in v1] + [0])
        n_out = [(b.n if mode == BOW_KF_F else a.n) for a, b in zip(v1, v2)]
        self.stride = max(n_out + [1])
        self.d_v1 = self._upload_structs(v1, BowView)
        self.d_v2 = self._upload_structs(v2, BowView)
        self.d_tp = self._upload_structs(tps, TriangParams) if tps else None
        self.match = torch.empty((self.npairs, self.stride), dtype=torch.int32, device=self.dev)
        self.nmatches = torch.empty((self.npairs,), dtype=torch.int32, device=self.dev)

    def _t(self, a, dtype):
        import torch
        if isinstance(a, torch.Tensor):
            t = a.contiguous()
        else:
            t = torch.from_numpy(np.ascontiguousarray(a)).to(self.dev)
        self._keep.append(t)
        return t.data_ptr()

    def _view(self, s):
        import torch
        kps = s["kps"]
        n = kps.shape[0] if isinstance(kps, torch.Tensor) else len(kps)
        if not isinstance(kps, torch.Tensor):
            kps = np.ascontiguousarray(kps, KEYPOINT_DTYPE).view(np.int32).reshape(-1, 7)
        node, ptr, idx = (np.ascontiguousarray(a, np.int32) for a in s["fv"])
        return BowView(self._t(kps, None), self._t(s["desc"], None),
                       self._t(np.ascontiguousarray(s["has_mp"], np.uint8), None) if s.get("has_mp") is not None
                       else None,
                       self._t(np.ascontiguousarray(s["u_right"], np.float32), None) if s.get("u_right") is not None
                       else None,
                       self._t(node, None), self._t(ptr, None), self._t(idx if len(idx) else np.zeros(1, np.int32),
                                                                         None),
                       n, len(node))

    def _upload_structs(self, items, cls):
        import torch
        raw = b"".join(bytes(memoryview(x)) for x in items)
        t = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(self.dev)
        self._keep.append(t)
        return t

    def run(self, nnratio=0.6, check_ori=True, stream=None):
        rc = lib.orbm_bow_search_device(self.mode, _ptr(self.d_v1), _ptr(self.d_v2),
                                        _ptr(self.d_tp) if self.d_tp is not None else None, self.npairs,
                                        self.max_nodes1, nnratio, 1 if check_ori else 0, _ptr(self.match),
                                        self.stride, _ptr(self.nmatches), _stream(stream))
        _check("orbm_bow_search_device", rc)
        return self.match, self.nmatches


def allpairs_host(q, t, mode=TOP2, device=0):
    """orbm_allpairs on host arrays: TOP2 -> (best_idx, best, second); FULL_U16 -> (nq, nt) uint16."""
    q = np.ascontiguousarray(q, np.uint8)
    nq, nt = len(q), len(t)
    t = np.ascontiguousarray(t if nt else np.zeros((1, 32), np.uint8), np.uint8)
    if mode == TOP2:
        out = [np.zeros(max(nq, 1), np.int32) for _ in range(3)]
        _check("orbm_allpairs", lib.orbm_allpairs(device, _u8(q), nq, _u8(t), nt, TOP2, out[0].ctypes.data,
                                                  out[1].ctypes.data, out[2].ctypes.data, None))
        return tuple(o[:nq].copy() for o in out)
    full = np.zeros((max(nq, 1), max(nt, 1)), np.uint16)
    _check("orbm_allpairs", lib.orbm_allpairs(device, _u8(q), nq, _u8(t), nt, FULL_U16, None, None, None,
                                              full.ctypes.data))
    return full[:nq, :nt].copy()
