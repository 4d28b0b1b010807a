"""ctypes binding of oracle/liboracle.so (test infrastructure only).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load the
oracle, and only as the checker / the timed CPU baseline (oracle/usv_oracle.h).
"""
import ctypes
import os
from ctypes import POINTER, c_double, c_float, c_int, c_int64, c_void_p

ROOT = os.path.abspath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
ORACLE_PATH = os.path.join(ROOT, "oracle", "liboracle.so")
REF_MATCH_PATH = os.path.join(ROOT, "oracle", "_ref", "libref_match.so")


class oracle_match(ctypes.Structure):
    _fields_ = [("left", ctypes.c_uint), ("right", ctypes.c_uint), ("value", c_double)]


_SIGS = {
    "usv_oracle_sad_naive": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int,
                                     c_void_p, c_int]),
    "usv_oracle_sad_sliding": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int,
                                       c_void_p, c_int, c_int]),
    "usv_oracle_sad_sliding_rows": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int,
                                            c_int, c_void_p, c_int, c_int, c_int, c_int]),
    "usv_oracle_distance_cm": (c_double, [c_int]),
    "usv_oracle_canny_distance_cm": (c_double, [c_int]),
    "usv_oracle_disparity_to_distance_cm": (None, [c_void_p, c_int, c_int, c_int, c_void_p, c_int]),
    "usv_oracle_moving_object_distance": (c_int, [c_int, c_int64, POINTER(c_float), c_int,
                                                  POINTER(c_float), c_int, POINTER(c_float), c_int,
                                                  POINTER(c_float), c_int, POINTER(c_float), c_int,
                                                  POINTER(c_int), c_int, c_int64, c_int64, c_int64,
                                                  POINTER(c_double)]),
    "usv_oracle_coordinate_position": (c_int, [c_int, POINTER(c_double), c_int, POINTER(c_float), c_int,
                                               c_int, POINTER(c_double)]),
    "usv_oracle_resolve_match_list": (c_int, [POINTER(oracle_match), c_int, POINTER(oracle_match)]),
    "usv_oracle_id_matcher": (c_int, [POINTER(oracle_match), c_int, POINTER(oracle_match), c_int,
                                      POINTER(c_int)]),
    "usv_oracle_hu_moments": (None, [c_void_p, c_int, c_void_p]),
    "usv_oracle_match_shapes_i1": (c_double, [c_void_p, c_int, c_void_p, c_int]),
    "usv_oracle_contour_area": (c_double, [c_void_p, c_int]),
    "usv_oracle_generate_matching_list": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int,
                                                  POINTER(oracle_match)]),
    "usv_oracle_convex_hull_cw": (c_int, [c_void_p, c_int, c_void_p]),
    "usv_oracle_min_area_rect": (c_int, [c_void_p, c_int, c_void_p]),
    "usv_oracle_rect_points": (None, [c_void_p, c_void_p]),
    "usv_oracle_match_centroids": (c_int, [c_void_p, c_void_p, c_int, POINTER(oracle_match), c_int, c_void_p]),
    "usv_oracle_invert3": (c_int, [c_void_p, c_void_p]),
    "usv_oracle_rectify_params": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p]),
    "usv_oracle_rectify_map": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p]),
    "usv_oracle_remap_linear": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_int,
                                        c_void_p, c_int]),
    "usv_oracle_bgr2hsv": (None, [c_void_p, c_int, c_int, c_int, c_void_p, c_int]),
    "usv_oracle_equalize_lut": (None, [c_void_p, c_int, c_void_p]),
    "usv_oracle_hsv2bgr": (None, [c_void_p, c_int, c_int, c_int, c_void_p, c_int]),
    "usv_oracle_bgr2gray": (None, [c_void_p, c_int, c_int, c_int, c_void_p, c_int]),
    "usv_oracle_frame_prep": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "usv_oracle_motion_mask": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int]),
    "usv_oracle_colour_mask": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                       c_void_p, c_int]),
}

_lib = None


def load_oracle():
    global _lib
    if _lib is None:
        lib = ctypes.CDLL(ORACLE_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


def oracle_sad(L, R, D, w, metric="sad", variant="sliding", threads=0):
    """numpy (H, W) u8 pair -> (H, W) u8 disparity from the C oracle."""
    import numpy as np
    lib = load_oracle()
    L = np.ascontiguousarray(L)
    R = np.ascontiguousarray(R)
    H, W = L.shape
    out = np.zeros((H, W), dtype=np.uint8)
    m = 0 if metric == "sad" else 1
    if variant == "naive":
        rc = lib.usv_oracle_sad_naive(L.ctypes.data, R.ctypes.data, W, H, W, D, w, m, out.ctypes.data, W)
    else:
        rc = lib.usv_oracle_sad_sliding(L.ctypes.data, R.ctypes.data, W, H, W, D, w, m, out.ctypes.data,
                                        W, threads)
    assert rc == 0, rc
    return out


def _p(a):
    return a.ctypes.data


def _pts(c):
    import numpy as np
    return np.ascontiguousarray(np.asarray(c, dtype=np.int32).reshape(-1)) if len(c) else np.zeros(2, np.int32)


def _flat(contours):
    import numpy as np
    pts = [p for c in contours for p in c]
    off = np.zeros(len(contours) + 1, dtype=np.int32)
    off[1:] = np.cumsum([len(c) for c in contours])
    flat = np.asarray(pts, dtype=np.int32).reshape(-1) if pts else np.zeros(2, dtype=np.int32)
    return np.ascontiguousarray(flat), off


def oracle_hu(c):
    import numpy as np
    out = np.zeros(7)
    pc = _pts(c)  # keep the array alive across the call
    load_oracle().usv_oracle_hu_moments(_p(pc), len(c), _p(out))
    return out


def oracle_match_shapes_i1(a, b):
    pa, pb = _pts(a), _pts(b)
    return load_oracle().usv_oracle_match_shapes_i1(_p(pa), len(a), _p(pb), len(b))


def oracle_contour_area(c):
    pc = _pts(c)
    return load_oracle().usv_oracle_contour_area(_p(pc), len(c))


def oracle_generate_matching_list(A, B):
    pa, oa = _flat(A)
    pb, ob = _flat(B)
    out = (oracle_match * max(len(A) * len(B), 1))()
    n = load_oracle().usv_oracle_generate_matching_list(_p(pa), _p(oa), len(A), _p(pb), _p(ob), len(B), out)
    return [(out[i].left, out[i].right, out[i].value) for i in range(n)]


def oracle_convex_hull(c):
    import numpy as np
    out = np.zeros(2 * max(len(c), 1), np.int32)
    pc = _pts(c)
    n = load_oracle().usv_oracle_convex_hull_cw(_p(pc), len(c), _p(out))
    return [tuple(int(v) for v in out[2 * i:2 * i + 2]) for i in range(n)]


def oracle_min_area_rect(c):
    """-> ((cx, cy), (w, h), angle) float32 values, as host.min_area_rect."""
    import numpy as np
    out = np.zeros(5, np.float32)
    pc = _pts(c)
    load_oracle().usv_oracle_min_area_rect(_p(pc), len(c), _p(out))
    return (out[0], out[1]), (out[2], out[3]), out[4]


def oracle_match_centroids(contours, matches):
    import numpy as np
    p, off = _flat(contours)
    arr = (oracle_match * max(len(matches), 1))()
    for i, (l, r, v) in enumerate(matches):
        arr[i].left, arr[i].right, arr[i].value = l, r, v
    out = np.zeros(2 * max(len(matches), 1), np.float32)
    n = load_oracle().usv_oracle_match_centroids(_p(p), _p(off), len(contours), arr, len(matches), _p(out))
    return [(out[2 * i], out[2 * i + 1]) for i in range(n)]


def oracle_rectify_params(K, dist, R, P):
    """25 doubles: ir[9], fx, fy, u0, v0, k1..s4 (rectify_oracle.c)."""
    import numpy as np
    lib = load_oracle()
    K = np.ascontiguousarray(K, dtype=np.float64)
    P = np.ascontiguousarray(P, dtype=np.float64)
    d = np.ascontiguousarray(dist if dist is not None else np.zeros(0), dtype=np.float64).ravel()
    Rm = None if R is None else np.ascontiguousarray(R, dtype=np.float64)
    out = np.zeros(25, dtype=np.float64)
    rc = lib.usv_oracle_rectify_params(_p(K), _p(d) if d.size else None, int(d.size),
                                       _p(Rm) if Rm is not None else None, _p(P), int(P.shape[1]), _p(out))
    assert rc == 0, rc
    return out


def oracle_rectify_map(params, W, H):
    import numpy as np
    lib = load_oracle()
    params = np.ascontiguousarray(params, dtype=np.float64)
    m1 = np.zeros((H, W, 2), dtype=np.int16)
    m2 = np.zeros((H, W), dtype=np.uint16)
    assert lib.usv_oracle_rectify_map(_p(params), W, H, _p(m1), _p(m2)) == 0
    return m1, m2


def oracle_remap(src, m1, m2):
    import numpy as np
    lib = load_oracle()
    src = np.ascontiguousarray(src)
    sH, sW = src.shape[:2]
    cn = 1 if src.ndim == 2 else src.shape[2]
    H, W = m2.shape
    out = np.zeros((H, W) if cn == 1 else (H, W, cn), dtype=np.uint8)
    rc = lib.usv_oracle_remap_linear(_p(src), sW, sH, sW * cn, cn, _p(np.ascontiguousarray(m1)),
                                     _p(np.ascontiguousarray(m2)), W, H, _p(out), W * cn)
    assert rc == 0, rc
    return out


def oracle_frame_prep(bgr):
    """(H, W, 3) u8 -> (hsv', bgr', gray)."""
    import numpy as np
    lib = load_oracle()
    bgr = np.ascontiguousarray(bgr)
    H, W = bgr.shape[:2]
    hsv = np.zeros((H, W, 3), np.uint8)
    out = np.zeros((H, W, 3), np.uint8)
    gray = np.zeros((H, W), np.uint8)
    assert lib.usv_oracle_frame_prep(_p(bgr), W, H, 3 * W, _p(hsv), _p(out), _p(gray)) == 0
    return hsv, out, gray


def oracle_motion_mask(gray, prev, thresh=40):
    import numpy as np
    lib = load_oracle()
    gray, prev = np.ascontiguousarray(gray), np.ascontiguousarray(prev)
    H, W = gray.shape
    out = np.zeros((H, W), np.uint8)
    assert lib.usv_oracle_motion_mask(_p(gray), _p(prev), W, H, W, thresh, _p(out), W) == 0
    return out


def oracle_colour_mask(hsv, lo1, hi1, lo2, hi2):
    import numpy as np
    lib = load_oracle()
    hsv = np.ascontiguousarray(hsv)
    H, W = hsv.shape[:2]
    b = [np.ascontiguousarray(v, dtype=np.int32) for v in (lo1, hi1, lo2, hi2)]
    out = np.zeros((H, W), np.uint8)
    assert lib.usv_oracle_colour_mask(_p(hsv), W, H, 3 * W, *[_p(v) for v in b], _p(out), W) == 0
    return out
