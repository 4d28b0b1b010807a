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
