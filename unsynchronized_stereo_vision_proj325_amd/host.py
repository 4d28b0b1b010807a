"""Host object path: the reference's C++ matcher / distance API through the C ABI.

These call the C++ restatements in libusv.so (csrc/host/*.cpp) -- the same
code a C++ caller reaches through include/Match.hpp, include/Matching.hpp and
include/DistanceCalculator.hpp.  Function names follow the reference:
  ResolveMatchList            P/Main.cpp:432-477
  IDMatcher                   P/Main.cpp:483-499
  GenerateMatchingList        P/Main.cpp:403-426 (OpenCV maths restated; parity unpinned)
  MatchCentroids              P/Main.cpp:1120-1143 (minAreaRect restated; parity unpinned)
  MovingObjectDistanceCalculator  P/DistanceCalculator.cpp:15-88
  CooridinatePositionCalculator   P/DistanceCalculator.cpp:90-141 (reference spelling)
"""
from __future__ import annotations

import ctypes
from ctypes import POINTER, c_double, c_float, c_int

import numpy as np

from . import _lib

LeftCam, RightCam = True, False


def _matches(seq):
    arr = (_lib.usv_match * max(len(seq), 1))()
    for i, (l, r, v) in enumerate(seq):
        arr[i].left_index, arr[i].right_index, arr[i].match_value = int(l), int(r), float(v)
    return arr


def ResolveMatchList(matcher):
    """list[(left, right, value)] -> tentative list (may contain duplicates, as the reference)."""
    lib = _lib.load()
    src = _matches(matcher)
    out = (_lib.usv_match * max(len(matcher), 1))()
    n = c_int(0)
    _lib.check("usv_resolve_match_list", lib.usv_resolve_match_list(src, len(matcher), out, ctypes.byref(n)))
    return [(out[i].left_index, out[i].right_index, out[i].match_value) for i in range(n.value)]


def IDMatcher(cur, old):
    """-> list[(x, y, z)] triples ((old.RightIndex, 0, 0) by the reference's comma operator)."""
    lib = _lib.load()
    a, b = _matches(cur), _matches(old)
    out = (c_int * max(3 * len(cur) * len(old), 3))()
    n = c_int(0)
    _lib.check("usv_id_matcher", lib.usv_id_matcher(a, len(cur), b, len(old), out, ctypes.byref(n)))
    return [(out[3 * i], out[3 * i + 1], out[3 * i + 2]) for i in range(n.value)]


def _flatten(contours):
    pts = [p for c in contours for p in c]
    off = np.zeros(len(contours) + 1, dtype=np.int32)
    off[1:] = np.cumsum([len(c) for c in contours])
    flat = np.asarray(pts, dtype=np.int32).reshape(-1) if pts else np.zeros(2, dtype=np.int32)
    return np.ascontiguousarray(flat), off


def GenerateMatchingList(contours_l, contours_r):
    """Contours as lists of (x, y) int points -> list[(i, j, score)] with score < 0.75."""
    lib = _lib.load()
    pa, oa = _flatten(contours_l)
    pb, ob = _flatten(contours_r)
    cap = max(len(contours_l) * len(contours_r), 1)
    out = (_lib.usv_match * cap)()
    n = c_int(0)
    ip = POINTER(c_int)
    _lib.check("usv_generate_matching_list", lib.usv_generate_matching_list(
        pa.ctypes.data_as(ip), oa.ctypes.data_as(ip), len(contours_l),
        pb.ctypes.data_as(ip), ob.ctypes.data_as(ip), len(contours_r), out, cap, ctypes.byref(n)))
    return [(out[i].left_index, out[i].right_index, out[i].match_value) for i in range(n.value)]


def match_shapes_i1(a, b) -> float:
    lib = _lib.load()
    pa = np.ascontiguousarray(np.asarray(a, dtype=np.int32).reshape(-1))
    pb = np.ascontiguousarray(np.asarray(b, dtype=np.int32).reshape(-1))
    ip = POINTER(c_int)
    return lib.usv_match_shapes_i1(pa.ctypes.data_as(ip), len(a), pb.ctypes.data_as(ip), len(b))


def contour_area(c) -> float:
    lib = _lib.load()
    p = np.ascontiguousarray(np.asarray(c, dtype=np.int32).reshape(-1))
    return lib.usv_contour_area(p.ctypes.data_as(POINTER(c_int)), len(c))


def min_area_rect(c):
    """OpenCV 3.0 minAreaRect of int points -> ((cx, cy), (w, h), angle_deg), float32 values."""
    lib = _lib.load()
    p = np.ascontiguousarray(np.asarray(c, dtype=np.int32).reshape(-1)) if len(c) else np.zeros(2, np.int32)
    out = (c_float * 5)()
    _lib.check("usv_min_area_rect", lib.usv_min_area_rect(p.ctypes.data_as(POINTER(c_int)), len(c), out))
    return (out[0], out[1]), (out[2], out[3]), out[4]


def MatchCentroids(contours, tentative_match):
    """Centre point of minAreaRect(contours[left]) per match (P/Main.cpp:1120-1143) -> list[(x, y)] float32."""
    lib = _lib.load()
    p, off = _flatten(contours)
    m = _matches(tentative_match)
    out = (c_float * max(2 * len(tentative_match), 2))()
    n = c_int(0)
    ip = POINTER(c_int)
    _lib.check("usv_match_centroids", lib.usv_match_centroids(
        p.ctypes.data_as(ip), off.ctypes.data_as(ip), len(contours), m, len(tentative_match), out,
        ctypes.byref(n)))
    return [(out[2 * i], out[2 * i + 1]) for i in range(n.value)]


def _f32(pts):
    a = np.ascontiguousarray(np.asarray(pts, dtype=np.float32).reshape(-1))
    return a, len(a) // 2


def MovingObjectDistanceCalculator(camera_side_left, ts_this, this_pts, cur_pts, old_pts, older_pts,
                                   triples, ts_other, ts_other_old, ts_other_older,
                                   return_interpolated=False, interpolated=()):
    """Time stamps are steady_clock ticks (ns).  Returns the appended dist list (cm).

    `interpolated` is the caller's InterpolatedVectorCenter_pointOtherCamera (by value in the
    reference, normally empty); with return_interpolated the grown vector (those points, then one
    extrapolated point per triple, P/DistanceCalculator.cpp:67) is returned as well."""
    lib = _lib.load()
    t, nt = _f32(this_pts)
    c, nc = _f32(cur_pts)
    o, no = _f32(old_pts)
    q, nq = _f32(older_pts)
    ii, ni = _f32(interpolated) if len(interpolated) else (np.zeros(2, np.float32), 0)
    tri = np.ascontiguousarray(np.asarray(triples, dtype=np.int32).reshape(-1))
    ntri = len(tri) // 3
    dist = np.zeros(max(ntri, 1), dtype=np.float64)
    interp = np.zeros(2 * max(ni + ntri, 1), dtype=np.float32)
    n = c_int(0)
    fp, ip, dp = POINTER(c_float), POINTER(c_int), POINTER(c_double)
    _lib.check("usv_moving_object_distance", lib.usv_moving_object_distance(
        int(bool(camera_side_left)), int(ts_this), t.ctypes.data_as(fp), nt, c.ctypes.data_as(fp), nc,
        o.ctypes.data_as(fp), no, q.ctypes.data_as(fp), nq, ii.ctypes.data_as(fp), ni,
        tri.ctypes.data_as(ip), ntri,
        int(ts_other), int(ts_other_old), int(ts_other_older), dist.ctypes.data_as(dp),
        interp.ctypes.data_as(fp), ctypes.byref(n)))
    d = dist[:n.value].tolist()
    if return_interpolated:
        return d, interp[:2 * (ni + n.value)].reshape(-1, 2)
    return d


def CooridinatePositionCalculator(camera_side_left, dist, this_pts, coordinate_display=True):
    """-> list[(x, y, z)] cm; empty unless coordinate_display (the reference's global gate)."""
    lib = _lib.load()
    d = np.ascontiguousarray(np.asarray(dist, dtype=np.float64))
    t, nt = _f32(this_pts)
    out = np.zeros(3 * max(len(d), 1), dtype=np.float64)
    n = c_int(0)
    dp, fp = POINTER(c_double), POINTER(c_float)
    _lib.check("usv_coordinate_position", lib.usv_coordinate_position(
        int(bool(camera_side_left)), d.ctypes.data_as(dp), len(d), t.ctypes.data_as(fp), nt,
        int(bool(coordinate_display)), out.ctypes.data_as(dp), ctypes.byref(n)))
    return [tuple(out[3 * i:3 * i + 3]) for i in range(n.value)]
