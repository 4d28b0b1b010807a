"""Stereo calibration file I/O.

The reference loads its calibration with OpenCV's FileStorage from an XML file
(``LoadCalibrationData``, P/Main.cpp:329-349) into ``CalibrationDataParameters``
(P/Main.cpp:175-180): thirteen named matrices.  OpenCV is absent here, so this
module reads and writes the same ``<opencv_storage>`` XML layout directly
(``type_id="opencv-matrix"`` nodes with ``rows``, ``cols``, ``dt`` and
whitespace-separated ``data``).  The reference's calibration file itself is not
in its repository; tests round-trip files written here and a hand-written file
in OpenCV's layout.
"""
from __future__ import annotations

import os
import xml.etree.ElementTree as ET
from dataclasses import dataclass, field, fields

import numpy as np

# FileStorage element type codes -> numpy dtypes
_DT = {"u": np.uint8, "c": np.int8, "w": np.uint16, "s": np.int16, "i": np.int32, "f": np.float32,
       "d": np.float64}
_DT_OF = {np.dtype(v): k for k, v in _DT.items()}


@dataclass
class CalibrationDataParameters:
    """P/Main.cpp:175-180 (the maps are built by rectify.Rectifier, not stored)."""
    intrinsicL: np.ndarray | None = None
    distCoeffsL: np.ndarray | None = None
    intrinsicR: np.ndarray | None = None
    distCoeffsR: np.ndarray | None = None
    RotationMat: np.ndarray | None = None
    TranslationMat: np.ndarray | None = None
    EssentailMat: np.ndarray | None = None  # the reference's spelling (P/Main.cpp:341)
    FundamentalMat: np.ndarray | None = None
    RectificationTransformMatL: np.ndarray | None = None
    RectificationTransformMatR: np.ndarray | None = None
    ProjectionMatL: np.ndarray | None = None
    ProjectionMatR: np.ndarray | None = None
    Disparity2DepthMappingMat: np.ndarray | None = None
    extra: dict = field(default_factory=dict)  # any other node of the file, by name

    def camera(self, left: bool):
        """(K, dist, Rrect, P) of one camera, the arguments initUndistortRectifyMap takes (P/Main.cpp:352,357)."""
        if left:
            return self.intrinsicL, self.distCoeffsL, self.RectificationTransformMatL, self.ProjectionMatL
        return self.intrinsicR, self.distCoeffsR, self.RectificationTransformMatR, self.ProjectionMatR


_NAMES = [f.name for f in fields(CalibrationDataParameters) if f.name != "extra"]


def _parse_matrix(node: ET.Element) -> np.ndarray:
    rows = int(node.findtext("rows"))
    cols = int(node.findtext("cols"))
    dt = node.findtext("dt").strip()
    channels = 1
    if len(dt) > 1 and dt[:-1].isdigit():  # e.g. "3d": multi-channel element
        channels, dt = int(dt[:-1]), dt[-1]
    if dt not in _DT:
        raise ValueError(f"{node.tag}: unsupported element type {dt!r}")
    text = node.findtext("data") or ""
    vals = np.array(text.split(), dtype=np.float64)
    if vals.size != rows * cols * channels:
        raise ValueError(f"{node.tag}: {vals.size} values for a {rows}x{cols}x{channels} matrix")
    out = vals.astype(_DT[dt]).reshape(rows, cols, channels) if channels > 1 else \
        vals.astype(_DT[dt]).reshape(rows, cols)
    return out


def load_calibration(path: str | os.PathLike) -> CalibrationDataParameters:
    """LoadCalibrationData (P/Main.cpp:329-349): every opencv-matrix node of the file, by name;
    names the reference reads that are missing stay None (FileStorage leaves the Mat empty)."""
    root = ET.parse(os.fspath(path)).getroot()
    if root.tag != "opencv_storage":
        raise ValueError(f"{path}: not an OpenCV FileStorage XML file (root <{root.tag}>)")
    cal = CalibrationDataParameters()
    for node in root:
        if node.get("type_id") != "opencv-matrix":
            continue
        m = _parse_matrix(node)
        if node.tag in _NAMES:
            setattr(cal, node.tag, m)
        else:
            cal.extra[node.tag] = m
    return cal


def _fmt(v, dt: str) -> str:
    if dt in "fd":
        return repr(float(v))  # shortest round-trip form
    return str(int(v))


def save_calibration(path: str | os.PathLike, cal: CalibrationDataParameters) -> None:
    """Write the matrices in FileStorage's XML layout (readable by cv::FileStorage and load_calibration)."""
    lines = ['<?xml version="1.0"?>', "<opencv_storage>"]
    items = [(n, getattr(cal, n)) for n in _NAMES] + list(cal.extra.items())
    for name, m in items:
        if m is None:
            continue
        a = np.asarray(m)
        if a.ndim == 1:
            a = a.reshape(-1, 1)
        channels = a.shape[2] if a.ndim == 3 else 1
        code = _DT_OF.get(a.dtype)
        if code is None:
            a = a.astype(np.float64)
            code = "d"
        dt = f"{channels}{code}" if channels > 1 else code
        data = " ".join(_fmt(v, code) for v in a.ravel())
        lines += [f'<{name} type_id="opencv-matrix">', f"  <rows>{a.shape[0]}</rows>", f"  <cols>{a.shape[1]}</cols>",
                  f"  <dt>{dt}</dt>", f"  <data>\n    {data}</data></{name}>"]
    lines.append("</opencv_storage>")
    with open(os.fspath(path), "w") as f:
        f.write("\n".join(lines) + "\n")
