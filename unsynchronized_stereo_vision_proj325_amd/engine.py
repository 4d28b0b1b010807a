"""GPU path: disparity and distance maps of rectified u8 stereo pairs.

Thin host layer over the C ABI (include/usv.h).  Tensors are torch device
tensors (PyTorch supplies device memory and the stream); the compute is the
gfx950 kernels in libusv.so.  Every call checks that its operands live on a
GPU and raises otherwise: there is no CPU path here.

Reference mapping: the engine is the new per-pixel block matcher SURVEY.md
§8(a) A1 (absent from the reference; nearest primitive P/Main.cpp:304) and the
per-pixel form A11 of the distance law P/DistanceCalculator.cpp:84.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib

_METRICS = {"sad": _lib.METRIC_SAD, "ssd": _lib.METRIC_SSD}
_MODELS = {"moving_object": _lib.DIST_MOVING_OBJECT, "canny": _lib.DIST_CANNY}
_KERNELS = {"auto": _lib.KERNEL_AUTO, "fast": _lib.KERNEL_FAST, "generic": _lib.KERNEL_GENERIC,
            "tiled": _lib.KERNEL_TILED, "matrix": _lib.KERNEL_MATRIX}


def distance_lut_cm(model: str = "moving_object") -> np.ndarray:
    """256-entry host table: lut[d] = distance in cm of integer disparity d.

    model "moving_object": P/DistanceCalculator.cpp:84 (d = 0 -> +inf);
    model "canny": P/Main.cpp:694.
    """
    lib = _lib.load()
    out = np.empty(256, dtype=np.float64)
    _lib.check("usv_distance_lut_cm",
               lib.usv_distance_lut_cm(_MODELS[model], out.ctypes.data_as(ctypes.POINTER(ctypes.c_double))))
    return out


def distance_lut_mm(model: str = "moving_object") -> np.ndarray:
    """The same table in mm (north_star's unit): lut_mm[d] = 10 * lut_cm[d] (usv_distance_lut_mm)."""
    lib = _lib.load()
    out = np.empty(256, dtype=np.float64)
    _lib.check("usv_distance_lut_mm",
               lib.usv_distance_lut_mm(_MODELS[model], out.ctypes.data_as(ctypes.POINTER(ctypes.c_double))))
    return out


_UNITS = {"cm": distance_lut_cm, "mm": distance_lut_mm}
# (model, unit, device index) -> device copy of the table; built once, never freed, so no launch
# ever has to wait for (or synchronise on) a temporary table
_LUT_CACHE: dict[tuple[str, str, int], torch.Tensor] = {}


def lut_device(model: str, unit: str, device: torch.device) -> torch.Tensor:
    """Device copy of the distance table for (model, unit), cached per device."""
    if model not in _MODELS or unit not in _UNITS:
        raise ValueError(f"model must be one of {sorted(_MODELS)}, unit one of {sorted(_UNITS)}")
    idx = device.index if device.index is not None else torch.cuda.current_device()
    key = (model, unit, idx)
    if key not in _LUT_CACHE:
        _LUT_CACHE[key] = torch.from_numpy(_UNITS[unit](model)).to(torch.device("cuda", idx))
        torch.cuda.synchronize(idx)  # the copy is complete before any stream may read the table
    return _LUT_CACHE[key]


def _stream(stream) -> int:
    s = torch.cuda.current_stream() if stream is None else stream
    return s.cuda_stream


def _check_image(t: torch.Tensor, name: str) -> None:
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise ValueError(f"{name} must be a CUDA (HIP) tensor; the engine has no CPU path")
    if t.dtype != torch.uint8:
        raise ValueError(f"{name} must be uint8, got {t.dtype}")
    if t.dim() not in (2, 3) or t.stride(-1) != 1:
        raise ValueError(f"{name} must be (H, W) or (B, H, W) with unit column stride")


@dataclass
class StereoBlockMatcher:
    """Block-match configuration: D disparities, w x w window.

    compute() returns the u8 disparity map and, when with_distance, the fused
    per-pixel distance map in cm (float64, bit-exact with the reference law).
    """

    num_disparities: int
    window: int
    metric: str = "sad"
    distance_model: str = "moving_object"
    kernel: str = "auto"
    distance_unit: str = "cm"

    def __post_init__(self):
        if self.metric not in _METRICS:
            raise ValueError(f"metric must be one of {sorted(_METRICS)}")
        if self.kernel not in _KERNELS:
            raise ValueError(f"kernel must be one of {sorted(_KERNELS)}")
        if self.distance_model not in _MODELS:
            raise ValueError(f"distance_model must be one of {sorted(_MODELS)}")
        if self.distance_unit not in _UNITS:
            raise ValueError(f"distance_unit must be one of {sorted(_UNITS)}")

    def lut_device(self, device: torch.device) -> torch.Tensor:
        return lut_device(self.distance_model, self.distance_unit, device)

    def compute(self, left: torch.Tensor, right: torch.Tensor, *, with_distance: bool = False,
                out_disp: torch.Tensor | None = None, out_dist: torch.Tensor | None = None,
                stream=None):
        _check_image(left, "left")
        _check_image(right, "right")
        if left.shape != right.shape or left.stride() != right.stride():
            raise ValueError("left and right must have the same shape and strides")
        if left.device != right.device:
            raise ValueError("left and right must be on the same device")
        batched = left.dim() == 3
        B = left.shape[0] if batched else 1
        H, W = left.shape[-2], left.shape[-1]
        pitch = left.stride(-2)
        if out_disp is None:
            out_disp = torch.empty(left.shape, dtype=torch.uint8, device=left.device)
        _check_image(out_disp, "out_disp")
        if tuple(out_disp.shape) != tuple(left.shape):
            raise ValueError("out_disp shape mismatch")
        if out_disp.device != left.device:
            raise ValueError("out_disp must be on the same device as left/right")
        lut = None
        if with_distance:
            lut = self.lut_device(left.device)
            if out_dist is None:
                out_dist = torch.empty(left.shape, dtype=torch.float64, device=left.device)
            if out_dist.dtype != torch.float64 or tuple(out_dist.shape) != tuple(left.shape) \
                    or out_dist.stride(-1) != 1 or not out_dist.is_cuda:
                raise ValueError("out_dist must be a float64 CUDA tensor shaped like left")
            if out_dist.device != left.device:
                raise ValueError("out_dist must be on the same device as left/right")
        lib = _lib.load()
        with torch.cuda.device(left.device):
            s = _stream(stream)
            if not batched:
                st = lib.usv_sad_disparity_ex(
                    left.data_ptr(), right.data_ptr(), W, H, pitch, self.num_disparities,
                    self.window, _METRICS[self.metric], out_disp.data_ptr(), out_disp.stride(-2),
                    out_dist.data_ptr() if with_distance else None,
                    out_dist.stride(-2) if with_distance else 0,
                    lut.data_ptr() if with_distance else None, _KERNELS[self.kernel], s)
                _lib.check("usv_sad_disparity_ex", st)
            else:
                if self.kernel != "auto":
                    raise ValueError("batched compute uses kernel='auto'")
                st = lib.usv_sad_disparity_batch(
                    left.data_ptr(), right.data_ptr(), B, left.stride(0), W, H, pitch,
                    self.num_disparities, self.window, _METRICS[self.metric], out_disp.data_ptr(),
                    out_disp.stride(0), out_disp.stride(-2),
                    out_dist.data_ptr() if with_distance else None,
                    out_dist.stride(0) if with_distance else 0,
                    out_dist.stride(-2) if with_distance else 0,
                    lut.data_ptr() if with_distance else None, s)
                _lib.check("usv_sad_disparity_batch", st)
        return (out_disp, out_dist) if with_distance else out_disp

    def bind(self, left: torch.Tensor, right: torch.Tensor, *, out_disp: torch.Tensor,
             out_dist: torch.Tensor | None = None, stream=None):
        """A zero-argument launcher for repeated matches over the same (resident) buffers.

        Validates once -- the same checks and errors as compute(), plus one real match through compute() --
        then prepares a usv_match_plan (include/usv.h: arguments checked, distance table and kernel resolved
        once) and returns a callable that enqueues one match per call with usv_match_plan_launch: one
        pointer argument, so a caller stepping a frame stream from Python pays the launch itself instead of
        compute()'s per-call validation and argument marshalling.  The buffers must stay alive (and
        unmoved) while the callable is used; the plan is freed with the callable.

        The callable always launches on the stream that was current (or passed as `stream`) when bind() ran,
        also when it is called inside another ``torch.cuda.stream(...)`` context -- unlike compute(), which
        follows the current stream on every call.  The callable holds that stream object alive with its buffers.
        """
        import weakref

        with_distance = out_dist is not None
        self.compute(left, right, with_distance=with_distance, out_disp=out_disp, out_dist=out_dist,
                     stream=stream)  # validation + one real launch (raises exactly as compute() does)
        lib = _lib.load()
        with torch.cuda.device(left.device):
            stream_obj = torch.cuda.current_stream() if stream is None else stream
            s = stream_obj.cuda_stream
            lut = self.lut_device(left.device) if with_distance else None
            batched = left.dim() == 3
            H, W = left.shape[-2], left.shape[-1]
            plan = ctypes.c_void_p()
            _lib.check("usv_match_plan_create", lib.usv_match_plan_create(
                left.data_ptr(), right.data_ptr(), left.shape[0] if batched else 1, left.stride(0) if batched else 0,
                W, H, left.stride(-2), self.num_disparities, self.window, _METRICS[self.metric],
                out_disp.data_ptr(), out_disp.stride(0) if batched else 0, out_disp.stride(-2),
                out_dist.data_ptr() if with_distance else None,
                out_dist.stride(0) if (with_distance and batched) else 0,
                out_dist.stride(-2) if with_distance else 0, lut.data_ptr() if with_distance else None,
                _KERNELS[self.kernel] if not batched else _lib.KERNEL_AUTO, s, ctypes.byref(plan)))
        keep = (left, right, out_disp, out_dist, lut, stream_obj)  # the callable holds its buffers and stream alive
        fn, handle, check = lib.usv_match_plan_launch, plan.value, _lib.check

        def launch():
            st = fn(handle)
            if st:
                check("usv_match_plan_launch", st)
            return keep[2]

        weakref.finalize(launch, lib.usv_match_plan_destroy, handle)
        return launch


def sad_disparity(left: torch.Tensor, right: torch.Tensor, num_disparities: int, window: int,
                  metric: str = "sad", kernel: str = "auto", stream=None) -> torch.Tensor:
    """One-shot disparity map (u8) of a rectified pair; see StereoBlockMatcher."""
    return StereoBlockMatcher(num_disparities, window, metric, kernel=kernel).compute(
        left, right, stream=stream)


def disparity_to_distance(disp: torch.Tensor, model: str = "moving_object",
                          out: torch.Tensor | None = None, stream=None, unit: str = "cm") -> torch.Tensor:
    """Per-pixel distance map (float64, cm or mm) of a u8 disparity map.
    Stream-ordered, no host synchronisation: the table is the cached per-device copy."""
    _check_image(disp, "disp")
    if disp.dim() != 2:
        raise ValueError("disparity_to_distance takes one (H, W) map")
    H, W = disp.shape
    if out is None:
        out = torch.empty((H, W), dtype=torch.float64, device=disp.device)
    if out.dtype != torch.float64 or tuple(out.shape) != (H, W) or out.stride(-1) != 1 \
            or out.device != disp.device:
        raise ValueError("out must be a float64 (H, W) tensor on disp's device")
    lut = lut_device(model, unit, disp.device)
    lib = _lib.load()
    with torch.cuda.device(disp.device):
        _lib.check("usv_disparity_to_distance",
                   lib.usv_disparity_to_distance(disp.data_ptr(), W, H, disp.stride(0), lut.data_ptr(),
                                                 out.data_ptr(), out.stride(0), _stream(stream)))
    return out
