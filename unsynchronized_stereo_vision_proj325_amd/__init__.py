"""MI355X (gfx950) stereo block-match + distance engine.

Drop-in for the hot path of 6dwavenminer/Unsynchronized_Stereo_Vision_Proj325:
the per-pixel SAD/SSD disparity search (new) and the
reference's distance / matcher API (Match.hpp, DistanceCalculator.hpp), plus
the per-frame stages around it: rectification, the colour chain and masks, and
the calibration file.
Compute runs in libusv.so (hand-written HIP for gfx950 behind a C ABI,
include/usv.h); this package is the Python host layer used by tests and bench.
"""
from . import _lib  # noqa: F401
from .calibration import CalibrationDataParameters, load_calibration, save_calibration  # noqa: F401
from .engine import (StereoBlockMatcher, disparity_to_distance, distance_lut_cm, distance_lut_mm,  # noqa: F401
                     sad_disparity)

__all__ = ["StereoBlockMatcher", "sad_disparity", "disparity_to_distance", "distance_lut_cm",
           "CalibrationDataParameters", "load_calibration", "save_calibration"]
# GPU stages around the matcher: .rectify (Rectifier, rectify_pair) and
# .preproc (FramePrep, frame_prep, ABSDiffSearch, ColourSearch).
