// Calibration.hpp -- LoadCalibrationData for C++ callers (P/Main.cpp:329-349).
//
// The reference defines CalibrationDataParameters and LoadCalibrationData inside
// Main.cpp (P/Main.cpp:175-180, 329-349) and reads a hard-coded Windows path.  A
// maintainer dropping the engine in deletes those two and includes this header:
// the struct keeps the reference's member names (EssentailMat spelling
// included) as usv_mat matrices, and the maps the reference recomputes every
// frame are built once from it (usv_calibration_rectify_params -> usv_rectify_map).
#pragma once
#include <string>

#include "usv.h"

struct CalibrationDataParameters : usv_calibration {
    CalibrationDataParameters() : usv_calibration() {}
};

// Reads `filename` (OpenCV FileStorage XML).  void and no-throw as in the reference: an
// unreadable file leaves every matrix empty.
void LoadCalibrationData(CalibrationDataParameters& CalibrationData, const std::string& filename);
// The reference's signature: the file named by $USV_CALIBRATION_FILE, else
// StereoCalibration4r3.xml in the working directory (the reference's file name, P/Main.cpp:331).
void LoadCalibrationData(CalibrationDataParameters& CalibrationData);
