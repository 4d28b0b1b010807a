// LoadCalibrationData from C++ (include/Calibration.hpp, P/Main.cpp:329-349) and the
// rectification parameters built from it: prints one JSON object per line for
// tests/test_calibration_cpp.py, which compares with the Python loader.
#include <cmath>
#include <cstdio>
#include <cstdlib>

#include "Calibration.hpp"

static void pmat(const char* name, const usv_mat& m, bool last = false) {
    std::printf("\"%s\": {\"rows\": %d, \"cols\": %d, \"data\": [", name, m.rows, m.cols);
    for (int i = 0; i < m.rows * m.cols; ++i) std::printf("%s%.17g", i ? ", " : "", m.data[i]);
    std::printf("]}%s", last ? "" : ", ");
}

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    setenv("USV_CALIBRATION_FILE", argv[1], 1);
    CalibrationDataParameters cal;
    LoadCalibrationData(cal);  // the reference's one-argument form
    std::printf("{");
    pmat("intrinsicL", cal.intrinsicL);
    pmat("distCoeffsL", cal.distCoeffsL);
    pmat("intrinsicR", cal.intrinsicR);
    pmat("distCoeffsR", cal.distCoeffsR);
    pmat("RotationMat", cal.RotationMat);
    pmat("RectificationTransformMatL", cal.RectificationTransformMatL);
    pmat("RectificationTransformMatR", cal.RectificationTransformMatR);
    pmat("ProjectionMatL", cal.ProjectionMatL);
    pmat("ProjectionMatR", cal.ProjectionMatR);
    pmat("Disparity2DepthMappingMat", cal.Disparity2DepthMappingMat, true);
    std::printf("}\n");
    for (int left = 1; left >= 0; --left) {
        double p[25];
        const int st = usv_calibration_rectify_params(&cal, left, p);
        std::printf("{\"params%s\": {\"status\": %d, \"values\": [", left ? "L" : "R", st);
        for (int i = 0; i < 25 && st == 0; ++i) std::printf("%s%.17g", i ? ", " : "", p[i]);
        std::printf("]}}\n");
    }
    CalibrationDataParameters missing;
    LoadCalibrationData(missing, "/nonexistent/StereoCalibration4r3.xml");
    std::printf("{\"missing_rows\": %d}\n", missing.intrinsicL.rows);
    return 0;
}
