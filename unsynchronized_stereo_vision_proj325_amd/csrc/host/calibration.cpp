// calibration.cpp -- LoadCalibrationData (P/Main.cpp:329-349) for C++ callers.
//
// The reference reads thirteen named matrices with OpenCV's FileStorage from an
// XML file into CalibrationDataParameters (P/Main.cpp:175-180), then builds the
// rectification maps from four of them per camera (P/Main.cpp:352,357).  OpenCV
// is absent from the image, so this reads FileStorage's XML layout itself:
// <opencv_storage> root, <name type_id="opencv-matrix"> nodes holding <rows>,
// <cols>, <dt> and whitespace-separated <data>.  Values are parsed with strtod
// (correctly rounded, the same doubles Python's float() gives: the Python
// loader calibration.py is the cross-check, tests/test_calibration_cpp.py).
// A name the file lacks leaves its matrix empty (rows = cols = 0), as
// FileStorage leaves the Mat empty.
#include "Calibration.hpp"

#include <cctype>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>

namespace {

struct Named {
    const char* name;
    usv_mat usv_calibration::*field;
};
// P/Main.cpp:335-347, the reference's spellings (EssentailMat)
const Named kNames[] = {
    {"intrinsicL", &usv_calibration::intrinsicL},
    {"intrinsicR", &usv_calibration::intrinsicR},
    {"distCoeffsL", &usv_calibration::distCoeffsL},
    {"distCoeffsR", &usv_calibration::distCoeffsR},
    {"RotationMat", &usv_calibration::RotationMat},
    {"TranslationMat", &usv_calibration::TranslationMat},
    {"EssentailMat", &usv_calibration::EssentailMat},
    {"FundamentalMat", &usv_calibration::FundamentalMat},
    {"RectificationTransformMatL", &usv_calibration::RectificationTransformMatL},
    {"RectificationTransformMatR", &usv_calibration::RectificationTransformMatR},
    {"ProjectionMatL", &usv_calibration::ProjectionMatL},
    {"ProjectionMatR", &usv_calibration::ProjectionMatR},
    {"Disparity2DepthMappingMat", &usv_calibration::Disparity2DepthMappingMat},
};

// Text between <tag> and </tag> inside [from, to) of s; npos when absent.
bool child_text(const std::string& s, size_t from, size_t to, const std::string& tag, std::string* out) {
    const std::string open = "<" + tag + ">", close = "</" + tag + ">";
    const size_t a = s.find(open, from);
    if (a == std::string::npos || a >= to) return false;
    const size_t b = s.find(close, a + open.size());
    if (b == std::string::npos || b > to) return false;
    *out = s.substr(a + open.size(), b - a - open.size());
    return true;
}

usv_status parse_matrix(const std::string& s, size_t from, size_t to, usv_mat* m) {
    std::string rows, cols, dt, data;
    if (!child_text(s, from, to, "rows", &rows) || !child_text(s, from, to, "cols", &cols) ||
        !child_text(s, from, to, "dt", &dt) || !child_text(s, from, to, "data", &data))
        return USV_ERR_INVALID_ARG;
    const int r = std::atoi(rows.c_str()), c = std::atoi(cols.c_str());
    size_t i0 = dt.find_first_not_of(" \t\r\n"), i1 = dt.find_last_not_of(" \t\r\n");
    if (i0 == std::string::npos) return USV_ERR_INVALID_ARG;
    const std::string code = dt.substr(i0, i1 - i0 + 1);
    // one channel of u, c, w, s, i, f or d (multi-channel matrices are not calibration data)
    if (code.size() != 1 || !std::strchr("ucwsifd", code[0])) return USV_ERR_UNSUPPORTED;
    if (r < 0 || c < 0 || (long)r * c > 16) return USV_ERR_UNSUPPORTED;
    const char* p = data.c_str();
    int n = 0;
    for (;;) {
        while (*p && std::isspace((unsigned char)*p)) ++p;
        if (!*p) break;
        char* end = nullptr;
        const double v = std::strtod(p, &end);
        if (end == p) return USV_ERR_INVALID_ARG;
        if (n >= r * c) return USV_ERR_INVALID_ARG;  // more values than rows x cols
        // integer element types hold integers; float ('f') is stored as the float the file meant
        m->data[n++] = code[0] == 'f' ? (double)(float)v : v;
        p = end;
    }
    if (n != r * c) return USV_ERR_INVALID_ARG;
    m->rows = r;
    m->cols = c;
    return USV_OK;
}

}  // namespace

extern "C" usv_status usv_load_calibration(const char* path, usv_calibration* out) {
    if (!path || !out) return USV_ERR_INVALID_ARG;
    std::memset(out, 0, sizeof(*out));
    std::ifstream f(path, std::ios::binary);
    if (!f) return USV_ERR_INVALID_ARG;
    std::stringstream ss;
    ss << f.rdbuf();
    const std::string s = ss.str();
    const size_t root = s.find("<opencv_storage>");
    const size_t root_end = s.rfind("</opencv_storage>");
    if (root == std::string::npos || root_end == std::string::npos || root_end < root)
        return USV_ERR_INVALID_ARG;
    for (const Named& nm : kNames) {
        const std::string open = std::string("<") + nm.name + " ";
        const std::string close = std::string("</") + nm.name + ">";
        size_t a = s.find(open, root);
        if (a == std::string::npos || a > root_end) continue;  // absent: empty matrix
        const size_t head_end = s.find('>', a);
        if (head_end == std::string::npos) return USV_ERR_INVALID_ARG;
        if (s.substr(a, head_end - a).find("opencv-matrix") == std::string::npos) continue;
        const size_t b = s.find(close, head_end);
        if (b == std::string::npos || b > root_end) return USV_ERR_INVALID_ARG;
        const usv_status st = parse_matrix(s, head_end + 1, b, &(out->*nm.field));
        if (st != USV_OK) return st;
    }
    return USV_OK;
}

extern "C" usv_status usv_calibration_rectify_params(const usv_calibration* cal, int left, double* params) {
    if (!cal || !params) return USV_ERR_INVALID_ARG;
    const usv_mat& K = left ? cal->intrinsicL : cal->intrinsicR;
    const usv_mat& d = left ? cal->distCoeffsL : cal->distCoeffsR;
    const usv_mat& R = left ? cal->RectificationTransformMatL : cal->RectificationTransformMatR;
    const usv_mat& P = left ? cal->ProjectionMatL : cal->ProjectionMatR;
    if (K.rows != 3 || K.cols != 3 || P.rows != 3 || (P.cols != 3 && P.cols != 4)) return USV_ERR_INVALID_ARG;
    const bool has_r = R.rows * R.cols != 0;
    if (has_r && (R.rows != 3 || R.cols != 3)) return USV_ERR_INVALID_ARG;
    const int nd = d.rows * d.cols;
    return usv_rectify_params(K.data, nd ? d.data : nullptr, nd, has_r ? R.data : nullptr, P.data, P.cols,
                              params);
}

void LoadCalibrationData(CalibrationDataParameters& CalibrationData, const std::string& filename) {
    // the reference's void, no-throw convention: a file it cannot read leaves the matrices empty
    if (usv_load_calibration(filename.c_str(), &CalibrationData) != USV_OK)
        std::memset(static_cast<usv_calibration*>(&CalibrationData), 0, sizeof(usv_calibration));
}

void LoadCalibrationData(CalibrationDataParameters& CalibrationData) {
    const char* env = std::getenv("USV_CALIBRATION_FILE");
    LoadCalibrationData(CalibrationData, env && *env ? std::string(env) : std::string("StereoCalibration4r3.xml"));
}
