/*
 * match_oracle.c -- CPU ORACLE (test infrastructure only; see usv_oracle.h).
 *
 * Restates the two OpenCV-free matcher stages of P/Main.cpp, with their quirks.
 */
#include "usv_oracle.h"

/* P/Main.cpp:432-477.  The outer while(AnyConflict) loop runs the pass once:
 * the input is cleared at line 475, so a second iteration finds it empty.  A
 * candidate that conflicts with a WORSE tentative entry overwrites every such
 * entry (possibly several -> duplicates); a candidate whose conflicts are all
 * better (or equal) is still appended (line 463-466). */
int usv_oracle_resolve_match_list(const usv_oracle_match* in, int n_in, usv_oracle_match* out) {
    int n_out = 0;
    for (int m = 0; m < n_in; ++m) {
        if (n_out == 0) { out[n_out++] = in[m]; continue; }
        int conflict = 0;
        for (int i = 0; i < n_out; ++i) {
            if (out[i].left == in[m].left || out[i].right == in[m].right) {
                if (out[i].value > in[m].value) { out[i] = in[m]; conflict = 1; }
            }
        }
        if (!conflict) out[n_out++] = in[m];
    }
    return n_out;
}

/* P/Main.cpp:483-499.  Line 492 builds (Point3i)(cur[i], old[j].RightIndex):
 * the comma operator discards cur[i] and Point3i(Vec3i(old[j].RightIndex))
 * gives (old[j].RightIndex, 0, 0). */
int usv_oracle_id_matcher(const usv_oracle_match* cur, int n_cur, const usv_oracle_match* old,
                          int n_old, int* out_xyz) {
    int n = 0;
    for (int i = 0; i < n_cur; ++i) {
        if (n_old == 0) continue;
        for (int j = 0; j < n_old; ++j) {
            if (cur[i].right == old[j].left) {
                out_xyz[3 * n + 0] = (int)old[j].right;
                out_xyz[3 * n + 1] = 0;
                out_xyz[3 * n + 2] = 0;
                ++n;
            }
        }
    }
    return n;
}
