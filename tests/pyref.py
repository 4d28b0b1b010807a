"""Pure-Python restatement of the A1 block-match spec.

Independent of oracle/sad_oracle.c (written separately, plain loops), used
only on tiny inputs to pin the C oracle.  Test infrastructure only.
"""


def sad_disparity_py(L, R, D, w, metric="sad"):
    H, W = len(L), len(L[0])
    r = (w - 1) // 2

    def cl(v, hi):
        return 0 if v < 0 else (hi if v > hi else v)

    out = [[0] * W for _ in range(H)]
    for y in range(H):
        for x in range(W):
            best, bd = None, 0
            for d in range(D):
                c = 0
                for dy in range(-r, r + 1):
                    yy = cl(y + dy, H - 1)
                    for dx in range(-r, r + 1):
                        t = int(L[yy][cl(x + dx, W - 1)]) - int(R[yy][cl(x + dx - d, W - 1)])
                        c += abs(t) if metric == "sad" else t * t
                if best is None or c < best:
                    best, bd = c, d
            out[y][x] = bd
    return out
