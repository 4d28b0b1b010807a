#!/bin/bash
# GPU box (round 5): parity of the in-tree build, then the interleaved timing A/B of build_variants/*.so
# against it on configs C and E.  Each GPU step has its own limit; the first failure ends the call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
OUT=gpurun_out/${TAG:-r05ab}; mkdir -p $OUT
echo "=== parity ($(date +%T))"
timeout -k 10 ${PARITY_TO:-600} python -u -m pytest ${TESTS:-tests/test_gpu_parity.py} -m gpu -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -n 5 $OUT/pytest.log; [ $rc -ne 0 ] && { echo "parity FAILED rc=$rc"; exit $rc; }
[ -n "$NO_AB" ] && exit 0
ROUNDS=${ROUNDS:-2} bash scripts/gpu_timing_ab.sh || exit 1
cp gpurun_out/tab_C.txt gpurun_out/tab_E.txt $OUT/ 2>/dev/null
exit 0
