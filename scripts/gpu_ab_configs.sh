#!/bin/bash
# GPU box: full GPU test suite, then interleaved A/Bs of the in-tree build and build_variants/*.so on
# configs B, A and C (and E with AB_E=1).  Each step has its own limit; the first failure ends the call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-abcfg}; mkdir -p $OUT
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
      > $OUT/pytest.log 2>&1 || { echo "FAILED pytest"; tail -30 $OUT/pytest.log; exit 1; }
  tail -2 $OUT/pytest.log
fi
common="--no-cpu-baseline --pipeline-steps 0 --extra-steps 0"
run_ab() {  # run_ab <name> <args>
  ROUNDS=${ROUNDS:-3} ARGS="$2" timeout -k 10 600 bash scripts/ab_interleaved.sh > $OUT/ab_$1.log 2>&1 || { echo "FAILED ab $1"; tail $OUT/ab_$1.log; exit 1; }
  echo "== $1"; grep median $OUT/ab_$1.log
}
run_ab B "--steps 100 --warmup 10 $common --kernel-steps 200 --width 640 --height 480 --disparities 64 --window 7"
run_ab A "--steps 100 --warmup 10 $common --kernel-steps 200 --width 320 --height 240 --disparities 32 --window 5"
run_ab C "--steps 100 --warmup 10 $common --kernel-steps 200"
[ "${AB_E:-0}" = 1 ] && run_ab E "--steps 20 --warmup 3 $common --kernel-steps 20 --width 3840 --height 2160 --disparities 256 --window 15"
exit 0
