#!/bin/bash
# GPU box: rectify parity of each ${VARIANTS_DIR}/*.so, then the per-kernel pipeline A/B (rocprof).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for v in ${VARIANTS_DIR:-build_variants_ua}/*.so; do
  n=$(basename $v .so)
  USV_LIB_PATH=$PWD/$v timeout -k 10 300 python -u -m pytest tests/test_rectify.py tests/test_preproc.py -m gpu -x -q -p no:cacheprovider \
      --timeout 120 --timeout-method thread > gpurun_out/rp_$n.log 2>&1
  rc=$?; echo "parity $n: $(tail -1 gpurun_out/rp_$n.log)"
  [ $rc -ne 0 ] && { tail -30 gpurun_out/rp_$n.log; exit $rc; }
done
for r in 1 2; do PP_ITERS=300 VARIANTS_DIR=${VARIANTS_DIR:-build_variants_ua} bash scripts/prof_pipeline_ab.sh | grep -E "==|remap_kernel<3, true>|remap_tile|rectify_hsv"; done
