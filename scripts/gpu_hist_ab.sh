#!/bin/bash
# GPU box: the default library and build_variants_hc/*.so (LDS histogram copies per wave) on the preproc /
# rectify GPU parity tests, then per-kernel rocprof times of the pipeline stages (scripts/prof_pipeline_ab.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for v in default build_variants_hc/*.so; do
  n=$(basename $v .so); lib=""; [ "$v" != default ] && lib=$PWD/$v
  USV_LIB_PATH=$lib timeout -k 10 300 python -u -m pytest tests/test_preproc.py tests/test_rectify.py -m gpu -x -q -p no:cacheprovider \
      --timeout 120 --timeout-method thread > gpurun_out/hp_$n.log 2>&1
  rc=$?; echo "parity $n: $(tail -1 gpurun_out/hp_$n.log)"
  [ $rc -ne 0 ] && { tail -30 gpurun_out/hp_$n.log; exit $rc; }
done
PP_ITERS=300 VARIANTS_DIR=build_variants_hc bash scripts/prof_pipeline_ab.sh
