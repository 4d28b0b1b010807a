#!/bin/bash
# GPU box, round-4 batch b: the remap variants (build_variants_rm/) -- rectify parity on each, per-kernel
# A/B of the pipeline stages -- then the round's profiles (scripts/gpu_profiles.sh r04: C, B, E with the
# cold-cache FETCH / WRITE / request-size passes).  Every step has its own limit; the first failure ends it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
step() {  # step <name> <cmd...>
  echo "=== $1 ($(date +%T))"; local n=$1; shift
  "$@" > gpurun_out/b_$n.log 2>&1; local rc=$?
  tail -n 12 gpurun_out/b_$n.log
  [ $rc -ne 0 ] && { echo "FAILED rc=$rc in $n: stopping"; exit $rc; }
  return 0
}
for v in ${RM_DIR:-build_variants_rm}/*.so; do
  [ -e "$v" ] || continue
  step "rm_parity_$(basename $v .so)" env USV_LIB_PATH=$PWD/$v timeout -k 10 300 python -u -m pytest tests/test_rectify.py tests/test_preproc.py \
      -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
done
step rm_ab env PP_ITERS=300 VARIANTS_DIR=${RM_DIR:-build_variants_rm} bash scripts/prof_pipeline_ab.sh
[ "${SKIP_PROFILES:-0}" = 1 ] || step profiles timeout -k 10 900 bash scripts/gpu_profiles.sh r04
exit 0
