#!/bin/bash
# GPU box, one iteration: (1) the GPU tests named by $TESTS (default: rectify + preproc), (2) parity of
# every build_variants/*.so on the small-frame and border cases, (3) an interleaved A/B of the in-tree
# build and the variants on the workload in $AB_ARGS (default config B), (4) the bench pipeline legs.
# Each GPU step has its own limit; the first failure ends the call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-iter}
mkdir -p $OUT
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 4 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "FAILED rc=$rc in $name: stopping"; exit $rc; fi
}
step tests 400 python -u -m pytest ${TESTS:-tests/test_rectify.py tests/test_preproc.py} -m gpu -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread
SEL=${SEL:-"baseline_configs or ragged or border or fixtures"}
for v in build_variants/*.so; do
  [ -e "$v" ] || continue
  n=$(basename $v .so)
  USV_LIB_PATH=$PWD/$v step parity_$n 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider \
      --timeout 120 --timeout-method thread -k "$SEL"
done
if [ "${AB:-1}" = 1 ]; then
  ROUNDS=${ROUNDS:-3} ARGS=${AB_ARGS:-"--steps 100 --warmup 10 --no-cpu-baseline --pipeline-steps 0 --extra-steps 0 --kernel-steps 200 --width 640 --height 480 --disparities 64 --window 7"} \
    step ab 900 bash scripts/ab_interleaved.sh
  cp gpurun_out/ab.txt $OUT/ab.txt
fi
[ "${PIPE:-1}" = 1 ] && step bench 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --extra-steps 0
exit 0
