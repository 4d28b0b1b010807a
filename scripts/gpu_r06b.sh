#!/bin/bash
# GPU box (round 6): targeted tests on the product library, the K = 16 variant's parity suite, then an
# interleaved A/B of the variants in build_variants/ against the product (scripts/ab_interleaved.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06b}; mkdir -p $OUT
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 4 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "FAILED rc=$rc in $name: stopping"; exit $rc; fi
}
PT="python -u -m pytest -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread"
[ -z "$NO_TESTS" ] && step tests 600 $PT ${TESTS:-tests/test_ssd_matrix.py tests/test_streaming.py tests/test_gpu_contours.py tests/test_sharding.py}
for v in ${VARIANT_TESTS}; do
  step "vt_$v" 600 env USV_LIB_PATH=$PWD/build_variants/$v.so $PT ${VT_FILES:-tests/test_gpu_parity.py}
done
[ -z "$NO_AB" ] && step ab 900 env ROUNDS=${ROUNDS:-3} bash scripts/ab_interleaved.sh
cp gpurun_out/ab.txt $OUT/ab.txt 2>/dev/null
exit 0
