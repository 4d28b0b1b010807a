#!/bin/bash
# GPU box: smoke, the driver's bench command, and a rocprofv3 kernel-trace of a short bench run.
# Each GPU step has its own limit; the first failure ends the call.  Usage: scripts/gpu_bench_prof.sh <tag> [bench args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
TAG=${1:-r03}; shift
BARGS=${*:---steps 20 --warmup 5}
OUT=gpurun_out/$TAG
mkdir -p $OUT
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 4 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "FAILED rc=$rc in $name: stopping"; exit $rc; fi
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[ -n "$TESTS" ] && step pytest 600 python -u -m pytest $TESTS -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread
step bench 300 python bench.py $BARGS
step trace 240 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --extra-steps 0
exit 0
