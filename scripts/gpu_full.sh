#!/bin/bash
# GPU box: smoke, the whole -m gpu suite, the driver's bench command, a rocprofv3 kernel trace of it.
# Each GPU step has its own limit; the first failure ends the call.  TAG names gpurun_out/<TAG>.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06full}; mkdir -p $OUT
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 4 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "FAILED rc=$rc in $name: stopping"; exit $rc; fi
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[ -z "$NO_TESTS" ] && step pytest 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread
step bench 300 python bench.py --gpus 1 --steps 20 --warmup 5
cp $OUT/bench.log $OUT/bench.json
[ -n "$BENCH2" ] && step bench2 300 python bench.py --gpus 1 --steps 20 --warmup 5 && step bench_default 300 python bench.py
[ -z "$NO_TRACE" ] && step trace 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5
exit 0
