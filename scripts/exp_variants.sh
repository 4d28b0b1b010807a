#!/bin/bash
# GPU box: stamps breakdown (if built) + bench of the default build and each
# build_variants/*.so (config C).  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; tail -n 4 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "FAILED rc=$rc in $name: stopping"; exit $rc; fi; }
if [ -f build_variants/stamps.so ]; then
  USV_LIB_PATH=$PWD/build_variants/stamps.so step stamps 240 python scripts/stamps.py
fi
step bench_default 240 python bench.py --steps 200 --warmup 20 --no-cpu-baseline
for v in build_variants/*.so; do
  n=$(basename $v .so); [ "$n" = stamps ] && continue
  USV_LIB_PATH=$PWD/$v step bench_$n 240 python bench.py --steps 200 --warmup 20 --no-cpu-baseline
done
step bench_default2 240 python bench.py --steps 200 --warmup 20 --no-cpu-baseline
step bench_nodist 240 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-distance
exit 0
