#!/bin/bash
# A/B experiment on the GPU box: LDS-DMA probe, GPU parity tests, bench of the
# default build and of build_variants/*.so.  Each GPU step time-limited; a
# fatal exit stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; esac; [ "$1" -gt 128 ] && return 0; return 1; }
step() { local name=$1 to=$2; shift 2; echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; tail -n 6 "gpurun_out/$name.log"
  if fatal $rc || [ $rc -ne 0 ]; then echo "FAILED rc=$rc in $name: stopping"; exit $rc; fi; return $rc; }
[ -x scripts/probes/glds_probe ] && step probe 60 scripts/probes/glds_probe
step pytest_gpu 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider
step bench_default 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline
for v in build_variants/*.so; do
  n=$(basename $v .so)
  USV_LIB_PATH=$PWD/$v step bench_$n 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline
done
exit 0
