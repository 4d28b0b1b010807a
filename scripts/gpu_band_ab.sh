#!/bin/bash
# GPU box: parity tests, per-workgroup timeline of the weighted band plan, interleaved A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -20 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
if [ -f build_variants/wgtime_g1.so ]; then
  USV_LIB_PATH=$PWD/build_variants/wgtime_g1.so timeout -k 10 120 python scripts/wgtime.py > gpurun_out/wgtime_g1.txt 2>&1 || exit 1
  mv build_variants/wgtime_g1.so /tmp/
fi
ROUNDS=${ROUNDS:-3} bash scripts/ab_interleaved.sh
