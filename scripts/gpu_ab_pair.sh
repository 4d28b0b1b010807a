#!/bin/bash
# GPU box: parity tests of the in-tree library, then an interleaved A/B of it against the
# build_variants/*.so (config C, kernel_ms by HIP events).  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_isa_lint.py -m gpu -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread > gpurun_out/ab_parity.log 2>&1
rc=$?; tail -3 gpurun_out/ab_parity.log
[ $rc -ne 0 ] && { echo "parity FAILED rc=$rc"; exit $rc; }
ROUNDS=${ROUNDS:-4} ARGS=${ARGS:---steps 200 --warmup 20 --no-cpu-baseline --no-parity --extra-steps 0 --pipeline-steps 0} \
    bash scripts/ab_interleaved.sh
