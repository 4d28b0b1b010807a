#!/bin/bash
# GPU box: parity of each ${VARIANTS_DIR:-build_variants}/*.so, then interleaved A/Bs on configs B and A
# (the grouped kernel's shapes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for v in ${VARIANTS_DIR:-build_variants}/*.so; do
  n=$(basename $v .so)
  [ "$n" = r03_kernels ] && continue
  USV_LIB_PATH=$PWD/$v timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider \
      --timeout 120 --timeout-method thread > gpurun_out/vp_$n.log 2>&1
  rc=$?; echo "parity $n: $(tail -1 gpurun_out/vp_$n.log)"
  [ $rc -ne 0 ] && { tail -30 gpurun_out/vp_$n.log; exit $rc; }
done
ROUNDS=${ROUNDS:-3} ARGS="--steps 300 --warmup 20 --no-cpu-baseline --no-parity --extra-steps 0 --pipeline-steps 0 --width 640 --height 480 --disparities 64 --window 7" \
    bash scripts/ab_interleaved.sh && cp gpurun_out/ab.txt gpurun_out/ab_B.txt || exit 1
ROUNDS=${ROUNDS:-3} ARGS="--steps 300 --warmup 20 --no-cpu-baseline --no-parity --extra-steps 0 --pipeline-steps 0 --width 320 --height 240 --disparities 32 --window 5" \
    bash scripts/ab_interleaved.sh && cp gpurun_out/ab.txt gpurun_out/ab_A.txt
