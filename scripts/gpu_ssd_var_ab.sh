set -e
export TMPDIR=/tmp
for v in build_variants/*.so; do
  USV_LIB_PATH=$PWD/$v timeout -k 10 300 python -u -m pytest tests/test_ssd_matrix.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/vp_$(basename $v .so).log 2>&1 || { echo "PARITY FAIL $v"; tail -20 gpurun_out/vp_$(basename $v .so).log; exit 1; }
  echo "parity $v: $(tail -1 gpurun_out/vp_$(basename $v .so).log)"
done
ROUNDS=3 timeout -k 10 500 python -u scripts/gpu_ssd_ab.py
