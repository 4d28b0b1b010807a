cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_sad.log 2>&1 || { tail -30 gpurun_out/pytest_sad.log; exit 1; }
tail -1 gpurun_out/pytest_sad.log
ROUNDS=2 ARGS="--steps 20 --warmup 3 --no-cpu-baseline --pipeline-steps 0 --extra-steps 0 --width 3840 --height 2160 --disparities 256 --window 15" bash scripts/ab_interleaved.sh && cp gpurun_out/ab.txt gpurun_out/abE.txt && ROUNDS=3 ARGS="--steps 200 --warmup 20 --no-cpu-baseline --pipeline-steps 0 --extra-steps 0" bash scripts/ab_interleaved.sh
