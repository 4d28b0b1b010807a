set -o pipefail
export TMPDIR=/tmp
TESTS="tests/test_gpu_parity.py" SEL="baseline_configs or ragged or group or fixtures or border" AB=1 PIPE=0 TAG=it2 bash scripts/gpu_iter.sh || exit 1
cp gpurun_out/ab.txt gpurun_out/it2/abB.txt
ROUNDS=3 ARGS="--steps 100 --warmup 10 --no-cpu-baseline --pipeline-steps 0 --extra-steps 0 --kernel-steps 200 --width 320 --height 240 --disparities 32 --window 5" timeout -k 10 600 bash scripts/ab_interleaved.sh > gpurun_out/it2/abA.log 2>&1 || exit 1
cp gpurun_out/ab.txt gpurun_out/it2/abA.txt; tail -6 gpurun_out/it2/abA.log
