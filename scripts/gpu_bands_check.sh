#!/bin/bash
# Band sharding on the GPU: parity test, then a 2-rank one-GPU rehearsal of bench.py --split bands.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "band" > gpurun_out/bands_pytest.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 50 --warmup 10 > gpurun_out/bands_bench1.log 2>&1 &&
USV_BENCH_REHEARSE=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --split bands \
    --gather none --no-cpu-baseline > gpurun_out/bands_bench2.log 2>&1
rc=$?
tail -3 gpurun_out/bands_pytest.log; tail -2 gpurun_out/bands_bench1.log; tail -2 gpurun_out/bands_bench2.log
exit $rc
