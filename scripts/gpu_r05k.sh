#!/bin/bash
# round 5: SSD band-size A/B + matrix SSD parity, then bench.py over 1..4 alternating streams (interleaved)
set -o pipefail
OUT=gpurun_out/r05k
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ssd_matrix.py > $OUT/pytest_ssd.txt 2>&1 || exit $?
timeout -k 10 600 python scripts/gpu_ssd_ab.py > $OUT/ssd_ab.txt 2>&1 || exit $?
for r in 1 2; do
  for ns in 1 2 3 4; do
    for k in 20 200; do
      timeout -k 10 180 python bench.py --steps $k --warmup 5 --streams $ns --no-cpu-baseline --no-parity \
        > $OUT/bench_s${ns}_k${k}_r${r}.json 2> $OUT/bench_s${ns}_k${k}_r${r}.err || exit $?
    done
  done
done
tail -n 3 $OUT/pytest_ssd.txt
tail -n 8 $OUT/ssd_ab.txt
for f in $OUT/bench_s*.json; do python -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['ms_per_step']*1e3,2), 'us/step', round(d['kernel_ms']*1e3,2), 'kernel us', round(d['span_ms_per_step']*1e3,2),'span')"; done
