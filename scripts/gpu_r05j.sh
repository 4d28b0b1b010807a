#!/bin/bash
# round 5: SSD grid/occupancy A/B, then bench.py with one vs two alternating streams (interleaved)
set -o pipefail
OUT=gpurun_out/r05j
mkdir -p $OUT
timeout -k 10 600 python scripts/gpu_ssd_ab.py > $OUT/ssd_ab.txt 2>&1 || exit $?
for r in 1 2; do
  for ns in 1 2; do
    timeout -k 10 180 python bench.py --steps 200 --warmup 20 --streams $ns --no-cpu-baseline --no-parity \
      > $OUT/bench_s${ns}_r${r}.json 2> $OUT/bench_s${ns}_r${r}.err || exit $?
  done
done
tail -n 40 $OUT/ssd_ab.txt
for f in $OUT/bench_s*.json; do python -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['ms_per_step']*1e3,2), 'us/step', round(d['kernel_ms']*1e3,2), 'kernel us', round(d['span_ms_per_step']*1e3,2),'span')"; done
