#!/bin/bash
# GPU box: bench.py's extra legs (pipeline, e2e, chains) for the in-tree library and every build_variants/*.so,
# interleaved ROUNDS times (no CPU baseline, no parity); prints the frame-stage legs and the host expansion.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out/leg_ab; mkdir -p $OUT
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in default $(ls build_variants/*.so 2>/dev/null | xargs -n1 basename 2>/dev/null | sed 's/\.so$//'); do
    lib=""; [ $v != default ] && lib=$PWD/build_variants/$v.so
    USV_LIB_PATH=$lib timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity \
        > $OUT/${v}_$r.json 2> $OUT/${v}_$r.err || { echo "FAILED $v $r"; tail -5 $OUT/${v}_$r.err; exit 1; }
    python3 - "$OUT/${v}_$r.json" "$v" "$r" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
p = d['pipeline']
print(sys.argv[2], sys.argv[3], {k: round(v['us'], 2) for k, v in p.items() if isinstance(v, dict)},
      'expand', round(d['e2e']['host_distance_expand_ms_16_threads'], 3), 'step', round(d['ms_per_step'] * 1e3, 2))
PY
  done
done
