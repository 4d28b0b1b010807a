#!/bin/bash
# Interleaved A/B on the GPU box: each build_variants/*.so (and the in-tree
# default) benched ROUNDS times in rotation, so drift hits every variant alike.
# Prints kernel_ms (HIP events) per run, then the per-variant medians.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
ROUNDS=${ROUNDS:-3}
ARGS=${ARGS:---steps 200 --warmup 20 --no-cpu-baseline --extra-steps 0}
out=gpurun_out/ab.txt; : > $out
for r in $(seq $ROUNDS); do
  for v in default ${VARIANTS_DIR:-build_variants}/*.so; do
    n=$(basename $v .so)
    if [ "$v" = default ]; then lib=""; else lib=$PWD/$v; fi
    res=$(USV_LIB_PATH=$lib timeout -k 10 120 python bench.py $ARGS 2>/dev/null | tail -1)
    rc=$?
    if [ $rc -ne 0 ] || [ -z "$res" ]; then echo "FAILED $n rc=$rc"; exit 1; fi
    k=$(echo "$res" | python -c "import json,sys; d=json.load(sys.stdin); print(round(d['kernel_ms']*1e3,2), round(d['ms_per_step']*1e3,2))")
    echo "$r $n $k" | tee -a $out
  done
done
python - <<'PY'
import collections, statistics
d = collections.defaultdict(list)
for line in open("gpurun_out/ab.txt"):
    r, n, k, w = line.split()
    d[n].append((float(k), float(w)))
for n, v in sorted(d.items()):
    print(f"{n:14s} kernel median {statistics.median(x[0] for x in v):7.2f} us  step median {statistics.median(x[1] for x in v):7.2f} us  ({len(v)} runs)")
PY
