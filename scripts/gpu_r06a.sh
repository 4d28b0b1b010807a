cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r06a; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_ssd_matrix.py tests/test_streaming.py tests/test_gpu_contours.py tests/test_gpu_parity.py tests/test_sharding.py  -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d.get('kernel_ms'), d.get('fallbacks',{}).get('ssd_matrix'))"
