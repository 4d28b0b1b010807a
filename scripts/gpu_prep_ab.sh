#!/bin/bash
# GPU box: frame-prep and rectification parity, then kernel traces of scripts/prof_prep.py for the in-tree library
# and every build_variants/*.so, interleaved twice.  Summaries: gpurun_out/prep_ab/<variant>_<round>/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/prep_ab; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_preproc.py tests/test_rectify.py -m gpu \
    > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 1; }
tail -2 $OUT/pytest.txt
for r in 1 2; do
  for v in default $(ls build_variants/*.so 2>/dev/null | xargs -n1 basename 2>/dev/null | sed 's/\.so$//'); do
    lib=""; [ $v != default ] && lib=$PWD/build_variants/$v.so
    USV_LIB_PATH=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/${v}_$r -o t --output-format csv \
        -- python3 scripts/prof_prep.py 200 > $OUT/${v}_$r.log 2>&1 || { echo "FAILED $v $r"; exit 1; }
  done
done
python3 - <<'PY'
import csv, glob
for f in sorted(glob.glob('gpurun_out/prep_ab/*/**/*kernel_trace.csv', recursive=True)):
    rows = list(csv.DictReader(open(f)))
    by = {}
    for r in rows:
        n = r['Kernel_Name']
        if not any(k in n for k in ('hist', 'equalize', 'remap')):
            continue
        key = (n.split('(')[0].split('::')[-1][:28], int(r.get('Grid_Size_X', r.get('Grid_Size', 0)) or 0))
        by.setdefault(key, []).append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
    print(f.split('/')[2])
    for k, v in sorted(by.items()):
        v = sorted(v)
        print('   %-30s grid %8d  n %4d  median %.2f us  min %.2f' % (k[0], k[1], len(v), v[len(v) // 2], v[0]))
PY
