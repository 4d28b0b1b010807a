#!/bin/bash
# GPU box: FETCH_SIZE / WRITE_SIZE calibration (scripts/probes/traffic_probe.hip, prebuilt as
# scripts/probes/bin_traffic_probe): kernel trace, then one --pmc pass per counter, each under its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/traffic
mkdir -p $OUT
timeout -k 10 60 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace --output-format csv -- scripts/probes/bin_traffic_probe > $OUT/trace.log 2>&1 || { echo "trace failed"; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o fetch --output-format csv -- scripts/probes/bin_traffic_probe > $OUT/fetch.log 2>&1 || { echo "fetch pass failed"; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o write --output-format csv -- scripts/probes/bin_traffic_probe > $OUT/write.log 2>&1 || { echo "write pass failed"; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum -d $OUT/rdreq -o rdreq --output-format csv -- scripts/probes/bin_traffic_probe > $OUT/rdreq.log 2>&1 || echo "rdreq pass failed (optional)"
find $OUT -name "*.csv"
exit 0
