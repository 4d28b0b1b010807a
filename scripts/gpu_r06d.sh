#!/bin/bash
# GPU box (round 6): K = 16 variants (parity + interleaved A/B at config C), then PMC passes of config E on the
# product library (scripts/gpu_profiles.sh) and the warm SSD matrix-kernel profile (scripts/gpu_pmc_ssd.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
TAG=r06d NO_TESTS=1 VARIANT_TESTS="${VT:-k16ra4}" bash scripts/gpu_r06b.sh || exit 1
[ -n "$NO_PROF" ] && exit 0
echo "=== E profile ($(date +%T))"
CONFIGS=E bash scripts/gpu_profiles.sh ${PTAG:-r06} > gpurun_out/r06d/prof_E.log 2>&1 || { tail -5 gpurun_out/r06d/prof_E.log; exit 1; }
echo "=== SSD profile ($(date +%T))"
TAG=${PTAG:-r06}_ssd16 bash scripts/gpu_pmc_ssd.sh > gpurun_out/r06d/prof_ssd.log 2>&1 || { tail -5 gpurun_out/r06d/prof_ssd.log; exit 1; }
tail -20 gpurun_out/r06d/prof_ssd.log
exit 0
