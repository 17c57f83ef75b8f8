#!/bin/bash
# Kernel-trace summary of one bench configuration: CONFIG (2A/2B/3/3F/5), TAG (output name).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$PWD"
mkdir -p gpurun_out/r02
export TMPDIR=/tmp
cd /tmp
timeout -k 10 ${LIMIT:-300} rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r02/prof_${TAG}" -o run -- python3 "$R/bench.py" \
  --config ${CONFIG} --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline --no-host-path ${ARGS:-} > "$R/gpurun_out/r02/prof_${TAG}.log" 2>&1
rc=$?; echo "prof rc=$rc"; tail -c 400 "$R/gpurun_out/r02/prof_${TAG}.log"; exit $rc
