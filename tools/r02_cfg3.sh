#!/bin/bash
# Round-2 config-3 session: parity (incl. 3F full size), 3F bench for the default build and the
# old chain geometry, kernel-trace summary of 3F. Each GPU step has its own limit; stop on failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$PWD"
mkdir -p gpurun_out/r02
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -k "not config2_full and not config5_full" > gpurun_out/r02/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r02/tests.log; [ $rc -ne 0 ] && exit $rc
for v in default ch8x8; do
  lib="$R/skyvault-rs_amd/skv/libskv.so"; [ $v != default ] && lib="$R/skyvault-rs_amd/skv/variants/libskv_$v.so"
  SKV_LIB=$lib timeout -k 10 300 python bench.py --config 3F --steps 3 --warmup 1 --no-cpu-baseline --no-host-path > gpurun_out/r02/cfg3F_$v.log 2>&1
  rc=$?; echo "3F $v rc=$rc"; tail -c 600 gpurun_out/r02/cfg3F_$v.log; echo; [ $rc -ne 0 ] && exit $rc
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r02/prof3F" -o run -- python3 "$R/bench.py" --config 3F --steps 2 --warmup 1 --no-cpu-baseline --no-host-path > "$R/gpurun_out/r02/prof3F.log" 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
