#!/bin/bash
# span opt-in test + a host-traced config-5 call (where the host time of a 10^6-stream call goes)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "span_parse" -x -q --timeout 200 --timeout-method thread > $O/span_test.log 2>&1 || { tail -30 $O/span_test.log; exit 1; }
tail -2 $O/span_test.log
SKV_HOST_TRACE=1 timeout -k 10 300 python -u bench.py --config 5 --steps 2 --warmup 1 --no-cpu-baseline --no-host-path > $O/c5trace.log 2>&1 || { tail -30 $O/c5trace.log; exit 1; }
tail -1 $O/c5trace.log | cut -c1-400
