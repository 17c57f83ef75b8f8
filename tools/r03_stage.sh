#!/bin/bash
# staged chunk walks: parity tests, then config 3 A/B (SKV_STAGE=0 vs auto) and a traced general
# host pipeline call (P = 8)
set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r03/stage_tests.log 2>&1 || { tail -30 gpurun_out/r03/stage_tests.log; exit 1; }
tail -2 gpurun_out/r03/stage_tests.log
for v in 0 1; do
  SKV_STAGE=$v timeout -k 10 300 python bench.py --config 3 --steps 10 --warmup 2 --no-cpu-baseline --no-host-path > gpurun_out/r03/stage_b3_$v.json 2> gpurun_out/r03/stage_b3_$v.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/r03/stage_b3_$v.json'));print('STAGE=$v', d['ms_per_step'], d['value'], d['phases_ms'])"
done
SKV_HOST_TRACE=1 timeout -k 10 300 python tools/hp_cfg3.py 8 > gpurun_out/r03/hp_trace.log 2>&1 || exit 1
grep -v "^\[skv host\]" gpurun_out/r03/hp_trace.log | tail -3
