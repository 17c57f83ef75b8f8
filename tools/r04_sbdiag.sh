#!/bin/bash
# k_sort_bucket timing diagnostics (tools/build_variants_r04.sh sbdiag) on config 5: the kernel trace
# shows k_sort_bucket<D> per skipped part next to the product kernel k_sort_bucket<0>.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$PWD"
O="$R/gpurun_out/r04"
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_sort.py -m gpu -x -q --timeout 120 --timeout-method thread > "$O/sbdiag_tests.log" 2>&1 \
  || { tail -20 "$O/sbdiag_tests.log"; exit 1; }
tail -1 "$O/sbdiag_tests.log"
cd /tmp
SKV_LIB="$R/skyvault-rs_amd/skv/variants/libskv_sbdiag.so" timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
  -d "$O/sbdiag_prof" -o run -- python3 "$R/bench.py" --config 5 --steps 2 --warmup 1 --no-cpu-baseline --no-host-path \
  > "$O/sbdiag_bench.log" 2>&1 || { tail -5 "$O/sbdiag_bench.log"; exit 1; }
cd "$R"
cp "$(ls $O/sbdiag_prof/*kernel_stats.csv | head -1)" "$O/sbdiag_stats.csv"
rm -rf "$O/sbdiag_prof"
grep -E "k_sort_bucket|k_sort_tile|k_sort_scatter" "$O/sbdiag_stats.csv" | cut -d, -f1-5
