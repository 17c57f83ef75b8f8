#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R="$PWD"
SKV_LIB=$R/skyvault-rs_amd/skv/variants/libskv_tprof.so timeout -k 10 300 python3 tools/r06/tileprof.py 16 2>&1 | grep -E "call|tile phase" || exit 1
bash tools/r06/probe2.sh
