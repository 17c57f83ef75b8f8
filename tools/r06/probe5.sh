#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R="$PWD"
for v in ${VARIANTS:-tp4 tp8 tp16}; do
  echo "== $v"
  SKV_LIB=$R/skyvault-rs_amd/skv/variants/libskv_$v.so timeout -k 10 300 python3 tools/r06/tileprof.py 16 2>&1 | grep -E "call 3|tile phase" || exit 1
done
