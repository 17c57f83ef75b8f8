#!/bin/bash
# Config-5 host entry (10^6 pinned WAL runs) under pipeline knobs; traces in gpurun_out/r05/c5/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05/c5; mkdir -p $O
run() {  # tag env...
  local tag=$1; shift
  env "$@" SKV_HOST_TRACE=1 timeout -k 10 200 python tools/r05/c5host.py 1000000 table > $O/$tag.log 2>&1 || { echo "$tag failed"; tail -3 $O/$tag.log; return 1; }
  echo "$tag: $(grep 'rep 2' $O/$tag.log)"
}
run serial SKV_HOST_PIPE=0 && run base X=1 && run thr16 SKV_HOST_THREADS=16 && run ig128 SKV_INGEST_BLOCKS=128 && \
run ig1024 SKV_INGEST_BLOCKS=1024 && run wg SKV_INGEST_WG=1 && run p6 SKV_HOST_PARTS=6
grep gpipe $O/base.log | tail -11
