#!/bin/bash
# Builds the round-4 measurement variants of libskv.so (skv/variants/libskv_<tag>.so) from the
# current sources, one object directory per tag (skyvault-rs_amd/Makefile `variant`). CPU only.
#   diag3    k_fx_tile copy-only diagnostic (no key phase; wrong output)
#   diag4    k_fx_tile keys from a compact (hi, lo) array (k_fx_keys) instead of the record lines
#   u1, u1w8 k_fx_tile unroll 1 / unroll 1 with 8 waves (occupancy A/B)
#   cap1024  fused tiles of 1024 records
#   tile2k   general merge tiles of 2048 elements, 512 threads (2 workgroups per CU)
#   seg512, seg1024  k_gather segments of 512 / 1024 records
#   span8k, span32k  span parse spans of 8 / 32 KiB (128 / 512 threads)
#   sbtop256, sbtop2048, sbper8, sbper32  record-sort bucket search: LDS top-level entries, elements per thread
#   sortprof  the record sort's phase ticks (SKV_SORT_PROF_PRINT=1 prints them; diagnostic)
#   t512     general merge tiles of 4096 elements on 512 threads (8 per thread)
#   sbatom2  record-sort bucket pass with a second returning atomic per element (diagnostic: their cost)
#   sortlds  record-sort bucket network in LDS (the round-3 form) instead of registers
#   sbilp2   record-sort bucket pass searching 2 elements per thread at once (fewer registers)
#   sbdiag   record-sort bucket pass timing diagnostics: k_sort_bucket<D> launches with parts skipped
#   sa8, sa32, sbb4, sbb16  two-pass bucketing: elements per thread of pass A / pass B (default 16 / 8)
#   ov12, ov20  record sort: samples per bucket (default 16: 768-element buckets)
#   ev32, ev24  record sort: one sample per 32 / 24 elements (24 / 32 per bucket: the same 768 target)
#   tie4, tie8, tie16, tie64  bucket sort: longest tie run sorted by one thread (default 8)
#   tileprof merge-tile phase ticks (printed when the ctx is destroyed; diagnostic)
#   gu4, gu1, gnt0, gpage  k_gather: 4 / 1 blocks per lane in flight, plain stores, the page gather
set -eu
cd "$(dirname "$0")/../skyvault-rs_amd"
J=${J:-8}
declare -A F=(
  [diag3]="-DSKV_FX_DIAG=3"
  [diag4]="-DSKV_FX_DIAG=4"
  [u1]="-DSKV_FX_U=1"
  [u1w8]="-DSKV_FX_U=1 -DSKV_FX_WAVES=8"
  [cap1024]="-DSKV_FX_CAP=1024"
  [tile2k]="-DSKV_TILE_CAP=2048 -DSKV_TILE_TARGET=1536 -DSKV_TILE_THREADS=512"
  [seg512]="-DSKV_GATHER_SEG=512"
  [seg1024]="-DSKV_GATHER_SEG=1024"
  [span8k]="-DSKV_SPAN_BYTES=8192"
  [span32k]="-DSKV_SPAN_BYTES=32768"
  [sbtop256]="-DSKV_SB_TOP=256"
  [sbtop2048]="-DSKV_SB_TOP=2048"
  [sbper8]="-DSKV_SB_PER=8"
  [sbper32]="-DSKV_SB_PER=32"
  [sortprof]="-DSKV_SORT_PROF=1"
  [t512]="-DSKV_TILE_THREADS=512"
  [sbatom2]="-DSKV_SB_ATOM2=1"
  [sortlds]="-DSKV_SORT_REGS=0"
  [sbilp2]="-DSKV_SB_ILP=2"
  [sbdiag]="-DSKV_SB_DIAGK=1"
  [sa8]="-DSKV_SA_PER=8"
  [sa32]="-DSKV_SA_PER=32"
  [sbb4]="-DSKV_SBB_PER=4"
  [sbb16]="-DSKV_SBB_PER=16"
  [ov12]="-DSKV_SORT_OV=12"
  [ov20]="-DSKV_SORT_OV=20"
  [tileprof]="-DSKV_TILE_PROF=1"
  [ev32]="-DSKV_SORT_EVERY=32 -DSKV_SORT_OV=24"
  [ev24]="-DSKV_SORT_EVERY=24 -DSKV_SORT_OV=32"
  [tie4]="-DSKV_SORT_TIE_MAX=4"
  [tie8]="-DSKV_SORT_TIE_MAX=8"
  [tie16]="-DSKV_SORT_TIE_MAX=16"
  [tie64]="-DSKV_SORT_TIE_MAX=64"
  [gu4]="-DSKV_GATHER_U=4"
  [gu1]="-DSKV_GATHER_U=1"
  [gnt0]="-DSKV_GATHER_NT=0"
  [gpage]="-DSKV_PAGE_GATHER=1"
)
for tag in ${TAGS:-${!F[@]}}; do
  make -s -j"$J" variant TAG="$tag" VFLAGS="${F[$tag]}"
  echo "built skv/variants/libskv_$tag.so (${F[$tag]})"
done
