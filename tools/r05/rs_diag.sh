for b in noht nohtst; do
  TAUS=384 BIN=tools/ubench/rs_tile_$b bash tools/r05/rsprobe.sh | sed "s/^/$b /" || exit 1
done
