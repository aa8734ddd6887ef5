#!/usr/bin/env bash
# Round 4: does the gap between consecutive 1 GiB operands (dest placed `gap` bytes past the end of
# the source) change the copy / a + b rate?  The product shapes of tools/stream_variants.hip,
# interleaved over the gaps, two passes.  Usage: scripts/layout_gap_ab.sh TAG
set -u
TAG="$1"
OUT=gpurun_out/$TAG
mkdir -p $OUT
for rep in 1 2; do
  for gap in 0 256 4096 8192 65536 1048576 3145728; do
    echo "== rep $rep gap $gap" >> $OUT/layout_gap.txt
    timeout -k 10 60 build/stream_variants 7 prod dskew:$gap >> $OUT/layout_gap.txt 2>&1 || exit $?
  done
done
cat $OUT/layout_gap.txt
