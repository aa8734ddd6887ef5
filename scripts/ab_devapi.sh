#!/usr/bin/env bash
# Device-API work-group reduce, member-batched loads (default build) vs the round-2 shape
# (build/ab/reduce_bw_old: -DISHMEMX_DEV_MEMBER_BATCH=1 -DISHMEMX_DEV_AG_UNROLL=4), interleaved.
set -u
TAG="$1"; OUT=gpurun_out/$TAG; mkdir -p $OUT
for rep in 1 2; do
  for v in new old; do
    if [ $v = new ]; then EXE=build/reduce_bw; else EXE=build/ab/reduce_bw_old; fi
    EXE=$EXE bash scripts/reduce_bw_p2.sh 1048576 $OUT/bw_${v}_r$rep.csv || exit $?
    echo "== $v r$rep"; grep -E "device_grp1|device_subgroup" $OUT/bw_${v}_r$rep.csv | awk -F, '$10>=1048576' | cut -d, -f7,9,10,12,13
  done
done
