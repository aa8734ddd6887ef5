#!/usr/bin/env bash
# Round 4: ramped first / last chunks of the staged host pipeline (ISHMEM_STAGED_RAMP=1, default)
# against uniform 64 MiB chunks (=0), interleaved, the N=1 bench's host-memory legs (1 GiB, dest
# checked in full): pinned blocking, pinned on-stream back to back, pageable.
set -u
TAG="$1"; OUT=gpurun_out/$TAG; mkdir -p $OUT
for rep in 1 2 3; do
  for v in 0 1; do
    ISHMEM_STAGED_RAMP=$v timeout -k 10 240 python bench.py --steps 8 --warmup 2 --no-combine --no-cpu-baseline \
      > $OUT/b_ramp${v}_r$rep.json 2> $OUT/b_ramp${v}_r$rep.err || exit $?
    python -c "import json; d=json.load(open('$OUT/b_ramp${v}_r$rep.json')); e=d['e2e_host']; p=d['e2e_host_pageable']; print('ramp$v r$rep pinned %.2f b2b %.2f pageable %.2f b2b %.2f warm %s checked %s %s' % (e['value'], e.get('on_stream_back_to_back_GiBps', 0), p['value'], p.get('on_stream_back_to_back_GiBps', 0), e.get('warmup_GiBps_per_call'), e['checked'], p['checked']))" | tee -a $OUT/ab.txt
  done
done
