#!/usr/bin/env bash
# Round 5: where the misaligned 2-PE phased reduce loses (phase times, 1 GiB), aligned vs src+4.
set -u
OUT=gpurun_out/r05q; mkdir -p $OUT
for rep in 1 2; do
  for off in 0 4; do
    ISHMEM_BENCH_SAME_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port 29631 tools/sweep.py --min-bytes 1073741824 --max-mib 1024 --iters 10 \
      --src-offset $off --phases > $OUT/p2_off${off}_r$rep.csv 2> $OUT/p2_off${off}_r$rep.err || exit $?
    echo "== off $off r$rep"; grep -v "Gloo\|peer ranks" $OUT/p2_off${off}_r$rep.csv
  done
done
