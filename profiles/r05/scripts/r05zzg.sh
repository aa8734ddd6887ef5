#!/usr/bin/env bash
# Round 5: blocking host calls (ishmem_float_sum_reduce / fcollectmem / sum_inscan / broadcastmem),
# host clock per call, 2 PEs with one-PE-per-GPU launch shapes, 8 B - 256 KiB.
set -u
OUT=gpurun_out/r05zzg; mkdir -p $OUT
for c in reduce fcollect inscan broadcast; do
  ISHMEM_BENCH_SAME_DEVICE=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29733 tools/sweep.py --coll $c --blocking --min-bytes 8 --max-mib 1 --factor 8 --iters 200 \
    --emulate-share1 > $OUT/p2_$c.csv 2> $OUT/p2_$c.err || exit $?
  echo "p2 blocking $c: $(grep -v 'Gloo\|peer ranks\|^#\|bytes' $OUT/p2_$c.csv | tr '\n' ' ')" | tee -a $OUT/ab.txt
done
