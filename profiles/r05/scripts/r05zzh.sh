#!/usr/bin/env bash
# Round 5: blocking host calls — hipStreamSynchronize (block_spin=0, default) against a host spin
# on a stream-written completion word (1: then hipStreamSynchronize; 2: the spin alone), 2 PEs with
# one-PE-per-GPU launch shapes, 8 B - 256 KiB, reduce and fcollect, interleaved x2.
set -u
OUT=gpurun_out/r05zzh; mkdir -p $OUT
for rep in 1 2; do
  for c in reduce fcollect; do
    for b in 0 1 2; do
      ISHMEM_BENCH_SAME_DEVICE=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port 29735 tools/sweep.py --coll $c --blocking --min-bytes 8 --max-mib 1 --factor 8 --iters 200 \
        --emulate-share1 --param block_spin=$b > $OUT/${c}_b${b}_r$rep.csv 2> $OUT/${c}_b${b}_r$rep.err || exit $?
      echo "p2 blocking $c block_spin=$b r$rep: $(grep -v 'Gloo\|peer ranks\|^#\|bytes' $OUT/${c}_b${b}_r$rep.csv | tr '\n' ' ')" | tee -a $OUT/ab.txt
    done
  done
done
