#!/usr/bin/env bash
# Round 5: mid sizes (64 KiB - 16 MiB) with sources 4 B off dest's phase vs aligned, 2 PEs with
# one-PE-per-GPU launch shapes (persistent kernel below 4 MiB: element-granular when misaligned).
set -u
OUT=gpurun_out/r05zb; mkdir -p $OUT
for rep in 1 2; do
  for off in 0 4; do
    ISHMEM_BENCH_SAME_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port 29691 tools/sweep.py --min-bytes 65536 --max-mib 16 --factor 4 --iters 50 \
      --src-offset $off --emulate-share1 > $OUT/p2_off${off}_r$rep.csv 2> $OUT/p2_off${off}_r$rep.err || exit $?
    echo "off$off r$rep: $(grep -v 'Gloo\|peer ranks\|^#\|bytes' $OUT/p2_off${off}_r$rep.csv | tr '\n' ' ')" | tee -a $OUT/ab.txt
  done
done
