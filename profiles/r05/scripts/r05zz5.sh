#!/usr/bin/env bash
# Round 5: default paths of the final tree, 2 / 4 PEs with one-PE-per-GPU launch shapes,
# 4 KiB - 256 MiB (granule to 512 KiB, two-member whole-array fold to 32 MiB, phased above).
set -u
OUT=gpurun_out/r05zz5; mkdir -p $OUT
for np_ in 2 4; do
  ISHMEM_BENCH_SAME_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $np_ \
    --master-addr 127.0.0.1 --master-port 29721 tools/sweep.py --min-bytes 4096 --max-mib 256 --factor 2 --iters 20 \
    --emulate-share1 > $OUT/p${np_}.csv 2> $OUT/p${np_}.err || exit $?
  echo "p$np_: $(grep -v 'Gloo\|peer ranks\|^#\|bytes' $OUT/p${np_}.csv | tr '\n' ' ')" | tee -a $OUT/ab.txt
done
