#!/usr/bin/env bash
# Round 5: small-size latency of fcollect and inscan next to reduce (which has the granule path),
# 2 / 4 PEs with one-PE-per-GPU launch shapes, 1 KiB - 1 MiB per PE.
set -u
OUT=gpurun_out/r05zn; mkdir -p $OUT
for np_ in 2 4; do
  for c in reduce fcollect inscan; do
    ISHMEM_BENCH_SAME_DEVICE=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node $np_ \
      --master-addr 127.0.0.1 --master-port 29705 tools/sweep.py --coll $c --min-bytes 1024 --max-mib 1 --factor 4 --iters 50 \
      --emulate-share1 > $OUT/p${np_}_$c.csv 2> $OUT/p${np_}_$c.err || exit $?
    echo "p$np_ $c: $(grep -v 'Gloo\|peer ranks\|^#\|bytes' $OUT/p${np_}_$c.csv | tr '\n' ' ')" | tee -a $OUT/ab.txt
  done
done
