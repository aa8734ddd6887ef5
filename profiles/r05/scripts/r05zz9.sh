#!/usr/bin/env bash
# Round 5: default paths after the 3-/4-member whole-array fold (direct_max_pes=4), 3 / 4 PEs with
# one-PE-per-GPU launch shapes, 512 KiB - 32 MiB.
set -u
OUT=gpurun_out/r05zz9; mkdir -p $OUT
for np_ in 3 4; do
  ISHMEM_BENCH_SAME_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $np_ \
    --master-addr 127.0.0.1 --master-port 29727 tools/sweep.py --min-bytes 524288 --max-mib 32 --factor 2 --iters 20 \
    --emulate-share1 > $OUT/p${np_}.csv 2> $OUT/p${np_}.err || exit $?
  echo "p$np_: $(grep -v 'Gloo\|peer ranks\|^#\|bytes' $OUT/p${np_}.csv | tr '\n' ' ')" | tee -a $OUT/ab.txt
done
