#!/usr/bin/env bash
# Round 5: the product library with the granule ring laid out by team size (capacity 1 MiB / p,
# the default threshold) against the persistent kernel (ISHMEM_LL_MAX_BYTES=0), 2 / 3 / 4 PEs with
# one-PE-per-GPU launch shapes, 16 KiB - 1 MiB.
set -u
OUT=gpurun_out/r05zi; mkdir -p $OUT
for np_ in 2 3 4; do
  for ll in 0 default; do
    if [ $ll = 0 ]; then export ISHMEM_LL_MAX_BYTES=0; else unset ISHMEM_LL_MAX_BYTES; fi
    ISHMEM_BENCH_SAME_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $np_ \
      --master-addr 127.0.0.1 --master-port 29697 tools/sweep.py --min-bytes 16384 --max-mib 1 --factor 2 --iters 50 \
      --emulate-share1 > $OUT/p${np_}_ll${ll}.csv 2> $OUT/p${np_}_ll${ll}.err || exit $?
    echo "p$np_ ll$ll: $(grep -v 'Gloo\|peer ranks\|^#\|bytes' $OUT/p${np_}_ll${ll}.csv | tr '\n' ' ')" | tee -a $OUT/ab.txt
  done
done
