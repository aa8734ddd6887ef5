#!/usr/bin/env bash
# Round 5: small broadcasts on the granule path (kLLBroadcast) against the pull kernel
# (ISHMEM_LL_MAX_BYTES=0), 2 / 4 PEs with one-PE-per-GPU launch shapes, 1 KiB - 1 MiB.
set -u
OUT=gpurun_out/r05zz; mkdir -p $OUT
for np_ in 2 4; do
  for ll in 0 default; do
    if [ $ll = 0 ]; then export ISHMEM_LL_MAX_BYTES=0; else unset ISHMEM_LL_MAX_BYTES; fi
    ISHMEM_BENCH_SAME_DEVICE=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node $np_ \
      --master-addr 127.0.0.1 --master-port 29715 tools/sweep.py --coll broadcast --min-bytes 1024 --max-mib 1 --factor 4 --iters 50 \
      --emulate-share1 > $OUT/p${np_}_ll${ll}.csv 2> $OUT/p${np_}_ll${ll}.err || exit $?
    echo "p$np_ broadcast ll$ll: $(grep -v 'Gloo\|peer ranks\|^#\|bytes' $OUT/p${np_}_ll${ll}.csv | tr '\n' ' ')" | tee -a $OUT/ab.txt
  done
done
