#!/usr/bin/env bash
# Round 5: granule ring of 8 MiB per team (capacity 2 MiB / p, default threshold 512 KiB) against
# the persistent kernel (ISHMEM_LL_MAX_BYTES=0), 2 / 3 / 4 PEs with one-PE-per-GPU launch shapes,
# 128 KiB - 1 MiB, interleaved x2.
set -u
OUT=gpurun_out/r05zr; mkdir -p $OUT
for rep in 1 2; do
  for np_ in 2 3 4; do
    for ll in 0 default; do
      if [ $ll = 0 ]; then export ISHMEM_LL_MAX_BYTES=0; else unset ISHMEM_LL_MAX_BYTES; fi
      ISHMEM_BENCH_SAME_DEVICE=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node $np_ \
        --master-addr 127.0.0.1 --master-port 29709 tools/sweep.py --min-bytes 131072 --max-mib 1 --factor 2 --iters 50 \
        --emulate-share1 > $OUT/p${np_}_ll${ll}_r$rep.csv 2> $OUT/p${np_}_ll${ll}_r$rep.err || exit $?
      echo "p$np_ ll$ll r$rep: $(grep -v 'Gloo\|peer ranks\|^#\|bytes' $OUT/p${np_}_ll${ll}_r$rep.csv | tr '\n' ' ')" | tee -a $OUT/ab.txt
    done
  done
done
