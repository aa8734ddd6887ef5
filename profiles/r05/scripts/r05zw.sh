#!/usr/bin/env bash
# Round 5: granule ring layout — items grouped by 64 so each granule store / poll of a wave covers
# 512 contiguous bytes (product) against the paired layout (item i at granules 2i, 2i+1;
# build/ab/libishmem_amd_llpaired.so, -DISHMEMI_LL_PAIRED=1), 2 / 4 PEs with one-PE-per-GPU launch
# shapes, 16 KiB - 512 KiB, interleaved x2.
set -u
OUT=gpurun_out/r05zw; mkdir -p $OUT
for rep in 1 2; do
  for np_ in 2 4; do
    for lay in wave paired; do
      if [ $lay = paired ]; then export ISHMEM_AMD_LIB=$PWD/build/ab/libishmem_amd_llpaired.so; else unset ISHMEM_AMD_LIB; fi
      ISHMEM_BENCH_SAME_DEVICE=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node $np_ \
        --master-addr 127.0.0.1 --master-port 29713 tools/sweep.py --min-bytes 16384 --max-mib 1 --factor 2 --iters 100 \
        --emulate-share1 > $OUT/p${np_}_${lay}_r$rep.csv 2> $OUT/p${np_}_${lay}_r$rep.err || exit $?
      echo "p$np_ $lay r$rep: $(grep -v 'Gloo\|peer ranks\|^#\|bytes' $OUT/p${np_}_${lay}_r$rep.csv | tr '\n' ' ')" | tee -a $OUT/ab.txt
    done
  done
done
