#!/usr/bin/env bash
# Round 5: granule (LL) path past 64 KiB — an A/B build with 1 MiB rings
# (-DISHMEMI_LL_MAX_BYTES=1048576, build/ab/libishmem_amd_ll1m.so) — against the persistent kernel
# for the same sizes (ISHMEM_LL_MAX_BYTES=0), 2 / 4 / 8 PEs with one-PE-per-GPU launch shapes,
# 16 KiB - 1 MiB, interleaved x2.
set -u
OUT=gpurun_out/r05zh; mkdir -p $OUT
export ISHMEM_AMD_LIB=$PWD/build/ab/libishmem_amd_ll1m.so
for rep in 1 2; do
  for np_ in 2 4 8; do
    for ll in 0 1M; do
      ISHMEM_LL_MAX_BYTES=$ll ISHMEM_BENCH_SAME_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $np_ \
        --master-addr 127.0.0.1 --master-port 29695 tools/sweep.py --min-bytes 16384 --max-mib 1 --factor 2 --iters 50 \
        --emulate-share1 > $OUT/p${np_}_ll${ll}_r$rep.csv 2> $OUT/p${np_}_ll${ll}_r$rep.err || exit $?
      echo "p$np_ ll$ll r$rep: $(grep -v 'Gloo\|peer ranks\|^#\|bytes' $OUT/p${np_}_ll${ll}_r$rep.csv | tr '\n' ' ')" | tee -a $OUT/ab.txt
    done
  done
done
