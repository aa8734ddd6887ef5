#!/usr/bin/env bash
# Round 5: multi-PE reduce with sources on another 16-B phase than dest (rs_phase_realign_kernel),
# 2 and 4 PEs on the one GPU, 16 MiB - 1 GiB, round-4 library (build/ab/libishmem_amd_r04.so) vs
# this tree, interleaved A B A B; aligned operands of this tree as the reference line.
set -u
OUT=gpurun_out/r05o; mkdir -p $OUT
for np_ in 2 4; do
  for rep in 1 2; do
    for v in r04 r05 aligned; do
      if [ $v = r04 ]; then export ISHMEM_AMD_LIB=$PWD/build/ab/libishmem_amd_r04.so; else unset ISHMEM_AMD_LIB; fi
      off="--src-offset 4"; [ $v = aligned ] && off=""
      ISHMEM_BENCH_SAME_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $np_ \
        --master-addr 127.0.0.1 --master-port 2961$np_ tools/sweep.py --min-bytes 16777216 --max-mib 1024 --factor 4 --iters 10 $off \
        > $OUT/p${np_}_${v}_r$rep.csv 2> $OUT/p${np_}_${v}_r$rep.err || exit $?
      echo "== p$np_ $v r$rep"; grep -v "^#\|Gloo" $OUT/p${np_}_${v}_r$rep.csv
    done
  done
done
