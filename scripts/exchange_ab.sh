#!/usr/bin/env bash
# Blocking fcollect / sum_inscan latency: the round-4 agreement exchange (one LL
# launch on host-mapped memory) against round 3's (H2D copy + fcollect launch + D2H copy, built as
# build/ab/libishmem_amd_exch_fcollect.so), 2 and 4 PEs on the one GPU, interleaved A B A B.
set -u
TAG="$1"; OUT=gpurun_out/$TAG; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 ISHMEM_BENCH_SAME_DEVICE=1 ISHMEM_TIMEOUT_MS=10000
for np_ in 2 4; do
  for coll in fcollect inscan; do
    for rep in 1 2; do
      for v in r4 r3; do
        if [ $v = r3 ]; then export ISHMEM_AMD_LIB=build/ab/libishmem_amd_exch_fcollect.so; else unset ISHMEM_AMD_LIB; fi
        timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node $np_ --master-addr 127.0.0.1 \
          --master-port 2976$np_ tools/sweep.py --blocking --coll $coll --max-mib 1 --min-bytes 8 --factor 8 \
          --iters 200 > $OUT/exch_${v}_${coll}_p${np_}_r$rep.csv 2> $OUT/exch_${v}_${coll}_p${np_}_r$rep.err || exit $?
        echo "== $v $coll p$np_ rep$rep"; grep -E "^[0-9]" $OUT/exch_${v}_${coll}_p${np_}_r$rep.csv | tr '\n' ' '; echo
      done
    done
  done
done
unset ISHMEM_AMD_LIB
