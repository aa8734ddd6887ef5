#!/usr/bin/env bash
# Size sweep of the reduce paths at 2 and 4 PEs sharing the one GPU: default (LL / two-member
# one-shot fold / persistent / phased by size), phased forced (no one-shot fold), persistent only.
set -u
TAG="$1"; OUT=gpurun_out/$TAG; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 ISHMEM_BENCH_SAME_DEVICE=1
for np_ in 2 4; do
  for v in default phased persistent; do
    case $v in
      default) unset ISHMEM_PHASED_MIN_BYTES ISHMEM_ONESHOT_P2_MAX_BYTES ;;
      phased) export ISHMEM_PHASED_MIN_BYTES=0 ISHMEM_ONESHOT_P2_MAX_BYTES=0 ;;
      persistent) export ISHMEM_PHASED_MIN_BYTES=-1 ISHMEM_ONESHOT_P2_MAX_BYTES=0 ;;
    esac
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $np_ --master-addr 127.0.0.1 \
      --master-port 2964$np_ tools/sweep.py --max-mib 256 --min-bytes 4194304 --factor 2 --iters 30 \
      > $OUT/sweep_${v}_p$np_.csv 2> $OUT/sweep_${v}_p$np_.err || exit $?
    echo "== $v p$np_"; grep -E "^[0-9]" $OUT/sweep_${v}_p$np_.csv
  done
done
