#!/usr/bin/env bash
# Host-memory leg: staging copies on the DMA engines (0) or by the copy kernel out (1), in (2),
# both (3) — tools/host_flavours_ab.py per setting, interleaved twice.
set -u
TAG="$1"; OUT=gpurun_out/$TAG; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 AB_ROUNDS=2 AB_KINDS=hostmalloc,registered,pageable
for rep in 1 2; do
  for v in 0 1 2 3; do
    ISHMEM_STAGED_COPY_KERNEL=$v timeout -k 10 150 python -u tools/host_flavours_ab.py \
      > $OUT/staged_copy_k${v}_r$rep.jsonl 2>&1 || exit $?
    echo "== staged_copy_kernel=$v rep$rep"; grep summary $OUT/staged_copy_k${v}_r$rep.jsonl | cut -c1-600
  done
done
