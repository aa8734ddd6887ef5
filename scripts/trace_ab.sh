#!/usr/bin/env bash
# Phase traces of the 2-PE kernel (same device) (dev tool; one run per argument).
set -u
TAG="$1"; shift
mkdir -p gpurun_out/$TAG
export HSA_ENABLE_IPC_MODE_LEGACY=0 ISHMEM_BENCH_SAME_DEVICE=1
for f in "$@"; do
  timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port 29801 tools/phase_trace.py --sizes ${SIZES:-4194304,4194304,4194304} \
      > gpurun_out/$TAG/trace_f$f.log 2>&1 || exit $?
done
