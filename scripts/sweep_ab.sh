#!/usr/bin/env bash
# Same-device size sweeps for A/B comparisons of the multi-PE kernel (dev tool).
# Usage: scripts/sweep_ab.sh TAG "NPES..." [MAX_MIB]
set -u
TAG="$1"; NPS="$2"; MAXMIB="${3:-1024}"
mkdir -p gpurun_out/$TAG
export HSA_ENABLE_IPC_MODE_LEGACY=0 ISHMEM_BENCH_SAME_DEVICE=1
for np_ in $NPS; do
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $np_ --master-addr 127.0.0.1 \
      --master-port $((29600 + np_)) tools/sweep.py --max-mib $MAXMIB > gpurun_out/$TAG/sweep$np_.log 2>&1 || exit $?
done
