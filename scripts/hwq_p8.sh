#!/usr/bin/env bash
# 8 PEs as processes on the one GPU: small-message latency with the default hardware queues per
# process and with GPU_MAX_HW_QUEUES=1 / 2 (co-location effect: queues across processes vs the
# scheduler's mapped set).  Each run bounded; stops at the first failure.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/${1:-hwq}"
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0 ISHMEM_BENCH_SAME_DEVICE=1 ISHMEM_MAX_BLOCKS=64
cd "$R"
for q in default 1 2; do
  if [ "$q" = default ]; then unset GPU_MAX_HW_QUEUES; else export GPU_MAX_HW_QUEUES=$q; fi
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
    --master-port $((29610 + ${q/default/0})) tools/sweep.py --max-mib 4 --min-bytes 4096 --factor 4 --iters 50 \
    > "$OUT/p8_hwq_$q.csv" 2> "$OUT/p8_hwq_$q.err" || { echo "rc=$? at q=$q"; exit 1; }
done
echo done
