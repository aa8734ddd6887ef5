#!/usr/bin/env bash
# A/B of the launch finish: flat single-line count for grids <= 64 (tree) vs sharded only
# (abtest_flat0/), 2 and 4 PEs on the one GPU, interleaved twice.  Dev tool.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/${1:-abfin}"
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0 ISHMEM_BENCH_SAME_DEVICE=1
cd "$R"
for rep in 1 2; do
  for np_ in 2 4; do
    for v in flat sharded; do
      sw=tools/sweep.py; [ "$v" = sharded ] && sw=abtest_flat0/tools/sweep.py
      timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $np_ --master-addr 127.0.0.1 \
        --master-port $((29700 + np_ + rep * 10)) $sw --max-mib 64 --min-bytes 262144 --factor 4 --iters 50 \
        > "$OUT/${v}_p${np_}_r$rep.csv" 2> "$OUT/${v}_p${np_}_r$rep.err" || { echo "rc=$? $v p$np_"; exit 1; }
    done
  done
done
echo done
