#!/usr/bin/env bash
# Round 5: sum_inscan at 3 / 4 PEs, 512 KiB - 8 MiB, after the direct fold was opened to 3- and
# 4-member teams ((p - 1) * B <= 8 MiB); one-PE-per-GPU launch shapes.  Before: profiles/r05/scan/
# ab_direct_vs_scratch.txt (phased_min=default rows).
set -u
OUT=gpurun_out/r05zzb; mkdir -p $OUT
for np_ in 3 4; do
  ISHMEM_BENCH_SAME_DEVICE=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node $np_ \
    --master-addr 127.0.0.1 --master-port 29729 tools/sweep.py --coll inscan --min-bytes 524288 --max-mib 8 --factor 2 --iters 30 \
    --emulate-share1 > $OUT/p${np_}.csv 2> $OUT/p${np_}.err || exit $?
  echo "p$np_ inscan: $(grep -v 'Gloo\|peer ranks\|^#\|bytes' $OUT/p${np_}.csv | tr '\n' ' ')" | tee -a $OUT/ab.txt
done
