#!/usr/bin/env bash
# Round 5: persistent kernel with the source 4 B off dest's phase, 64 KiB - 16 MiB, 2 PEs with
# one-PE-per-GPU launch shapes: shifted-source vector items (ar_shifted=1) against the
# element-granular instantiation (ar_shifted=0) and the aligned call.
set -u
OUT=gpurun_out/r05zd; mkdir -p $OUT
for rep in 1 2; do
  for cfg in "0 1" "4 1" "4 0"; do
    set -- $cfg; off=$1; sh=$2
    ISHMEM_BENCH_SAME_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port 29691 tools/sweep.py --min-bytes 65536 --max-mib 16 --factor 4 --iters 50 \
      --src-offset $off --emulate-share1 --param ar_shifted=$sh > $OUT/p2_off${off}_sh${sh}_r$rep.csv 2> $OUT/p2_off${off}_sh${sh}_r$rep.err || exit $?
    echo "off$off sh$sh r$rep: $(grep -v 'Gloo\|peer ranks\|^#\|bytes' $OUT/p2_off${off}_sh${sh}_r$rep.csv | tr '\n' ' ')" | tee -a $OUT/ab.txt
  done
done
