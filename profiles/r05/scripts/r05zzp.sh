#!/usr/bin/env bash
# Round 5: in-place reduces (source == dest) at 512 KiB - 32 MiB: the whole-array fold into the
# staging region + barrier + local copy (direct_inplace=1, default) against the persistent kernel /
# phased path (0), 2 and 4 PEs with one-PE-per-GPU launch shapes, granule path off, interleaved x2.
set -u
OUT=gpurun_out/r05zzp; mkdir -p $OUT
for rep in 1 2; do
  for np_ in 2 4; do
    for d in 1 0; do
      ISHMEM_LL_MAX_BYTES=0 ISHMEM_BENCH_SAME_DEVICE=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node $np_ \
        --master-addr 127.0.0.1 --master-port 29739 tools/sweep.py --inplace --min-bytes 524288 --max-mib 32 --factor 2 --iters 20 \
        --emulate-share1 --param direct_inplace=$d > $OUT/p${np_}_d${d}_r$rep.csv 2> $OUT/p${np_}_d${d}_r$rep.err || exit $?
      echo "p$np_ inplace direct_inplace=$d r$rep: $(grep -v 'Gloo\|peer ranks\|^#\|bytes' $OUT/p${np_}_d${d}_r$rep.csv | tr '\n' ' ')" | tee -a $OUT/ab.txt
    done
  done
done
