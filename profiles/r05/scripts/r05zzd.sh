#!/usr/bin/env bash
# Round 5: granule path vs the whole-array fold at 256 KiB - 1 MiB for 3 / 4 PEs (ll_max_bytes
# 512 KiB, the default, against 256 KiB), reduce and inscan, one-PE-per-GPU launch shapes,
# interleaved x2.
set -u
OUT=gpurun_out/r05zzd; mkdir -p $OUT
for rep in 1 2; do
  for np_ in 3 4; do
    for c in reduce inscan; do
      for ll in 524288 262144; do
        ISHMEM_BENCH_SAME_DEVICE=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node $np_ \
          --master-addr 127.0.0.1 --master-port 29731 tools/sweep.py --coll $c --min-bytes 131072 --max-mib 1 --factor 2 --iters 50 \
          --emulate-share1 --param ll_max_bytes=$ll > $OUT/p${np_}_${c}_ll${ll}_r$rep.csv 2> $OUT/p${np_}_${c}_ll${ll}_r$rep.err || exit $?
        echo "p$np_ $c ll_max=$ll r$rep: $(grep -v 'Gloo\|peer ranks\|^#\|bytes' $OUT/p${np_}_${c}_ll${ll}_r$rep.csv | tr '\n' ' ')" | tee -a $OUT/ab.txt
      done
    done
  done
done
