#!/usr/bin/env bash
# Round 5: sum_inscan at 512 KiB - 16 MiB: default paths (persistent scan kernel below 4 MiB) vs
# ISHMEM_PHASED_MIN_BYTES=0 (2 PEs: the direct fold between barriers; 3-4 PEs: the phased
# fold + pull grids), 2 / 3 / 4 PEs with one-PE-per-GPU launch shapes, interleaved x2.
set -u
OUT=gpurun_out/r05zz2; mkdir -p $OUT
for rep in 1 2; do
  for np_ in 2 3 4; do
    for pm in default 0; do
      if [ $pm = 0 ]; then export ISHMEM_PHASED_MIN_BYTES=0; else unset ISHMEM_PHASED_MIN_BYTES; fi
      ISHMEM_BENCH_SAME_DEVICE=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node $np_ \
        --master-addr 127.0.0.1 --master-port 29717 tools/sweep.py --coll inscan --min-bytes 524288 --max-mib 16 --factor 2 --iters 30 \
        --emulate-share1 > $OUT/p${np_}_pm${pm}_r$rep.csv 2> $OUT/p${np_}_pm${pm}_r$rep.err || exit $?
      echo "p$np_ inscan phased_min=$pm r$rep: $(grep -v 'Gloo\|peer ranks\|^#\|bytes' $OUT/p${np_}_pm${pm}_r$rep.csv | tr '\n' ' ')" | tee -a $OUT/ab.txt
    done
  done
done
