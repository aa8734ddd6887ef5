#!/usr/bin/env bash
# Round 5: the whole-array fold between barriers for 3- and 4-member teams (set_param
# direct_max_pes=4, oneshot_p2_max_bytes raised) against the default paths (persistent below 4 MiB,
# phased above), one-PE-per-GPU launch shapes, 512 KiB - 32 MiB, interleaved x2.
set -u
OUT=gpurun_out/r05zz8; mkdir -p $OUT
for rep in 1 2; do
  for np_ in 3 4; do
    for d in 2 4; do
      ISHMEM_ONESHOT_P2_MAX_BYTES=64M ISHMEM_BENCH_SAME_DEVICE=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node $np_ \
        --master-addr 127.0.0.1 --master-port 29725 tools/sweep.py --min-bytes 524288 --max-mib 32 --factor 2 --iters 20 \
        --emulate-share1 --param direct_max_pes=$d > $OUT/p${np_}_d${d}_r$rep.csv 2> $OUT/p${np_}_d${d}_r$rep.err || exit $?
      echo "p$np_ direct_max_pes=$d r$rep: $(grep -v 'Gloo\|peer ranks\|^#\|bytes' $OUT/p${np_}_d${d}_r$rep.csv | tr '\n' ' ')" | tee -a $OUT/ab.txt
    done
  done
done
