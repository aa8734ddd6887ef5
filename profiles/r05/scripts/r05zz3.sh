#!/usr/bin/env bash
# Round 5: two-member reduces, 512 KiB - 256 MiB: barrier + whole-array fold grid + barrier
# (direct_p2=1, default) against the persistent kernel's one-shot mode below 4 MiB and the phased
# path from 4 MiB (direct_p2=0); one-PE-per-GPU launch shapes, sources aligned and 4 B off,
# interleaved x2.  oneshot_p2_max_bytes raised to 256 MiB so the direct path runs at every size.
set -u
OUT=gpurun_out/r05zz3; mkdir -p $OUT
for rep in 1 2; do
  for off in 0 4; do
    for d in 1 0; do
      ISHMEM_ONESHOT_P2_MAX_BYTES=256M ISHMEM_BENCH_SAME_DEVICE=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port 29719 tools/sweep.py --min-bytes 524288 --max-mib 256 --factor 2 --iters 20 \
        --src-offset $off --emulate-share1 --param direct_p2=$d > $OUT/off${off}_d${d}_r$rep.csv 2> $OUT/off${off}_d${d}_r$rep.err || exit $?
      echo "off$off direct$d r$rep: $(grep -v 'Gloo\|peer ranks\|^#\|bytes' $OUT/off${off}_d${d}_r$rep.csv | tr '\n' ' ')" | tee -a $OUT/ab.txt
    done
  done
done
