#!/usr/bin/env bash
# Round 5: the one-wave realigned reduce-scatter (default) — parity on the phased / offsets /
# stream-barrier / timeout tests, then 2 and 4 PEs x 1 GiB misaligned vs aligned.
set -u
OUT=gpurun_out/r05t; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_multi.py \
  -k "phased or inplace or missing or stream_memop or config3" > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
for np_ in 2 4; do
  for off in 4 0; do
    ISHMEM_BENCH_SAME_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $np_ \
      --master-addr 127.0.0.1 --master-port 2965$np_ tools/sweep.py --min-bytes 16777216 --max-mib 1024 --iters 10 \
      --src-offset $off --phases > $OUT/p${np_}_off$off.csv 2> $OUT/p${np_}_off$off.err || exit $?
    echo "p$np_ off$off $(grep -v 'Gloo\|peer ranks\|^#\|bytes' $OUT/p${np_}_off$off.csv | tr '\n' ' ') $(grep phases $OUT/p${np_}_off$off.csv)" | tee -a $OUT/ab.txt
  done
done
