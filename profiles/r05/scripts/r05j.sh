#!/usr/bin/env bash
# Round 5: the stream-memory-op team barrier (ISHMEM_BARRIER_KIND=stream): parity at 2 / 3 / 8 PEs,
# then per-call us of the phased path at 1-16 MiB with each barrier kind, 2 PEs with one-PE-per-GPU
# launch shapes, interleaved A B A B.
set -u
OUT=gpurun_out/r05j; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -p no:cacheprovider -m gpu \
  "tests/test_gpu_multi.py::test_phased_path_with_stream_memop_barriers" > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 1; }
tail -2 $OUT/pytest.txt
for rep in 1 2; do
  for kind in kernel stream; do
    ISHMEM_BENCH_SAME_DEVICE=1 ISHMEM_BARRIER_KIND=$kind ISHMEM_PHASED_MIN_BYTES=0 timeout -k 10 180 \
      python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 \
      tools/sweep.py --min-bytes 1048576 --max-mib 16 --factor 2 --iters 50 --emulate-share1 > $OUT/sweep_${kind}_r$rep.csv 2> $OUT/sweep_${kind}_r$rep.err || exit $?
    echo "== $kind r$rep"; grep -v "^#" $OUT/sweep_${kind}_r$rep.csv
  done
done
