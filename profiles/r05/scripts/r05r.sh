#!/usr/bin/env bash
# Round 5: realigned reduce-scatter block size A/B (512 product / 256 / 64 / round-4 library),
# 2 PEs x 1 GiB, sources 4 B off dest's phase, phase times; aligned reference; parity of the
# product on the phased offsets scenarios first.
set -u
OUT=gpurun_out/${TAG:-r05r}; mkdir -p $OUT
true || timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  "tests/test_gpu_multi.py::test_phased_reduce_scatter_allgather_path" "tests/test_gpu_multi.py::test_inplace_offsets_edges" \
  > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
for rep in 1 2; do
  for v in rsr512 rsr64p0 rsr64p1 rsr512p1 aligned; do
    case $v in rsr512|aligned) unset ISHMEM_AMD_LIB;; r04) export ISHMEM_AMD_LIB=$PWD/build/ab/libishmem_amd_r04.so;;
      *) export ISHMEM_AMD_LIB=$PWD/build/ab/libishmem_amd_$v.so;; esac
    off=4; [ $v = aligned ] && off=0
    ISHMEM_BENCH_SAME_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port 29641 tools/sweep.py --min-bytes 1073741824 --max-mib 1024 --iters 10 \
      --src-offset $off --phases > $OUT/p2_${v}_r$rep.csv 2> $OUT/p2_${v}_r$rep.err || exit $?
    echo "$v r$rep $(grep -v 'Gloo\|peer ranks\|^#\|bytes' $OUT/p2_${v}_r$rep.csv | tr '\n' ' ') $(grep phases $OUT/p2_${v}_r$rep.csv)" | tee -a $OUT/ab.txt
  done
done
