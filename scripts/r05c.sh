#!/usr/bin/env bash
# Round 5: the 512-thread DPP + LDS realigned kernels (fan-in and phased reduce-scatter): parity,
# then the misaligned 1-PE copy / a + b at 1 GiB, three times.
set -u
OUT=gpurun_out/r05c; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_single.py "tests/test_gpu_multi.py::test_phased_reduce_scatter_allgather_path" \
  "tests/test_gpu_multi.py::test_inplace_offsets_edges" > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 1; }
tail -2 $OUT/pytest.txt
for r in 1 2 3; do
  MISALIGNED_MIB=1024 timeout -k 10 120 python tools/misaligned_probe.py > $OUT/probe_r$r.json 2> $OUT/probe_r$r.err || exit $?
  python -c "import json; d=json.load(open('$OUT/probe_r$r.json')); print('r$r', ' '.join('%s=%.4f%s' % (k, v['ms'], '' if v.get('ok', True) else '!BAD') for k, v in d.items()))" | tee -a $OUT/probe.txt
done
