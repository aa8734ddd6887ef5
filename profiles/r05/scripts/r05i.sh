#!/usr/bin/env bash
# Round 5: realigned kernels (serial per-source issue, one-shot): parity, misaligned probe x3,
# then FETCH_SIZE / WRITE_SIZE passes over the 1 GiB probe (separate --pmc runs).
set -u
OUT=gpurun_out/r05i; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_single.py "tests/test_gpu_multi.py::test_phased_reduce_scatter_allgather_path" \
  "tests/test_gpu_multi.py::test_inplace_offsets_edges" > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 1; }
tail -2 $OUT/pytest.txt
for r in 1 2 3; do
  MISALIGNED_MIB=1024 timeout -k 10 120 python tools/misaligned_probe.py > $OUT/probe_r$r.json 2> $OUT/probe_r$r.err || exit $?
  python -c "import json; d=json.load(open('$OUT/probe_r$r.json')); print('r$r', ' '.join('%s=%.4f%s' % (k, v['ms'], '' if v.get('ok', True) else '!BAD') for k, v in d.items()))" | tee -a $OUT/probe.txt
done
MISALIGNED_MIB=1024 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python tools/misaligned_probe.py > $OUT/pmc_fetch.log 2>&1 || exit $?
MISALIGNED_MIB=1024 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python tools/misaligned_probe.py > $OUT/pmc_write.log 2>&1 || exit $?
find $OUT -name "*counter_collection.csv" | head
