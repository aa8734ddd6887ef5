#!/usr/bin/env bash
# Round 5 first GPU call: realign variants microbench (k = 4, 12, 1 B) and the tests the round's
# first changes touch (IPC-mode default, test-hooks library, device checker at configs[4]).
set -u
OUT=gpurun_out/r05a; mkdir -p $OUT
for k in 4 12 1; do
  timeout -k 10 120 ./tools/bin/realign_variants 1024 3 10 $k > $OUT/rv_k$k.txt 2>&1 || exit $?
done
timeout -k 10 60 ./tools/bin/streamop_probe 2000 > $OUT/streamop.txt 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_examples.py tests/test_gpu_multi.py::test_coarse_grained_flags_across_devices_refused_at_init \
  "tests/test_gpu_multi.py::test_all_ops_types_vs_oracle_and_mpich_golden" \
  "tests/test_gpu_multi.py::test_one_pe_per_gpu_configuration_emulated" \
  "tests/test_gpu_multi.py::test_config5_min_max_prod_int32_f64_4KiB_to_4GiB" \
  tests/test_gpu_cpp.py > $OUT/pytest.txt 2>&1
rc=$?
tail -3 $OUT/pytest.txt
exit $rc
