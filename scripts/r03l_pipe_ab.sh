mkdir -p gpurun_out/r03l && timeout -k 10 200 tools/bin/stream_variants 5 r3 > gpurun_out/r03l/stream_r3.txt 2>&1 && \
ISHMEM_AMD_LIB=build/ab/libishmem_amd_pipe.so timeout -k 10 400 python -u -m pytest tests/test_gpu_multi.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "golden or inplace or config3 or two_pe or eight_pes_compile or stress" > gpurun_out/r03l/pytest_pipe.log 2>&1 && \
bash scripts/ab_occ.sh r03l product=product pipe=build/ab/libishmem_amd_pipe.so > gpurun_out/r03l/ab.txt 2>&1
