#!/bin/bash
# Round 6 (late): the shifted phased reduce-scatter in 512-thread workgroups (set_param "rs_block")
# against one-wave workgroups in block / XCD-grouped order; 2 / 4 PEs x 1 GiB on the one GPU,
# sources 4 B off dest's phase, with one-PE-per-GPU launch shapes (--emulate-share1, the fold off,
# as r06c) and co-located (share = p); interleaved x2, aligned sources as the reference.
set -u
O=gpurun_out/r06r
mkdir -p $O
export ISHMEM_BENCH_SAME_DEVICE=1 HSA_ENABLE_IPC_MODE_LEGACY=0
port=29400
for r in 1 2; do
  for p in 2 4; do
    for cfg in e:64:1 e:64:0 e:512:0 e:512:1 e:0:1 c:64:1 c:512:1 c:0:1; do
      IFS=: read mode bs x <<< "$cfg"
      off=4; [ $bs = 0 ] && { bs=64; off=0; }
      extra=""; [ $mode = e ] && extra="--emulate-share1 --param xgmi_fold_max_bytes=0"
      f=$O/p${p}_${mode}_off${off}_b${bs}_x${x}_r$r
      port=$((port + 1))
      timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node $p --master-addr 127.0.0.1 \
        --master-port $port tools/sweep.py --min-bytes 1073741824 --max-mib 1024 --iters 10 $extra \
        --src-offset $off --phases --param rs_block=$bs --param rs_xcd=$x \
        > $f.csv 2> $f.err || { echo "FAIL $f"; tail -5 $f.err; exit 1; }
      echo "$(basename $f): $(grep -v '^#\|Gloo\|peer ranks\|bytes' $f.csv | tr '\n' ' ') $(grep '# phases' $f.csv)"
    done
  done
done | tee $O/ab.txt
