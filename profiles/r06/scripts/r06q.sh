#!/bin/bash
# Round 6 (late): unaligned-load a + b / copy with consecutive 1 KiB blocks per one-wave workgroup
# (tools/realign_variants.hip k_unalc) against block order and the XCD-grouped order, 1 GiB,
# shifts 4 and 12 B.  From the repo root; results in profiles/r06/realign/r06q/.
set -u
O=gpurun_out/r06q
mkdir -p $O
timeout -k 10 100 ./tools/bin/realign_variants 1024 5 10 4 > $O/rv_k4.txt 2>&1 || exit 1
timeout -k 10 100 ./tools/bin/realign_variants 1024 5 10 12 > $O/rv_k12.txt 2>&1
