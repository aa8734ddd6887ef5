#!/usr/bin/env bash
# Two PEs (processes) on the box's one GPU running the reference-shaped reduce_bw harness
# (tests/cpp/reduce_bw.cpp); CSV on PE 0's stdout.  Usage: scripts/reduce_bw_p2.sh MAX_NELEMS OUT
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
KEY="bw$$"
export HSA_ENABLE_IPC_MODE_LEGACY=0 ISHMEM_NPES=2 ISHMEM_DEVICE=0 ISHMEM_BOOTSTRAP_KEY=$KEY ISHMEM_MAX_BLOCKS=${MB:-128}
ISHMEM_PE=1 timeout -k 10 500 "${EXE:-$R/build/reduce_bw}" --csv -m "$1" > /dev/null 2>&1 &
P1=$!
ISHMEM_PE=0 timeout -k 10 500 "${EXE:-$R/build/reduce_bw}" --csv -m "$1" > "$2" 2>&1
RC=$?
wait $P1
RC1=$?
exit $(( RC != 0 ? RC : RC1 ))
