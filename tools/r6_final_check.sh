#!/bin/bash
# Round-6 closing GPU pass: (1) the unweighted-free-state segment test against the kernel with the pivot
# check compiled out (nofb), which should fail -- evidence that the test reaches the fallback; (2) the full
# GPU suite, smoke() and the driver's bench command on the final kernel (tools/r6_check.sh).
# bash tools/r6_final_check.sh OUTDIR
OUT=${1:?outdir}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p "$OUT"
GPMPC_LIB=$PWD/gp-mpc_amd/gpmpc/lib/libgpmpc_mi355x_nofb.so timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 \
    --timeout-method thread tests/test_gpu_launch.py -m gpu -k free_state > "$OUT/nofb_free_state.log" 2>&1
rc=$?
echo "free-state test without the pivot check: exit $rc (1 = failed, as expected)"
tail -n 4 "$OUT/nofb_free_state.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/r6_check.sh "$OUT/check"
