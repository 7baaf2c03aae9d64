#!/bin/bash
# Round 4, call 4: OP_L1PROD diagnostic variants (launch knob "diag", see l1prod_op).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/r4d_bisect.log
L1_DIAGS=${L1_DIAGS:-256} timeout -k 10 300 python -u scripts/l1prod_bisect.py 16 3 16 8 > gpurun_out/r4d_bisect.log 2>&1 || { tail -20 gpurun_out/r4d_bisect.log; exit 1; }
grep -v "^/opt" gpurun_out/r4d_bisect.log | cut -c1-400
