#!/bin/bash
# Round 4, call 3: OP_L1PROD with every lambda word read before any r term is written (two-phase), bisection;
# gradient epilogue with packed slot bytes + v_cvt_rpi: HEA GPU tests and adjoint timing.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/l1prod_bisect.py 16 3 16 8 > gpurun_out/r4c_bisect_16x8.log 2>&1 || { tail -20 gpurun_out/r4c_bisect_16x8.log; exit 1; }
grep variant gpurun_out/r4c_bisect_16x8.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_hea.py > gpurun_out/r4c_hea_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4c_hea_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/hea_ab.py --rounds 5 --variants "w8:adj_waves=8,w8f:adj_waves=8;full13=1" > gpurun_out/r4c_ab.log 2>&1 || { tail -20 gpurun_out/r4c_ab.log; exit 1; }
tail -1 gpurun_out/r4c_ab.log
