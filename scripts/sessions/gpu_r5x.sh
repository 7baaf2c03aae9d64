#!/bin/bash
# Round 5, call 24: the readout op's |amplitude|^2 as one v_dot2_f32_f16 per word (two converts, a multiply and an fma
# before): MFMA-engine GPU tests on the new tree, interleaved kbench A/B of the two built trees, stall table.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5x
timeout -k 10 400 python -u -m pytest tests/test_gpu_hea.py -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r5x/hea_tests.log 2>&1
rc=$?; echo "hea_tests rc=$rc"; tail -2 gpurun_out/r5x/hea_tests.log
for c in 64 8; do
  for r in 1 2 3; do for v in base dot2; do
    QFX_PKG_ROOT=$PWD/ab/$v timeout -k 10 200 python scripts/hea_kbench.py --iters 30 --clients $c > gpurun_out/r5x/ab_${v}_${c}_$r.log 2>&1 || exit 1
    echo "$v c=$c r=$r $(tail -1 gpurun_out/r5x/ab_${v}_${c}_$r.log)"
  done; done
done
timeout -k 10 300 python -u scripts/hea_stamps.py --clients 64 --out gpurun_out/r5x/stamps64.jsonl > gpurun_out/r5x/stamps64.log 2>&1
rc=$?; echo "stamps64 rc=$rc"; tail -4 gpurun_out/r5x/stamps64.log
