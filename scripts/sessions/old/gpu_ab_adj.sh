#!/bin/bash
# A/B of adjoint-kernel variants: correctness of the new tree under each wave count, then interleaved kernel
# timing (scripts/hea_kbench.py) of ab/base vs ab/v1 at 8 and 4 adjoint waves, 64- and 8-client steps.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for w in 8 4; do
  QFEDX_HEA_ADJ_WAVES=$w timeout -k 10 300 python -u -m pytest tests/test_gpu_hea.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/hea_tests_w$w.log 2>&1
  rc=$?; echo "hea tests w$w rc=$rc"; tail -2 gpurun_out/hea_tests_w$w.log; [ $rc -eq 0 ] || exit $rc
done
for r in 1 2; do
  for K in 64 8; do
    for v in base v1_8 v1_4; do
      tree=${v%%_*}; w=${v#*_}; [ "$w" = "$v" ] && w=8
      QFEDX_HEA_ADJ_WAVES=$w QFX_PKG_ROOT=$PWD/ab/$tree timeout -k 10 200 python scripts/hea_kbench.py --iters 30 --clients $K > gpurun_out/ab_${v}_${K}_$r.log 2>&1 || exit 1
      echo "$v K=$K r$r $(tail -1 gpurun_out/ab_${v}_${K}_$r.log)"
    done
  done
done
