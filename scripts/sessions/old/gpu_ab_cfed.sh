#!/bin/bash
# CFed GPU tests, then interleaved cfed128 / cfed128_epoch suite runs of ab/old (previous tree) vs this tree.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
root=$PWD
timeout -k 10 600 python -u -m pytest tests/test_gpu_cnn.py -x -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/cfed_tests.log 2>&1
rc=$?; tail -2 gpurun_out/cfed_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do for v in old new; do for c in cfed128 cfed128_epoch; do
  d=$root; [ $v = old ] && d=$root/ab/old
  (cd $d && timeout -k 10 300 python bench_suite.py --config $c --steps 10 --warmup 5) > gpurun_out/abcf_${v}_${c}_$r.log 2>&1 || exit 1
  echo "$v $c r=$r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abcf_${v}_${c}_$r.log)"
done; done; done
