#!/bin/bash
# Interleaved bench.py A/B of the working tree against a built copy of another tree in ab/old (same box):
# headline (64 clients) and the 8-client per-rank share, ROUNDS rounds each.  TESTS: GPU tests to run first.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
root=$PWD
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/abtree_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/abtree_tests.log; [ $rc -eq 0 ] || exit $rc
fi
for r in $(seq ${ROUNDS:-3}); do for v in old new; do for cl in 64 8; do
  d=$root; [ $v = old ] && d=$root/ab/old
  (cd $d && timeout -k 10 300 python bench.py --steps 40 --warmup 5 --clients $cl) > gpurun_out/abtree_${v}_${cl}_$r.log 2>&1 || exit 1
  echo "$v clients=$cl r=$r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abtree_${v}_${cl}_$r.log)"
done; done; done
