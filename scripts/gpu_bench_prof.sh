#!/bin/bash
# bench (graph + async rounds) and a kernel-trace profile of it (for GPU idle-gap analysis)
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 600 python bench.py --steps 20 --warmup 3 "$@" > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep metric gpurun_out/bench.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py --steps 10 --warmup 2 "$@" > gpurun_out/prof_bench.log 2>&1
rc=$?; echo "prof rc=$rc"; grep '"metric"' gpurun_out/prof_bench.log
exit $rc
