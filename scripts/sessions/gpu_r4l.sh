#!/bin/bash
# Round 4, call 12: where the ~26 us between two round graphs goes (graph_gap.py under rocprofv3: boundary gap vs
# kernels per graph, dirty-L2 size at the boundary, graph packet capture), and the host-side profile of the share-8
# bench.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/gap
run() {
  local name=$1; shift
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gap -o $name -- "$@" > gpurun_out/gap/$name.log 2>&1
  local rc=$?
  [ $rc -eq 0 ] || { echo "$name rc=$rc"; exit $rc; }
}
run k1 python3 scripts/graph_gap.py --kernels 1 --reps 200
run k12 python3 scripts/graph_gap.py --kernels 12 --reps 200
run k12d64 python3 scripts/graph_gap.py --kernels 12 --reps 200 --dirty-mb 64
run k12d512 python3 scripts/graph_gap.py --kernels 12 --reps 200 --dirty-mb 512
for n in k1:1 k12:12 k12d64:13 k12d512:13; do
  name=${n%%:*}; kp=${n##*:}
  echo -n "$name: "; python3 scripts/gap_split.py gpurun_out/gap/${name}_kernel_trace.csv $kp
  grep us_per_replay gpurun_out/gap/$name.log
done
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 120 python3 scripts/graph_gap.py --kernels 12 --reps 200
DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 timeout -k 10 120 python3 scripts/graph_gap.py --kernels 12 --reps 200
timeout -k 10 300 python -m cProfile -o gpurun_out/share8.pstats bench.py --steps 300 --warmup 5 --clients 8 > gpurun_out/r4l_share8_cprof.log 2>&1
rc=$?; [ $rc -eq 0 ] || exit $rc
python3 -c "import pstats; pstats.Stats('gpurun_out/share8.pstats').sort_stats('tottime').print_stats(25)" > gpurun_out/r4l_share8_pstats.txt
head -60 gpurun_out/r4l_share8_pstats.txt
