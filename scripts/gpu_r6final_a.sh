#!/bin/bash
# Round 6 final validation, part A: GPU test suite -> smoke -> headline bench -> rocprofv3 kernel trace + round timeline.
source "$(dirname "$0")/gpu_step.sh"
mkdir -p gpurun_out/prof_final
step gpu_tests 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py --steps 20 --warmup 3
step bench8 600 python bench.py --steps 20 --warmup 3 --clients 8
step prof_bench 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_final -o bench -- python3 bench.py --steps 10 --warmup 2
