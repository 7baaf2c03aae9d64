#!/bin/bash
# Round 6: CFed forward W2 tap records padded to 5 chunks (staging stores 12-way -> 6.5-way) - CNN tests, diagnostics,
# interleaved cfed128 suite lines (base = HEAD, new = padded W2 records) and kernel traces.
source "$(dirname "$0")/gpu_step.sh"
step cnn_tests 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_cnn.py
for v in base new; do
  QFX_PKG_ROOT=$PWD/ab/$v TAILN=1 step diag_$v 200 python scripts/cnn_flip_diag.py
done
for r in 1 2 3; do for v in base new; do
  (cd ab/$v && timeout -k 10 300 python bench_suite.py --config cfed128 --steps 50 --warmup 3 > ../../gpurun_out/cfab_${v}$r.log 2>&1) || { echo "cfab_${v}$r failed"; tail -5 gpurun_out/cfab_${v}$r.log; exit 1; }
  grep '"metric"' gpurun_out/cfab_${v}$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], {k: d[k] for k in d if 'err' in k})"
done; done
for v in base new; do
  mkdir -p gpurun_out/cfprof_$v
  (cd ab/$v && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ../../gpurun_out/cfprof_$v -o cf -- python3 bench_suite.py --config cfed128 --steps 10 --warmup 2 > ../../gpurun_out/cfprof_$v.log 2>&1) || { echo "cfprof_$v failed"; exit 1; }
done
