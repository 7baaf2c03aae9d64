"""Launcher dry run (ROADMAP.md:81-83,95-96 Slurm smoke test: 10 clients + 1 server).

``scripts/slurm/qfedx.sbatch`` runs unmodified under stand-in ``scontrol`` / ``srun`` shims: ``srun`` executes its
command once on this host, so the job's own torchrun line (c10d rendezvous on the head node, 2 ranks on the CPU
with gloo here instead of 8 MI355X ranks with RCCL) trains the smoke config end to end and writes the run
directory (metrics JSONL, checkpoint, MLflow-layout tracking) the batch script asks for.  No Slurm is installed
in this image; the shims stand in for exactly the two commands the script calls.
"""
import json
import os
import socket
import stat
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _shim(path, body):
    with open(path, "w") as f:
        f.write("#!/bin/bash\n" + body)
    os.chmod(path, os.stat(path).st_mode | stat.S_IEXEC)


def test_sbatch_script_dry_run_trains_smoke_config(tmp_path):
    bin_dir = tmp_path / "bin"
    bin_dir.mkdir()
    # scontrol show hostnames <list> -> the head node; srun [--opt=..]... cmd -> run cmd once here
    _shim(str(bin_dir / "scontrol"), 'echo 127.0.0.1\n')
    _shim(str(bin_dir / "srun"), 'while [[ "$1" == --* ]]; do shift; done\nexec "$@"\n')
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    run_dir = tmp_path / "run"
    env = dict(os.environ, PATH=f"{bin_dir}:{os.environ['PATH']}", SLURM_JOB_NODELIST="node001", SLURM_NNODES="1",
               SLURM_JOB_NAME="qfedx", SLURM_JOB_ID="4242", QFEDX_GPUS_PER_NODE="2", QFEDX_PORT=str(port),
               QFEDX_RUN_DIR=str(run_dir), PYTHONPATH=ROOT, MASTER_ADDR="127.0.0.1")
    cmd = ["bash", os.path.join(ROOT, "scripts", "slurm", "qfedx.sbatch"), "configs/smoke_10clients.yaml",
           "train.num_rounds=2", "runtime.device=cpu", "runtime.dist_backend=gloo", "runtime.log_every=100",
           "runtime.checkpoint_every=1"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    recs = [json.loads(x) for x in open(run_dir / "metrics.jsonl") if x.strip()]
    rounds = [x for x in recs if x.get("round", 0) >= 1 and "train_loss" in x]
    assert [x["round"] for x in rounds] == [1, 2] and all(x["participants"] == 10 for x in rounds)
    assert os.path.isdir(run_dir / "ckpt") and os.path.isdir(run_dir / "mlruns")
