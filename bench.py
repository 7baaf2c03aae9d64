"""Headline benchmark: federated rounds/s + client local-steps/s, 16-qubit VQC x 64 clients.

Metric/config from BASELINE.json ("federated rounds/sec + client local-steps/sec, 16-qubit VQC x 64
clients").  One bench step = one full federated round: every one of the 64 clients (sharded over
the N GPUs, one process per GPU, RCCL all-reduce) runs ``--local-steps`` local Adam steps on a
minibatch of ``--batch`` samples from its synthetic non-IID shard (forward statevector passes +
readout CE + adjoint backward + fused Adam, all gfx950 HIP kernels), then the fused FedAvg local
reduce (angle-wrapped deltas) and ONE all-reduce update the global model.  Nothing is skipped in
the timed region.  Total clients are fixed as N grows -> strong scaling.

Usage: python bench.py [--gpus N --steps K --warmup W]   (N>1: launched by torch.distributed.run)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def timed_rounds(cfg, device, backend, world, warmup: int, steps: int, counts: list | None = None):
    """Build this rank's runner, run ``warmup`` untimed rounds, then time exactly ``steps`` rounds
    bracketed by barrier + device sync on both sides; returns (runner, max-over-ranks seconds).  ``counts``
    (optional list) receives each timed round's number of training clients (participants - dropouts, over all
    ranks: the sampling is keyed, identical on every rank)."""
    import torch
    from qfedx_amd.data.datasets import build_federated_data
    from qfedx_amd.fl.adapters import make_adapter
    from qfedx_amd.fl.server import FederatedRunner
    from qfedx_amd.parallel.dist import barrier, max_over_ranks, shard_clients

    my = shard_clients(cfg.data.num_clients, world.world_size, world.rank)
    data = build_federated_data(cfg, clients=my)
    adapter = make_adapter(cfg, device, backend)
    runner = FederatedRunner(cfg, adapter, data, world, device, backend)

    def sync():
        barrier(world)
        if device.type == "cuda":
            torch.cuda.synchronize()

    for r in range(warmup):
        runner.run_round(r, sync=False)
    sync()
    runner.timer.enabled = False            # no phase events inside the timed rounds (phase_ms calibrates after)
    from qfedx_amd.fl import trainer as _tr
    w0 = _tr.WAIT_S[0]
    t0 = time.perf_counter()
    for r in range(warmup, warmup + steps):
        rec = runner.run_round(r, sync=False)
        runner.comm_bytes = rec.get("comm_bytes_per_rank", 0)
        if counts is not None:
            counts.append(rec["participants"] - rec["dropped"])
    # host time to build and enqueue a round, without the time it waited for the GPU to free a pinned buffer
    runner.host_ms = 1e3 * (time.perf_counter() - t0 - (_tr.WAIT_S[0] - w0)) / max(steps, 1)
    sync()
    dt = time.perf_counter() - t0
    return runner, max_over_ranks(dt, world)


def phase_ms(runner, world, steps: int, calib: int = 5) -> dict:
    """Per-round milliseconds of the runner's phases (HIP events; max over ranks), from ``calib`` untimed rounds run
    after the timed ones (the timed rounds record no events: each one idles the GPU between graph launches):
    ``local_train_ms`` = the round graph (every local step + the fused FedAvg reduce, and the collective + apply when
    they are captured with it), ``comm_ms`` = whatever of the all-reduce + finalize/apply runs outside the graph."""
    import torch
    from qfedx_amd.parallel.dist import barrier, max_over_ranks
    tm = runner.timer
    tm.reset()
    tm.enabled, tm.every = True, 1
    for r in range(10_000, 10_000 + calib):
        runner.run_round(r, sync=False)
    barrier(world)
    if runner.device.type == "cuda":
        torch.cuda.synchronize()
    return {f"{k}_ms": round(max_over_ranks(v, world), 4) for k, v in sorted(tm.per_phase().items())}


def precision_check(runner, batch: int) -> dict:
    """Accuracy evidence for the fp16-state MFMA engine at the bench shape: ONE untimed adjoint VJP of this
    rank's clients (first ``batch`` samples of each shard, the current global params) on the MFMA engine and
    on the fp32 VALU engine (ahead-of-time interpreter kernels, no JIT), same inputs and readout weights.
    Returns the max abs differences of <Z> and of the parameter gradient, and the gradient's max magnitude."""
    import torch
    from qfedx_amd.ops.statevec_hip import HipProgram
    eng = runner.adapter.engine
    spec = runner.adapter.spec
    if getattr(eng, "hip", None) is None or not hasattr(eng.hip, "vjp") or isinstance(eng.hip, HipProgram):
        return {}
    store = runner.store
    # at most ~4 GiB of fp32 reference states (all clients at the 16q headline; a few at 24q)
    kmax = max(1, (4 << 30) // (batch * (8 << spec.n_qubits)))
    xang = spec.encode_features(store.X[:kmax, :batch].float())
    K, B = xang.shape[:2]
    th = runner.params[: spec.n_theta].float()[None].expand(K, -1).contiguous()
    g = torch.Generator(device="cpu").manual_seed(1234)
    w = (torch.randn(K * B, spec.n_classes, generator=g) / B).to(xang.device)
    z_m, g_m = eng.hip.vjp(xang, th, w)
    ref = HipProgram(eng.ops, eng.coef, spec.n_qubits, spec.readout, xang.device, n_theta=spec.n_theta,
                     state_dtype="fp32", jit=False, x_width=spec.x_width)
    z_r, g_r = ref.vjp(xang, th, w)
    torch.cuda.synchronize()
    return {"max_abs_err_expz": float((z_m - z_r).abs().max()), "max_abs_err_grad": float((g_m - g_r).abs().max()),
            "max_abs_grad": float(g_r.abs().max()), "precision_ref": "fp32 VALU engine (interpreter kernels)",
            "precision_samples": int(K * B)}


def make_config(args):
    """The bench's experiment config (BASELINE.json headline: 16-qubit VQC x 64 clients, synthetic non-IID)."""
    from qfedx_amd.config import ExperimentConfig
    cfg = ExperimentConfig(name="bench")
    cfg.data.dataset = "synthetic"
    cfg.data.num_clients = args.clients
    cfg.data.partition_type = "non_iid"
    cfg.data.alpha = 0.5
    cfg.data.samples_per_client = max(4 * args.batch, 64)
    cfg.data.test_samples = 256
    cfg.data.n_features = args.qubits
    cfg.model.n_qubits = args.qubits
    cfg.model.n_layers = args.layers
    cfg.model.n_classes = args.classes
    cfg.model.readout_scale = 3.0
    cfg.model.state_dtype = {"mfma": "mfma", "mfma_bf16": "bf16"}.get(args.engine, "fp32")
    cfg.train.batch_size = args.batch
    cfg.train.local_steps = args.local_steps
    cfg.train.learning_rate = 0.05
    cfg.train.optimizer = "adam"
    cfg.train.grad_method = "adjoint"
    cfg.privacy.dp = args.dp
    cfg.privacy.clip_norm = 1.0
    cfg.privacy.noise_multiplier = 1.0
    cfg.runtime.backend = args.backend
    cfg.runtime.device = args.device
    cfg.runtime.dist_backend = getattr(args, "dist_backend", "auto")
    return cfg


def relaunch_if_needed(gpus: int) -> None:
    """``--gpus N`` must match the launched world.  Started without a launcher (no WORLD_SIZE) and N > 1,
    re-run this command under ``torch.distributed.run`` (one rank per GPU, 127.0.0.1 rendezvous) as a
    CHILD process - nothing here has touched the GPU yet - and exit with its status."""
    ws = os.environ.get("WORLD_SIZE")
    if ws is None:
        if gpus <= 1:
            return
        import socket
        import subprocess
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
               "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(sys.argv[0]), *sys.argv[1:]]
        sys.exit(subprocess.call(cmd))
    if int(ws) != gpus:
        sys.exit(f"bench.py: --gpus {gpus} but WORLD_SIZE={ws}; launch one rank per GPU "
                 f"(torch.distributed.run --nproc-per-node {gpus}) or pass --gpus {ws}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--qubits", type=int, default=16)
    ap.add_argument("--layers", type=int, default=3)
    ap.add_argument("--clients", type=int, default=64)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--local-steps", type=int, default=1)
    ap.add_argument("--classes", type=int, default=3)
    ap.add_argument("--dp", action="store_true")
    ap.add_argument("--backend", default="auto")
    ap.add_argument("--device", default="auto")
    ap.add_argument("--dist-backend", default="auto", choices=["auto", "nccl", "gloo"],
                    help="process-group backend (auto: nccl = RCCL on GPUs, gloo on CPU); gloo on GPUs lets "
                         "several ranks share one GPU in tests")
    ap.add_argument("--engine", default="mfma", choices=["mfma", "mfma_bf16", "valu"],
                    help="mfma: fp16-state MFMA group-unitary engine (ops/hea_mfma.py); mfma_bf16: the same engine "
                         "with bf16 state storage; valu: fp32 pass engine")
    ap.add_argument("--precision-check", type=int, default=1,
                    help="after timing, one untimed VJP on the fp32 VALU engine at the bench shape: report the "
                         "MFMA engine's max abs <Z> / gradient differences (0 = skip)")
    args = ap.parse_args()
    relaunch_if_needed(args.gpus)

    import torch
    from qfedx_amd.api import setup
    from qfedx_amd.parallel.dist import shutdown

    cfg = make_config(args)
    device, backend, world = setup(cfg)
    runner, dt = timed_rounds(cfg, device, backend, world, args.warmup, args.steps)
    # clients trained by each rank (the 8-GPU operating point is 8 of the 64 headline clients per rank)
    from qfedx_amd.parallel.dist import all_gather_cat
    per_rank = [int(v) for v in all_gather_cat(torch.tensor([len(runner.local_ids)], dtype=torch.int64,
                                                             device=device), world).cpu().tolist()]
    phases = phase_ms(runner, world, args.steps)
    ev = runner.evaluate()
    prec = precision_check(runner, args.batch) if (args.precision_check and device.type == "cuda") else {}
    local_steps_total = args.clients * args.local_steps * args.steps
    value = local_steps_total / dt
    rounds_per_s = args.steps / dt
    # label what actually ran: the MFMA engine exists only on the HIP backend (ops/engine.py)
    sdt = getattr(runner.adapter, "state_dtype", "")
    mfma = backend == "hip" and sdt in ("mfma", "fp16", "mfma_bf16")
    import torch.distributed as tdist
    from qfedx_amd.parallel.dist import max_over_ranks
    rccl_ws = tdist.get_world_size() if tdist.is_initialized() else 0
    fallbacks = max_over_ranks(float(getattr(runner.adapter.trainer, "capture_fallbacks", 0)), world)
    graph_comm = runner.graph_comm_mode if fallbacks == 0 else "mixed"
    engine = "mfma" if mfma else ("valu" if backend == "hip" else backend)
    if world.is_main:
        rec = {
            "metric": f"client local-steps/sec ({args.qubits}-qubit VQC x {args.clients} clients federated rounds)",
            "value": round(value, 3),
            "unit": "client local-steps/s",
            "n_gpus": world.world_size,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * dt / args.steps, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": (("bf16" if sdt == "mfma_bf16" else "fp16") + "-state/fp32-accumulate (MFMA)") if mfma else "fp32",
            "engine": engine,
            "data": "synthetic non-IID (Dirichlet alpha=0.5) client shards, random-init VQC",
            "rounds_per_sec": round(rounds_per_s, 4),
            "samples_per_sec": round(value * args.batch, 1),
            "backend": backend,
            "test_acc_after": round(ev["test_acc"], 4),
            "dist_backend": world.backend,
            # ranks in the process group as torch.distributed sees it (0: no group) and whether the round's
            # all-reduce ran captured in the round hipGraph on every rank (agreed at startup; "mixed" if a later
            # shape had to fall back to an eager collective on some rank)
            "rccl_world_size": rccl_ws,
            "graph_comm": graph_comm,
            # CC4: round r + 1's upload + minibatch gather on a side stream against round r's graph + collective
            # (on with more than one rank; QFEDX_CC4 overrides)
            "cc4_overlap": bool(getattr(runner.adapter.trainer, "cc4", False)),
            # MFMA engine tiling: forward / adjoint tile bits (2^13 forward tiles for small per-rank batches)
            "mfma_tiles": ([int(runner.adapter.engine.hip.tile_bits), int(runner.adapter.engine.hip.adj_tile_bits)]
                           if mfma else None),
            "host_ms_per_round": round(getattr(runner, "host_ms", 0.0), 4),   # enqueue time (GPU runs behind)
            "clients_per_rank": per_rank,
            # bytes each rank all-reduces per round: ONE fused [exact int64 update | weight | metrics] buffer
            "allreduce_bytes_per_round": int(getattr(runner, "comm_bytes", 0)),
            **phases,
            **prec,
            "config": {
                "model": f"vqc-{args.qubits}q-{args.layers}L-hea-cnot-chain",
                "global_batch": args.clients * args.batch,
                "seq_len": args.qubits,
                "parallelism": f"client-parallel dp{world.world_size}",
                "n_qubits": args.qubits,
                "n_clients": args.clients,
                "local_steps_per_round": args.local_steps,
                "grad": "adjoint",
                "optimizer": "adam",
                "dp": bool(args.dp),
            },
        }
        print(json.dumps(rec), flush=True)
    shutdown(world)


if __name__ == "__main__":
    main()
