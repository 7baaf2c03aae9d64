"""Benchmarks of the other BASELINE.json configs (bench.py is the headline 16q x 64-client VQC).

    python bench_suite.py --config cfed128 --steps 10 --warmup 2
    torchrun --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 bench_suite.py --config vqc20q_dp64

One step = one federated round of the named config (every participating client runs its local steps,
fused local reduce, one all-reduce, global update).  Prints one JSON line (rank 0) in bench.py's
format; ``vs_baseline`` is set where BASELINE.md has a measured reference number (CFed: 258 client
local-steps/s for the reference TinyCNN ``client_update`` on an 8-vCPU host).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

SUITE = {
    # name: (config file, overrides, metric label, reference client-local-steps/s or None)
    "cfed128": ("configs/baseline4_cfed_128clients.yaml", ["train.local_steps=1"],
                "client local-steps/sec (CFed TinyCNN x 128 clients, batch 32)", 258.0),
    "cfed128_epoch": ("configs/baseline4_cfed_128clients.yaml", [],
                      "client local-steps/sec (CFed TinyCNN x 128 clients, 1 local epoch)", 258.0),
    "vqc20q_dp64": ("configs/baseline3_20q_dp_64clients.yaml", ["model.state_dtype=fp32"],
                    "client local-steps/sec (20-qubit VQC x 64 non-IID clients, DP)", None),
    "vqc24q_ps256": ("configs/baseline5_24q_256clients_paramshift_shots.yaml", ["model.state_dtype=fp32"],
                     "client local-steps/sec (24-qubit VQC x 256 clients, param-shift + shots)", None),
    "vqc24q_ps256_mfma": ("configs/baseline5_24q_256clients_paramshift_shots.yaml", ["model.state_dtype=mfma"],
                          "client local-steps/sec (24-qubit VQC x 256 clients, param-shift + shots, fp16 MFMA engine)",
                          None),
    # config 2 as written (state_dtype: bf16) runs the bf16 MFMA engine (csrc/hea_mfma_bf16.hip)
    "vqc16q_bf16_8": ("configs/baseline2_16q_bf16_8clients.yaml", ["train.local_steps=1"],
                      "client local-steps/sec (16-qubit VQC bf16 state x 8 clients)", None),
    "vqc16q_bf16_8_mfma": ("configs/baseline2_16q_bf16_8clients.yaml", ["train.local_steps=1"],
                           "client local-steps/sec (16-qubit VQC bf16 state x 8 clients, bf16 MFMA engine)", None),
    "vqc16q_bf16_8_valu": ("configs/baseline2_16q_bf16_8clients.yaml", ["train.local_steps=1",
                                                                        "model.state_dtype=bf16_valu"],
                           "client local-steps/sec (16-qubit VQC bf16 state x 8 clients, VALU pass engine)", None),
    "vqc16q_fp16_8_mfma": ("configs/baseline2_16q_bf16_8clients.yaml", ["train.local_steps=1", "model.state_dtype=mfma"],
                           "client local-steps/sec (16-qubit VQC x 8 clients, fp16 MFMA engine in place of bf16 "
                           "storage)", None),
    "vqc16q_64": ("configs/headline_16q_64clients.yaml", ["model.state_dtype=fp32"],
                  "client local-steps/sec (16-qubit VQC x 64 clients federated rounds)", None),
    "vqc16q_64_mfma": ("configs/headline_16q_64clients.yaml", ["model.state_dtype=mfma"],
                       "client local-steps/sec (16-qubit VQC x 64 clients, fp16 MFMA engine)", None),
    "vqc16q_64_mfma_secagg": ("configs/headline_16q_64clients.yaml",
                              ["model.state_dtype=mfma", "privacy.secure_agg=true"],
                              "client local-steps/sec (16-qubit VQC x 64 clients, pairwise-mask SecAgg on the device)",
                              None),
    "cfed128_secagg": ("configs/baseline4_cfed_128clients.yaml", ["train.local_steps=1", "privacy.secure_agg=true"],
                       "client local-steps/sec (CFed TinyCNN x 128 clients, batch 32, SecAgg on the device)", 258.0),
    "cfed128_secagg_sparse": ("configs/baseline4_cfed_128clients.yaml",
                              ["train.local_steps=1", "privacy.secure_agg=true", "privacy.secagg_graph=sparse"],
                              "client local-steps/sec (CFed TinyCNN x 128 clients, batch 32, SecAgg+ sparse "
                              "neighbour masks on the device)", 258.0),
    "vqc16q_64_mfma_secagg_sparse": ("configs/headline_16q_64clients.yaml",
                                     ["model.state_dtype=mfma", "privacy.secure_agg=true",
                                      "privacy.secagg_graph=sparse"],
                                     "client local-steps/sec (16-qubit VQC x 64 clients, SecAgg+ sparse neighbour "
                                     "masks on the device)", None),
    # DP lines key their noise by the public seed (privacy.deterministic_noise: reproducible accuracy; NOT private)
    "vqc20q_dp64_mfma": ("configs/baseline3_20q_dp_64clients.yaml",
                         ["model.state_dtype=mfma", "privacy.deterministic_noise=true"],
                         "client local-steps/sec (20-qubit VQC x 64 non-IID clients, DP, fp16 MFMA engine)", None),
    # distributed DP: each client adds sigma^2 C^2 / m, the SecAgg sum carries the accounted sigma C
    "vqc20q_ddp64_mfma": ("configs/baseline3_20q_dp_64clients.yaml",
                          ["model.state_dtype=mfma", "privacy.deterministic_noise=true",
                           "privacy.noise_mode=distributed", "privacy.secure_agg=true", "train.weighting=uniform"],
                          "client local-steps/sec (20-qubit VQC x 64 non-IID clients, distributed DP + SecAgg, "
                          "fp16 MFMA engine)", None),
    "vqc48q_mps64": ("configs/mps_48q_64clients.yaml", [],
                     "client local-steps/sec (48-qubit VQC x 64 clients, MPS tensor-network backend)", None),
    "vqc4q_2_cpu": ("configs/baseline1_4q_2clients_cpu.yaml", ["train.local_steps=1"],
                    "client local-steps/sec (4-qubit VQC x 2 clients, CPU gloo)", None),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfed128", choices=sorted(SUITE))
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("overrides", nargs="*")
    args = ap.parse_args()
    from bench import relaunch_if_needed
    relaunch_if_needed(args.gpus)

    from bench import timed_rounds
    from qfedx_amd.api import setup
    from qfedx_amd.config import load_config
    from qfedx_amd.parallel.dist import shutdown

    path, ov, metric, ref = SUITE[args.config]
    cfg = load_config(os.path.join(ROOT, path), ov + list(args.overrides))
    device, backend, world = setup(cfg)
    counts = []
    runner, dt = timed_rounds(cfg, device, backend, world, args.warmup, args.steps, counts)
    t = cfg.train
    # local steps actually run in the timed rounds (all clients): the fixed step count per training client
    # (participants of each round: Poisson sampling under DP varies them), or epochs x ceil(n/B) at full
    # participation
    if t.local_steps > 0:
        total = sum(counts) * t.local_steps
    else:
        import math
        per_round = sum(t.local_epochs * math.ceil(int(n) / t.batch_size) for n in runner.store.counts)
        total = int(per_round * world.world_size) * args.steps   # store holds this rank's clients
    value = total / dt
    ev = runner.evaluate()
    if world.is_main:
        kind = cfg.model.kind
        rec = {
            "metric": metric, "value": round(value, 3), "unit": "client local-steps/s",
            "n_gpus": world.world_size, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(1e3 * dt / args.steps, 3), "higher_is_better": True, "scaling": "strong",
            "vs_baseline": round(value / ref, 2) if ref else None,
            "dtype": {"bf16": "bf16-state/fp32-compute", "mfma": "fp16-state/fp32-accumulate (MFMA)",
                      "mfma_bf16": "bf16-state/fp32-accumulate (MFMA)",
                      "fp16": "fp16-state/fp32-accumulate (MFMA)"}.get(
                          getattr(runner.adapter, "state_dtype", cfg.model.state_dtype)
                          if backend == "hip" else "fp32", "fp32"),   # the MFMA/bf16 engines exist only on HIP
            "data": "synthetic non-IID client shards, random init", "rounds_per_sec": round(args.steps / dt, 4),
            "samples_per_sec": round(value * t.batch_size, 1), "backend": backend,
            # host time to build and enqueue a round (bench.timed_rounds): a round is host-bound when this nears ms_per_step
            "host_ms_per_round": round(float(getattr(runner, "host_ms", 0.0)), 4),
            "test_acc_after": round(ev["test_acc"], 4),
            "config": {"name": cfg.name, "model": kind if kind != "vqc" else
                       f"vqc-{cfg.model.n_qubits}q-{cfg.model.n_layers}L",
                       "global_batch": cfg.data.num_clients * t.batch_size,
                       "seq_len": cfg.model.n_qubits if kind == "vqc" else 784,
                       "parallelism": f"client-parallel dp{world.world_size}", "n_clients": cfg.data.num_clients,
                       "grad": t.grad_method, "optimizer": t.optimizer, "dp": cfg.privacy.dp,
                       "secure_agg": cfg.privacy.secure_agg,
                       "shots": cfg.noise.shots},
        }
        if cfg.privacy.dp:
            rec["dp"] = {"noise_mode": cfg.privacy.noise_mode, "noise_multiplier": cfg.privacy.noise_multiplier,
                         "clip_norm": cfg.privacy.clip_norm, "delta": cfg.privacy.delta,
                         # accounted rounds = the sum of the history's step counts (the accountant merges equal
                         # (q, sigma) rounds into one record); q next to epsilon.  Every round that ran is charged:
                         # warm-up, timed and calibration rounds alike.
                         "rounds_accounted": int(sum(h[2] for h in runner.accountant.history)),
                         "sampling_rate_q": sorted({round(float(h[0]), 6) for h in runner.accountant.history}),
                         "epsilon": round(float(runner.accountant.get_epsilon(cfg.privacy.delta)), 4),
                         "deterministic_noise": cfg.privacy.deterministic_noise}
        eng = getattr(runner.adapter, "engine", None)
        if kind == "vqc" and backend == "hip":
            from bench import precision_check
            rec.update(precision_check(runner, t.batch_size))     # untimed: MFMA vs fp32 VALU engine
            if cfg.model.state_dtype == "mfma" and "bf16" in path:
                rec["dtype_note"] = ("BASELINE config 2 names bf16 state storage; the fp16 MFMA engine stores "
                                     "fp16 amplitudes (11-bit significand vs bf16's 8), so the substitution is more "
                                     "precise, not less: see max_abs_err_* against the fp32 engine")
        if kind == "tinycnn" and backend == "hip":
            from qfedx_amd.ops.cnn_hip import precision_check as cnn_precision
            rec.update(cnn_precision(cfg.model.n_classes, device))   # untimed: kernels vs float64 autograd
            rec["dtype"] = ("fp32 (conv2 forward, dgrad and wgrad as a 3-term fp16 split on v_mfma_f32_16x16x32_f16 "
                            "with fp32 accumulation; conv1 and the fc layers on v_mfma_f32_16x16x4_f32)")
        if t.grad_method == "param_shift" and eng is not None and hasattr(eng.hip, "shift_pass_counts"):
            # pass launches per sample of one gradient: naive shifted circuits vs prefix reuse + pi identity
            rec["param_shift"] = dict(eng.hip.shift_pass_counts(), reuse=bool(eng.ps_reuse))
        print(json.dumps(rec), flush=True)
    shutdown(world)


if __name__ == "__main__":
    main()
