"""Federated round loop ("server.py", ROADMAP.md:34-39; reference ``federated_learning``,
``Classical_FL.py:104-157``).

Reference behaviour kept: round-0 evaluation, ``num_rounds`` rounds of (all clients train ->
FedAvg -> load -> test eval), an accuracy history list, progress print every 5 rounds, return
``{'model', 'accuracies'}``.  Redesigned for MI355X:

* every rank holds an identical global parameter vector; clients are sharded over ranks and a
  rank's participating clients train as ONE batch (no per-client Python loop);
* client sampling (fraction q) and dropouts are keyed by (seed, round) so all ranks agree without
  communication; dropped clients simply contribute weight 0 (SecAgg orphan masks are removed);
* aggregation = fused local reduce on-device + ONE all-reduce of [update | weight | metrics];
* the test set is sharded over ranks and metrics are all-reduced;
* RDP accountant step + epsilon per round, JSONL metrics, checkpoint every K rounds, resume.
"""
from __future__ import annotations

import json
import math
import os
import time
from typing import Optional

import numpy as np
import torch

from ..parallel.dist import (ShardedServerState, World, agree_graph_comm, all_gather_cat, all_reduce_,
                             all_reduce_async, barrier, broadcast_, shard_clients)
from ..privacy.accountant import RDPAccountant
from ..privacy.dp import noise_scale, draw_noise_seed
from ..privacy.secure_agg import SecureAggregator
from ..utils.device import h2d
from ..utils.checkpoint import latest_checkpoint, load_checkpoint, save_checkpoint
from ..utils.logging import MetricsWriter, get_logger
from ..utils.seeding import generator, np_rng
from ..utils.timing import PhaseTimer
from .aggregator import EXACT_SCALE, Aggregator
from .trainer import ShardStore

# single-rank rounds apply the update inside the FedAvg reduce launch (FusedApply: every block arrives on one counter)
# up to this many buffer entries: past it the arrivals, one same-address atomic per 64-parameter block, cost more
# than the round_apply launch they save (CFed TinyCNN, 128 clients: +9 us per round, profiles/r4_round_structure_ab.txt)
FUSED_APPLY_MAX = 4096


def sample_participants(num_clients: int, fraction: float, seed: int, round_num: int,
                        poisson: bool = False) -> list[int]:
    """Clients taking part in round ``round_num`` (ROADMAP.md:35,106), keyed by (seed, round) so every
    rank draws the same set without communication.

    ``poisson=False``: a fixed-size subset of m = round(q N) drawn without replacement.
    ``poisson=True``: every client independently with probability q (the set may be empty) - the
    sampling the subsampled-Gaussian RDP bound of ``privacy/accountant.py`` assumes."""
    if fraction >= 1.0:
        return list(range(num_clients))
    if poisson:
        u = np_rng(seed, "sample_clients_poisson", round_num).random(num_clients)
        return [int(c) for c in np.flatnonzero(u < fraction)]
    m = max(1, int(round(fraction * num_clients)))
    g = generator(seed, "sample_clients", round_num)
    return sorted(torch.randperm(num_clients, generator=g)[:m].tolist())


def sample_dropouts(participants: list[int], prob: float, seed: int, round_num: int) -> list[int]:
    if prob <= 0:
        return []
    out = []
    for c in participants:
        if np_rng(seed, "client_drop", round_num, c).random() < prob:
            out.append(c)
    return out


class FederatedRunner:
    """Drives federated training for one model adapter (VQC or TinyCNN) on this rank."""

    def __init__(self, cfg, adapter, data, world: World, device: torch.device, backend: str):
        self.cfg = cfg
        self.adapter = adapter
        self.data = data
        self.world = world
        self.device = device
        self.backend = backend
        self.log = get_logger()
        t, p = cfg.train, cfg.privacy
        self.num_clients = data.num_clients
        self.local_ids = list(data.client_ids)
        self.store = ShardStore(data.clients, data.client_ids, device)
        self.P = adapter.n_params
        # DP noise + DP client sampling key: a per-run secret (rank 0's OS randomness, broadcast, never
        # persisted or logged); the public train.seed only under privacy.deterministic_noise
        self.noise_seed = draw_noise_seed(world, p.deterministic_noise, t.seed) if p.dp else t.seed
        sampling = t.sampling if t.sampling != "auto" else ("poisson" if p.dp else "fixed")
        if sampling not in ("fixed", "poisson"):
            raise ValueError(f"train.sampling must be auto | fixed | poisson, got {t.sampling!r}")
        self.poisson = sampling == "poisson"
        noise_scale(getattr(p, "noise_mode", "local"), 1)           # validates privacy.noise_mode
        if p.dp and getattr(p, "noise_mode", "local") == "distributed" and not p.secure_agg:
            # each client's share of the noise is too small to protect its update on its own: only the SecAgg sum
            # (which the server sees instead of the shares) carries the accounted sigma C
            raise ValueError("privacy.noise_mode=distributed needs privacy.secure_agg=true")
        if p.dp and getattr(p, "noise_mode", "local") == "distributed" and t.weighting != "uniform":
            # the shares are scaled by each client's FedAvg weight AFTER noising: the sum then carries noise std
            # sigma C sqrt(sum w_k^2 / m) against a sensitivity of max_k w_k C, an effective multiplier of
            # sigma RMS(w) / max(w) < sigma for unequal weights - the accountant would under-report epsilon
            raise ValueError("privacy.noise_mode=distributed needs train.weighting=uniform (with sample weighting "
                             "the aggregate noise falls below the accounted sigma)")
        self.secagg = None
        if p.secure_agg:
            # each client's DH secret comes from OS randomness on the rank hosting it; only public keys
            # are exchanged (all-gather), so no process holds another rank's client secrets
            self.secagg = SecureAggregator(None, p.secagg_bits, p.secagg_scale, getattr(p, "secagg_graph", "full"),
                                           getattr(p, "secagg_min_live", 0))
            self.secagg.setup(self.local_ids, world)
        self.aggregator = Aggregator(self.P, adapter.angle_mask(), device, backend, t.aggregate,
                                     t.wrap_angles, p.dp, p.clip_norm, p.noise_multiplier, p.secure_agg,
                                     self.secagg, self.noise_seed, num_clients=self.num_clients)
        self.accountant = RDPAccountant()
        # test shard for this rank
        Xt, yt = data.test
        sl = shard_clients(int(yt.shape[0]), world.world_size, world.rank)
        self.X_test = Xt[sl[0]: sl[-1] + 1].to(device) if sl else Xt[:0].to(device)
        self.y_test = yt[sl[0]: sl[-1] + 1].to(device) if sl else yt[:0].to(device)
        self.metrics = MetricsWriter(cfg.runtime.metrics_path, world.rank, cfg.to_dict(), cfg.runtime.tracking_dir,
                                     cfg.runtime.experiment or cfg.name)
        self.timer = PhaseTimer(device, every=int(getattr(cfg.runtime, "timer_every", 0) or
                                                  (16 if torch.device(device).type == "cuda" else 1)))
        self.start_round = 0
        self.history: list[dict] = []
        self.server_opt = None
        if t.server_optimizer != "fedavg" or t.server_lr != 1.0:
            if p.secure_agg:
                raise ValueError("server_optimizer needs plain (non-SecAgg) aggregation of the update sums")
            self.server_opt = ShardedServerState(self.P, world, device, t.server_optimizer, t.server_lr,
                                                 t.server_momentum)
        self.params = adapter.init_params(t.seed).to(device)
        broadcast_(self.params, world)                      # CC1: identical theta on all ranks
        # CC6: per-client update norms in the round all-reduce.  Opt-in NON-PRIVATE diagnostic: the raw pre-clip norms
        # (and the clip fraction / quantiles logged from them) are computed from private data without noise and are
        # not charged to the accountant, so a run that logs them is outside the epsilon it reports
        self.n_norm_slots = (self.num_clients if (p.dp and not p.secure_agg and
                                                  getattr(cfg.runtime, "log_client_norms", False)) else 0)
        # CC2: the round's collective captured into the round hipGraph - decided ONCE, agreed by every rank (each
        # rank captures and replays one all-reduce, compared bitwise with an eager one; fl/trainer.py keeps a per-shape
        # eager fallback that preserves the collective order)
        want = (bool(getattr(cfg.runtime, "graph_comm", True)) and backend == "hip" and self.server_opt is None
                and torch.device(device).type == "cuda" and (not world.distributed or world.backend == "nccl"))
        self.graph_comm = agree_graph_comm(world, want)
        cc4_env = os.environ.get("QFEDX_CC4")
        self.cc4 = (cc4_env == "1") or (cc4_env is None and world.distributed and
                                        bool(getattr(cfg.runtime, "overlap_comm", True)))
        # the graphed HIP round's side-stream upload + gather (opt-in: see RuntimeConfig.overlap_comm_device)
        adapter.trainer.cc4 = (cc4_env == "1") or (cc4_env is None and world.distributed and
                                                   bool(getattr(cfg.runtime, "overlap_comm_device", False)))
        self.graph_comm_mode = ("captured" if self.graph_comm else "eager") if backend == "hip" else "none"

    # ------------------------------------------------------------------ eval
    @torch.no_grad()
    def evaluate(self, params: Optional[torch.Tensor] = None) -> dict:
        params = self.params if params is None else params
        loss_sum, correct, n = self.adapter.evaluate(params, self.X_test, self.y_test)
        buf = torch.tensor([loss_sum, correct, n], dtype=torch.float64, device=self.device)
        all_reduce_(buf, self.world)
        n_tot = max(float(buf[2]), 1.0)
        return {"test_acc": float(buf[1]) / n_tot, "test_loss": float(buf[0]) / n_tot}

    @torch.no_grad()
    def test_auc(self, params: Optional[torch.Tensor] = None) -> float:
        """Macro one-vs-rest ROC AUC on the full (rank-sharded, gathered) test set (ROADMAP:112)."""
        if not hasattr(self.adapter, "logits"):
            return float("nan")
        params = self.params if params is None else params
        lg = self.adapter.logits(params, self.X_test).float()
        C = self.cfg.model.n_classes
        probs = all_gather_cat(torch.softmax(lg, -1).reshape(-1), self.world).reshape(-1, C).cpu().numpy()
        ys = all_gather_cat(self.y_test.to(lg.device).double(), self.world).cpu().numpy().astype(int)
        try:
            from sklearn.metrics import roc_auc_score
            if C == 2:
                return float(roc_auc_score(ys, probs[:, 1]))
            if len(set(ys.tolist())) < C:
                return float("nan")
            return float(roc_auc_score(ys, probs, multi_class="ovr", average="macro"))
        except Exception:
            return float("nan")

    # ------------------------------------------------------------------ checkpoint
    def save(self, round_num: int) -> None:
        rt = self.cfg.runtime
        if not rt.checkpoint_dir:
            return
        # the sharded server-optimizer moments are gathered on every rank (collective) before rank 0 writes
        server_state = self.server_opt.state_dict() if self.server_opt is not None else None
        if self.world.is_main:
            payload = {
                "global_state": self.adapter.state_dict(self.params),
                "accountant": json.dumps(self.accountant.state_dict()),
                "config": self.cfg.to_dict(),
                "metrics": self.history,
                "seed": torch.tensor(self.cfg.train.seed),   # public root seed (DP noise uses a run secret)
            }
            if server_state is not None:
                payload["server_state"] = server_state
            path = save_checkpoint(rt.checkpoint_dir, round_num, payload)
            self.metrics.tracker.log_artifact(path, "checkpoints")
        barrier(self.world)

    def maybe_resume(self) -> None:
        rt = self.cfg.runtime
        if not (rt.resume and rt.checkpoint_dir):
            return
        path = latest_checkpoint(rt.checkpoint_dir)
        if path is None:
            return
        ck = load_checkpoint(path)
        self.params = self.adapter.from_state_dict(ck["global_state"]).to(self.device)
        self.accountant.load_state_dict(json.loads(ck["accountant"]))
        self.history = list(ck.get("metrics", []))
        if self.server_opt is not None:
            if "server_state" not in ck:
                raise ValueError(f"{path} has no server_state but train.server_optimizer="
                                 f"{self.cfg.train.server_optimizer!r} needs its moments to resume")
            self.server_opt.load_state_dict(ck["server_state"])
        self.start_round = int(ck["round"])
        self.log.info(f"resumed from {path} at round {self.start_round}")

    # ------------------------------------------------------------------ main loop
    def _round_setup(self, r: int) -> dict:
        """Round r's public, theta-independent decisions: participants, dropouts, the SecAgg abort, this rank's live
        clients.  Keyed by (seed, round) only, so computing them a round early (CC4 prefetch) changes nothing."""
        t = self.cfg.train
        p = self.cfg.privacy
        # under DP the participant set is part of the mechanism: keyed by the secret like the noise
        participants = sample_participants(self.num_clients, t.client_fraction,
                                           self.noise_seed if p.dp else t.seed, r, self.poisson)
        dropped = sample_dropouts(participants, t.dropout_prob, t.seed, r)
        # SecAgg+ abort (Bell et al.): a survivor left with fewer than the threshold of live mask neighbours would be
        # unmasked by the orphan-mask removal, so the round aggregates nothing.  The decision uses public data only
        # (participants, dropouts, the round-keyed graph): every rank takes it alike and still posts its (zero)
        # contribution to the one collective.
        sa_abort = bool(p.secure_agg and self.secagg is not None and participants
                        and not self.secagg.round_ok(participants, dropped, r))
        if sa_abort:
            dropped = list(participants)
        dropped_set = set(dropped)
        part_set = set(participants)
        local_part = [i for i, c in enumerate(self.local_ids) if c in part_set]
        local_alive = [i for i in local_part if self.local_ids[i] not in dropped_set]
        return {"participants": participants, "dropped": dropped, "sa_abort": sa_abort, "dropped_set": dropped_set,
                "local_alive": local_alive}

    def _prefetch(self, r: int) -> None:
        """CC4: build round r's theta-independent inputs now - its setup and, through the trainer, the minibatch plan,
        the tables and the gathered, encoded minibatches - while the previous round's collective is in flight."""
        if r >= self.cfg.train.num_rounds or not hasattr(self.adapter.trainer, "prepare_round"):
            return
        st = self._round_setup(r)
        pre = self.adapter.trainer.prepare_round(self.store, st["local_alive"], r)
        self._pre = (r, st, pre)
        self.prefetches = getattr(self, "prefetches", 0) + 1

    def run_round(self, r: int, sync: bool = True) -> dict:
        """One federated round.  With ``sync=False`` nothing reads device memory back: the round is
        only enqueued (the host can build round r+1 while the GPU runs round r) and the returned
        record holds device tensors until :meth:`resolve_record`."""
        t = self.cfg.train
        p = self.cfg.privacy
        self.timer.step(r)
        pre_r = self.__dict__.pop("_pre", None)
        pre = None
        if pre_r is not None and pre_r[0] == r:
            st, pre = pre_r[1], pre_r[2]
        else:
            st = self._round_setup(r)
        participants, dropped, sa_abort = st["participants"], st["dropped"], st["sa_abort"]
        dropped_set, local_alive = st["dropped_set"], st["local_alive"]
        t0 = time.perf_counter()
        dev = self.device
        P = self.P
        ids = [self.local_ids[i] for i in local_alive]
        # distributed DP: each client's share of the noise is N(0, sigma^2 C^2 / m) for the round's m live participants
        # (public: every rank knows the participant set and the dropouts), so the SecAgg sum carries exactly sigma C
        dp_mode = getattr(p, "noise_mode", "local")
        dp_scale = noise_scale(dp_mode, len(participants) - len(dropped)) if (p.dp and dp_mode != "local") else None
        fast = self.backend == "hip" and self.server_opt is None
        trainer = self.adapter.trainer
        if fast:
            # round epilogue on the device, run by the trainer right after the local steps (captured into the
            # round's hipGraph): the fused local reduce writes the head of the all-reduce buffer and the last
            # block of the same launch appends the fixed-point metrics.  Round-dependent inputs (DP noise keys,
            # uniform FedAvg weights) travel as per-client tables with the round's upload, never as kernel
            # arguments.
            if getattr(self, "_round_buf", None) is None:
                self._round_buf = torch.zeros(P + 6 + self.n_norm_slots, dtype=torch.int64, device=dev)
                # FusedApply arrival counter (self-resetting); allocated here, eagerly: created inside the round
                # graph's capture, its zero fill would become a node replayed every round
                self._apply_cnt = torch.zeros(1, dtype=torch.int32, device=dev)
            buf = self._round_buf
            extra = {}
            if p.dp and ids:
                from ..ops.fedavg_hip import dp_noise_keys
                extra["dpkeys"] = dp_noise_keys(ids, r, self.noise_seed)
            if t.weighting == "uniform":
                extra["fw"] = torch.ones(len(ids), dtype=torch.float64)
            if dp_scale is not None and ids:
                extra["dpscale"] = torch.full((len(ids),), dp_scale, dtype=torch.float32)
            if p.secure_agg and ids:
                # SecAgg on the device: every local client's pair-seed keys and mask signs for this round ride with
                # the round's tables; the fused reduce masks each client's ring element (K18), so the round stays
                # one graph launch
                extra["sa_seed"], extra["sa_sign"] = self.secagg.round_tables(ids, participants, dropped,
                                                                              self.num_clients, r)
                extra["sa_round"] = torch.full((len(ids),), r, dtype=torch.int32)
            if self.n_norm_slots and ids:
                extra["cid"] = torch.tensor(ids, dtype=torch.int32)
            agg = self.aggregator
            NN = self.n_norm_slots
            if getattr(self, "_round_outs", None) is None:     # [metrics | sat | wsum | norms], one per graph variant
                self._round_outs = [torch.zeros(6 + NN, dtype=torch.float64, device=dev) for _ in range(2)]
                self._out_writes = [0, 0]
                self._flip = 0
            ring = (p.secagg_bits, p.secagg_scale) if p.secure_agg else (0, 1.0)
            world, params_g, outs = self.world, self.params, self._round_outs

            fused = self.__dict__.setdefault("_apply_fused", {})

            def post(v):
                # ONE collective per round (CC2+CC3), then finalize + apply in place; captured into the round
                # graph (variant v writes metrics buffer v) when the collective allows it.  A single-rank round whose
                # epilogue already applied (variant v, in the same capture) has nothing left to do.
                if fused.pop("variant", None) == v:
                    return
                all_reduce_(buf, world)
                from ..ops._ext import ext
                ext().round_apply(buf, P, params_g, 1.0, outs[v], *ring, NN)

            def apply_variant(tabs, theta):
                """The metrics buffer variant whose post() the single-rank apply may fold into (None: no fold)."""
                v = tabs.get("variant", self._flip if tabs.get("eager") else None)
                if (v is not None and not world.distributed and P + 6 + NN <= FUSED_APPLY_MAX
                        and os.environ.get("QFEDX_FUSED_APPLY", "1") != "0"
                        and theta.data_ptr() == params_g.data_ptr()):
                    return v
                return None

            def fused_tail(tabs, theta):
                # plain FedAvg (no DP noise / clipping, no SecAgg masks) folded into the MFMA engine's fused Adam
                # epilogue of the last local step (hea_step.hip, QfxFedTail): same fixed-point terms, int64 atomics
                # into the zeroed buffer head, metrics packed and (single rank) the round applied by the last client
                if p.dp or p.secure_agg or NN or agg.backend != "hip" or \
                        os.environ.get("QFEDX_FED_TAIL", "1") == "0":
                    return None
                if getattr(agg, "_mask_u8", None) is None:
                    agg._mask_u8 = agg.angle_mask.to(torch.uint8).contiguous()
                if getattr(self, "_tail_cnt", None) is None:
                    self._tail_cnt = torch.zeros(1, dtype=torch.int32, device=dev)
                fed = [buf, theta, agg._mask_u8, tabs.get("fw", tabs["w"]), tabs["loss"].reshape(-1),
                       tabs["correct"].reshape(-1), tabs["nvalid"].reshape(-1), tabs["act"].reshape(-1),
                       self._tail_cnt]
                v = apply_variant(tabs, theta)
                if v is not None:
                    fed += [params_g, outs[v]]
                return {"fed": fed, "wrap": bool(agg.wrap), "n_norms": NN, "zero": buf[: P + 1]}

            def epilogue(params_k, tabs, theta):
                # one launch: the fused reduce writes the buffer head, its last block packs the metrics.  Single
                # rank, with post(v) known to follow (captured right behind it: tabs["variant"] = v; eager: the
                # variant post will take) the same launch also applies the round (no collective in between), one
                # launch fewer per round.  tabs["fed_done"]: the engine already ran all of it (fused_tail).
                sa = (tabs["sa_seed"], tabs["sa_sign"], tabs["sa_round"]) if "sa_seed" in tabs else None
                v = apply_variant(tabs, theta)
                apply = None
                fused.pop("variant", None)
                if tabs.get("fed_done"):
                    if v is not None:
                        fused["variant"] = v
                    return
                if v is not None:
                    apply = (params_g, outs[v], self._apply_cnt, *ring, NN)
                    fused["variant"] = v
                agg.local_reduce(params_k, theta, tabs.get("fw", tabs["w"]), r, ids, out=buf[: P + 1],
                                 keys=tabs.get("dpkeys"), secagg_tabs=sa, norm_cid=tabs.get("cid"),
                                 pack=(buf, tabs["loss"].reshape(-1), tabs["correct"].reshape(-1),
                                       tabs["nvalid"].reshape(-1), tabs["act"].reshape(-1)), apply=apply,
                                 dp_scale=tabs.get("dpscale"))
            epilogue.fused_tail = fused_tail
            graph_comm = self.graph_comm
            with self.timer.phase("local_train"):
                res = trainer.run_round(self.store, local_alive, self.params, r, epilogue=epilogue,
                                        extra=extra or None, post=post if graph_comm else None)
            if not local_alive:
                buf.zero_()
        else:
            with self.timer.phase("local_train"):
                res = trainer.run_round(self.store, local_alive, self.params, r,
                                        **({"pre": pre} if pre is not None else {}))
            with self.timer.phase("aggregate"):
                if t.weighting == "uniform":
                    w = torch.ones(len(local_alive), dtype=torch.float64, device=dev)
                elif "weights" in res:            # uploaded with the round's tables (no gather launch)
                    w = res["weights"]
                else:
                    if getattr(self, "_counts_dev", None) is None:
                        self._counts_dev = self.store.counts.to(torch.float64).to(dev)
                    w = self._counts_dev[res["lid"]]
                if local_alive:
                    contrib = self.aggregator.local_reduce(res["params"], self.params, w, r, ids,
                                                           participants=participants, dropped=dropped,
                                                           dp_scale=dp_scale)
                else:
                    contrib = torch.zeros(P + 1, dtype=torch.int64, device=dev)
                loss_sum = (res["loss"].double() * res["nvalid"].double()).sum()
                correct = (res["correct"].double() * res["act"].double()).sum()
                host_m = h2d(torch.tensor([float(res.get("samples", 0.0)), float(res.get("steps", 0))],
                                          dtype=torch.float64), dev)
                sat = self.aggregator.last_saturation if local_alive else None
                sat = (sat.to(dev).double().reshape(1) if sat is not None
                       else torch.zeros(1, dtype=torch.float64, device=dev))
                # CC6: this rank's clients' norms in their global slots (zero elsewhere): the metric SUM all-reduce
                # gathers them
                nslots = torch.zeros(self.n_norm_slots, dtype=torch.float64, device=dev)
                if self.n_norm_slots and local_alive and self.aggregator.last_norms is not None:
                    nslots[torch.tensor(ids, device=dev)] = self.aggregator.last_norms.double().to(dev)
                metrics = torch.cat([torch.stack([loss_sum, correct]).to(dev), host_m, sat, nslots])
        norms = None
        comm_bytes = 0
        with self.timer.phase("comm"):
            if fast:
                if res.get("post_done"):
                    v = res["post_variant"]
                else:
                    v = self._flip
                    self._flip ^= 1
                    post(v)
                self._out_writes[v] += 1
                comm_bytes = self._round_buf.numel() * 8
                out = self._round_outs[v]
                metrics = out[:5]                                     # + saturated fixed-point terms
                norms = out[6:6 + NN] if NN else None
            elif self.server_opt is not None:
                # server optimizer (CC5): small all-reduce of [weight | metrics]; the update sums are
                # reduce-scattered inside the sharded step and the new params all-gathered
                tail = torch.cat([contrib[P:P + 1].to(torch.int64),
                                  torch.round(metrics.double() * EXACT_SCALE).to(torch.int64)])
                all_reduce_(tail, self.world)
                # + the reduce-scatter of the padded update sums and the all-gather of the new parameter slices
                comm_bytes = tail.numel() * 8 + 2 * self.server_opt.padded * 8
                wsum = tail[0].double() / EXACT_SCALE
                metrics = tail[1:].double() / EXACT_SCALE
                self._set_params(self.server_opt.step(self.params, contrib[:P].to(torch.int64), wsum))
            elif p.secure_agg:
                all_reduce_(contrib, self.world)          # int64 ring elements: exact, mod later
                all_reduce_(metrics, self.world)
                comm_bytes = contrib.numel() * contrib.element_size() + metrics.numel() * metrics.element_size()
                mean_upd, wsum = self.aggregator.finalize(contrib)
                self._set_params(self.aggregator.apply(self.params, mean_upd, wsum=wsum))
            else:
                # ONE collective per round (CC2+CC3): [exact fixed-point update | weight | metrics]
                buf = torch.cat([contrib.to(torch.int64),
                                 torch.round(metrics.double() * EXACT_SCALE).to(torch.int64)])
                if self.cc4:
                    # CC4: round r + 1's theta-independent work (setup, plan, minibatch gather + encode) runs while
                    # this round's all-reduce is in flight (gloo: on its worker thread); theta_{r+1} waits for it
                    work = all_reduce_async(buf, self.world)
                    self._prefetch(r + 1)
                    work.wait()
                else:
                    all_reduce_(buf, self.world)
                comm_bytes = buf.numel() * 8
                mean_upd, wsum = self.aggregator.finalize(buf[: P + 1])
                metrics = buf[P + 1:].double() / EXACT_SCALE
                self._set_params(self.aggregator.apply(self.params, mean_upd, wsum=wsum))
        if not fast and self.n_norm_slots:
            norms, metrics = metrics[5:], metrics[:5]
        if p.dp:
            # the subsampled-Gaussian RDP bound holds for Poisson sampling at rate q; a fixed-size subset
            # drawn without replacement is accounted conservatively with no amplification (q = 1)
            q = min(1.0, t.client_fraction) if self.poisson else 1.0
            self.accountant.step(q, p.noise_multiplier, 1)
        rec = {"round": r + 1, "participants": len(participants), "dropped": len(dropped), "secagg_aborted": sa_abort,
               "_metrics": metrics, "_t0": t0,
               "_out_stamp": (v, self._out_writes[v]) if fast else None,
               "_norms": (norms, [c for c in participants if c not in dropped_set]) if norms is not None else None,
               "comm_bytes_per_rank": int(comm_bytes),
               "upload_bytes": int(len(participants) - len(dropped)) * (self.P + 1) * 4}
        if p.dp:
            rec["epsilon"] = self.accountant.get_epsilon(p.delta)
        return self.resolve_record(rec) if sync else rec

    def _set_params(self, new: torch.Tensor) -> None:
        """Update the global params IN PLACE: the trainer's cached round hipGraph reads them at a fixed address,
        so a fresh tensor per round (SecAgg / server-optimizer paths) would miss the graph cache every round."""
        self.params.copy_(new.to(self.params.dtype))

    def resolve_record(self, rec: dict) -> dict:
        """Read a round's metrics back (syncs with the device) and fill the derived fields."""
        if "_metrics" not in rec:
            return rec
        stamp = rec.pop("_out_stamp", None)
        if stamp is not None and self._out_writes[stamp[0]] != stamp[1]:
            raise RuntimeError(f"round {rec['round']}: its metrics buffer was reused by a later round; resolve "
                               "records (resolve_record) within two rounds")
        m = rec.pop("_metrics").double().cpu().tolist()
        dt = time.perf_counter() - rec.pop("_t0")
        nrm = rec.pop("_norms", None)
        if nrm is not None:                      # CC6: every client's pre-clip update norm, clip fraction
            vals = nrm[0].double().cpu().numpy()[nrm[1]] if nrm[1] else np.zeros(0)
            if vals.size:
                C = self.cfg.privacy.clip_norm
                q = np.quantile(vals, [0.1, 0.5, 0.9])
                rec.update({"clip_frac": float((vals > C).mean()), "norm_p10": float(q[0]), "norm_p50": float(q[1]),
                            "norm_p90": float(q[2]),
                            "norms_private": False})   # raw, un-noised statistics (runtime.log_client_norms)
        if len(m) > 4 and m[4] > 0:
            raise RuntimeError(f"round {rec['round']}: {int(m[4])} fixed-point FedAvg terms saturated at 2^53 "
                               "(|w * Delta| > 2^21): lower the aggregation weights (train.weighting=uniform) or "
                               "the update magnitude (DP clipping / learning rate)")
        rec.update({"train_loss": m[0] / max(m[2], 1.0) if m[2] else float("nan"),
                    "train_acc": m[1] / max(m[2], 1.0) if m[2] else float("nan"),
                    "local_steps": int(round(m[3])), "round_time_s": dt,
                    "local_steps_per_s": m[3] / dt if dt > 0 else 0.0})
        return rec

    def run(self) -> dict:
        t = self.cfg.train
        self.maybe_resume()
        accs = []
        if self.start_round == 0:
            ev = self.evaluate()
            accs.append(ev["test_acc"])
            if self.world.is_main:
                self.log.info(f"Round 0: Test Accuracy = {ev['test_acc']:.4f}")
            self.metrics.log({"round": 0, **ev})
        else:
            accs = [h.get("test_acc") for h in self.history if "test_acc" in h]
        t_start = time.perf_counter()
        for r in range(self.start_round, t.num_rounds):
            rec = self.run_round(r)
            if (r + 1) % max(1, t.eval_every) == 0 or r + 1 == t.num_rounds:
                rec.update(self.evaluate())
                accs.append(rec["test_acc"])
            self.history.append(rec)
            self.metrics.log(rec)
            if self.world.is_main and ((r + 1) % self.cfg.runtime.log_every == 0 or r + 1 == t.num_rounds):
                eps = f" eps={rec['epsilon']:.3f}" if "epsilon" in rec else ""
                self.log.info(f"Round {r + 1}: Test Accuracy = {rec.get('test_acc', float('nan')):.4f} "
                              f"train_loss={rec['train_loss']:.4f} {rec['local_steps_per_s']:.1f} local-steps/s{eps}")
            ck = self.cfg.runtime.checkpoint_every
            if ck and (r + 1) % ck == 0:
                self.save(r + 1)
        wall = time.perf_counter() - t_start
        auc = self.test_auc()
        if self.world.is_main:
            self.metrics.log({"final": True, "test_auc": auc, "wall_s": wall})
        self.metrics.close()
        return {"model": self.adapter.state_dict(self.params), "params": self.params, "accuracies": accs,
                "auc": auc,
                "history": self.history, "wall_s": wall,
                # mean ms per TIMED round of each phase and how many rounds were timed (on the GPU only every
                # runtime.timer_every-th round is; raw totals would undercount the run by that factor)
                "phases_ms_per_round": self.timer.per_phase(), "phase_rounds_timed": dict(self.timer.counts),
                "epsilon": self.accountant.get_epsilon(self.cfg.privacy.delta) if self.cfg.privacy.dp else None}
