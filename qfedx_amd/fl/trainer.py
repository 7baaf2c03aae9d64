"""Client-batched local training ("client.py", ROADMAP.md:34-36; reference ``client_update``,
``Classical_FL.py:40-64``).

All of a rank's participating clients train in LOCKSTEP: step s of every client is one batched
kernel sequence over [K clients x B samples].  Clients keep their own minibatch order (Philox-keyed
permutation per (seed, round, client, epoch)), their own optimizer state row, and their own step
budget: with ``local_epochs`` E, client k runs E * ceil(n_k / B) steps (exactly the reference's
``epochs x len(dataloader)``); shorter clients are masked out of later steps, and a last partial
batch is handled by per-sample loss weights (padding rows weigh 0).  ``local_steps > 0`` instead
fixes the step count for every client (benchmarks).
"""
from __future__ import annotations

import math
import os
import time

import numpy as np
from typing import Optional

import torch

from ..utils.device import PackedUpload, h2d
from ..utils.seeding import _philox4x32_np, philox4x32, philox_key
from .optim import BatchedOptimizer

# The round prologue gathers every step's inputs up front below this buffer size.  The buffer lives in the round
# graph's private pool and up to _GRAPH_LRU graphs stay cached, so the cap bounds that reserve too (1.5 GiB).
UPFRONT_GATHER_BYTES = 1 << 28
# prologue gather blocks up to which the round prologue also does the host upload (its gather blocks read their indices
# from the pinned buffer): one launch fewer at the 8-client share (9.7 -> 8.1 us); at 2,048 one-row blocks the pinned
# index reads took 35 us.  Short rows are packed 16 to a block since (64 clients: 128 gather blocks).
FOLD_UPLOAD_MAX_BLOCKS = 512
FOLD_UPLOAD = os.environ.get("QFEDX_FOLD_UPLOAD", "1") != "0"     # (A/B knob)
_GRAPH_LRU = 6



def _wait_rounds(ent: dict, n: int) -> None:
    """Block until graph entry ``ent`` has finished the uploads of ``n`` replays (the round's first node, the upload
    kernel, publishes the count to a coherent pinned word once every block has read its pinned buffer): spins
    briefly, then yields; the GPU is normally far ahead of this."""
    if n <= 0:
        return
    flag = ent["flag"].view(torch.int64)
    if int(flag[0]) >= n:
        return
    spins, t0, tw = 0, None, time.perf_counter()
    while int(flag[0]) < n:
        spins += 1
        if spins > 64:
            time.sleep(20e-6)
            if t0 is None:
                t0 = time.perf_counter()
            elif time.perf_counter() - t0 > 5.0:     # never expected: drain the GPU, then the word must be there
                torch.cuda.synchronize()
                if int(flag[0]) < n:
                    raise RuntimeError(f"round signal stuck at {int(flag[0])} < {n}: device writes to the coherent "
                                       "pinned word are not visible to the host")
    WAIT_S[0] += time.perf_counter() - tw


WAIT_S = [0.0]     # host seconds spent waiting for the GPU in _wait_rounds (bench: host enqueue cost = loop - wait)

class ShardStore:
    """Device-resident padded shards: X [K, Nmax, F], y [K, Nmax], counts [K]."""

    def __init__(self, shards: list, client_ids: list, device, feature_fn=None):
        self.client_ids = list(client_ids)
        self.device = torch.device(device)
        K = len(shards)
        counts = [int(s[1].shape[0]) for s in shards]
        nmax = max(counts) if counts else 0
        feat_shape = tuple(shards[0][0].shape[1:]) if K else ()
        X = torch.zeros((K, nmax) + feat_shape, dtype=torch.float32)
        y = torch.zeros(K, nmax, dtype=torch.int64)
        for k, (Xs, ys) in enumerate(shards):
            X[k, : counts[k]] = Xs.float()
            y[k, : counts[k]] = ys.long()
        if feature_fn is not None:
            X = feature_fn(X)
        self.X = X.to(self.device)
        self.y = y.to(self.device)
        self.counts = torch.tensor(counts, dtype=torch.int64)
        self.nmax = nmax

    def __len__(self) -> int:
        return len(self.client_ids)


class BatchPlan:
    """Per-round minibatch schedule for a set of clients (host-side index tables, keyed RNG).

    Built by the native round scheduler (``csrc/runtime.cpp``: per-client Philox keys from one round key,
    keyed partial Fisher-Yates epoch orders, [S, K, B] index / weight / active tables) in microseconds; ``_plan_torch`` is the vectorised torch oracle / fallback.  Keyed by (seed, round,
    client id, epoch) only -> identical however clients are sharded over ranks.
    """

    def __init__(self, counts: torch.Tensor, client_ids: list, batch_size: int, round_num: int,
                 seed: int, local_epochs: int = 1, local_steps: int = 0, shuffle: bool = True,
                 native: bool | None = None):
        self.B = batch_size
        self.local_steps = local_steps
        C = _native_runtime() if native is not False else None
        if native and C is None:
            raise RuntimeError("native round scheduler requested but the extension is not built")
        rk = philox_key(seed, "batch", round_num) if shuffle else (0, 0)
        if C is not None:
            ids = torch.tensor([int(c) for c in client_ids], dtype=torch.int64)
            self.idx, self.wts, self.active, steps = C.batch_plan(counts.reshape(-1), ids, batch_size, rk[0], rk[1],
                                                                  local_epochs, local_steps, shuffle)
            self.steps_per_client = steps.tolist()
            self.max_steps = int(self.idx.shape[0])
        else:
            self._plan_torch(counts, client_ids, batch_size, rk, local_epochs, local_steps, shuffle)

    def _plan_torch(self, counts, client_ids, B, rk, local_epochs, local_steps, shuffle):
        K = len(client_ids)
        n = counts.to(torch.int64).reshape(-1)
        nb = (n + B - 1) // B                                   # batches per epoch
        if local_steps > 0:
            steps = torch.full((K,), local_steps, dtype=torch.int64)
            epochs = (steps * B + n.clamp(min=1) - 1) // n.clamp(min=1)
        else:
            steps = local_epochs * nb
            epochs = torch.full((K,), local_epochs, dtype=torch.int64)
        self.steps_per_client = steps.tolist()
        self.max_steps = int(steps.max()) if K else 0
        S, E, N = self.max_steps, max(int(epochs.max()) if K else 1, 1), max(int(n.max()) if K else 1, 1)
        perm = np.tile(np.arange(N, dtype=np.int64), (K, E, 1))
        if shuffle and K:
            ids = torch.tensor([int(c) for c in client_ids], dtype=torch.int64)
            ctr = torch.stack([ids & 0xFFFFFFFF, ids >> 32, torch.zeros_like(ids), torch.zeros_like(ids)], -1)
            keys = philox4x32(ctr, rk[0], rk[1])[:, :2].numpy()  # per-client key = Philox(round key, client id)
            nblk = (E * N + 3) // 4
            blk = np.arange(nblk, dtype=np.int64)
            c = np.stack([blk & 0xFFFFFFFF, blk >> 32, np.zeros_like(blk), np.zeros_like(blk)], -1)[None]
            w = _philox4x32_np(np.broadcast_to(c, (K, nblk, 4)), keys[:, 0:1], keys[:, 1:2])
            w = w.reshape(K, -1)[:, :E * N].reshape(K, E, N)      # raw words of elements e*N + j
            nn = n.numpy()[:, None]
            used = (steps.numpy() * B if local_steps > 0 else epochs.numpy() * np.maximum(n.numpy(), 1))[:, None]
            m = np.minimum(nn, used - np.arange(E)[None, :] * np.maximum(nn, 1))      # [K, E] prefix drawn
            jmax = np.minimum(m, nn - 1)
            kk_, ee_ = np.meshgrid(np.arange(K), np.arange(E), indexing="ij")
            for j in range(int(jmax.max()) if jmax.size else 0):   # partial Fisher-Yates, Lemire multiply-shift
                act = j < jmax
                span = np.maximum(nn - j, 0).astype(np.uint64)
                r = np.where(act, j + ((w[:, :, j] * span) >> np.uint64(32)).astype(np.int64), j)
                a, bvals = perm[:, :, j].copy(), perm[kk_, ee_, r]
                perm[:, :, j] = bvals
                perm[kk_, ee_, r] = a
        perm = torch.from_numpy(perm)
        s_ = torch.arange(S)[:, None, None]                       # [S, 1, 1]
        t_ = torch.arange(B)[None, None, :]                       # [1, 1, B]
        nk = n[None, :, None].clamp(min=1)
        kk = torch.arange(K)[None, :, None]
        if local_steps > 0:                                       # fixed steps: walk the epoch order cyclically
            pos = (s_ * B + t_) % (epochs[None, :, None] * nk)
            ep, i = pos // nk, pos % nk
            valid = torch.ones(S, K, B, dtype=torch.bool)
        else:                                                     # epochs x ceil(n/B) steps, last batch partial
            ep, jb = s_ // nb[None, :, None].clamp(min=1), s_ % nb[None, :, None].clamp(min=1)
            i = jb * B + t_
            valid = i < n[None, :, None]
            i = torch.where(valid, i, torch.zeros_like(i))
        active = (torch.arange(S)[:, None] < steps[None, :])      # [S, K]
        valid = valid & active[:, :, None]
        lin = (kk * E + ep.clamp(max=E - 1)) * N + i               # broadcast -> [S, K, B] linear indices
        # numpy gather: torch's OpenMP take on a few thousand elements can stall for tens of ms
        idx = torch.from_numpy(np.take(perm.contiguous().numpy(), lin.expand(S, K, B).contiguous().numpy()))
        cnt = valid.sum(-1, keepdim=True).clamp(min=1)
        self.idx = torch.where(valid, idx, torch.zeros_like(idx))
        self.wts = valid.float() / cnt.float()
        self.active = active.float()


def graph_bucket(k: int, k_max: int) -> int:
    """Captured client count for ``k`` participating clients: the next power of two up to 8, then the next
    multiple of 8, capped at the rank's client count ``k_max``.  Under Poisson client sampling the per-round
    count varies (Binomial(N, q)); bucketing keeps the number of distinct hipGraph shapes small, so rounds
    replay a cached graph instead of re-capturing (at the cost of < 8 idle client rows)."""
    if k <= 0:
        return 0
    b = 1 << (k - 1).bit_length() if k <= 8 else -(-k // 8) * 8
    return max(k, min(b, k_max))


def _pad_clients(tabs: dict, kp: int) -> dict:
    """Extend a round's client tables to ``kp`` clients with inactive rows: store slot of client 0, minibatch
    index 0, loss weight 0, step mask 0, FedAvg weight 0 (the optimizer leaves them untouched, the readout
    writes zero loss / hits for them); any other per-client table (first dim K) is zero-padded."""
    K = tabs["lid"].shape[0]
    if kp <= K:
        return tabs
    n = kp - K
    out = {}
    for name, t in tabs.items():
        if name == "lid":
            out[name] = torch.cat([t, t[:1].expand(n)])
        elif name in ("idx", "wts", "act", "nvalid"):              # [S, K, ...] step tables
            out[name] = torch.cat([t, torch.zeros_like(t[:, :1]).expand(-1, n, *t.shape[2:])], 1)
        else:                                                      # [K, ...] per-client tables (FedAvg weights, keys)
            out[name] = torch.cat([t, torch.zeros((n,) + tuple(t.shape[1:]), dtype=t.dtype)])
    return out


_NATIVE = []


def _native_runtime():
    if not _NATIVE:
        try:
            from .. import _qfedx_C as C
            _NATIVE.append(C if hasattr(C, "batch_plan") else None)
        except ImportError:
            _NATIVE.append(None)
    return _NATIVE[0]


def _tail(epilogue, dv, theta, variant=None, eager=False):
    """The round epilogue's FedAvg as a ``fed_tail`` maker for the last local step (``epilogue.fused_tail``), or None.
    The returned callable gets ``done = True`` when the engine ran the FedAvg itself (the epilogue then skips it)."""
    make = getattr(epilogue, "fused_tail", None)
    if make is None:
        return None

    def tail(loss_all, correct_all):
        tabs = dict(dv, loss=loss_all, correct=correct_all)
        if variant is not None:
            tabs["variant"] = variant
        if eager:
            tabs["eager"] = True
        return make(tabs, theta)
    tail.done = False
    return tail


class RoundPrefetch:
    """A round's theta-independent inputs, built ahead (CC4): plan, host tables, and on the portable path the
    gathered + encoded minibatches of every step."""

    def __init__(self, round_num: int, local_idx: list):
        self.round_num = round_num
        self.local_idx = local_idx
        self.plan = self.tabs = self.cids = self.common = self.batches = None
        self.method = None


class VQCClientTrainer:
    """Runs one federated round of local training for a rank's clients (batched)."""

    def __init__(self, spec, engine, train_cfg, device, backend: str = "torch"):
        self.spec = spec
        self.engine = engine
        self.cfg = train_cfg
        self.device = torch.device(device)
        self.backend = backend

    def encode(self, X: torch.Tensor) -> torch.Tensor:
        return self.spec.encode_features(X)

    @staticmethod
    def _gather_blocks(rows: int, F: int) -> int:
        """Gather blocks of the round prologue for ``rows`` rows of F features (csrc/train_kernels.hip: short rows are
        packed 256 / tps to a block)."""
        from ..ops._ext import ext
        tps = int(ext().prologue_gather_lanes(int(F)))
        return rows if tps == 0 else -(-rows // (256 // tps))

    def _gather_mode(self) -> int:
        spec = self.spec
        return 2 if spec.amplitude else (1 if spec.feature_scale == "minmax" else 0)

    def _body(self, X, Y, lid, theta, idx_d, wts_d, act_d, steps: int, round_num: int, method: str,
              traj_keys=None, ro_keys=None, tail=None, batches=None, xy=None):
        """Device work of one round (capturable): local steps of all clients.

        ``X`` [Nc, Nmax, F] / ``Y`` [Nc, Nmax] are the whole device-resident client store and ``lid`` [K]
        the round's store slots: on HIP each step's minibatch is gathered and angle-encoded straight from
        the store by one kernel (no per-round copy of the clients' shards), the round starts with one
        params/optimizer-state init kernel.

        Returns (params [K,P], loss [S,K], correct [S,K]): per-step, per-client weighted loss and hit
        counts are written straight into round buffers by the readout kernel (no per-step metric ops);
        the round epilogue reduces them.  With a noise model, every sample runs ``trajectories``
        Pauli-trajectory replicas (loss weights split evenly) and the readout is confused /
        shot-sampled, all keyed per client and step."""
        cfg, spec = self.cfg, self.spec
        noise = self.engine.noise
        T = noise.trajectories if (noise is not None and spec.noisy) else 1
        K = lid.shape[0]
        P = theta.numel()
        params = torch.empty(K, P, dtype=torch.float32, device=self.device)
        opt_kind = "sgd" if cfg.optimizer == "spsa" else cfg.optimizer
        opt = BatchedOptimizer(opt_kind, (K, P), self.device, cfg.learning_rate, cfg.momentum,
                               backend=self.backend, zero_init=False)
        loss_all = torch.empty(steps, K, dtype=torch.float32, device=self.device)
        correct_all = torch.empty(steps, K, dtype=torch.float32, device=self.device)
        BT = idx_d.shape[-1] * T
        fused = self.backend == "hip" and X.is_cuda
        # one prologue launch: client rows + optimizer state initialised and every step's minibatch gathered
        # and encoded up front (trajectory replicas, T > 1, and rounds whose inputs pass UPFRONT_GATHER_BYTES
        # gather per step)
        upfront = fused and T == 1 and steps * K * BT * X.shape[-1] * 4 <= UPFRONT_GATHER_BYTES
        # xy: every step's minibatches already gathered into these buffers on the side stream (CC4, _graphed): the
        # prologue only sets the client rows (and the first step's fragments); no upload or gather here
        pregathered = xy is not None and upfront
        # the round graph's host upload (_graphed): folded into the prologue launch while its gather is small (each
        # gather block reads its indices from the pinned buffer itself: csrc/train_kernels.hip UploadJob), else its
        # own copy kernel here, ahead of every reader of the uploaded tables
        pend = self.__dict__.pop("_pending_upload", None)
        if pend is not None and not (upfront and idx_d.is_contiguous() and FOLD_UPLOAD
                                     and self._gather_blocks(steps * K * BT, X.shape[-1]) <= FOLD_UPLOAD_MAX_BLOCKS):
            from ..ops._ext import ext
            ext().host_upload(*pend)
            pend = None
        if fused:
            from ..ops._ext import ext
            mode = self._gather_mode()
            if pregathered:
                xbuf, ybuf = xy
            else:
                xbuf = torch.empty(steps if upfront else 1, K, BT, X.shape[-1], dtype=torch.float32,
                                   device=self.device)
                ybuf = torch.empty((steps if upfront else 1) * K * BT, dtype=torch.int64, device=self.device)
            dummy = torch.zeros(K, BT, 0 if spec.noisy else 1, device=self.device) if spec.amplitude else None
        else:
            rows = lid[:, None]
        fj = None
        # ``tail(loss_all, correct_all)``: the round epilogue's FedAvg as a ``fed_tail`` for the last step's engine
        # call (the MFMA engine folds it into its fused Adam epilogue); ``tail.done`` says the engine ran it
        ft = tail(loss_all, correct_all) if (tail is not None and fused and method == "adjoint") else None
        if upfront:
            m, v, t = opt.init_state()
            # the MFMA engine's first-step fragments come from theta in the same launch (every row starts as theta);
            # the FedAvg tail's all-reduce buffer head is zeroed there too
            fj = self.engine.prologue_frag_job() if method == "adjoint" and noise is None else None
            gi = idx_d[:0] if pregathered else idx_d.contiguous()         # steps = 0: no gather blocks
            ext().round_prologue(theta.float().contiguous(), params, m, v, t, X, Y, lid, gi, mode,
                                 float(spec.alpha), xbuf[:0] if pregathered else xbuf, ybuf, frag_job=fj,
                                 frag_bf16=bool(getattr(self.engine.hip, "bf16", False)),
                                 zero=ft["zero"] if ft is not None else None,
                                 upload=list(pend) if pend is not None else None)
        else:
            ft = None                                  # (the tail needs the prologue's zeroed buffer head)
            opt.init_round(params, theta.float())
        for s in range(steps):
            bi = idx_d[s]
            ws = wts_d[s]
            if T > 1:
                bi = bi.repeat(1, T)
                ws = ws.repeat(1, T) / T
            if fused:
                if upfront:
                    xs, yb = xbuf[s], ybuf.view(steps, K, BT)[s]
                else:
                    ext().batch_gather(X, Y, lid, bi.contiguous(), mode, float(spec.alpha), xbuf[0], ybuf)
                    xs, yb = xbuf[0], ybuf.view(K, BT)
                init = xs if spec.amplitude else None
                xang = dummy if spec.amplitude else xs
            elif batches is not None:                 # gathered + encoded ahead (prepare_round, CC4)
                xang, yb = batches[s]
                init = None
            else:
                xb = X[rows, bi]                     # [K, B, F]
                yb = Y[rows, bi]
                init = xb if spec.amplitude else None
                xang = self.encode(xb)
            xang = self.engine.augment(xang, traj_keys, s)
            res = self.engine.loss_and_grads(xang, yb, ws, params, method, rng_keys=(cfg.seed, round_num, s),
                                             readout_keys=ro_keys, step=s, out_loss=loss_all[s],
                                             out_correct=correct_all[s], init=init, fused_opt=(opt, act_d[s]),
                                             shared_frags=fj[1] if (fj is not None and s == 0) else None,
                                             fed_tail=ft if s == steps - 1 else None)
            if res.get("fed_done", False):
                tail.done = True
            if not res.get("opt_done", False):      # the MFMA engine runs HIP Adam inside its gradient reduction
                opt.step(params, res["grad"], act_d[s])
        return params, loss_all, correct_all

    def prepare_round(self, store: ShardStore, local_idx: list, round_num: int, extra: Optional[dict] = None,
                      gather: bool = True) -> "RoundPrefetch":
        """The theta-INDEPENDENT part of a round (CC4): the keyed minibatch plan, the round's host tables and, on the
        portable path, every step's gathered and encoded minibatch.  The server builds round r + 1's while round r's
        collective is in flight (``all_reduce_async``); on the graphed HIP path the upload and the gather of round
        r + 1 run on a side stream against round r's graph (``_graphed``, ``cc4``).  ``gather=False``: tables only."""
        cfg = self.cfg
        K = len(local_idx)
        pre = RoundPrefetch(round_num, list(local_idx))
        if K == 0:
            return pre
        li = torch.tensor(local_idx, dtype=torch.int64)
        cids = [store.client_ids[i] for i in local_idx]
        plan = BatchPlan(store.counts[li], cids, cfg.batch_size, round_num, cfg.seed,
                         cfg.local_epochs, cfg.local_steps)
        nvalid = (plan.wts > 0).sum(-1).float() * plan.active
        pre.common = {"samples": float(nvalid.sum()), "steps": int(sum(plan.steps_per_client)), "client_ids": cids,
                      "n_samples": store.counts[li].to(torch.float64)}
        if plan.idx.numel() and int(plan.idx.max()) >= max(1, store.nmax):   # the gather kernel trusts the table
            raise RuntimeError("minibatch plan indexes past the client store")
        tabs = {"lid": li, "idx": plan.idx, "wts": plan.wts, "act": plan.active, "nvalid": nvalid,
                "w": store.counts[li].to(torch.float64)}   # FedAvg sample-count weights
        for name, t in (extra or {}).items():
            if name in tabs or t.shape[0] != K:
                raise ValueError(f"extra table {name!r} must be a new per-client [K, ...] table")
            tabs[name] = t
        pre.plan, pre.tabs, pre.cids = plan, tabs, cids
        pre.method = "spsa" if cfg.optimizer == "spsa" else cfg.grad_method
        fused = self.backend == "hip" and store.X.is_cuda
        if gather and not fused and self.engine.noise is None and not self.spec.amplitude:
            # portable path: every step's minibatch gathered and encoded now (theta-independent)
            rows = li.to(store.X.device)[:, None]
            pre.batches = []
            for s_ in range(plan.max_steps):
                bi = plan.idx[s_].to(store.X.device)
                pre.batches.append((self.encode(store.X[rows, bi]), store.y[rows, bi]))
        return pre

    def run_round(self, store: ShardStore, local_idx: list, theta_g: torch.Tensor, round_num: int,
                  epilogue=None, extra: Optional[dict] = None, post=None, pre: "RoundPrefetch" = None) -> dict:
        """Train clients ``store[local_idx]`` from the global params.

        Returns device tensors: ``params`` [K,P], ``loss`` / ``correct`` [S,K] per step, ``nvalid`` /
        ``act`` [S,K] (valid samples / active flag per client and step), ``lid`` [K] (store slots), plus
        host scalars ``samples`` / ``steps`` and ``n_samples`` (cpu, for weighting).

        ``extra``: more per-client host tables [K, ...] uploaded with the round's tables (e.g. DP noise keys).
        ``epilogue(params, tables, theta)``: device work run right after the local steps, on the trained
        params (possibly padded with inactive weight-0 rows), the round's device tables and the global params;
        on the hipGraph path it is captured into the round graph, so it may only launch device work on static
        buffers (no host values that change per round).
        ``post()``: the round's collective + global update (all-reduce of the epilogue's buffer, apply to
        ``theta_g`` in place), run after the epilogue: captured into the round graph too when possible (then the
        whole round - host upload, local steps, reduce, all-reduce, apply - is ONE graph launch), else run
        eagerly.  The returned ``post_done`` says it ran (the caller must not run it again).
        ``pre``: this round's ``prepare_round`` result, built ahead while the previous round's collective ran (CC4);
        used when it is for the same round and clients (else the tables are built here)."""
        K = len(local_idx)
        P = theta_g.numel()
        if K == 0:
            z = torch.zeros(0, 0, device=self.device)
            return {"params": torch.zeros(0, P, device=self.device), "loss": z, "correct": z, "nvalid": z, "act": z,
                    "lid": torch.zeros(0, dtype=torch.int64, device=self.device), "samples": 0.0, "steps": 0,
                    "client_ids": [], "n_samples": torch.zeros(0, dtype=torch.float64)}
        if pre is None or pre.round_num != round_num or pre.local_idx != list(local_idx) or pre.plan is None:
            pre = self.prepare_round(store, local_idx, round_num, extra, gather=False)
        else:
            self.prefetch_hits = getattr(self, "prefetch_hits", 0) + 1
        plan, tabs, cids, common, method = pre.plan, pre.tabs, pre.cids, pre.common, pre.method
        noise = self.engine.noise
        graphed = self.use_graph and method == "adjoint" and noise is None
        if graphed:
            tabs = _pad_clients(tabs, graph_bucket(K, len(store)))
            fit = getattr(self.engine, "fit_tiles", None)
            if fit is not None and not self.__dict__.get("_graph_cache"):
                # small per-rank batches: smaller MFMA tiles (decided once, before the first round graph)
                fit(int(tabs["lid"].shape[0]) * plan.B)
        up = PackedUpload(tabs)
        traj_keys = ro_keys = None
        if noise is not None:
            traj_keys = noise.client_keys("noise_traj", round_num, cids, self.device)
            ro_keys = noise.client_keys("shots", round_num, cids, self.device)
        post_v = None
        if graphed:
            params, loss_all, correct_all, dv, post_v = self._graphed(store, up, theta_g, plan, round_num,
                                                                      epilogue, post)
            # padding clients (inactive, weight 0) only fill the captured shape: the FedAvg reduce sees the
            # K real rows; their [S, Kpad] metric columns are all zero
            params = params[:K]
            dv = dict(dv, w=dv["w"][:K], lid=dv["lid"][:K])
        else:
            dv = up.to_device(self.device)
            theta = theta_g.to(self.device)
            tail = _tail(epilogue, dv, theta, eager=True)
            params, loss_all, correct_all = self._body(store.X, store.y, dv["lid"], theta, dv["idx"],
                                                       dv["wts"], dv["act"], plan.max_steps, round_num, method,
                                                       traj_keys, ro_keys, tail=tail, batches=pre.batches)
            if epilogue is not None:    # eager: ``post`` (if any) runs right after, on the caller's side
                epilogue(params, dict(dv, loss=loss_all, correct=correct_all, eager=True,
                                      fed_done=bool(tail and tail.done)), theta)
        return {"params": params, "loss": loss_all, "correct": correct_all, "nvalid": dv["nvalid"], "act": dv["act"],
                "lid": dv["lid"], "weights": dv["w"], "post_done": post_v is not None, "post_variant": post_v,
                **common}

    # ------------------------------------------------------------------ hipGraph capture
    @property
    def use_graph(self) -> bool:
        return self.backend == "hip" and self.device.type == "cuda" and getattr(self, "graphs", True)

    def _graphed(self, store, up, theta_g, plan, round_num, epilogue=None, post=None):
        """Replay the whole round as ONE hipGraph (static shapes: #clients, steps, batch).

        Captured once per SHAPE, not per client set, in two variants that differ only in the pinned host buffer
        their first node reads the round's packed tables from (client slots, minibatch indices, loss weights, step
        masks, per-client keys; a copy kernel, or the round prologue itself when its gather is small): round r
        fills pinned buffer r % 2 - free once round r - 2's
        replay has finished - and replays variant r % 2, so the host stays a round ahead with no upload launch
        of its own.  The captured launches gather every step's minibatches from the (static) client store by
        slot, so client sampling reuses the graph.  The global params are read in place when they are a float32
        device tensor (the runner updates them in place), otherwise copied into a static buffer.  ``epilogue``
        (the fused FedAvg reduce + metrics pack) and ``post`` (the collective + in-place apply) are captured
        after the local steps, so a round is one graph launch; if the collective cannot be captured, ``post``
        runs eagerly after the replay.  A small LRU bounds the live graphs.
        """
        K = up.layout[0][4][0]
        dev = self.device
        direct = theta_g.is_cuda and theta_g.dtype == torch.float32 and theta_g.is_contiguous()
        # CC4 (world_size > 1, or QFEDX_CC4=1): the round's host upload and minibatch gather leave the graph for a side
        # stream, into per-variant table / minibatch buffers, so round r + 1's upload + gather run while round r's
        # graph - its local steps, and its all-reduce + apply at the end - is still on the main stream
        F = store.X.shape[-1]
        cc4 = bool(getattr(self, "cc4", False)) and plan.max_steps * K * plan.B * F * 4 <= UPFRONT_GATHER_BYTES
        key = (K, plan.max_steps, plan.B, store.nmax, store.X.data_ptr(), tuple(l[0] for l in up.layout),
               theta_g.data_ptr() if direct else None, epilogue is not None, post is not None, cc4)
        cache = self.__dict__.setdefault("_graph_cache", {})
        ent = cache.pop(key, None)
        if ent is None:
            from ..ops._ext import ext
            E = ext()
            packs = [torch.empty(up.nbytes, dtype=torch.uint8, device=dev) for _ in range(2 if cc4 else 1)]
            dvs = [up.to_device(dev, pk) for pk in packs]
            pack, dv = packs[0], dvs[0]
            ent = {"pack": pack, "dv": dv, "theta": theta_g if direct else theta_g.to(dev).float().clone(),
                   "cc4": cc4, "packs": packs, "dvs": dvs,
                   "pin": [E.host_alloc(up.nbytes), E.host_alloc(up.nbytes)], "flip": 0,
                   # upload-completion counter (round count + block arrivals) and its coherent host mirror, both
                   # written by the graph's first node (the upload kernel's last block)
                   "ctr": torch.zeros(2, dtype=torch.int64, device=dev), "flag": E.host_alloc(8, True),
                   "launched": 0}
            ent["flag"].zero_()
            if cc4:
                ent["xy"] = [(torch.empty(plan.max_steps, K, plan.B, F, dtype=torch.float32, device=dev),
                              torch.empty(plan.max_steps * K * plan.B, dtype=torch.int64, device=dev))
                             for _ in range(2)]
                ent["side"] = torch.cuda.Stream(device=dev)
                ent["ev_g"] = [torch.cuda.Event() for _ in range(2)]
                ent["ev_c"] = [torch.cuda.Event() for _ in range(2)]
                ent["c_rec"] = [False, False]
                ent["pshape"] = torch.empty(K, theta_g.numel(), dtype=torch.float32, device=dev)

            def body(variant=None, bv=0):
                # ``variant``: set when post(variant) is captured right behind the epilogue (it may fold into it);
                # ``bv``: the variant whose tables / minibatch buffers the capture reads (CC4: one set per variant)
                d = dvs[bv] if cc4 else dv
                tail = _tail(epilogue, d, ent["theta"], variant=variant)
                out = self._body(store.X, store.y, d["lid"], ent["theta"], d["idx"], d["wts"], d["act"],
                                 plan.max_steps, round_num, "adjoint", tail=tail,
                                 xy=ent["xy"][bv] if cc4 else None)
                if epilogue is not None:
                    tabs = dict(d, loss=out[1], correct=out[2], fed_done=bool(tail and tail.done))
                    if variant is not None:
                        tabs["variant"] = variant
                    epilogue(out[0], tabs, ent["theta"])
                return out
            # the graph owns its workspaces: eager calls (evaluation) can never regrow/free them
            ent["ws"] = {}
            cur = torch.cuda.current_stream(dev)
            with self.engine.hip.private_workspace(ent["ws"]):
                side = torch.cuda.Stream(device=dev)
                side.wait_stream(cur)
                with torch.cuda.stream(side):       # warm-up (no collective / apply): modules loaded, sizes fixed
                    if cc4:     # gather only, from the device tables to_device filled (no pinned upload, no count)
                        self._cc4_gather(ent, store, up, 0, wait=False, upload=False)
                    body()
                cur.wait_stream(side)
                ent["graphs"], ent["out"] = [], []
                ent["post_in_graph"] = post is not None and getattr(self, "graph_comm", True)
                for v in range(2):
                    up._fill(ent["pin"][v][: up.nbytes])
                    g = torch.cuda.CUDAGraph()
                    try:
                        # thread-local capture: the RCCL watchdog thread queries its work events at any time, and in
                        # the global mode such a query during the capture aborted the process (hipErrorStreamCapture-
                        # Unsupported, seen once in tests/test_gpu_rccl.py)
                        with torch.cuda.graph(g, capture_error_mode="thread_local"):
                            if not cc4:
                                self._pending_upload = (ent["pin"][v][: up.nbytes], pack, ent["ctr"], ent["flag"])
                            out = body(v if ent["post_in_graph"] else None, v)
                            if ent["post_in_graph"]:
                                post(v)
                    except Exception as exc:
                        self.__dict__.pop("_pending_upload", None)
                        if not ent["post_in_graph"]:
                            raise
                        # the collective refused capture although the ranks agreed it could be captured
                        # (parallel/dist.py agree_graph_comm): graphs without it, post() runs eagerly right after
                        # the replay - the same point of this rank's collective sequence, so ranks stay matched
                        import warnings
                        warnings.warn(f"round collective capture failed ({exc!r}); running it eagerly on this rank")
                        self.capture_fallbacks = getattr(self, "capture_fallbacks", 0) + 1
                        self.graph_comm = False
                        ent["post_in_graph"] = False
                        torch.cuda.synchronize(dev)
                        ent["graphs"], ent["out"] = [], []
                        for v2 in range(2):
                            g = torch.cuda.CUDAGraph()
                            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                                if not cc4:
                                    self._pending_upload = (ent["pin"][v2][: up.nbytes], pack, ent["ctr"],
                                                            ent["flag"])
                                out = body(None, v2)
                            ent["graphs"].append(g)
                            ent["out"].append(out)
                        break
                    ent["graphs"].append(g)
                    ent["out"].append(out)
            while len(cache) >= _GRAPH_LRU:         # LRU: drop the oldest shape
                old = cache.pop(next(iter(cache)))
                # the counter only says its uploads are done: drain the device before the graph and its
                # workspaces are released (rare: more live shapes than the LRU holds)
                _wait_rounds(old, old["launched"])
                torch.cuda.current_stream(dev).synchronize()
        cache[key] = ent                            # most recently used last
        if not direct:
            ent["theta"].copy_(theta_g.float())
        v = ent["flip"]
        ent["flip"] ^= 1
        n = ent["launched"]
        _wait_rounds(ent, n - 1)                    # pinned buffer v: its last reader (replay n - 2) is done
        up._fill(ent["pin"][v][: up.nbytes])
        if cc4:
            # side stream: this round's upload + gather, behind only the graph that last read variant v's buffers
            # (round r - 2); it runs while round r - 1's graph, collective included, is still on the main stream
            self._cc4_gather(ent, store, up, v)
            torch.cuda.current_stream(dev).wait_event(ent["ev_g"][v])
        ent["graphs"][v].replay()
        if cc4:
            ent["ev_c"][v].record(torch.cuda.current_stream(dev))
            ent["c_rec"][v] = True
        ent["launched"] = n + 1
        if post is not None and not ent["post_in_graph"]:
            post(v)
        return (*ent["out"][v], ent["dvs"][v] if cc4 else ent["dv"], v if post is not None else None)

    def _cc4_gather(self, ent, store, up, v: int, wait: bool = True, upload: bool = True) -> None:
        """The round's theta-independent device work on the side stream (CC4): the upload of the round's tables from
        pinned buffer v into the variant's device tables and every step's minibatch gather + encode, one prologue
        launch without client rows (csrc/train_kernels.hip: its gather blocks read the indices from the pinned copy,
        its last block posts the upload-completion count).  Ordered after the graph that last read variant v."""
        from ..ops._ext import ext
        side = ent["side"]
        if wait and ent["c_rec"][v]:
            side.wait_event(ent["ev_c"][v])
        d = ent["dvs"][v]
        xb, yb = ent["xy"][v]
        with torch.cuda.stream(side):
            ext().round_prologue(ent["theta"], ent["pshape"], None, None, None, store.X, store.y, d["lid"],
                                 d["idx"].contiguous(), self._gather_mode(), float(self.spec.alpha), xb, yb,
                                 rows=False, upload=[ent["pin"][v][: up.nbytes], ent["packs"][v], ent["ctr"],
                                                     ent["flag"]] if upload else None)
            ent["ev_g"][v].record(side)
        if not wait:
            torch.cuda.current_stream(self.device).wait_stream(side)
