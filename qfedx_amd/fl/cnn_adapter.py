"""CFed adapter: client-batched TinyCNN local training (reference ``client_update``,
``Classical_FL.py:40-64``; BASELINE config 4 "CFed classical-CNN path, 128 clients").

Per local step all of a rank's clients run together: [K, B] minibatches (keyed shuffles), one
batched forward/backward (grouped convs + batched GEMMs; fused gfx950 kernels on the HIP backend),
keyed inverted-dropout masks, CE loss, then ONE fused multi-client SGD-momentum (or Adam) update of
the flat [K, P] buffer.  Optimizer state is fresh every round, like the reference's per-round
``optim.SGD(lr, momentum=0.9)`` (``:53``).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ..models import tinycnn as tc
from .optim import BatchedOptimizer
from ..utils.device import PackedUpload
from .trainer import UPFRONT_GATHER_BYTES, BatchPlan, ShardStore


class CNNClientTrainer:
    def __init__(self, num_classes: int, train_cfg, device, backend: str = "torch"):
        self.C = num_classes
        self.cfg = train_cfg
        self.device = torch.device(device)
        self.backend = backend
        self._hip = None
        if backend == "hip":
            from ..ops.cnn_hip import HipTinyCNN
            self._hip = HipTinyCNN(num_classes, self.device)

    def loss_and_grads(self, params, xb, yb, wts, mask, loss_out=None, correct_out=None, sgd=None):
        if self._hip is not None:
            return self._hip.loss_and_grads(params, xb, yb, wts, mask, loss_out, correct_out, sgd=sgd)
        if sgd is not None:
            raise ValueError("the fused SGD step exists on the HIP backend only")
        p = params.detach().requires_grad_(True)
        logits = tc.batched_forward(p, xb, self.C, mask)
        nll = F.cross_entropy(logits.reshape(-1, self.C), yb.reshape(-1), reduction="none").reshape(yb.shape)
        loss = (nll * wts).sum(-1)
        loss.sum().backward()
        correct = ((logits.argmax(-1) == yb) & (wts > 0)).sum(-1).float()
        return {"loss": loss.detach(), "grad": p.grad, "correct": correct}

    def run_round(self, store: ShardStore, local_idx: list, theta_g: torch.Tensor, round_num: int,
                  epilogue=None, extra=None, post=None) -> dict:
        """Same contract as ``VQCClientTrainer.run_round`` (per-step [S,K] loss/correct round buffers, optional
        ``extra`` per-client tables and device ``epilogue``, here run eagerly; ``post`` is left to the caller)."""
        cfg = self.cfg
        K = len(local_idx)
        P = theta_g.numel()
        if K == 0:
            z = torch.zeros(0, 0, device=self.device)
            return {"params": torch.zeros(0, P, device=self.device), "loss": z, "correct": z, "nvalid": z, "act": z,
                    "lid": torch.zeros(0, dtype=torch.int64, device=self.device), "samples": 0.0, "steps": 0,
                    "client_ids": [], "n_samples": torch.zeros(0, dtype=torch.float64)}
        li = torch.tensor(local_idx, dtype=torch.int64)
        cids = [store.client_ids[i] for i in local_idx]
        plan = BatchPlan(store.counts[li], cids, cfg.batch_size, round_num, cfg.seed, cfg.local_epochs,
                         cfg.local_steps)
        nvalid = (plan.wts > 0).sum(-1).float() * plan.active
        if plan.idx.numel() and int(plan.idx.max()) >= max(1, store.nmax):
            raise RuntimeError("minibatch plan indexes past the client store")
        tabs = {"lid": li, "idx": plan.idx, "wts": plan.wts, "act": plan.active, "nvalid": nvalid,
                "w": store.counts[li].to(torch.float64)}
        if self._hip is not None:   # dropout Philox keys ride with the round's tables; the head draws the masks
            tabs["dkeys"] = tc.dropout_keys(cids, cfg.seed, round_num)
        for name, t in (extra or {}).items():
            if name in tabs or t.shape[0] != K:
                raise ValueError(f"extra table {name!r} must be a new per-client [K, ...] table")
            tabs[name] = t
        dv = PackedUpload(tabs).to_device(self.device)
        params = torch.empty(K, P, dtype=torch.float32, device=self.device)
        opt = BatchedOptimizer(cfg.optimizer if cfg.optimizer != "spsa" else "sgd", (K, P), self.device,
                               cfg.learning_rate, cfg.momentum, backend=self.backend, zero_init=False)
        S = plan.max_steps
        loss_all = torch.empty(S, K, dtype=torch.float32, device=self.device)
        correct_all = torch.empty(S, K, dtype=torch.float32, device=self.device)
        fused = self.backend == "hip" and store.X.is_cuda
        # SGD-momentum fused into the gradient-producing kernels (HIP): the round's first step reads theta broadcast
        # and writes the stepped client rows, so no row init, no gradient buffer and no optimizer launch
        fuse_sgd = fused and self._hip is not None and opt.kind in ("sgd", "sgdm", "spsa") and \
            getattr(cfg, "fuse_optimizer", True)
        theta_dev = theta_g.to(self.device).float().contiguous()
        upfront = False
        if fused:   # minibatches gathered straight from the device store by slot (no per-round shard copy)
            from ..ops._ext import ext
            img = tuple(store.X.shape[2:])
            Xf = store.X.view(store.X.shape[0], store.X.shape[1], -1)
            B = plan.B
            # one prologue launch (client rows + optimizer state, every step's minibatch) while the round's
            # images fit a modest buffer; long rounds gather per step
            upfront = S * K * B * Xf.shape[-1] * 4 <= UPFRONT_GATHER_BYTES
            xbuf = torch.empty(S if upfront else 1, K, B, Xf.shape[-1], dtype=torch.float32, device=self.device)
            ybuf = torch.empty((S if upfront else 1) * K * B, dtype=torch.int64, device=self.device)
        else:
            rows = dv["lid"][:, None]
        if upfront:
            m, v, t = opt.init_state()
            ext().round_prologue(theta_dev, params, m, v, t, Xf, store.y, dv["lid"], dv["idx"].contiguous(), 2, 1.0,
                                 xbuf, ybuf, rows=not fuse_sgd)
        else:
            opt.init_round(params, theta_dev)
        for s in range(S):
            if upfront:
                xb, yb = xbuf[s].view(K, B, *img), ybuf.view(S, K, B)[s]
            elif fused:
                ext().batch_gather(Xf, store.y, dv["lid"], dv["idx"][s], 2, 1.0, xbuf[0], ybuf)
                xb, yb = xbuf[0].view(K, B, *img), ybuf.view(K, B)
            else:
                xb = store.X[rows, dv["idx"][s]]
                yb = store.y[rows, dv["idx"][s]]
            if self._hip is not None:   # the head draws the keyed mask itself (no upload or launches per step)
                mask = ("philox", dv["dkeys"], s, 0.5)
            else:
                mask = tc.dropout_masks(cids, cfg.batch_size, cfg.seed, round_num, s, self.device)
            if fuse_sgd:
                sgd = dict(opt.fused_sgdm(last=s == S - 1), pout=params, act=dv["act"][s])
                pin = theta_dev.expand(K, P) if s == 0 else params
                res = self.loss_and_grads(pin, xb, yb, dv["wts"][s], mask, loss_all[s], correct_all[s], sgd=sgd)
            else:
                res = self.loss_and_grads(params, xb, yb, dv["wts"][s], mask, loss_all[s], correct_all[s])
                opt.step(params, res["grad"], dv["act"][s], last=s == S - 1)
            if res["loss"].data_ptr() != loss_all[s].data_ptr():    # portable path: separate outputs
                loss_all[s].copy_(res["loss"])
                correct_all[s].copy_(res["correct"])
        if epilogue is not None:
            epilogue(params, dict(dv, loss=loss_all, correct=correct_all, eager=True), theta_g.to(self.device).float())
        return {"params": params, "loss": loss_all, "correct": correct_all, "nvalid": dv["nvalid"], "act": dv["act"],
                "lid": dv["lid"], "weights": dv["w"], "samples": float(nvalid.sum()), "steps": int(sum(plan.steps_per_client)),
                "client_ids": cids, "n_samples": store.counts[li].to(torch.float64)}


class TinyCNNAdapter:
    def __init__(self, cfg, device, backend: str):
        self.C = cfg.model.n_classes
        self.device = torch.device(device)
        self.trainer = CNNClientTrainer(self.C, cfg.train, device, backend)
        self.n_params = tc.n_params(self.C)
        self.eval_batch = 1024

    def init_params(self, seed: int) -> torch.Tensor:
        return tc.init_flat(self.C, seed)

    def angle_mask(self):
        return None

    def state_dict(self, params: torch.Tensor) -> dict:
        return dict(tc.flat_to_state_dict(params.detach().cpu(), self.C))

    def from_state_dict(self, sd: dict) -> torch.Tensor:
        return tc.state_dict_to_flat(sd, self.C)

    def _fwd(self, params: torch.Tensor, xb: torch.Tensor) -> torch.Tensor:
        x = xb.reshape(1, -1, 1, 28, 28).float()
        hip = self.trainer._hip
        if hip is not None:
            return hip.logits(params[None].float(), x)[0]
        return tc.batched_forward(params[None].float(), x, self.C)[0]

    @torch.no_grad()
    def logits(self, params: torch.Tensor, X: torch.Tensor) -> torch.Tensor:
        out = [self._fwd(params, X[s: s + self.eval_batch]) for s in range(0, X.shape[0], self.eval_batch)]
        return torch.cat(out) if out else torch.zeros(0, self.C, device=X.device)

    @torch.no_grad()
    def evaluate(self, params: torch.Tensor, X: torch.Tensor, y: torch.Tensor):
        if X.shape[0] == 0:
            return 0.0, 0.0, 0.0
        loss_sum = torch.zeros((), dtype=torch.float64, device=X.device)
        correct = torch.zeros((), dtype=torch.float64, device=X.device)
        hip = self.trainer._hip
        for s in range(0, X.shape[0], self.eval_batch):       # no per-batch host sync (reference :100)
            xb, yb = X[s: s + self.eval_batch], y[s: s + self.eval_batch]
            if hip is not None:                               # HIP: CE and argmax hits fused into the eval head
                _, ls, hits = hip.logits(params[None].float(), xb.reshape(1, -1, 1, 28, 28).float(), yb[None])
                loss_sum += ls
                correct += hits
                continue
            logits = self._fwd(params, xb)
            loss_sum += F.cross_entropy(logits, yb, reduction="sum").double()
            correct += (logits.argmax(-1) == yb).sum().double()
        return float(loss_sum), float(correct), float(X.shape[0])
