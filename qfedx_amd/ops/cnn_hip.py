"""Client-batched TinyCNN on gfx950 (CFed path; reference ``Classical_FL.py:21-64``).

One local step of K clients x B samples:
  1. ``cnn_forward``  - fused conv1/conv2 + bias + ReLU + 2x2 max-pool (fp32 MFMA implicit GEMM, per
                        client weights), writes pooled maps + argmax codes
  2. ``cnn_fc1_forward`` - fc1 as per-client MFMA tiles, split over the 1568 inputs into FC_KS partial sums (no
                        library GEMM: a batched GEMM's algorithm changes with the client count, so a client's result
                        would depend on how clients are sharded over ranks)
  3. ``cnn_head``     - fc1 partials (fixed order) + bias + ReLU + keyed dropout + fc2 + weighted CE, dlogits, fc2
                        grads, dL/dh1, fc1 bias grad
  4. fc1 backward     - ``cnn_fc1_dgrad`` (dL/dpool2) then ``cnn_fc1_wgrad`` (weight grad into the gradient rows)
  5. ``cnn_backward`` - unpool + ReLU masks, conv2 weight/input grads, conv1 weight grads (MFMA),
                        deterministic fixed-order reduction into the flat [K, P] gradient
With ``sgd`` (``loss_and_grads``) the local SGD-momentum step is fused into the kernels that produce the gradient
entries (head: fc2 + fc1 bias, fc1_wgrad: fc1 weights, the conv reduction: conv weights + biases; cnn_args.h): the
gradient is never written or re-read and no optimizer launch runs.  The first local step of a round may read the
global parameters broadcast (``theta.expand(K, P)``, row stride 0) and write the stepped client rows, so the round
prologue sets no per-client rows.
No autograd graph, no per-client Python loop, no library kernels; every buffer is sized [K, ...] once per shape.
Evaluation (reference ``evaluate_model``, ``Classical_FL.py:83-102``) runs the same conv + fc1 kernels and
``cnn_eval_head`` (logits, fused CE / argmax-hit sums).
"""
from __future__ import annotations

import torch

from ..models import tinycnn as tc
from ._ext import ext


class HipTinyCNN:
    def __init__(self, num_classes: int, device):
        self.C = num_classes
        self.device = torch.device(device)
        self.P = tc.n_params(num_classes)
        b = tc.layer_boundaries(num_classes)     # conv1.w conv1.b conv2.w conv2.b fc1.w fc1.b fc2.w fc2.b
        self.off_conv = [b[0], b[1], b[2], b[3]]
        self.fc1w, self.fc1b, self.fc2w, self.fc2b = b[4], b[5], b[6], b[7]
        self._ws = {}

    def _buf(self, name, shape, dtype=torch.float32):
        n = 1
        for s in shape:
            n *= s
        t = self._ws.get(name)
        if t is None or t.numel() < n or t.dtype != dtype:
            t = torch.empty(n, dtype=dtype, device=self.device)
            self._ws[name] = t
        return t[:n].view(shape)

    def conv_forward(self, params: torch.Tensor, X: torch.Tensor):
        """params [K, P]; X [K, B, 1, 28, 28] -> pool1, am1, pool2, am2 (flat per sample)."""
        K, B = X.shape[:2]
        S = K * B
        Xf = X.reshape(S, 784).float().contiguous()
        pool1 = self._buf("pool1", (S, 16 * 196))
        am1 = self._buf("am1", (S, 16 * 196), torch.uint8)
        pool2 = self._buf("pool2", (S, 32 * 49))
        am2 = self._buf("am2", (S, 32 * 49), torch.uint8)
        ext().cnn_forward(Xf, params, K, B, self.off_conv, pool1, am1, pool2, am2)
        return Xf, pool1, am1, pool2, am2

    def _fc1(self, params, pool2, K, B):
        """fc1 pre-activation partial sums [K, FC_KS, B, 64] (bias added by the heads)."""
        C = ext()
        h1p = self._buf("h1p", (K, C.cnn_fc1_splits(), B, 64))
        C.cnn_fc1_forward(pool2, params, self.fc1w, K, B, h1p)
        return h1p

    @torch.no_grad()
    def logits(self, params: torch.Tensor, X: torch.Tensor, y: torch.Tensor | None = None):
        """Eval forward (no dropout): logits [K, B, C]; with labels ``y`` [K, B] also the (CE sum, hits) float64
        device scalars, summed per 64-sample block by the head and over the blocks here."""
        params = params.float().contiguous()
        K, B = X.shape[:2]
        _, _, _, pool2, _ = self.conv_forward(params, X)
        h1p = self._fc1(params, pool2, K, B)
        C = ext()
        out = torch.empty(K * B, self.C, dtype=torch.float32, device=self.device)
        stats = self._buf("eval_stats", (K * C.cnn_eval_blocks(B), 2), torch.float64)
        yy = y.reshape(-1).long().contiguous() if y is not None else None
        C.cnn_eval_head(h1p, params, self.fc1b, self.fc2w, self.fc2b, self.C, K, B, yy, out, stats)
        if y is None:
            return out.view(K, B, self.C)
        s = stats.sum(0)
        return out.view(K, B, self.C), s[0], s[1]

    @torch.no_grad()
    def loss_and_grads(self, params: torch.Tensor, xb: torch.Tensor, yb: torch.Tensor, wts: torch.Tensor,
                       mask, loss_out: torch.Tensor | None = None,
                       correct_out: torch.Tensor | None = None, sgd: dict | None = None) -> dict:
        """``mask``: [K, B, 64] dropout mask, ``None`` (no dropout) or ``("philox", keys, stream, p)`` - per-client
        device Philox keys [K, 2] from which the head draws the inverted-dropout mask itself (u >= p kept x
        1/(1-p): ``tinycnn.dropout_masks``' exact values).  ``loss_out`` / ``correct_out``: optional contiguous fp32 [K] rows the head
        writes into directly.  ``sgd``: fuse the local SGD-momentum step (dict pout, buf, t_in, t_out, act, lr, mu,
        keep; cnn_args.h): ``params`` are the rows read (``theta.expand(K, P)`` on a round's first step) and the
        stepped rows go to ``pout``; the returned ``grad`` is then None."""
        C = ext()
        if params.stride(0) != 0:
            params = params.float().contiguous()
        K, B = xb.shape[:2]
        S = K * B
        Xf, pool1, am1, pool2, am2 = self.conv_forward(params, xb)
        h1 = self._fc1(params, pool2, K, B)                            # partial sums; the head adds them + bias
        if sgd is None:
            grad = torch.empty(K, self.P, dtype=torch.float32, device=self.device)   # every entry is written below
            sk = hy = None
        else:
            grad = torch.empty(0, 0, dtype=torch.float32, device=self.device)
            sk = [params, sgd["pout"], sgd["buf"], sgd["t_in"], sgd["t_out"], sgd["act"].float().contiguous()]
            hy = [float(sgd["lr"]), float(sgd["mu"]), 1.0 if sgd["keep"] else 0.0]
        dh1 = self._buf("dh1", (K, B, 64))
        dlog = self._buf("dlog", (S, 16))
        loss = loss_out if loss_out is not None else torch.empty(K, dtype=torch.float32, device=self.device)
        correct = correct_out if correct_out is not None else torch.empty(K, dtype=torch.float32, device=self.device)
        if isinstance(mask, tuple):
            _, dkeys, stream, p = mask
            m, dk, dst, dp, ds = None, dkeys.reshape(K, 2).long().contiguous(), int(stream), float(p), \
                float(torch.tensor(1.0) / (1 - p))
        else:
            m = mask.float().contiguous() if mask is not None else torch.ones(K, B, 64, device=self.device)
            dk, dst, dp, ds = None, 0, 0.0, 1.0
        C.cnn_head(h1, self.fc1b, m, dk, dst, dp, ds, params, self.fc2w, self.fc2b, self.C, K, B, yb.reshape(S).long().contiguous(),
                   wts.reshape(S).float().contiguous(), dh1, dlog, loss, correct, grad, sk, hy)
        # dL/dpool2 reads the fc1 weights BEFORE the weight-gradient launch may step them in place (fused SGD)
        dP2 = self._buf("dP2", (S, 1568))
        C.cnn_fc1_dgrad(dh1, params, self.fc1w, K, B, dP2)
        C.cnn_fc1_wgrad(dh1, pool2, K, B, grad, self.fc1w, sk, hy)      # straight into the gradient rows / step
        G = C.cnn_bwd_groups(K, B)
        part = self._buf("part", (K * G, C.cnn_partial_size()))
        C.cnn_backward(Xf, params, K, B, self.off_conv, pool1, am1, pool2, am2, dP2, part, grad, sk, hy)
        return {"loss": loss, "grad": grad if sgd is None else None, "correct": correct}


def precision_check(num_classes: int, device, K: int = 16, B: int = 32, seed: int = 0) -> dict:
    """Untimed evidence for the CFed kernels' arithmetic (bench_suite lines): logits and per-client gradients of
    ``HipTinyCNN`` on K clients x B MNIST-like samples against float64 torch autograd, as max |error| / max |value|
    (logits; each parameter tensor's gradient), and the same for float32 torch on the CPU - the fp32 yardstick."""
    import torch.nn.functional as F
    from ..models import tinycnn as tc
    C = num_classes
    g = torch.Generator().manual_seed(seed)
    params = torch.stack([tc.init_flat(C, seed + k) for k in range(K)]) + 0.02 * torch.randn(K, tc.n_params(C),
                                                                                              generator=g)
    X = torch.rand(K, B, 1, 28, 28, generator=g)
    X[X < 0.6] = 0.0
    y = torch.randint(0, C, (K, B), generator=g)
    w = torch.full((K, B), 1.0 / B)
    mask = (torch.rand(K, B, 64, generator=g) >= 0.5).float() * 2.0

    def ref(dtype):
        p = params.to(dtype).clone().requires_grad_(True)
        logits = tc.batched_forward(p, X.to(dtype), C, mask.to(dtype))
        nll = F.cross_entropy(logits.reshape(-1, C), y.reshape(-1), reduction="none").reshape(K, B)
        (nll * w.to(dtype)).sum().backward()
        return logits.detach().double(), p.grad.double()

    l64, g64 = ref(torch.float64)
    l32, g32 = ref(torch.float32)
    hip = HipTinyCNN(C, device)
    dev = torch.device(device)
    lh = hip.logits(params.to(dev), X.to(dev)).double().cpu()
    # logits() runs without dropout; the gradient check uses the same dropout mask as the reference
    lref = tc.batched_forward(params.double(), X.double(), C).detach()
    r = hip.loss_and_grads(params.to(dev), X.to(dev), y.to(dev), w.to(dev), mask.to(dev))
    gh = r["grad"].double().cpu()
    bounds = tc.layer_boundaries(C)

    def grad_err(gx):
        return max(float((gx[:, a:b] - g64[:, a:b]).abs().max() / g64[:, a:b].abs().max().clamp_min(1e-30))
                   for a, b in zip(bounds[:-1], bounds[1:]))

    return {"max_rel_err_logits": float((lh - lref).abs().max() / lref.abs().max()),
            "max_rel_err_grad": grad_err(gh),
            "fp32_torch_max_rel_err_logits": float((l32 - l64).abs().max() / l64.abs().max()),
            "fp32_torch_max_rel_err_grad": grad_err(g32),
            "precision_ref": "float64 torch autograd", "precision_samples": K * B}
