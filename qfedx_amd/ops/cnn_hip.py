"""Client-batched TinyCNN on gfx950 (CFed path; reference ``Classical_FL.py:21-64``).

One local step of K clients x B samples:
  1. ``cnn_forward``  - fused conv1/conv2 + bias + ReLU + 2x2 max-pool (fp32 MFMA implicit GEMM, per
                        client weights), writes pooled maps + argmax codes
  2. fc1              - ``bmm`` over the client batch (plain batched GEMM -> hipBLASLt/rocBLAS; bias in the head)
  3. ``cnn_head``     - fc1 bias + ReLU + keyed dropout + fc2 + weighted CE, dlogits, fc2 grads, dL/dh1, fc1 bias grad
  4. fc1 backward     - ``cnn_fc1_wgrad`` (weight grad into the gradient rows) + one batched GEMM (dL/dpool2)
  5. ``cnn_backward`` - unpool + ReLU masks, conv2 weight/input grads, conv1 weight grads (MFMA),
                        deterministic fixed-order reduction into the flat [K, P] gradient
No autograd graph, no per-client Python loop; every buffer is sized [K, ...] once per shape.
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
        w = params[:, self.fc1w: self.fc1b].view(K, 64, 1568)
        bias = params[:, self.fc1b: self.fc2w]
        return torch.baddbmm(bias[:, None, :], pool2.view(K, B, 1568), w.transpose(1, 2)), w

    @torch.no_grad()
    def logits(self, params: torch.Tensor, X: torch.Tensor) -> torch.Tensor:
        """Eval forward (no dropout): [K, B, C]."""
        params = params.float().contiguous()
        K, B = X.shape[:2]
        _, _, _, pool2, _ = self.conv_forward(params, X)
        h1, _ = self._fc1(params, pool2, K, B)
        w2 = params[:, self.fc2w: self.fc2b].view(K, self.C, 64)
        b2 = params[:, self.fc2b: self.fc2b + self.C]
        return torch.baddbmm(b2[:, None, :], torch.relu(h1), w2.transpose(1, 2))

    @torch.no_grad()
    def loss_and_grads(self, params: torch.Tensor, xb: torch.Tensor, yb: torch.Tensor, wts: torch.Tensor,
                       mask, loss_out: torch.Tensor | None = None,
                       correct_out: torch.Tensor | None = None) -> dict:
        """``mask``: [K, B, 64] dropout mask, ``None`` (no dropout) or ``("philox", keys, stream, p)`` - per-client
        device Philox keys [K, 2] from which the head draws the inverted-dropout mask itself (u >= p kept x
        1/(1-p): ``tinycnn.dropout_masks``' exact values).  ``loss_out`` / ``correct_out``: optional contiguous fp32 [K] rows the head
        writes into directly."""
        C = ext()
        params = params.float().contiguous()
        K, B = xb.shape[:2]
        S = K * B
        Xf, pool1, am1, pool2, am2 = self.conv_forward(params, xb)
        w1 = params[:, self.fc1w: self.fc1b].view(K, 64, 1568)
        h1 = torch.bmm(pool2.view(K, B, 1568), w1.transpose(1, 2))    # the head adds the fc1 bias
        grad = torch.empty(K, self.P, dtype=torch.float32, device=self.device)   # every entry is written below
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
                   wts.reshape(S).float().contiguous(), dh1, dlog, loss, correct, grad)
        C.cnn_fc1_wgrad(dh1, pool2, K, B, grad, self.fc1w)      # written straight into the gradient rows
        dP2 = torch.bmm(dh1, w1).reshape(S, 1568).contiguous()
        G = C.cnn_bwd_groups(K, B)
        part = self._buf("part", (K * G, C.cnn_partial_size()))
        C.cnn_backward(Xf, params, K, B, self.off_conv, pool1, am1, pool2, am2, dP2, part, grad)
        return {"loss": loss, "grad": grad, "correct": correct}
