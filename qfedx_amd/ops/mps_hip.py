"""HIP paths of the MPS backend.

* ``MpsChainProgram`` (csrc/mps_chain.hip; math: quantum/mps_chain.py): ``VQCEngine(backend="mps")`` routes <Z> and
  adjoint gradients here on a GPU when ``mps_chain.eligible(spec)`` (the angle-encoded RX/RZ + CNOT-chain ansatz with
  <= 3 layers: exact bond 2^L <= 8, any qubit count).
* ``MpsMpoProgram`` (csrc/mps_mpo.hip; tables: quantum/mps_mpo.py): any other lowered circuit whose MPO bonds stay
  <= 16 without recompression - ``MPSProgram.expz_vjp`` / ``expz_rows`` use it on the GPU.
The einsum-network MPS (``quantum/mps.py``) stays the path for truncating circuits and on the CPU."""
from __future__ import annotations

import torch

from ..quantum.mps_chain import _FEATURES, eligible
from ._ext import ext

_EMPTY = torch.zeros(0)


class MpsChainProgram:
    def __init__(self, spec, device):
        if not eligible(spec):
            raise ValueError("the MPS chain kernel covers angle-encoded RX/RZ + CNOT-chain VQCs with 1..3 layers")
        self.spec = spec
        self.n, self.L, self.C = spec.n_qubits, spec.n_layers, spec.n_classes
        self.n_theta = spec.n_theta
        self.readout = [int(q) for q in spec.readout]
        self.feature = _FEATURES[spec.feature_map.lower()]
        self.device = torch.device(device)
        self._ws = {}

    def _buf(self, name, numel):
        t = self._ws.get(name)
        if t is None or t.numel() < numel:
            t = torch.empty(numel, dtype=torch.float32, device=self.device)
            self._ws[name] = t
        return t[:numel]

    def _run(self, xang, theta, w=None):
        K, B, F = xang.shape
        S = K * B
        x = xang.reshape(S, F).float().contiguous()
        th = theta.float().contiguous()
        z = torch.empty(S, self.C, dtype=torch.float32, device=self.device)
        rp = self._buf("rp", S * self.n * 128)
        if w is None:
            ext().mps_chain(x, th, B, self.n, self.L, self.feature, self.readout, _EMPTY, z, _EMPTY, rp, _EMPTY)
            return z.view(K, B, self.C), None
        g = torch.empty(S, 2 * self.n * self.L, dtype=torch.float32, device=self.device)
        ro = self._buf("ro", S * (max(self.readout) + 1) * 128)
        ext().mps_chain(x, th, B, self.n, self.L, self.feature, self.readout, w.reshape(S, self.C).float().contiguous(),
                        z, g, rp, ro)
        return z.view(K, B, self.C), g.view(K, B, -1)

    @torch.no_grad()
    def expz(self, xang: torch.Tensor, theta: torch.Tensor) -> torch.Tensor:
        """<Z_c> [K, B, C] for encoded features [K, B, n] and per-client theta [K, >= n_theta]."""
        return self._run(xang, theta)[0]

    @torch.no_grad()
    def train(self, xang: torch.Tensor, params: torch.Tensor, y: torch.Tensor, wmask: torch.Tensor):
        """One launch for a noiseless training step: <Z>, the logits a <Z> + b, the weighted softmax cross entropy and
        dL/d<Z> per sample in the kernel (qfx_readout.h, as the MFMA engine's fused readout), then the gradient sweeps
        - the separate <Z> launch, its right sweep and the torch readout ops are gone.  params [K, n_theta + 2C]
        (theta | a | b) -> (loss [K], grad [K, n_theta + 2C], correct [K], expz [K, B, C]), ``ce_readout``'s
        definitions."""
        K, B, F = xang.shape
        S = K * B
        C = self.C
        x = xang.reshape(S, F).float().contiguous()
        p = params.float().contiguous()
        z = torch.empty(S, C, dtype=torch.float32, device=self.device)
        dl = torch.empty(S, C, dtype=torch.float32, device=self.device)
        lossv = torch.empty(S, dtype=torch.float32, device=self.device)
        hitv = torch.empty(S, dtype=torch.float32, device=self.device)
        g = torch.empty(S, 2 * self.n * self.L, dtype=torch.float32, device=self.device)
        rp = self._buf("rp", S * self.n * 128)
        ro = self._buf("ro", S * (max(self.readout) + 1) * 128)
        ext().mps_chain(x, p, B, self.n, self.L, self.feature, self.readout, _EMPTY, z, g, rp, ro,
                        y.reshape(S).long().contiguous(), wmask.reshape(S).float().contiguous(), self.n_theta, dl,
                        lossv, hitv)
        zk, dlk = z.view(K, B, C), dl.view(K, B, C)
        grad = torch.cat([g.view(K, B, -1).sum(1), (dlk * zk).sum(1), dlk.sum(1)], -1)
        return lossv.view(K, B).sum(1), grad, hitv.view(K, B).sum(1), zk

    @torch.no_grad()
    def grads(self, xang: torch.Tensor, theta: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
        """d/dtheta of sum_{b, c} w[k, b, c] <Z_c>_{k, b}: [K, n_theta] (per-sample gradients summed over each
        client's samples in order)."""
        return self._run(xang, theta, w)[1].sum(1)


class MpsMpoProgram:
    """HIP contraction (csrc/mps_mpo.hip) of an ``MPSProgram`` that is never recompressed (``autograd_ok``) and
    whose cuts carry at most 4 two-qubit gates (bond <= 16): any 1-qubit gate kinds, CX / CZ at any distance - the
    ring / all-to-all / custom circuits the chain kernel does not cover.  One workgroup per sample builds each
    qubit's tensor from its event list (``quantum/mps_mpo.py``) and runs the transfer-environment sweeps; the
    gradient launch pulls dL/d<Z> back to every rotation angle.  Replaces the einsum network's ~10 small batched
    GEMMs per gate (and their autograd tape) on the GPU; the CPU keeps the einsum network."""

    def __init__(self, prog):
        from ..quantum.mps_mpo import ROTATIONS, compile_mpo
        self.n = prog.n
        self.G = len(prog.ops_list)
        self.device = prog.device
        self.tab_host = compile_mpo(prog.ops_list, prog.n)
        self.tab = {k: v.to(self.device) for k, v in self.tab_host.items()}
        # dL/d(angle) is reported for the slot-carrying rotations, as MPSProgram.expz_vjp masks its AD gradient
        self.mask = torch.tensor([s >= 0 and k in ROTATIONS for k, _, _, s in prog.ops_list], device=self.device)
        self._ws = {}
        self.launches = 0

    @staticmethod
    def eligible(prog) -> bool:
        from ..quantum.mps_mpo import compile_mpo
        if prog.device.type != "cuda" or prog.dtype != torch.complex64 or not prog.autograd_ok or prog.n < 2:
            return False
        try:
            compile_mpo(prog.ops_list, prog.n)
        except ValueError:
            return False
        return True

    def _buf(self, name, numel):
        t = self._ws.get(name)
        if t is None or t.numel() < numel:
            t = torch.empty(numel, dtype=torch.float32, device=self.device)
            self._ws[name] = t
        return t[:numel]

    def run(self, ang: torch.Tensor, readout, w=None):
        """ang [S, G] gate angles -> (<Z_c> [S, C], dL/d(angle) [S, G] masked to rotations, or None without w)."""
        ro = [int(q) for q in readout]
        if not 1 <= len(ro) <= 8:
            raise ValueError("the MPO kernel reads out 1..8 qubits")
        ang = ang.float().contiguous()
        S = ang.shape[0]
        if ang.shape[1] != self.G:
            raise ValueError(f"angles [S, {ang.shape[1]}] for a {self.G}-gate program")
        z = torch.empty(S, len(ro), dtype=torch.float32, device=self.device)
        t, h = self.tab, self.tab_host
        rp = self._buf("rp", S * self.n * 512)
        self.launches += 1
        if w is None:
            ext().mps_mpo(ang, t["gkind"], t["events"], t["sinfo"], t["nbits"], h["sinfo"], h["nbits"], ro, _EMPTY,
                          z, _EMPTY, rp, _EMPTY)
            return z, None
        dang = torch.zeros(S, self.G, dtype=torch.float32, device=self.device)
        rob = self._buf("ro", S * (max(ro) + 1) * 512)
        ext().mps_mpo(ang, t["gkind"], t["events"], t["sinfo"], t["nbits"], h["sinfo"], h["nbits"], ro,
                      w.reshape(S, len(ro)).float().contiguous(), z, dang, rp, rob)
        return z, torch.where(self.mask, dang, torch.zeros_like(dang))
