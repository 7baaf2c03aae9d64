"""gfx950 statevector program: plans + workspaces + kernel launch sequences.

``HipProgram`` owns three plans of one lowered circuit (built once by the native planner):
  * ``eval``  : forward from the product state, last pass = readout partials only (no store)
  * ``train`` : forward, last pass stores psi and readout partials
  * ``adj``   : adjoint sweep (reverse program, psi + lambda, gradient slab)
and the device workspaces (psi, lambda, readout partials, gradient slab) sized for the largest batch
seen.  A local training step is then a fixed launch sequence (all on the current stream, capturable
in a hipGraph):  train passes -> readout+CE -> adjoint passes -> gradient reduce.

Each pass runs either as a circuit-specialised kernel (generated from the plan and compiled with
hiprtc for gfx950 by ``csrc/jit.cpp``; default) or through the ahead-of-time interpreter kernel
(``csrc/statevec.hip``; ``QFEDX_JIT=0`` or when specialisation is unavailable).  Both execute the
same plan and are tested against each other and the float64 oracle.
"""
from __future__ import annotations

import contextlib
import os

import torch

from ._ext import ext
from .plan_tools import FIN_READOUT, FIN_STORE, parse_blob

KMAX = 12        # tile = 2^12 amplitudes = 256 lanes x 16 registers
MODE_FWD_PRODUCT, MODE_FWD_LOAD, MODE_ADJ = 0, 1, 2
_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(_PKG, "csrc")
JIT_CACHE = os.environ.get("QFEDX_JIT_CACHE", os.path.join(os.path.dirname(_PKG), "build", "jit"))
ARCH = os.environ.get("QFEDX_ARCH", "gfx950")


_NO_KEYS = torch.zeros(0, dtype=torch.int64)


def _keys(keys, noise) -> torch.Tensor:
    if noise.shots > 0:
        if keys is None:
            raise ValueError("shot sampling needs per-client Philox keys")
        return keys.contiguous()
    return _NO_KEYS


def choose_R(n: int) -> int:
    return 16 if n >= 4 else 4


def jit_enabled() -> bool:
    return os.environ.get("QFEDX_JIT", "1") != "0"


def slot_csr(info: dict, n_theta: int) -> torch.Tensor:
    """slot -> gradient-gate CSR of a plan: int32 [offsets (n_theta + 1) | gate ids], gates in plan order
    (the order the device sums them in)."""
    lists = [[] for _ in range(n_theta)]
    for g, e in enumerate(info["gates"]):
        if 0 <= e["slot"] < n_theta and e["kind"] <= 3:          # rx / ry / rz / p carry gradients
            lists[e["slot"]].append(g)
    offs, ent = [0], []
    for lst in lists:
        ent += lst
        offs.append(len(ent))
    return torch.tensor(offs + ent, dtype=torch.int32)


class _Plan:
    def __init__(self, ops, coef, n, R, kmax, readout, n_theta, mode, final_flags, device, jit: bool,
                 bf16: bool = False):
        C = ext()
        blob = C.plan(torch.as_tensor(ops), torch.as_tensor(coef), n, R, kmax, list(readout), n_theta,
                      mode, final_flags)
        self.info = parse_blob(blob)
        self.blob_cpu = blob
        self.blob = blob.to(device)
        self.R = R
        self.adjoint = mode == MODE_ADJ
        self.passes = [(p["offset"], p["K"], p["NGRAD"], p["NOPS"]) for p in self.info["passes"]]
        self.k = self.info["passes"][0]["K"]
        self.n = n
        self.csr = slot_csr(self.info, n_theta).to(device) if self.adjoint else None
        self.jit_handles = None
        if jit:
            self.jit_handles = [C.jit_prepare(blob, i, self.adjoint, JIT_CACHE, CSRC, ARCH, bf16)[0]
                                for i in range(len(self.passes))]

    @property
    def tiles_per_state(self) -> int:
        return 1 << (self.n - self.k)


class HipProgram:
    def __init__(self, ops, coef, n_qubits: int, readout, device, n_theta: int, state_dtype: str = "fp32",
                 kmax: int = KMAX, jit: bool | None = None, x_width: int | None = None):
        if state_dtype not in ("fp32", "bf16"):
            raise ValueError(f"state_dtype must be fp32 or bf16, got {state_dtype!r}")
        self.bf16 = state_dtype == "bf16"
        self.n = n_qubits
        self.readout = list(readout)
        self.C = len(self.readout)
        self.device = torch.device(device)
        self.n_theta = n_theta
        self.x_width = n_qubits if x_width is None else x_width
        self.R = choose_R(n_qubits)
        self.jit = jit_enabled() if jit is None else jit
        if self.bf16 and not self.jit:
            raise RuntimeError("bf16 statevector storage needs the circuit-specialised (JIT) kernels; "
                               "unset QFEDX_JIT=0")
        args = (ops, coef, n_qubits, self.R, kmax, self.readout, n_theta)
        self._plan_args = (ops, coef, kmax)
        self.eval_plan = _Plan(*args, MODE_FWD_PRODUCT, FIN_READOUT, self.device, self.jit, self.bf16)
        self.train_plan = _Plan(*args, MODE_FWD_PRODUCT, FIN_STORE | FIN_READOUT, self.device, self.jit, self.bf16)
        self.adj_plan = _Plan(*args, MODE_ADJ, 0, self.device, self.jit, self.bf16)
        # statevector storage between passes: complex64, or packed bf16 (re, im) in one int32
        self.state_torch_dtype = torch.int32 if self.bf16 else torch.complex64
        self.G = self.train_plan.info["G"]
        self._ws = {}

    # ------------------------------------------------------------------ workspaces
    @contextlib.contextmanager
    def private_workspace(self, ws: dict):
        """Route workspace allocations to ``ws`` (owned by a captured hipGraph).

        A graph bakes buffer addresses into its kernel nodes, so its workspaces must never be
        regrown or freed by later eager calls (e.g. an evaluation with a larger batch)."""
        saved = self._ws
        self._ws = ws
        try:
            yield ws
        finally:
            self._ws = saved

    def _buf(self, name: str, numel: int, dtype) -> torch.Tensor:
        t = self._ws.get(name)
        if t is None or t.numel() < numel or t.dtype != dtype:
            t = torch.empty(numel, dtype=dtype, device=self.device)
            self._ws[name] = t
        return t[:numel]

    def _run_passes(self, plan: _Plan, adjoint: bool, psi, lam, params, spc, xang, w_read, part, slab, S):
        C = ext()
        for i, (off, k, ngrad, nops) in enumerate(plan.passes):
            if plan.jit_handles is not None:
                C.jit_launch(plan.jit_handles[i], plan.blob, off, psi, lam, params, spc, xang, w_read, part, slab,
                             S, ngrad)
            else:
                C.pass_launch(plan.R, adjoint, plan.blob, off, k, self.n, nops, plan.info["G"], psi, lam, params,
                              spc, xang, w_read, part, slab, S, ngrad)

    # ------------------------------------------------------------------ forward / eval
    @torch.no_grad()
    def expz(self, xang: torch.Tensor, theta: torch.Tensor, noise=None, keys=None, step: int = 0,
             init: torch.Tensor | None = None) -> torch.Tensor:
        K, B, F = xang.shape
        if F != self.x_width:
            raise ValueError(f"expected {self.x_width} x-slot values per sample, got {F}")
        S = K * B
        x = xang.reshape(S, F).float().contiguous()
        th = theta.float().contiguous()
        plan = self.eval_plan if init is None else self._load_plan(FIN_READOUT)
        psi = self._buf("psi", S << self.n, self.state_torch_dtype)
        part = self._buf("part", S * plan.tiles_per_state * self.C, torch.float32)
        if init is not None:
            self._state_in(psi, init.reshape(S, -1))
        self._run_passes(plan, False, psi, None, th, B, x, None, part, None, S)
        out = self._buf("expz", S * self.C, torch.float32)
        ext().readout_sum(part, plan.tiles_per_state, self.C, S, out)
        if noise is not None:
            ext().readout_noise(out, self.C, B, S, noise.p01, noise.p10, noise.shots, _keys(keys, noise),
                                int(step))
        return out.reshape(K, B, self.C).clone()

    # ------------------------------------------------------------------ generic simulation
    def _load_plan(self, fin: int) -> _Plan:
        """Plan that starts from a caller-provided state (amplitude encoding / initialize)."""
        cache = self.__dict__.setdefault("_load_plans", {})
        if fin not in cache:
            cache[fin] = _Plan(self._plan_args[0], self._plan_args[1], self.n, self.R, self._plan_args[2],
                               self.readout, self.n_theta, MODE_FWD_LOAD, fin, self.device, self.jit, self.bf16)
        return cache[fin]

    def _state_in(self, psi: torch.Tensor, init: torch.Tensor) -> None:
        """Initial states into the pass workspace.  Real ``init`` [S, F <= 2^n] = raw amplitudes, encoded
        on device (zero-pad, float64 L2 normalisation, zero row -> uniform) straight into the
        storage format; complex ``init`` [S, 2^n] = states used as given (complex64 storage)."""
        if init.is_complex():
            if self.bf16:
                raise NotImplementedError("explicit complex initial states need complex64 storage; pass real "
                                          "amplitudes to encode them on device")
            psi.view(init.shape[0], -1).copy_(init.to(torch.complex64))
            return
        x = init.reshape(init.shape[0], -1).float().contiguous()
        part = self._buf("amp_part", x.shape[0] * ext().amp_scratch(x.shape[1]), torch.float64)
        ext().amp_init(x, self.n, part, psi)

    @torch.no_grad()
    def statevector(self, xang: torch.Tensor, theta: torch.Tensor, init: torch.Tensor | None = None):
        """Final states [S, 2^n] complex64 (logical amplitude order) and <Z_readout> [S, C]."""
        K, B, F = xang.shape
        S = K * B
        x = xang.reshape(S, F).float().contiguous()
        th = theta.float().contiguous()
        plan = self.train_plan if init is None else self._load_plan(FIN_STORE | FIN_READOUT)
        psi = self._buf("psi", S << self.n, self.state_torch_dtype)
        part = self._buf("part", S * plan.tiles_per_state * self.C, torch.float32)
        if init is not None:
            self._state_in(psi, init)
        self._run_passes(plan, False, psi, None, th, B, x, None, part, None, S)
        z = self._buf("expz", S * self.C, torch.float32)
        ext().readout_sum(part, plan.tiles_per_state, self.C, S, z)
        state = psi.view(S, -1)
        if self.bf16:   # unpack (re, im) bf16 pairs
            u = state.view(torch.int32)
            re = (u << 16).view(torch.float32)
            im = (u & -65536).view(torch.float32)
            state = torch.complex(re, im)
        return state.clone(), z.view(S, self.C).clone()

    @torch.no_grad()
    def vjp(self, xang: torch.Tensor, theta: torch.Tensor, w: torch.Tensor, init: torch.Tensor | None = None):
        """Adjoint VJP of sum_c w[s, c] <Z_c>_s: returns (<Z> [S, C], d/dtheta [K, n_theta] summed over the
        B samples of each parameter row)."""
        K, B, F = xang.shape
        S = K * B
        C = ext()
        x = xang.reshape(S, F).float().contiguous()
        th = theta.float().contiguous()
        tr, adj = (self.train_plan if init is None else self._load_plan(FIN_STORE | FIN_READOUT)), self.adj_plan
        psi = self._buf("psi", S << self.n, self.state_torch_dtype)
        lam = self._buf("lam", S << self.n, self.state_torch_dtype)
        part = self._buf("part", S * tr.tiles_per_state * self.C, torch.float32)
        slab = self._buf("slab", S * adj.tiles_per_state * self.G, torch.float32)
        if init is not None:
            self._state_in(psi, init)
        self._run_passes(tr, False, psi, None, th, B, x, None, part, None, S)
        z = self._buf("expz", S * self.C, torch.float32)
        C.readout_sum(part, tr.tiles_per_state, self.C, S, z)
        wr = w.reshape(S, self.C).float().contiguous()
        self._run_passes(adj, True, psi, lam, th, B, x, wr, None, slab, S)
        grad = torch.zeros(K, th.shape[1], dtype=torch.float32, device=self.device)
        gpart = self._buf("gpart", K * C.grad_split(adj.tiles_per_state, B) * self.G, torch.float32)
        C.grad_reduce(slab, adj.tiles_per_state, B, K, self.G, adj.blob, adj.csr, grad, gpart)
        return z.view(S, self.C).clone(), grad[:, : self.n_theta]

    # ------------------------------------------------------------------ train step
    def loss_and_grads(self, xang, y, wmask, params, spec, noise=None, keys=None, step: int = 0, out_loss=None,
                       out_correct=None, init: torch.Tensor | None = None) -> dict:
        """One adjoint training step; ``init`` [K, B, 2^n] (amplitude encoding) starts the circuit from
        the given states through the planner's load-from-state forward plan."""
        K, B, F = xang.shape
        if F != self.x_width:
            raise ValueError(f"expected {self.x_width} x-slot values per sample, got {F}")
        S = K * B
        C = ext()
        x = xang.reshape(S, F).float().contiguous()
        p = params.float().contiguous()
        yy = y.reshape(S).long().contiguous()
        ww = wmask.reshape(S).float().contiguous()
        tr = self.train_plan if init is None else self._load_plan(FIN_STORE | FIN_READOUT)
        adj = self.adj_plan
        psi = self._buf("psi", S << self.n, self.state_torch_dtype)
        lam = self._buf("lam", S << self.n, self.state_torch_dtype)
        part = self._buf("part", S * tr.tiles_per_state * self.C, torch.float32)
        slab = self._buf("slab", S * adj.tiles_per_state * self.G, torch.float32)
        expz = self._buf("expz", S * self.C, torch.float32)
        if init is not None:
            self._state_in(psi, init.reshape(S, -1))
        wread = self._buf("wread", S * self.C, torch.float32)
        loss = torch.empty(K, dtype=torch.float32, device=self.device) if out_loss is None else out_loss
        correct = torch.empty(K, dtype=torch.float32, device=self.device) if out_correct is None else out_correct
        grad = torch.empty_like(p)      # every entry written: theta slots by grad_reduce, a/b by readout_ce
        self._run_passes(tr, False, psi, None, p, B, x, None, part, None, S)
        if noise is None:
            C.readout_ce(part, tr.tiles_per_state, self.C, B, K, yy, ww, p, self.n_theta, expz, wread, loss,
                         correct, grad, True, 0.0, 0.0, 0, _NO_KEYS, 0)
        else:
            C.readout_ce(part, tr.tiles_per_state, self.C, B, K, yy, ww, p, self.n_theta, expz, wread, loss,
                         correct, grad, True, noise.p01, noise.p10, noise.shots, _keys(keys, noise), int(step))
        self._run_passes(adj, True, psi, lam, p, B, x, wread, None, slab, S)
        gpart = self._buf("gpart", K * C.grad_split(adj.tiles_per_state, B) * self.G, torch.float32)
        C.grad_reduce(slab, adj.tiles_per_state, B, K, self.G, adj.blob, adj.csr, grad, gpart)
        return {"loss": loss, "grad": grad, "correct": correct, "expz": expz.reshape(K, B, self.C)}
