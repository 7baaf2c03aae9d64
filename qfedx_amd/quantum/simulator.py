"""Batched statevector simulation of arbitrary circuits on the gfx950 engine (public API).

    sim = Simulator(circuit, readout=[0, 3], device="cuda")            # any lowerable Circuit
    psi, z = sim.run(values)                     # values [S, n_slots] -> states [S, 2^n], <Z_c> [S, C]
    z, g = sim.vjp(values, w)                    # adjoint VJP of sum_c w[s,c] <Z_c>_s -> dL/dvalues [S, n_slots]
    psi, z = sim.run(values, initial_state=amp)  # start from given (e.g. amplitude-encoded) states
    sim = Simulator(circuit, readout=[0], backend="mps", chi_max=64)   # tensor network: run() returns an MPS

``values`` is one parameter row per circuit instance: the concatenation of the circuit's parameter
vectors in ``slots`` order (default: order of first appearance).  On a GPU the circuit is planned by the
native pass planner and executed by circuit-specialised kernels (the same engine as the VQC); on CPU the
portable torch executor runs the identical lowered program.  This is the GPU counterpart of the
reference's ``Statevector.from_instruction`` (``qAmplitude.py:44-46``), batched over instances.
"""
from __future__ import annotations

from typing import Optional

import torch

from .circuit import Circuit


class Simulator:
    def __init__(self, circuit: Circuit, readout: Optional[list] = None, device="cpu", backend: str = "auto",
                 slots: Optional[list] = None, state_dtype: str = "fp32", chi_max: int = 64):
        self.circuit = circuit
        self.n = circuit.n_qubits
        self.readout = list(range(min(self.n, 1))) if readout is None else list(readout)
        self.device = torch.device(device)
        if backend == "auto":
            backend = "hip" if self.device.type == "cuda" else "torch"
        self.backend = backend
        names = slots
        if names is None:
            names = []
            for p in circuit.parameters:
                if p.name not in names:
                    names.append(p.name)
        sizes = {}
        for p in circuit.parameters:
            sizes[p.name] = max(sizes.get(p.name, 0), p.index + 1)
        self.slot_of, off = {}, 0
        for nm in names:
            self.slot_of[nm] = off
            off += sizes.get(nm, 0)
        self.n_slots = max(off, 1)
        ops, coef = circuit.to_program(self.slot_of)
        self.ops, self.coef = ops, coef
        if backend == "mps":
            from .mps import MPSProgram
            self.prog = MPSProgram(ops, coef, self.n, self.device, chi_max=chi_max)
        elif backend == "hip":
            from ..ops.statevec_hip import HipProgram
            # every slot is a parameter row entry (n_theta = n_slots); the per-sample x row is a dummy
            self.prog = HipProgram(ops, coef, self.n, self.readout, self.device, n_theta=self.n_slots,
                                   state_dtype=state_dtype, x_width=1)
        else:
            from ..ops.statevec_torch import TorchProgram
            self.prog = TorchProgram(ops, coef, self.n, self.device)

    def _rows(self, values: torch.Tensor) -> torch.Tensor:
        v = torch.as_tensor(values, dtype=torch.float32, device=self.device)
        if v.dim() == 1:
            v = v[None]
        if v.shape[1] < self.n_slots:
            v = torch.cat([v, v.new_zeros(v.shape[0], self.n_slots - v.shape[1])], 1)
        return v.contiguous()

    def run(self, values, initial_state: Optional[torch.Tensor] = None):
        """-> (states [S, 2^n] complex64, <Z_readout> [S, C] float32); with backend="mps" the states are
        returned as a ``quantum.mps.MPS`` batch."""
        v = self._rows(values)
        S = v.shape[0]
        init = None if initial_state is None else torch.as_tensor(initial_state).to(self.device, torch.complex64)
        if self.backend == "mps" and init is None and self.prog.autograd_ok and self.prog.hip_program() is not None:
            z, back = self.prog.expz_vjp(v, self.readout)        # HIP contraction (csrc/mps_mpo.hip)
            g = slot_grads(back(w), torch.from_numpy(self.ops), torch.from_numpy(self.coef), self.n_slots).float()
            return z.float(), g
        if self.backend == "mps":
            st = self.prog.run(v, state=init)
            return st, self.prog.expz(st, self.readout).float()
        if self.backend == "hip":
            x = torch.zeros(S, 1, 1, device=self.device)
            return self.prog.statevector(x, v, init)
        psi = self.prog.run(v.double(), state=None if init is None else init.to(self.prog.dtype))
        z = self.prog.expz(psi, self.readout).float()
        return psi.to(torch.complex64), z

    def expectation_z(self, values, initial_state=None) -> torch.Tensor:
        return self.run(values, initial_state)[1]

    def vjp(self, values, w, initial_state=None):
        """Adjoint vector-Jacobian product of sum_c w[s, c] <Z_c>_s: -> (<Z> [S, C], grad [S, n_slots])."""
        v = self._rows(values)
        S = v.shape[0]
        w = torch.as_tensor(w, dtype=torch.float32, device=self.device).reshape(S, len(self.readout))
        init = None if initial_state is None else torch.as_tensor(initial_state).to(self.device, torch.complex64)
        if self.backend == "hip":
            x = torch.zeros(S, 1, 1, device=self.device)
            return self.prog.vjp(x, v, w, init)
        from ..ops.statevec_torch import slot_grads
        if self.backend == "mps" and init is None and self.prog.autograd_ok and self.prog.hip_program() is not None:
            z, back = self.prog.expz_vjp(v, self.readout)        # HIP contraction (csrc/mps_mpo.hip)
            g = slot_grads(back(w), torch.from_numpy(self.ops), torch.from_numpy(self.coef), self.n_slots).float()
            return z.float(), g
        if self.backend == "mps":
            st = self.prog.run(v, state=init)
            z = self.prog.expz(st, self.readout).float()
            gg = self.prog.adjoint_grads(v, st, w, self.readout, init=init)
            g = slot_grads(gg, torch.from_numpy(self.ops), torch.from_numpy(self.coef), self.n_slots).float()
            return z, g
        vd = v.double()
        psi = self.prog.run(vd, state=None if init is None else init.to(self.prog.dtype))
        z = self.prog.expz(psi, self.readout).float()
        gg = self.prog.adjoint_grads(vd, psi, w.double(), self.readout)
        g = slot_grads(gg, torch.from_numpy(self.ops), torch.from_numpy(self.coef), self.n_slots).float()
        return z, g
