"""Client-batched VQC compute engine (forward readout, loss, gradients).

One call processes ALL of a rank's clients at once: inputs are shaped [K, B, ...] (K clients x B
samples) with per-client parameters [K, P_total] - the client axis is a batch axis of the kernels,
replacing the reference's sequential per-client Python loop (``Classical_FL.py:132-140``).

Backends:
  * ``hip``   - gfx950 pass kernels of the in-tree extension (``ops/statevec_hip.py``)
  * ``torch`` - the portable program executor (``ops/statevec_torch.py``), CPU path + oracle
  * ``mps``   - batched matrix-product-state network (``quantum/mps.py``) for qubit counts past
                statevector memory (ROADMAP.md:85-87); ``adjoint`` = reverse-mode AD through the exact
                network, or parameter shift when the bond bound exceeds ``mps_chi``

Gradient methods (ROADMAP.md:23,38,130-135): ``adjoint`` (default; 1 forward + 1 reverse sweep),
``param_shift`` (2 shifted circuits per rotation gate, batched; on the MFMA engine the same shot-sampled
estimator from stored pass prefixes + the pi identity, ``HeaMfmaProgram.param_shift``), ``spsa`` (2 perturbed losses),
``autograd`` (torch complex autograd; CPU cross-check only).
"""
from __future__ import annotations

import math
import os
from typing import Optional

import torch
import torch.nn.functional as F

from ..models.vqc import VQCSpec, logits_from_expz
from ..utils.seeding import generator
from .statevec_torch import TorchProgram, slot_grads


def ce_readout(expz: torch.Tensor, y: torch.Tensor, wmask: torch.Tensor, a: torch.Tensor, b: torch.Tensor):
    """Weighted CE on logits a<Z>+b.  expz [K,B,C], y [K,B], wmask [K,B] (per-sample loss weight).

    Returns loss [K], dL/dexpz [K,B,C], grad_a [K,C], grad_b [K,C], correct [K] (weighted count of
    argmax hits, counting samples with wmask>0 as 1).
    """
    logits = logits_from_expz(expz, a, b)
    logp = torch.log_softmax(logits, -1)
    nll = -logp.gather(-1, y.unsqueeze(-1)).squeeze(-1)
    loss = (nll * wmask).sum(-1)
    p = logp.exp()
    dlog = (p - F.one_hot(y, expz.shape[-1]).to(p)) * wmask.unsqueeze(-1)
    w = dlog * a.unsqueeze(-2)
    grad_a = (dlog * expz).sum(-2)
    grad_b = dlog.sum(-2)
    correct = ((logits.argmax(-1) == y) & (wmask > 0)).sum(-1).to(expz.dtype)
    return loss, w, grad_a, grad_b, correct


class VQCEngine:
    def __init__(self, spec: VQCSpec, device="cpu", backend: str = "torch", state_dtype: str = "fp32",
                 noise=None, mps_chi: int = 64):
        self.spec = spec
        self.mps_hip = None
        # noiseless MPS-chain training steps fuse the readout cross entropy into the gradient launch (MpsChainProgram.
        # train); False runs the <Z> launch, the torch readout and the gradient launch (tests compare the two)
        self.fused_mps_readout = True
        self.noise = noise          # quantum.noise.NoiseModel or None
        self.device = torch.device(device)
        self.backend = backend
        ops, coef = spec.program()
        self.ops = torch.from_numpy(ops)
        self.coef = torch.from_numpy(coef)
        self.n_slots = spec.n_theta + spec.x_width
        self.state_dtype = state_dtype
        self.ps_reuse = os.environ.get("QFEDX_PS_REUSE", "1") != "0"   # 0: naive shifted rows (A/B, tests)
        if backend == "torch":
            self.prog = TorchProgram(ops, coef, spec.n_qubits, self.device)
            self.hip = None
        elif backend == "mps":
            from ..quantum.mps import MPSProgram
            if spec.amplitude and spec.n_qubits > 26:
                raise ValueError("amplitude-encoded initial states need a dense 2^n vector (n <= 26 with mps)")
            self.prog = MPSProgram(ops, coef, spec.n_qubits, self.device, chi_max=mps_chi)
            self.hip = None
            # the CNOT-chain VQC (<= 3 layers, exact at bond 2^L) runs on one HIP kernel per step on a GPU - only
            # when mps_chi admits the exact bond: with mps_chi < 2^L the einsum network truncates, and the same
            # config must give the same (truncated) result on every device
            from ..quantum.mps_chain import eligible as chain_ok
            if (self.device.type == "cuda" and chain_ok(spec) and noise is None
                    and int(mps_chi) >= (1 << spec.n_layers)):
                from .mps_hip import MpsChainProgram
                self.mps_hip = MpsChainProgram(spec, self.device)
        elif backend == "density":
            # exact density matrices with the Kraus gate channel (HIP kernel on a GPU, torch on CPU)
            from .density import DensityProgram
            kraus = noise.kraus() if (noise is not None and noise.gate_noise) else None
            self.prog = DensityProgram(ops, coef, spec.n_qubits, spec.readout, self.device, kraus=kraus)
            self.hip = None
        elif backend == "hip" and state_dtype in ("mfma", "fp16", "mfma_bf16"):
            # fp16 (or bf16) states + MFMA group unitaries (ops/hea_mfma.py) for the hardware-efficient ansatz
            from .hea_mfma import HeaMfmaProgram
            self.hip = HeaMfmaProgram(spec, self.device, storage="bf16" if state_dtype == "mfma_bf16" else "fp16")
            self.prog = TorchProgram(ops, coef, spec.n_qubits, self.device)
        elif backend == "hip":
            from .statevec_hip import HipProgram
            self.hip = HipProgram(ops, coef, spec.n_qubits, spec.readout, self.device,
                                  n_theta=spec.n_theta, state_dtype=state_dtype, x_width=spec.x_width)
            self.prog = TorchProgram(ops, coef, spec.n_qubits, self.device)  # for param-shift/autograd
        else:
            raise ValueError(f"unknown backend '{backend}'")

    def fit_tiles(self, samples: int) -> bool:
        """Small-batch tiling of the MFMA engine (BASELINE config 2's per-GPU point, 1 client x 32 samples): when a
        step's forward would launch fewer than two workgroups per CU at 2^14-amplitude tiles (16q: 4 tiles per
        sample, 128 workgroups at 32 samples), rebuild the program on 2^13 forward tiles (two passes still; 256
        workgroups) - measured 0.084 -> 0.076 ms per 1-client step (profiles/r6_config2_1client.txt).  Decided once,
        by the trainer before its first round graph is captured (eager evaluation workspaces of the old program are
        simply dropped); QFEDX_HEA_TILE pins the tiling.  Returns True if it switched."""
        import os
        hip = self.hip
        if (getattr(self, "_tiles_fitted", False) or hip is None or not hasattr(hip, "tile_bits")
                or os.environ.get("QFEDX_HEA_TILE") or self.device.type != "cuda"):
            return False
        self._tiles_fitted = True
        if hip.tile_bits < 14 or samples <= 0:
            return False
        cus = torch.cuda.get_device_properties(self.device).multi_processor_count
        if samples * hip.tiles_last >= 2 * cus:
            return False
        from .hea_mfma import HeaMfmaProgram
        small = HeaMfmaProgram(self.spec, self.device, tile_bits=13, storage=hip.storage)
        if small.n_passes != hip.n_passes:
            return False
        small.fused_readout = hip.fused_readout
        self.hip = small
        return True

    # ------------------------------------------------------------------ helpers
    def _states(self, init: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
        """Initial states [.., 2^n] complex: real ``init`` holds raw amplitudes (encoded here, on the HIP
        backend by the device kernel instead); complex ``init`` is used as given."""
        if init is None or init.is_complex():
            return init
        return self.spec.initial_states(init)

    def _init_rows(self, init: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
        """[K,B,..] initial states -> [K*B, 2^n] in the torch executor's dtype (None passes through)."""
        st = self._states(init)
        return None if st is None else st.reshape(-1, st.shape[-1]).to(self.prog.dtype)

    def _check(self, xang: torch.Tensor, init: Optional[torch.Tensor] = None) -> None:
        if self.spec.amplitude:
            N = 1 << self.spec.n_qubits
            if (init is None or init.shape[:-1] != xang.shape[:-1]
                    or (init.shape[-1] != N if init.is_complex() else init.shape[-1] > N)):
                raise ValueError("amplitude-encoded VQC needs init [K, B, <=2^n] raw amplitudes (or complex "
                                 "states [K, B, 2^n])")
        elif init is not None:
            raise ValueError("initial states are only used by feature_map='amplitude'")
        # the angle feature map reads one feature per qubit: a narrower input would make the
        # kernels read past each sample's row
        if xang.shape[-1] != self.spec.x_width:
            raise ValueError(f"VQC needs {self.spec.n_qubits} features per sample (one per qubit)"
                             f"{' + %d noise selectors' % self.spec.n_noise_ops if self.spec.noisy else ''}, "
                             f"got {xang.shape[-1]}; set data.n_features = model.n_qubits")

    def prologue_frag_job(self):
        """The MFMA engine's (slot_tab, frags) for the round prologue (None for every other engine)."""
        job = getattr(self.hip, "prologue_frag_job", None)
        return job() if job is not None else None

    def augment(self, xang: torch.Tensor, keys: Optional[torch.Tensor], step: int) -> torch.Tensor:
        """Append this step's noise-trajectory Pauli selectors to the encoded features [K, B, n]."""
        if not self.spec.noisy:
            return xang
        K, B, _ = xang.shape
        sel = self.noise.pauli_columns(keys, B, self.spec.n_noise_ops, step).to(xang)
        return torch.cat([xang, sel], -1)

    def _readout(self, expz, keys, step):
        if self.noise is None or not self.noise.readout_noise:
            return expz
        return self.noise.apply_readout(expz, keys, step)

    def _rows(self, xang: torch.Tensor, theta: torch.Tensor) -> torch.Tensor:
        K, B, n = xang.shape
        th = theta[:, None, :].expand(K, B, theta.shape[-1])
        return torch.cat([th, xang.to(th.dtype)], -1).reshape(K * B, -1)

    # ------------------------------------------------------------------ forward
    @torch.no_grad()
    def expz(self, xang: torch.Tensor, theta: torch.Tensor, readout_keys: Optional[torch.Tensor] = None,
             step: int = 0, init: Optional[torch.Tensor] = None) -> torch.Tensor:
        """<Z_c> for [K,B,x_width] encoded features and per-client theta [K,P] -> [K,B,C] (with the
        readout noise model applied when one is configured).  ``init`` (amplitude encoding): raw
        amplitudes [K,B,F<=2^n] (normalised on device) or complex initial states [K,B,2^n]."""
        K, B, _ = xang.shape
        self._check(xang, init)
        if self.backend == "hip":
            nz = self.noise if (self.noise is not None and self.noise.readout_noise) else None
            return self.hip.expz(xang, theta, nz, readout_keys, step, init)
        if self.backend == "density":
            if init is not None:
                raise ValueError("the density-matrix simulator starts from |0><0| (angle feature maps)")
            z = self.prog.expz(self._rows(xang, theta)).reshape(K, B, -1).float()
            return self._readout(z, readout_keys, step)
        if self.mps_hip is not None and init is None:
            return self._readout(self.mps_hip.expz(xang, theta), readout_keys, step)
        if self.backend == "mps" and init is None:
            z = self.prog.expz_rows(self._rows(xang, theta), self.spec.readout).reshape(K, B, -1).float()
            return self._readout(z, readout_keys, step)
        psi = self.prog.run(self._rows(xang, theta), state=self._init_rows(init))
        z = self.prog.expz(psi, self.spec.readout).reshape(K, B, -1).float()
        return self._readout(z, readout_keys, step)

    @torch.no_grad()
    def predict(self, xang: torch.Tensor, params: torch.Tensor, readout_keys=None, step: int = 0,
                init: Optional[torch.Tensor] = None) -> torch.Tensor:
        th, a, b = self.spec.split(params)
        return logits_from_expz(self.expz(xang, th, readout_keys, step, init), a, b)

    # ------------------------------------------------------------------ training
    def loss_and_grads(self, xang: torch.Tensor, y: torch.Tensor, wmask: torch.Tensor,
                       params: torch.Tensor, method: str = "adjoint", spsa_c: float = 0.1,
                       rng_keys: tuple = (0,), readout_keys: Optional[torch.Tensor] = None,
                       step: int = 0, out_loss: Optional[torch.Tensor] = None,
                       out_correct: Optional[torch.Tensor] = None, init: Optional[torch.Tensor] = None,
                       fused_opt=None, shared_frags=None, fed_tail=None) -> dict:
        """Loss [K], gradient [K,P], correct [K] for [K,B] minibatches.  ``out_loss`` / ``out_correct``
        (optional [K] views, e.g. rows of a round buffer) receive the loss / hit counts in place.
        ``init`` = raw amplitudes [K,B,F<=2^n] or complex states (amplitude encoding; None otherwise).
        ``fused_opt`` = (BatchedOptimizer, active [K]): an engine that can fuse the local optimizer step into its
        own launches (the MFMA engine: HIP Adam in the gradient reduction) does so and returns ``opt_done``.
        ``shared_frags``: the MFMA engine's unitary fragments of this step, already built by the round prologue
        (``prologue_frag_job``; a round's first step only, when every client row is the global vector).
        ``fed_tail``: the round's FedAvg to fold into this (last) step's fused Adam epilogue (``QfxFedTail``); the
        result says ``fed_done`` when the engine did."""
        spec = self.spec
        self._check(xang, init)
        if self.backend == "hip" and method == "adjoint":
            nz = self.noise if (self.noise is not None and self.noise.readout_noise) else None
            if fused_opt is not None and getattr(self.hip, "fuses_optimizer", False):
                return self.hip.loss_and_grads(xang, y, wmask, params, spec, nz, readout_keys, step, out_loss,
                                               out_correct, init, fused_opt=fused_opt, shared_frags=shared_frags,
                                               fed_tail=fed_tail)
            return self.hip.loss_and_grads(xang, y, wmask, params, spec, nz, readout_keys, step, out_loss,
                                           out_correct, init)
        res = self._loss_and_grads(xang, y, wmask, params, method, spsa_c, rng_keys, readout_keys, step, init)
        if out_loss is not None:
            out_loss.copy_(res["loss"])
            res["loss"] = out_loss
        if out_correct is not None:
            out_correct.copy_(res["correct"])
            res["correct"] = out_correct
        return res

    def _loss_and_grads(self, xang, y, wmask, params, method, spsa_c, rng_keys, readout_keys, step,
                        init=None) -> dict:
        spec = self.spec
        th, a, b = spec.split(params)
        if method == "autograd" and self.backend == "mps":
            method = "adjoint"               # the MPS adjoint IS reverse-mode AD through the network
        if method in ("adjoint", "autograd") and self.backend == "density":
            # mixed states: the parameter-shift rule holds for exp(-i theta P / 2) rotations with channels that do
            # not depend on theta in between; the statevector adjoint does not apply
            method = "param_shift"
        if method == "autograd":
            return self._autograd(xang, y, wmask, params, init)
        K, B, _ = xang.shape
        P = spec.n_theta
        with torch.no_grad():
            rows = psi = None
            if (method == "adjoint" and self.mps_hip is not None and init is None and self.noise is None
                    and self.fused_mps_readout):
                # one HIP launch (csrc/mps_chain.hip): <Z>, the readout cross entropy and dL/d<Z> in the kernel, then
                # the gradient sweeps
                loss, grad, correct, expz = self.mps_hip.train(xang, params, y, wmask)
                return {"loss": loss, "grad": grad, "correct": correct, "expz": expz}
            if method == "adjoint" and self.mps_hip is not None and init is None:
                # HIP column contraction (csrc/mps_chain.hip): <Z>, then the gradient sweep with dL/d<Z>
                expz = self._readout(self.mps_hip.expz(xang, th), readout_keys, step)
                loss, w, ga, gb, correct = ce_readout(expz, y, wmask, a, b)
                gth = self.mps_hip.grads(xang, th, w)
                return {"loss": loss, "grad": torch.cat([gth, ga, gb], -1), "correct": correct, "expz": expz}
            if (method == "adjoint" and self.backend == "mps" and self.prog.autograd_ok and init is None):
                # one recorded MPS contraction: readout now, reverse-mode pull-back of dL/d<Z> below
                rows = self._rows(xang, th)
                zt, back = self.prog.expz_vjp(rows, spec.readout)
                expz = self._readout(zt.reshape(K, B, -1).float(), readout_keys, step)
                loss, w, ga, gb, correct = ce_readout(expz, y, wmask, a, b)
                if self.noise is not None:
                    w = w * (1.0 - self.noise.p01 - self.noise.p10)
                gg = back(w.reshape(K * B, -1))
                gs = slot_grads(gg, self.ops, self.coef, self.n_slots)[:, :P]
                gth = gs.reshape(K, B, P).sum(1).float()
                return {"loss": loss, "grad": torch.cat([gth, ga, gb], -1), "correct": correct, "expz": expz}
            if method == "adjoint":          # torch backend: keep psi for the reverse sweep
                rows = self._rows(xang, th)
                psi = self.prog.run(rows, state=self._init_rows(init))
                expz = self._readout(self.prog.expz(psi, spec.readout).reshape(K, B, -1).float(), readout_keys, step)
            else:                            # HIP or torch forward, readout noise applied
                expz = self.expz(xang, th, readout_keys, step, init)
            loss, w, ga, gb, correct = ce_readout(expz, y, wmask, a, b)
            if method == "adjoint":
                if self.noise is not None:   # straight-through d<Z>_noisy / d<Z> for the exact adjoint
                    w = w * (1.0 - self.noise.p01 - self.noise.p10)
                if self.backend == "mps":
                    gg = self.prog.adjoint_grads(rows, psi, w.reshape(K * B, -1), spec.readout,
                                                 init=self._init_rows(init))
                else:
                    gg = self.prog.adjoint_grads(rows, psi, w.reshape(K * B, -1), spec.readout)
                gs = slot_grads(gg, self.ops, self.coef, self.n_slots)[:, :P]
                gth = gs.reshape(K, B, P).sum(1).float()
            elif method == "param_shift":
                # shifted expectations carry the readout channel themselves: w = dL/d<Z>_noisy unscaled
                if (self.backend == "hip" and hasattr(self.hip, "param_shift") and init is None
                        and self.ps_reuse):
                    # MFMA engine: prefix reuse + the pi identity (same estimator, ~2.5x fewer pass launches)
                    nz = self.noise if (self.noise is not None and self.noise.readout_noise) else None
                    gth = self.hip.param_shift(xang, params, w, nz, readout_keys, step)
                elif self._simple_shift_slots():
                    gth = self.param_shift_batched(xang, params, w, readout_keys, step, init)
                else:
                    gth = self._param_shift(self._rows(xang, th), w, K, B, init=init)
            elif method == "spsa":
                gth = self._spsa(xang, y, wmask, params, spsa_c, rng_keys, init)
            else:
                raise ValueError(f"unknown grad method '{method}'")
        grad = torch.cat([gth, ga, gb], -1)
        return {"loss": loss, "grad": grad, "correct": correct, "expz": expz}

    def _param_shift(self, rows: torch.Tensor, w: torch.Tensor, K: int, B: int,
                     chunk: int = 32, init: Optional[torch.Tensor] = None) -> torch.Tensor:
        """d<O>/dangle_g = 0.5 (<O>(angle+pi/2) - <O>(angle-pi/2)) for every theta gate."""
        prog, spec = self.prog, self.spec
        P = spec.n_theta
        base = prog.angles(rows)                                   # [KB, G]
        gates = [g for g, (k, q0, q1, s) in enumerate(prog.ops_list) if 0 <= s < P]
        gg = torch.zeros(rows.shape[0], len(prog.ops_list), dtype=base.dtype, device=rows.device)
        wflat = w.reshape(K * B, -1).to(base.dtype)
        for c0 in range(0, len(gates), chunk):
            sub = gates[c0:c0 + chunk]
            G2 = len(sub)
            ang = base.unsqueeze(0).repeat(2 * G2, 1, 1)            # [2G2, KB, G]
            for i, g in enumerate(sub):
                ang[2 * i, :, g] += math.pi / 2
                ang[2 * i + 1, :, g] -= math.pi / 2
            ang = ang.reshape(-1, base.shape[1])
            if init is None:
                st = prog.initial_state(ang.shape[0])
            else:
                st = self._init_rows(init).repeat(2 * G2, 1)
            for g in range(len(prog.ops_list)):
                st = prog.apply_gate(st, g, ang[:, g])
            z = prog.expz(st, spec.readout).reshape(G2, 2, rows.shape[0], -1)
            dz = 0.5 * (z[:, 0] - z[:, 1])                           # [G2, KB, C]
            for i, g in enumerate(sub):
                gg[:, g] = (dz[i] * wflat).sum(-1)
        gs = slot_grads(gg, self.ops, self.coef, self.n_slots)[:, :P]
        return gs.reshape(K, B, P).sum(1).float()

    # ------------------------------------------------------------------ batched parameter shift
    def _simple_shift_slots(self) -> bool:
        """True when every theta slot drives exactly one RX/RY/RZ gate with unit scale, so shifting the
        slot by +-pi/2 IS the gate's parameter shift (then shifts batch as parameter rows)."""
        if getattr(self, "_simple", None) is None:
            P = self.spec.n_theta
            seen = {}
            ok = True
            for (kind, q0, q1, slot), (sc, off) in zip(self.ops.tolist(), self.coef.tolist()):
                if 0 <= slot < P:
                    ok &= kind in (0, 1, 2) and abs(sc - 1.0) < 1e-12
                    seen[slot] = seen.get(slot, 0) + 1
            self._simple = bool(ok and all(v == 1 for v in seen.values()) and len(seen) == P)
        return self._simple

    def state_budget_bytes(self) -> int:
        if getattr(self, "_budget", None) is None:
            if self.device.type == "cuda":
                free, _ = torch.cuda.mem_get_info(self.device)
                self._budget = int(0.4 * free)
            else:
                self._budget = 1 << 31
        return self._budget

    def param_shift_batched(self, xang: torch.Tensor, params: torch.Tensor, w: torch.Tensor,
                            readout_keys: Optional[torch.Tensor] = None, step: int = 0,
                            init: Optional[torch.Tensor] = None) -> torch.Tensor:
        """dL/dtheta by the parameter-shift rule (ROADMAP.md:23,130-135).

        Every (client k, slot j, sign) is one parameter row theta_k +- pi/2 e_j over the client's B
        samples: the rows are one forward batch (the HIP eval kernels see them as ordinary samples),
        chunked so that the live statevectors fit ``state_budget_bytes``.  With a readout noise model
        each shifted evaluation is confused / shot-sampled from its own keyed stream, so the
        estimator is the finite-shot hardware estimator.  w = dL/d<Z> [K,B,C].  -> [K, n_theta]
        """
        K, B, F = xang.shape
        P = self.spec.n_theta
        R = 2 * P
        state_bytes = (self.spec.n_qubits * 2 * 8 * self.prog.chi_max ** 2 if self.backend == "mps"
                       else self.prog.state_bytes() if self.backend == "density"
                       else (1 << self.spec.n_qubits) * 8)
        rows_per_chunk = max(1, min(K * R, self.state_budget_bytes() // max(1, B * state_bytes)))
        contrib_all = torch.zeros(K * R, dtype=torch.float64, device=params.device)
        half_pi = math.pi / 2
        for r0 in range(0, K * R, rows_per_chunk):
            r = torch.arange(r0, min(K * R, r0 + rows_per_chunk), device=params.device)
            k, j = r // R, r % R
            slot, sign = j // 2, 1.0 - 2.0 * (j % 2).to(params.dtype)
            th = params[k, :P].clone()
            th[torch.arange(len(r), device=th.device), slot] += sign * half_pi
            keys = None
            if readout_keys is not None:
                # independent stream per shifted evaluation: mix the row index into the client key
                keys = readout_keys[k].clone()
                keys[:, 0] = (keys[:, 0] ^ ((j + 1) * 0x9E3779B9)) & 0xFFFFFFFF
                keys[:, 1] = (keys[:, 1] + (j + 1) * 0x85EBCA6B) & 0xFFFFFFFF
            z = self.expz(xang[k], th, keys, step, None if init is None else init[k]).double()                       # [rows, B, C]
            contrib_all[r] = (z * w[k].double()).sum((1, 2)) * (0.5 * sign.double())   # [rows]
        # row r = (k, slot, sign): fixed-order pair sum (no atomics -> deterministic)
        return contrib_all.view(K, P, 2).sum(-1).float()

    def _loss_only(self, xang, y, wmask, params, init=None):
        th, a, b = self.spec.split(params)
        z = self.expz(xang, th, init=init)
        return ce_readout(z, y, wmask, a, b)[0]

    def _spsa(self, xang, y, wmask, params, c: float, rng_keys: tuple, init=None) -> torch.Tensor:
        P = self.spec.n_theta
        K = params.shape[0]
        g = generator(*rng_keys, "spsa")
        delta = (torch.randint(0, 2, (K, P), generator=g) * 2 - 1).to(params)
        pad = torch.zeros(K, params.shape[1] - P, dtype=params.dtype, device=params.device)
        d = torch.cat([delta.to(params.device), pad], -1)
        lp = self._loss_only(xang, y, wmask, params + c * d, init)
        lm = self._loss_only(xang, y, wmask, params - c * d, init)
        return ((lp - lm) / (2 * c)).unsqueeze(-1) * delta.to(params.device)

    def _autograd(self, xang, y, wmask, params, init=None):
        spec = self.spec
        K, B, _ = xang.shape
        p = params.detach().clone().double().requires_grad_(True)
        th, a, b = spec.split(p)
        prog = TorchProgram(self.ops, self.coef, spec.n_qubits, params.device, torch.complex128)
        rows = self._rows(xang.double(), th)
        st = self._states(init)
        psi = prog.run(rows, state=None if st is None else st.reshape(K * B, -1).to(prog.dtype))
        expz = prog.expz(psi, spec.readout).reshape(K, B, -1)
        logits = logits_from_expz(expz, a, b)
        nll = -torch.log_softmax(logits, -1).gather(-1, y.unsqueeze(-1)).squeeze(-1)
        loss = (nll * wmask.double()).sum(-1)
        loss.sum().backward()
        correct = ((logits.argmax(-1) == y) & (wmask > 0)).sum(-1).float()
        return {"loss": loss.detach().float(), "grad": p.grad.float(), "correct": correct,
                "expz": expz.detach().float()}
