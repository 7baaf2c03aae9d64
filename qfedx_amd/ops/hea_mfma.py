"""MFMA statevector engine for the hardware-efficient VQC (host side).

``HeaMfmaProgram`` runs the pass plans of ``ops/hea_plan.py`` on the gfx950 kernels of
``csrc/hea_mfma.hip``: per local step

    hea_frags (per-client 16 x 16 group unitaries -> MFMA A fragments, hi + lo fp16)
    forward passes  (product state generated in-tile; intermediate pass outputs stored as fp16 (re, im))
    readout_ce      (shared with the VALU engine: <Z>, CE loss, dL/d<Z>, a/b gradients)
    adjoint passes  (reverse pass order; per-workgroup gradient partials)
    hea_grad_reduce (fixed-order sum over each client's samples and tiles)

It exposes the subset of ``HipProgram``'s interface the engine / trainer use (``expz``, ``vjp``,
``loss_and_grads``, ``private_workspace``), so ``VQCEngine(..., backend="hip", state_dtype="mfma")``
swaps it in for circuits ``hea_plan.eligible`` accepts.  Amplitudes are stored as fp16 scaled by
2^(n/2) (unit-magnitude typical values); MFMAs accumulate in fp32 and the unitaries carry a hi/lo fp16
split, so the only rounding is the fp16 state between ops (~2^-12 relative per op).
"""
from __future__ import annotations

import contextlib
import os

import numpy as np
import torch

from ._ext import ext
from .hea_plan import (OP_APPLY, OP_APPLY2, OP_BACK, OP_BACK2, OP_GRAD2, OP_GRAD_L1, OP_READOUT, TILE_BITS, W_CODE, build_plan, eligible, fo_table, obs_table,
                       pass_programs)

ADJ_TILE_BITS = 13   # adjoint tiles: 2^13 amplitudes x (psi, lambda) = 64 KB of LDS -> two workgroups per CU


def _same_passes(a, b) -> bool:
    """Two plans run the same rotation groups (and unitary slots) in the same passes - only their tile geometry
    differs.  The layer-1 gradient groups may sit in other passes: they exist only in the adjoint programs
    (the forward generates the whole layer-1 product state in its first pass)."""
    def sig(plan):
        return [sorted((g.slot, g.layer, tuple(g.qubits), g.frame) for g in p.groups) for p in plan.passes]
    return a.n_slots == b.n_slots and sig(a) == sig(b)

_FEATURE = {"ry": 0, "rx": 1, "rz": 2}


def _frag_index(ops: np.ndarray) -> torch.Tensor:
    """Per op the unitary fragments it multiplies by (slot * 4 + 0: U, + 2: U^H; a pair op names its two groups'),
    -1 for none: int32 [nops, 2] (prefetch table)."""
    from .hea_plan import OP_APPLY, OP_APPLY2, OP_BACK, OP_BACK2, W_CODE, W_SLOT, W_SLOT2
    out = np.full((len(ops), 2), -1, dtype=np.int32)
    for i, w in enumerate(ops):
        code = int(w[W_CODE])
        if code in (OP_APPLY, OP_APPLY2):
            out[i, 0] = 4 * int(w[W_SLOT])
        elif code in (OP_BACK, OP_BACK2):
            out[i, 0] = 4 * int(w[W_SLOT]) + 2
        if code == OP_APPLY2:
            out[i, 1] = 4 * int(w[W_SLOT2])
        elif code == OP_BACK2:
            out[i, 1] = 4 * int(w[W_SLOT2]) + 2
    return torch.from_numpy(out).contiguous()
_NO_KEYS = torch.zeros(0, dtype=torch.int64)
_NODBG = torch.zeros(0, dtype=torch.int64)     # no stall-attribution buffer (stamps build only)


NT_STORE_MIN_BYTES = 128 << 20   # pass states above which tiles are stored non-temporally (_nt_store)
FUSED_ADAM_MAX_BLOCKS = 256   # hea_grad_reduce blocks (clients x gradient ops) up to which Adam is fused


class HeaMfmaProgram:
    def __init__(self, spec, device, tile_bits: int | None = None, adj_tile_bits: int | None = None,
                 storage: str = "fp16"):
        """``storage``: fp16 (default) or bf16 (BASELINE config 2) amplitudes and unitary fragments
        (csrc/hea_mfma_bf16.hip: v_mfma_f32_16x16x32_bf16, fp32 accumulation; 2^-9 per-op state rounding)."""
        if storage not in ("fp16", "bf16"):
            raise ValueError(f"MFMA engine storage must be fp16 | bf16, got {storage!r}")
        self.storage = storage
        self.bf16 = storage == "bf16"
        if not eligible(spec):
            raise ValueError("the MFMA engine covers angle-encoded RX/RZ + CNOT-chain VQCs with 8..30 qubits, "
                             "no gate noise and <= 8 classes")
        self.spec = spec
        self.n = spec.n_qubits
        self.C = spec.n_classes
        self.n_theta = spec.n_theta
        self.device = torch.device(device)
        if tile_bits is None:
            tile_bits = int(os.environ.get("QFEDX_HEA_TILE", TILE_BITS))
        if adj_tile_bits is None:
            adj_tile_bits = int(os.environ.get("QFEDX_HEA_ADJ_TILE", min(tile_bits, ADJ_TILE_BITS)))
        self.tile_bits = tile_bits
        self.plan = build_plan(self.n, spec.n_layers, spec.readout, spec.entangler == "chain", spec.feature_map,
                               tile_bits)
        # The adjoint may run on smaller tiles than the forward (2^13 amplitudes: two adjoint workgroups per
        # CU, one's tile load hidden behind the other's group ops) when that plan has the same passes, rotation
        # groups and unitary slots: pass outputs are stored in memory order, so the tiling of a pass is free to
        # differ.
        plan_a = self.plan
        if adj_tile_bits != tile_bits:
            cand = build_plan(self.n, spec.n_layers, spec.readout, spec.entangler == "chain", spec.feature_map,
                              adj_tile_bits)
            if _same_passes(self.plan, cand):
                plan_a = cand
        self.adj_plan = plan_a
        self.adj_tile_bits = plan_a.passes[0].t if plan_a.passes else tile_bits
        C = ext()
        self.n_slots = self.plan.n_slots
        self.passes = []
        gmeta = []
        fplan = self.plan
        progs_f = pass_programs(fplan, [])
        # Forward passes after the last one that applies a unitary are identities on the state (they exist for
        # the adjoint's layer-1 gradient tiles, e.g. every pass of an L = 1 circuit): the forward stops at that
        # pass, reads out there, and later passes' stored outputs alias its output.
        applies = [j for j, (_, fwd, _) in enumerate(progs_f)
                   if any(int(w[W_CODE]) in (OP_APPLY, OP_APPLY2) for w in fwd)]
        self.fwd_last = applies[-1] if applies else 0
        J = len(progs_f)
        progs_a = pass_programs(plan_a, gmeta)
        self.n_gradops = len(gmeta)
        # the fused Adam epilogue of hea_grad_reduce updates each parameter in the block that formed its gradient:
        # it needs every theta parameter owned by exactly one gradient record (else the separate Adam launch runs)
        owned = []
        for row in gmeta:
            nr = int(row[1]) & 15
            owned += [int(v) for v in row[2:2 + nr]] + [int(v) for v in row[6:6 + nr]]
        self.grad_cover_exact = sorted(owned) == list(range(self.n_theta))
        if self.fwd_last < J - 1:
            pr, fr_ops, ar = progs_f[self.fwd_last]
            fr_ops = np.concatenate([fr_ops, obs_table(fplan, pr, OP_READOUT)[None]], 0)
            progs_f = [(p, f if j < self.fwd_last else (fr_ops if j == self.fwd_last else f[:0]), a)
                       for j, (p, f, a) in enumerate(progs_f)]
        self.n_regions = []       # per pass: gradient records of its adjoint program (LDS regions)
        for (p, fwd, _), (pa, _, adj) in zip(progs_f, progs_a):
            f = torch.from_numpy(fwd.astype(np.int32)).contiguous()
            a = torch.from_numpy(adj.astype(np.int32)).contiguous()
            ff, fa = _frag_index(fwd), _frag_index(adj)
            C.hea_check_ops(f, ff, self.n_slots, self.n_theta, False, p.t, self.n_gradops)
            C.hea_check_ops(a, fa, self.n_slots, self.n_theta, True, pa.t, self.n_gradops)
            self.n_regions.append(sum(2 if int(w[W_CODE]) in (OP_BACK2, OP_GRAD2) else
                                      int(int(w[W_CODE]) in (OP_BACK, OP_GRAD_L1)) for w in adj))
            of = torch.from_numpy(fo_table(fwd, p, self.n).reshape(-1)).to(self.device)
            oa = torch.from_numpy(fo_table(adj, pa, self.n).reshape(-1)).to(self.device)
            self.passes.append((p, (f.to(self.device), ff.to(self.device), of),
                                (a.to(self.device), fa.to(self.device), oa), pa))
        slot_tab = np.zeros((max(self.n_slots, 1), 9), dtype=np.int32)
        owner = np.zeros(self.n_theta, dtype=np.int32)
        for p in self.plan.passes:
            nt = 1 << (self.n - p.t)
            for g in p.groups:
                slot_tab[g.slot, 0] = len(g.qubits)
                for j, q in enumerate(g.qubits):
                    slot_tab[g.slot, 1 + j] = self.plan.theta_slot(g.layer, q)
                    slot_tab[g.slot, 5 + j] = self.plan.theta_slot(g.layer, q) + 1
            for g in p.groups + p.l1:
                for q in g.qubits:
                    owner[self.plan.theta_slot(g.layer, q)] = nt
                    owner[self.plan.theta_slot(g.layer, q) + 1] = nt
        if (owner == 0).any():
            raise RuntimeError("a parameter has no owning pass")
        self.slot_tab = torch.from_numpy(slot_tab).to(self.device)
        self.gmeta = torch.tensor(gmeta, dtype=torch.int32).reshape(-1).to(self.device)
        self.slab_tiles = max(1 << (self.n - p.t) for p in plan_a.passes)
        self.scale = float(1 << (self.n // 2))
        self.feature = _FEATURE[spec.feature_map.lower()]
        self._ws = {}
        self._ps_budget = None
        # noiseless steps compute the readout in the first adjoint pass (profiles/r5_fused_readout_ab.txt: a tie at 64
        # clients, -2.7% at 8); the readout kernel runs for readout noise - and for tests comparing the two (False)
        self.fused_readout = True
        if self.device.type == "cuda":
            self._shift_budget()      # query free HBM now, never inside a graph capture

    # ------------------------------------------------------------------ workspaces
    @contextlib.contextmanager
    def private_workspace(self, ws: dict):
        """Route workspace allocations to ``ws`` (owned by a captured hipGraph)."""
        saved = self._ws
        self._ws = ws
        try:
            yield ws
        finally:
            self._ws = saved

    def _zbuf(self, name: str, numel: int, dtype) -> torch.Tensor:
        """Workspace that is zero when created (e.g. arrival counters that their kernel resets after use): created
        outside graph capture (the capture's warm-up run), so no fill is ever captured."""
        t = self._ws.get(name)
        if t is None or t.numel() < numel or t.dtype != dtype:
            t = torch.zeros(numel, dtype=dtype, device=self.device)
            self._ws[name] = t
        return t[:numel]

    def _buf(self, name: str, numel: int, dtype) -> torch.Tensor:
        t = self._ws.get(name)
        if t is None or t.numel() < numel or t.dtype != dtype:
            t = torch.empty(numel, dtype=dtype, device=self.device)
            self._ws[name] = t
        return t[:numel]

    @property
    def n_passes(self) -> int:
        return len(self.passes)

    @property
    def tiles_last(self) -> int:
        """Tiles per sample of the pass that reads out <Z> (the last forward pass that runs)."""
        return 1 << (self.n - self.passes[self.fwd_last][0].t)

    def _geom(self, p, gen, load_lam, store_psi, store_lam, B, p_stride, S, x_stride, K, in_rep: int = 1,
              n_regions: int = 0, shared: bool = False):
        return [self.n, p.t, p.c, p.lo, p.hi, 1 << (self.n - p.t), int(gen), int(load_lam), int(store_psi),
                int(store_lam), B, self.C, self.n_theta, p_stride, self.feature, S, x_stride, self.n_slots,
                self.slab_tiles, K] + [int(h) for h in p.H] + [self.n_gradops, int(in_rep), int(self.bf16),
                                                                 int(n_regions), int(shared), int(self._nt_store(S))]

    def _nt_store(self, S: int) -> bool:
        """Non-temporal pass-output stores once a pass's states (S x 2^n x 4 bytes) outgrow half the 256 MB Infinity
        Cache: 16q x 2048 samples (512 MB) 1.820 -> 1.784 ms per step, while 8 clients' 64 MB are re-read faster from
        the cache with plain stores (profiles/r6_tile_nt_priority_ab.txt).  QFEDX_HEA_NT=0 / 1 overrides."""
        env = os.environ.get("QFEDX_HEA_NT")
        if env is not None:
            return env == "1"
        return S * (4 << self.n) > NT_STORE_MIN_BYTES

    def _frags(self, params: torch.Tensor, K: int, tag: str = "") -> torch.Tensor:
        fr = self._buf(f"{tag}frags", max(K * self.n_slots * 4 * 128 * 4, 1), torch.int32)
        if self.n_slots:
            ext().hea_frags(params, params.shape[1], self.slot_tab, self.n_slots, K, fr, self.bf16)
        return fr

    def _forward(self, x, params, fr, K, B, part, store_last: bool = False, tag: str = "", dbg=None,
                 shared: bool = False):
        """Forward passes up to the readout pass ``fwd_last``; returns the stored pass outputs (all of them with
        ``store_last``: the adjoint starts each pass from its output; identity passes after ``fwd_last`` alias
        its output).  ``tag`` names the workspaces; ``dbg`` (stamps build): per-pass stall-attribution buffers."""
        C = ext()
        S = K * B
        N = S << self.n
        stored = []
        empty = torch.empty(0, dtype=torch.int32, device=self.device)
        fempty = torch.empty(0, dtype=torch.float32, device=self.device)
        J, R = self.n_passes, self.fwd_last
        for j in range(R + 1):
            p, fwd = self.passes[j][0], self.passes[j][1]
            keep = j < R or store_last
            # evaluation only needs the previous pass output: two ping-pong buffers instead of one per pass
            name = f"{tag}psi{j}" if store_last else f"{tag}pe{j % 2}"
            out = self._buf(name, N, torch.int32) if keep else empty
            psi_in = stored[-1] if j > 0 else empty
            geom = self._geom(p, j == 0, False, keep, False, B, params.shape[1], S, x.shape[1], K, shared=shared)
            C.hea_pass(False, fwd[0], fwd[1], fwd[2], geom, self.scale, psi_in, out, empty, empty, x, params, fr, fempty,
                       part if j == R else fempty, fempty, dbg[f"fwd{j}"] if dbg else _NODBG)
            if keep:
                stored.append(out)
        if store_last:
            stored += [stored[R]] * (J - 1 - R)
        return stored

    def _adjoint(self, x, params, fr, K, B, stored, wread, gslab, tag: str = "", readout=None, dbg=None,
                 shared: bool = False):
        """Adjoint passes, last pass first.  ``readout`` = (part, y, wts, expz, rec): the first adjoint pass computes
        every sample's readout and dL/d<Z> itself (fused readout; ``wread`` is then its output, read by the later
        passes) instead of taking ``wread`` from the readout kernel."""
        C = ext()
        S = K * B
        N = S << self.n
        empty = torch.empty(0, dtype=torch.int32, device=self.device)
        fempty = torch.empty(0, dtype=torch.float32, device=self.device)
        J = self.n_passes
        lam_in = empty
        for j in range(J - 1, -1, -1):
            _, _, adj, p = self.passes[j]
            lam_out = self._buf(f"{tag}lam{j % 2}", N, torch.int32) if j > 0 else empty
            geom = self._geom(p, False, j < J - 1, False, j > 0, B, params.shape[1], S, x.shape[1], K,
                              n_regions=self.n_regions[j], shared=shared)
            if readout is not None and j == J - 1:
                part, yy, ww, expz, rec = readout
                C.hea_pass(True, adj[0], adj[1], adj[2], geom, self.scale, stored[j], empty, lam_in, lam_out, x,
                           params, fr, fempty, part, gslab, dbg[f"adj{j}"] if dbg else _NODBG,
                           [yy, ww, expz, wread, rec], self.tiles_last)
            else:
                C.hea_pass(True, adj[0], adj[1], adj[2], geom, self.scale, stored[j], empty, lam_in, lam_out, x,
                           params, fr, wread, fempty, gslab, dbg[f"adj{j}"] if dbg else _NODBG)
            lam_in = lam_out

    def _prep(self, xang, params):
        K, B, F = xang.shape
        if F < self.n:
            raise ValueError(f"expected >= {self.n} feature angles per sample, got {F}")
        x = xang.reshape(K * B, F).float().contiguous()
        p = params.float().contiguous()
        if p.shape[0] != K:
            raise ValueError("one parameter row per client expected")
        return x, p, K, B

    # ------------------------------------------------------------------ forward / eval
    @torch.no_grad()
    def expz(self, xang: torch.Tensor, theta: torch.Tensor, noise=None, keys=None, step: int = 0,
             init: torch.Tensor | None = None) -> torch.Tensor:
        if init is not None:
            raise ValueError("the MFMA engine starts from the angle feature map (no initial states)")
        x, th, K, B = self._prep(xang, theta)
        if th.shape[1] < self.n_theta + 2 * self.C:    # pad theta-only rows to the kernel's param stride
            th = torch.cat([th, th.new_zeros(K, self.n_theta + 2 * self.C - th.shape[1])], 1)
        S = K * B
        out = self._buf("expz", S * self.C, torch.float32)
        # clients per launch: two live states per sample fit the HBM budget (24q: 128 MiB per sample)
        Kc = max(1, min(K, self._shift_budget() // max(1, 2 * B * ((1 << self.n) * 4))))
        for k0 in range(0, K, Kc):
            k1 = min(K, k0 + Kc)
            Sc = (k1 - k0) * B
            thc = th[k0:k1] if Kc < K else th
            fr = self._frags(thc, k1 - k0)
            part = self._buf("part", Sc * self.tiles_last * self.C, torch.float32)
            self._forward(x[k0 * B:k1 * B], thc, fr, k1 - k0, B, part)
            ext().readout_sum(part, self.tiles_last, self.C, Sc, out[k0 * B * self.C:k1 * B * self.C])
        if noise is not None:
            from .statevec_hip import _keys
            ext().readout_noise(out, self.C, B, S, noise.p01, noise.p10, noise.shots, _keys(keys, noise), int(step))
        return out.reshape(K, B, self.C).clone()

    @torch.no_grad()
    def vjp(self, xang: torch.Tensor, theta: torch.Tensor, w: torch.Tensor, init: torch.Tensor | None = None):
        """Adjoint VJP of sum_c w[s, c] <Z_c>_s -> (<Z> [S, C], d/dtheta [K, n_theta])."""
        if init is not None:
            raise ValueError("the MFMA engine starts from the angle feature map (no initial states)")
        x, th, K, B = self._prep(xang, theta)
        if th.shape[1] < self.n_theta + 2 * self.C:
            th = torch.cat([th, th.new_zeros(K, self.n_theta + 2 * self.C - th.shape[1])], 1)
        S = K * B
        fr = self._frags(th, K)
        part = self._buf("part", S * self.tiles_last * self.C, torch.float32)
        stored = self._forward(x, th, fr, K, B, part, store_last=True)
        z = self._buf("expz", S * self.C, torch.float32)
        ext().readout_sum(part, self.tiles_last, self.C, S, z)
        wr = w.reshape(S, self.C).float().contiguous()
        gslab = self._buf("gslab", S * self.slab_tiles * self.n_gradops * 32, torch.int64)
        self._adjoint(x, th, fr, K, B, stored, wr, gslab)
        grad = torch.zeros(K, th.shape[1], dtype=torch.float32, device=self.device)
        ext().hea_grad_reduce(gslab, self.slab_tiles, self.n_gradops, self.gmeta, B, K, th, grad, th.shape[1])
        return z.view(S, self.C).clone(), grad[:, : self.n_theta]

    # ------------------------------------------------------------------ parameter shift (prefix reuse)
    def shift_owners(self) -> list:
        """Per forward pass j <= fwd_last: the theta indices whose rotation it applies (layer 1 is generated in
        pass 0; rotation group g of pass j carries theta_slot(layer, q) and its phase partner)."""
        own = [[] for _ in range(self.fwd_last + 1)]
        for q in range(self.n):
            own[0] += [self.plan.theta_slot(1, q), self.plan.theta_slot(1, q) + 1]
        for j in range(self.fwd_last + 1):
            for g in self.plan.passes[j].groups:
                for q in g.qubits:
                    own[j] += [self.plan.theta_slot(g.layer, q), self.plan.theta_slot(g.layer, q) + 1]
        flat = sorted(i for o in own for i in o)
        if flat != list(range(self.n_theta)):
            raise RuntimeError("forward passes do not own every parameter exactly once")
        return own

    def shift_pass_counts(self) -> dict:
        """Pass launches per sample of one parameter-shift gradient: naive (2 n_theta shifted circuits, every
        forward pass each) vs prefix reuse + the pi identity (one +pi branch per parameter from its pass on, the
        unshifted forward, C adjoint sweeps)."""
        F = self.fwd_last + 1
        own = self.shift_owners()
        branch = sum(len(o) * (F - j) for j, o in enumerate(own))
        return {"naive_fwd_passes": 2 * self.n_theta * F, "reuse_fwd_passes": branch + F,
                "reuse_adj_passes": self.C * self.n_passes, "branch_fwd_passes": branch}

    def _shift_budget(self) -> int:
        """Bytes of HBM the chunked evaluation / parameter-shift paths may hold in live states."""
        if self._ps_budget is None:
            env = os.environ.get("QFEDX_PS_BUDGET_MB")
            if env:
                self._ps_budget = int(env) << 20
            else:
                free, _ = torch.cuda.mem_get_info(self.device)
                self._ps_budget = int(0.4 * free)
        return self._ps_budget

    @torch.no_grad()
    def shifted_expz(self, xang: torch.Tensor, params: torch.Tensor, with_mean: bool = True) -> torch.Tensor:
        """Exact <Z> at theta +- pi/2 e_j for every client, parameter j, sign and sample -> [K, n_theta, 2, B, C]
        (sign 0: +pi/2), from the prefix-reuse identities of ``param_shift``.  ``with_mean=False`` drops the
        common term m (only the +- difference is wanted) and skips the +pi branches."""
        f0, fpi, jac = self._shift_parts(xang, params, with_mean)
        jt = jac.permute(0, 3, 1, 2)                        # [K, P, B, C]
        m = 0.5 * (f0.unsqueeze(1) + fpi) if with_mean else torch.zeros_like(jt)
        return torch.stack([m + jt, m - jt], 2).contiguous()

    @torch.no_grad()
    def _shift_parts(self, xang: torch.Tensor, params: torch.Tensor, with_mean: bool):
        """f(theta) [K, B, C], f(theta + pi e_j) [K, P, B, C] (None without the mean term) and the per-sample
        Jacobian d<Z_c>/dtheta_j [K, B, C, P]."""
        E = ext()
        x, th, K, B = self._prep(xang, params)
        P, C, n = self.n_theta, self.C, self.n
        if th.shape[1] < P + 2 * C:
            th = torch.cat([th, th.new_zeros(K, P + 2 * C - th.shape[1])], 1)
        ps = th.shape[1]
        F = self.fwd_last + 1
        own = self.shift_owners()
        sb = (1 << n) * 4                                   # fp16 (re, im) per amplitude
        budget = self._shift_budget()
        Kc = max(1, min(K, (budget // 2) // max(1, (F + 3) * B * sb)))
        rows_max = max(B, (budget // 2) // (2 * sb))        # samples per +pi chunk (two ping-pong states)
        f0 = torch.empty(K, B, C, dtype=torch.float32, device=self.device)
        jac = torch.empty(K, B, C, P, dtype=torch.float32, device=self.device)
        fpi = torch.empty(K, P, B, C, dtype=torch.float32, device=self.device) if with_mean else None
        empty = torch.empty(0, dtype=torch.int32, device=self.device)
        eye = torch.eye(C, dtype=torch.float32, device=self.device)
        for k0 in range(0, K, Kc):
            k1 = min(K, k0 + Kc)
            nk, S = k1 - k0, (k1 - k0) * B
            xs, ths = x[k0 * B:k1 * B], th[k0:k1].contiguous()
            fr = self._frags(ths, nk, "ps")
            part = self._buf("pspart", S * self.tiles_last * C, torch.float32)
            stored = self._forward(xs, ths, fr, nk, B, part, store_last=True, tag="ps")
            z = self._buf("psz", S * C, torch.float32)
            E.readout_sum(part, self.tiles_last, C, S, z)
            f0[k0:k1] = z.view(nk, B, C)
            # per-sample Jacobian rows: one adjoint sweep per class over the stored forward, reduced with spc = 1
            gslab = self._buf("psgslab", S * self.slab_tiles * self.n_gradops * 32, torch.int64)
            th_rep = ths.repeat_interleave(B, 0).contiguous()
            g = torch.zeros(S, ps, dtype=torch.float32, device=self.device)
            for c in range(C):
                wr = eye[c].expand(S, C).contiguous()
                self._adjoint(xs, ths, fr, nk, B, stored, wr, gslab, "ps")
                E.hea_grad_reduce(gslab, self.slab_tiles, self.n_gradops, self.gmeta, 1, S, th_rep, g, ps)
                jac[k0:k1, :, c] = g[:, :P].view(nk, B, P)
            if not with_mean:
                continue
            # +pi branches: parameter rows (client, owned parameter) from their pass on
            per = max(1, rows_max // B)                     # parameter rows per chunk
            for j, sl in enumerate(own):
                if not sl:
                    continue
                Pj = len(sl)
                slots = torch.tensor(sl, dtype=torch.long, device=self.device)
                nr = min(Pj, per)
                nkc = max(1, per // Pj) if nr == Pj else 1
                for a0 in range(0, nk, nkc):
                    a1 = min(nk, a0 + nkc)
                    for r0 in range(0, Pj, nr):
                        r1 = min(Pj, r0 + nr)
                        src = stored[j - 1][(a0 * B) << n:(a1 * B) << n] if j > 0 else empty
                        zb = self._pi_branch(j, xs[a0 * B:a1 * B], ths[a0:a1], slots[r0:r1], B, src)
                        fpi[k0 + a0:k0 + a1].index_copy_(1, slots[r0:r1], zb)
        return f0, fpi, jac

    @torch.no_grad()
    def param_shift(self, xang: torch.Tensor, params: torch.Tensor, w: torch.Tensor, noise=None, keys=None,
                    step: int = 0, exact_only: bool = False) -> torch.Tensor:
        """dL/dtheta by the parameter-shift rule with prefix reuse (ROADMAP.md:23,130-135).

        The naive estimator runs 2 n_theta shifted circuits per sample from |0>, each shot-sampled.  Two exact
        identities for a rotation exp(-i theta P / 2) (P^2 = 1) give the SAME shifted expectations with far
        fewer pass launches (``shift_pass_counts``):

          * f(theta +- pi/2) = m +- f'(theta),  m = (f(theta) + f(theta + pi)) / 2   (f = a + b cos + c sin)
          * f'(theta) for every parameter, sample and class = C adjoint sweeps (one per class, w = e_c) over the
            stored unshifted forward, reduced per sample (spc = 1)
          * f(theta + pi) for a parameter applied in forward pass j starts from the stored unshifted OUTPUT of
            pass j - 1 (the kernel's ``in_rep`` maps each shifted row to its client's stored sample) and runs
            only passes j..fwd_last; layer-1 parameters regenerate the product state in pass 0

        The exact shifted expectations are then readout-confused / shot-sampled exactly as the naive estimator
        samples them (same Philox key per (client, slot, sign) row: ``VQCEngine.param_shift_batched``), so the
        estimator's distribution is the hardware one.  With ``shots == 0`` the sampled difference is affine in
        f', so m is not needed (no +pi branches).  Work is chunked over clients and over shifted rows to fit
        ``_shift_budget`` (0.4 of free HBM).  ``exact_only``: skip the readout model (tests).
        w = dL/d<Z>_noisy [K, B, C] -> [K, n_theta]."""
        K, B, C = w.shape
        P = self.n_theta
        noisy = noise is not None and not exact_only
        need_m = noisy and noise.shots > 0
        f0, fpi, jac = self._shift_parts(xang, params, with_mean=need_m)
        # shifted expectations, their readout model and the shift rule in one device launch (HIP, qfx_ps_combine)
        out = torch.empty(K, P, dtype=torch.float32, device=self.device)
        kk = keys.to(self.device).long().contiguous() if (need_m and keys is not None) else _NO_KEYS.to(self.device)
        if need_m and keys is None:
            raise ValueError("shot sampling needs per-client Philox keys")
        fe = torch.empty(0, device=self.device)
        ext().ps_combine(f0 if need_m else fe, fpi if need_m else fe, jac.contiguous(), w.float().contiguous(), kk,
                         noise.p01 if noisy else 0.0, noise.p10 if noisy else 0.0, noise.shots if noisy else 0,
                         int(step), int(noisy), out)
        return out

    def _pi_branch(self, j, xs, ths, slots, B, src) -> torch.Tensor:
        """<Z> of theta + pi e_slot for clients ths [na, ps] x slots [nr] owned by forward pass j: passes
        j..fwd_last, the first reading the clients' stored pass j - 1 outputs ``src`` [na B 2^n] (each row
        shared by nr parameter rows: in_rep) or, for j = 0, regenerating the product state.  -> [na, nr, B, C]"""
        E = ext()
        na, nr = ths.shape[0], slots.numel()
        Kr, S = na * nr, na * nr * B
        ps = ths.shape[1]
        thr = ths.repeat_interleave(nr, 0).view(na, nr, ps).clone()
        thr[:, torch.arange(nr, device=self.device), slots] += float(np.pi)
        thr = thr.view(Kr, ps).contiguous()
        fr = self._frags(thr, Kr, "pb")
        R = self.fwd_last
        part = self._buf("pbpart", S * self.tiles_last * self.C, torch.float32)
        N = S << self.n
        empty = torch.empty(0, dtype=torch.int32, device=self.device)
        fempty = torch.empty(0, dtype=torch.float32, device=self.device)
        psi_in = src
        for jj in range(j, R + 1):
            p, fwd = self.passes[jj][0], self.passes[jj][1]
            keep = jj < R
            out = self._buf(f"pbpsi{(jj - j) % 2}", N, torch.int32) if keep else empty
            first = jj == j
            geom = self._geom(p, jj == 0, False, keep, False, B, ps, S, xs.shape[1], Kr, nr if first else 1)
            E.hea_pass(False, fwd[0], fwd[1], fwd[2], geom, self.scale, psi_in, out, empty, empty, xs, thr, fr, fempty,
                       part if jj == R else fempty, fempty, _NODBG)
            psi_in = out
        z = self._buf("pbz", S * self.C, torch.float32)
        E.readout_sum(part, self.tiles_last, self.C, S, z)
        return z.view(na, nr, B, self.C)

    # ------------------------------------------------------------------ train step
    fuses_optimizer = True    # VQCEngine: loss_and_grads(fused_opt=...) may run the Adam step in the reduction

    def _fused_readout(self, noise) -> bool:
        """Noiseless steps compute the readout in the first adjoint pass (``fused_readout``)."""
        return noise is None and self.fused_readout and self.tiles_last * self.C <= 64

    def prologue_frag_job(self):
        """(slot_tab, frags) for the round prologue to build the first local step's fragments from the global
        parameters (one shared set: every client row starts as theta), or None without unitary slots.  The trainer
        then passes ``shared_frags=frags`` to that step's ``loss_and_grads`` (hea_frag.h; one launch fewer)."""
        if not self.n_slots:
            return None
        return [self.slot_tab, self._buf("pfrags", self.n_slots * 4 * 128 * 4, torch.int32)]

    def _step(self, x, p, yy, ww, K, B, loss, correct, grad, expz, noise, keys, step, adam=None, dbg=None,
              shared_frags=None, fed=None):
        """Forward, readout + CE, adjoint and gradient reduction of clients [0, K).
        ``adam`` = (tensors, hyper) from ``BatchedOptimizer.fused_adam``: the clients' Adam step runs in the
        gradient reduction's epilogue (one launch fewer per local step).  ``dbg``: stall-attribution buffers per
        pass (``stamp_buffers``, stamps build only)."""
        C = ext()
        S = K * B
        shared = shared_frags is not None
        fr = shared_frags if shared else self._frags(p, K)
        part = self._buf("part", S * self.tiles_last * self.C, torch.float32)
        wread = self._buf("wread", S * self.C, torch.float32)
        gslab = self._buf("gslab", S * self.slab_tiles * self.n_gradops * 32, torch.int64)
        stored = self._forward(x, p, fr, K, B, part, store_last=True, dbg=dbg, shared=shared)
        # Fused readout: the first adjoint pass computes each sample's <Z>, cross entropy and dL/d<Z> from the readout
        # partials, and the gradient reduction sums the clients' loss, hits and readout gradients - one launch fewer
        # per local step.
        ro = None
        if self._fused_readout(noise):
            rec = self._buf("rorec", S * (2 * self.C + 2), torch.float32)
            ro = [rec, loss, correct]
            self._adjoint(x, p, fr, K, B, stored, wread, gslab, readout=(part, yy, ww, expz, rec), dbg=dbg,
                          shared=shared)
        else:
            if noise is None:
                C.readout_ce(part, self.tiles_last, self.C, B, K, yy, ww, p, self.n_theta, expz, wread, loss,
                             correct, grad, True, 0.0, 0.0, 0, _NO_KEYS, 0)
            else:
                from .statevec_hip import _keys
                C.readout_ce(part, self.tiles_last, self.C, B, K, yy, ww, p, self.n_theta, expz, wread, loss,
                             correct, grad, True, noise.p01, noise.p10, noise.shots, _keys(keys, noise), int(step))
            self._adjoint(x, p, fr, K, B, stored, wread, gslab, dbg=dbg, shared=shared)
        if adam is None:
            C.hea_grad_reduce(gslab, self.slab_tiles, self.n_gradops, self.gmeta, B, K, p, grad, p.shape[1],
                              None, None, ro, self.C, self.n_theta)
        else:
            cnt = self._zbuf("adamcnt", K, torch.int32)
            f = fed if fed is not None else {}
            C.hea_grad_reduce(gslab, self.slab_tiles, self.n_gradops, self.gmeta, B, K, p, grad, p.shape[1],
                              adam[0] + [cnt], adam[1], ro, self.C, self.n_theta, f.get("fed"),
                              bool(f.get("wrap", False)), int(f.get("n_norms", 0)))

    def stamp_buffers(self) -> dict:
        """Zeroed stall-attribution buffers, one per pass launch (``fwd{j}``, ``adj{j}``), for the stamps build
        (``QFEDX_STAMPS=1``, scripts/hea_stamps.py)."""
        rows = int(getattr(ext(), "HEA_STAMP_ROWS", 0)) * 16
        names = [f"fwd{j}" for j in range(self.fwd_last + 1)] + [f"adj{j}" for j in range(self.n_passes)]
        return {nm: torch.zeros(rows, dtype=torch.int64, device=self.device) for nm in names}

    def loss_and_grads(self, xang, y, wmask, params, spec, noise=None, keys=None, step: int = 0, out_loss=None,
                       out_correct=None, init: torch.Tensor | None = None, fused_opt=None, dbg=None,
                       shared_frags=None, fed_tail=None) -> dict:
        """One adjoint training step (same contract as ``HipProgram.loss_and_grads``).
        ``fused_opt`` = (BatchedOptimizer, active): with params updated in place (a contiguous fp32 tensor) and HIP
        Adam, the optimizer step runs in the gradient reduction's epilogue and the result says ``opt_done``;
        otherwise the caller steps the optimizer itself."""
        if init is not None:
            raise ValueError("the MFMA engine starts from the angle feature map (no initial states)")
        x, p, K, B = self._prep(xang, params)
        S = K * B
        yy = y.reshape(S).long().contiguous()
        ww = wmask.reshape(S).float().contiguous()
        expz = self._buf("expz", S * self.C, torch.float32)
        loss = torch.empty(K, dtype=torch.float32, device=self.device) if out_loss is None else out_loss
        correct = torch.empty(K, dtype=torch.float32, device=self.device) if out_correct is None else out_correct
        grad = torch.empty_like(p)
        adam = None
        # Fused only while the reduction has at most one block per CU.  Every block publishes its gradient entries
        # with one agent-scope release (an L2 writeback here): at 16q x 64 clients (832 blocks) the fused launch took
        # 33.6 us against 13 + 5.4 us for the two launches; at the 8-client share (104 blocks) it saves a launch
        # (round 387 -> 382 us; profiles/r3_fused_adam_ab.txt).
        ro_rows = 1 if self._fused_readout(noise) else 0
        # (the readout parameters are owned by the fused readout block, and the row must hold nothing else)
        want = (K * (self.n_gradops + ro_rows) <= FUSED_ADAM_MAX_BLOCKS and ro_rows == 1 and self.grad_cover_exact
                and p.shape[1] == self.n_theta + 2 * self.C)
        if want and fused_opt is not None and self.n_gradops > 0 and p.data_ptr() == params.data_ptr():
            adam = fused_opt[0].fused_adam(p, fused_opt[1])
        fed = fed_tail if (adam is not None and fed_tail is not None) else None
        self._step(x, p, yy, ww, K, B, loss, correct, grad, expz, noise, keys, step, adam=adam, dbg=dbg,
                   shared_frags=shared_frags, fed=fed)
        res = {"loss": loss, "grad": grad, "correct": correct, "expz": expz.reshape(K, B, self.C)}
        if adam is not None:
            res["opt_done"] = True
        if fed is not None:
            res["fed_done"] = True     # the round's FedAvg ran in the Adam epilogue (QfxFedTail)
        return res
