"""Stall attribution of the MFMA pass kernels (verdict r4 item 1a): where each wave of a pass spends its cycles.

Needs the stamps build (``python -m qfedx_amd._build --stamps``) and runs with ``QFEDX_STAMPS=1`` (set here): every wave
of the first STAMP_WG workgroups of each pass launch sums s_memtime deltas per phase (csrc/hea_mfma.hip, enum Ph):

  PRO    kernel start -> tile-load issue          LOAD   tile load / product-state generation -> first barrier
  BAR    op barriers, arrival -> release          SETUP  fragment registers, next-op staging, gradient-region flush
  BACK   BACK op bodies   GRADL1 cross-only op bodies   APPLY forward group ops   OTHER OBS / READOUT
  EPI    gradient epilogue (fixed point + u64 LDS atomics)                        TAIL   last barrier, reduction, store
  GEN1   first forward pass: layer-1 factors (wave 0) + barrier   GEN2 half-index tables + barrier (LOAD: the quads)

Each stamp costs ~40 cycles and drains the wave's LDS operations (s_waitcnt lgkmcnt(0)), so read SHARES, never the
build's run time.  Prints one JSON line per pass (mean cycles per wave per phase, per-op means, shares) and a text
table.  python scripts/hea_stamps.py [--qubits 16 --layers 3 --clients 64 --batch 32]
"""
import argparse
import json
import os
import sys

os.environ["QFEDX_STAMPS"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PH = ["PRO", "LOAD", "BAR", "SETUP", "BACK", "GRADL1", "APPLY", "OTHER", "EPI", "TAIL", "GEN1", "GEN2"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--qubits", type=int, default=16)
    ap.add_argument("--layers", type=int, default=3)
    ap.add_argument("--clients", type=int, default=64)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    import numpy as np
    import torch
    from qfedx_amd.models.vqc import VQCSpec
    from qfedx_amd.ops._ext import ext
    from qfedx_amd.ops.hea_mfma import HeaMfmaProgram
    from qfedx_amd.ops.hea_plan import OP_BACK, OP_BACK2, OP_GRAD2, OP_GRAD_L1, W_CODE

    E = ext()
    assert getattr(E, "__name__", "").endswith("_stamps"), "needs the stamps build (QFEDX_STAMPS=1)"
    dev = torch.device("cuda", 0)
    spec = VQCSpec(args.qubits, args.layers, 3)
    K, B = args.clients, args.batch
    g = torch.Generator().manual_seed(0)
    x = spec.encode_features(torch.rand(K, B, args.qubits, generator=g)).to(dev)
    y = torch.randint(0, 3, (K, B), generator=g).to(dev)
    w = torch.full((K, B), 1.0 / B, device=dev)
    params = torch.stack([spec.init_params(k) for k in range(K)]).to(dev)
    prog = HeaMfmaProgram(spec, dev)
    for _ in range(3):                                  # warm caches / clocks
        prog.loss_and_grads(x, y, w, params, spec)
    dbg = prog.stamp_buffers()
    prog.loss_and_grads(x, y, w, params, spec, dbg=dbg)
    torch.cuda.synchronize()
    lines = []
    for name, buf in dbg.items():
        j = int(name[3:])
        adjoint = name.startswith("adj")
        p = prog.passes[j][3] if adjoint else prog.passes[j][0]
        ops = prog.passes[j][2][0] if adjoint else prog.passes[j][1][0]
        codes = [int(c) for c in ops[:, W_CODE].cpu()]
        nw = (1 << (p.t - 4)) // 64 if adjoint else 8
        rows = buf.view(-1, 16).cpu().numpy().astype(np.float64)
        rows = rows[rows[:, 15] > 0]                     # waves that wrote a row
        if len(rows) == 0:
            continue
        tot = rows[:, 15].mean()
        mean = {ph: float(rows[:, i].mean()) for i, ph in enumerate(PH)}
        n_back = sum(c in (OP_BACK, OP_BACK2) for c in codes)        # op records (a pair record = one body)
        n_l1 = sum(c in (OP_GRAD_L1, OP_GRAD2) for c in codes)
        rec = {"pass": name, "t": p.t, "waves_per_wg": nw, "waves_stamped": int(len(rows)), "ops": len(codes),
               "op_codes": codes, "cycles_per_wave": round(tot), "phase_cycles": {k: round(v) for k, v in mean.items()},
               "phase_share": {k: round(v / tot, 4) for k, v in mean.items()},
               "per_op": {"BAR": round(mean["BAR"] / max(1, len(codes))), "SETUP": round(mean["SETUP"] / max(1, len(codes))),
                          "BACK_body": round(mean["BACK"] / n_back) if n_back else None,
                          "GRADL1_body": round(mean["GRADL1"] / n_l1) if n_l1 else None,
                          "EPI": round(mean["EPI"] / max(1, n_back + n_l1)) if (n_back + n_l1) else None},
               # barrier wait spread: the slowest wave of a workgroup waits least
               "bar_wave_p10_p90": [round(float(np.percentile(rows[:, 2], 10))), round(float(np.percentile(rows[:, 2], 90)))]}
        # per wave index (which waves the others wait for at the barriers): mean cycles of each phase
        ww = buf.view(-1, nw, 16).cpu().numpy().astype(np.float64)
        ww = ww[ww[:, :, 15].min(axis=1) > 0]
        rec["per_wave"] = {ph: [round(float(v)) for v in ww[:, :, i].mean(axis=0)] for i, ph in enumerate(PH)
                           if ww[:, :, i].mean() > 0}
        lines.append(rec)
        print(json.dumps(rec), flush=True)
    print()
    for r in lines:
        print(f"{r['pass']} per wave index (mean cycles):")
        for ph, v in r["per_wave"].items():
            print(f"  {ph:7s} " + " ".join(f"{x:6d}" for x in v))
    print(f"{'pass':6s} {'cyc/wave':>9s} " + " ".join(f"{ph:>7s}" for ph in PH))
    for r in lines:
        print(f"{r['pass']:6s} {r['cycles_per_wave']:9d} " + " ".join(f"{100 * r['phase_share'][ph]:6.1f}%" for ph in PH))
    if args.out:
        with open(args.out, "w") as f:
            for r in lines:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
