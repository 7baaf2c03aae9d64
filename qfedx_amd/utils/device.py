"""Device / backend selection (reference: one global ``device``, ``Classical_FL.py:19``).

Each process owns exactly one GPU (``LOCAL_RANK``) - the MI355X-native scaling model is one
process per GPU with RCCL between them.  ``backend`` chooses the statevector/CNN compute path:
``hip`` = the in-tree gfx950 extension (mandatory on a GPU: it fails loudly if the extension
is missing rather than silently falling back), ``torch`` = the portable reference
implementation used on CPU and as the numerics oracle in tests.
"""
from __future__ import annotations

import os

import torch


def resolve_device(spec: str = "auto") -> torch.device:
    if spec == "cpu":
        return torch.device("cpu")
    if spec in ("auto", "cuda") and torch.cuda.is_available():
        local = int(os.environ.get("LOCAL_RANK", "0"))
        idx = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(idx)
        return torch.device("cuda", idx)
    if spec == "cuda":
        raise RuntimeError("runtime.device=cuda requested but no GPU is visible")
    return torch.device("cpu")


def resolve_backend(spec: str, device: torch.device) -> str:
    if spec == "auto":
        return "hip" if device.type == "cuda" else "torch"
    if spec == "hip" and device.type != "cuda":
        raise RuntimeError("backend=hip requires a GPU device")
    return spec


def h2d(t: torch.Tensor, device) -> torch.Tensor:
    """Host -> device copy that never stalls the host on the GPU queue.

    A pageable-memory copy blocks until the stream reaches it (i.e. a hidden device sync).  Staging
    through pinned memory makes it a true async DMA; torch's caching host allocator keeps the pinned
    block alive until the copy has completed, so the staging buffer is never overwritten early.
    """
    device = torch.device(device)
    if device.type != "cuda" or t.device.type == "cuda":
        return t.to(device)
    return t.pin_memory().to(device, non_blocking=True)


class PackedUpload:
    """Several small host tensors -> ONE pinned staging buffer -> ONE async H2D copy.

    A federated round needs a handful of tiny host-built tables on the device (client slots, minibatch
    indices, loss weights, step masks); uploading them together replaces one copy launch (and one
    pinned staging allocation) per table.  ``to_device`` returns dtype/shape views into the device
    buffer (or into ``dst``, a preallocated uint8 device buffer, e.g. a hipGraph's static input).
    """

    ALIGN = 16

    def __init__(self, tensors: dict):
        self.layout = []
        off = 0
        for name, t in tensors.items():
            t = t.contiguous()
            nbytes = t.numel() * t.element_size()
            self.layout.append((name, off, nbytes, t.dtype, tuple(t.shape), t))
            off += (nbytes + self.ALIGN - 1) // self.ALIGN * self.ALIGN
        self.nbytes = max(off, self.ALIGN)

    def _staging(self, pin: bool) -> torch.Tensor:
        buf = torch.empty(self.nbytes, dtype=torch.uint8, pin_memory=pin)
        for _, off, nb, _, _, t in self.layout:
            if nb:
                buf[off: off + nb].copy_(t.reshape(-1).view(torch.uint8))
        return buf

    def to_device(self, device, dst: torch.Tensor | None = None) -> dict:
        device = torch.device(device)
        if device.type == "cuda":
            src = self._staging(True)
            if dst is None:
                dst = src.to(device, non_blocking=True)
            else:
                dst.copy_(src, non_blocking=True)
        else:
            dst = self._staging(False) if dst is None else dst.copy_(self._staging(False))
        return self.views(dst)

    def views(self, buf: torch.Tensor) -> dict:
        out = {}
        for name, off, nb, dt, shape, _ in self.layout:
            out[name] = buf[off: off + nb].view(dt).view(shape)
        return out
