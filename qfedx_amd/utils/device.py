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


class _PinnedRing:
    """Reusable pinned staging slots for host -> device uploads.

    Slot i is handed out again only after the event recorded behind its upload has completed, which
    blocks the host only when the GPU is ``SLOTS`` uploads behind.  The upload itself is a copy KERNEL
    that reads the pinned slot (``host_upload``): a small ``hipMemcpyAsync`` queued behind a hipGraph
    launch was measured to block the host until the stream drained every few rounds, which left the GPU
    idle while the host built the next round.
    """

    SLOTS = 16

    def __init__(self):
        self.bufs = [None] * self.SLOTS
        self.events = [None] * self.SLOTS
        self.i = 0

    def acquire(self, nbytes: int, alloc):
        i = self.i
        self.i = (i + 1) % self.SLOTS
        if self.events[i] is not None:
            self.events[i].synchronize()
        buf = self.bufs[i]
        if buf is None or buf.numel() < nbytes:
            # mapped + portable pinned memory.  hipHostMalloc is slow (~0.2 ms): the first use sizes EVERY slot,
            # so the allocations land in a run's first round instead of one per round for the next 15
            size = max(65536, 1 << (nbytes - 1).bit_length())
            for j in range(self.SLOTS):
                if self.bufs[j] is None or self.bufs[j].numel() < nbytes:
                    if self.events[j] is not None:
                        self.events[j].synchronize()
                    self.bufs[j] = alloc(size)
            buf = self.bufs[i]
        return i, buf[:nbytes]

    def release(self, i: int, device) -> None:
        ev = self.events[i]
        if ev is None:
            ev = self.events[i] = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(device))


_RING = None
_UPLOAD_BACKEND: list = []   # resolved once: [extension with host_alloc/host_upload] or [None]


def _upload_ext():
    """The extension's pinned-ring upload entry points, resolved ONCE per process (a failed import is not
    retried per upload, and a stale build without ``host_alloc``/``host_upload`` takes the plain-copy path)."""
    if not _UPLOAD_BACKEND:
        try:
            from ..ops._ext import ext
            E = ext()
            ok = hasattr(E, "host_alloc") and hasattr(E, "host_upload")
        except Exception:   # no extension (portable torch backend): plain pinned async copies
            E, ok = None, False
        _UPLOAD_BACKEND.append(E if ok else None)
    return _UPLOAD_BACKEND[0]


def _upload(fill, nbytes: int, device, dst: torch.Tensor | None = None) -> torch.Tensor:
    """``fill(pinned_uint8_view)`` writes ``nbytes`` (a multiple of 16); returns the device uint8 buffer."""
    global _RING
    E = _upload_ext()
    if E is None:
        src = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
        fill(src)
        if dst is None:
            return src.to(device, non_blocking=True)
        return dst.copy_(src, non_blocking=True)
    if _RING is None:
        _RING = _PinnedRing()
    i, src = _RING.acquire(nbytes, E.host_alloc)
    fill(src)
    if dst is None:
        dst = torch.empty(nbytes, dtype=torch.uint8, device=device)
    E.host_upload(src, dst[:nbytes])
    _RING.release(i, device)
    return dst


def h2d(t: torch.Tensor, device) -> torch.Tensor:
    """Host -> device copy that never stalls the host on the GPU queue (see ``_PinnedRing``)."""
    device = torch.device(device)
    if device.type != "cuda" or t.device.type == "cuda":
        return t.to(device)
    t = t.contiguous()
    nb = t.numel() * t.element_size()
    if nb == 0:
        return torch.empty(t.shape, dtype=t.dtype, device=device)
    padded = (nb + 15) // 16 * 16

    def fill(buf):
        buf[:nb].copy_(t.reshape(-1).view(torch.uint8))

    out = _upload(fill, padded, device)
    return out[:nb].view(t.dtype).view(t.shape)


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

    def _fill(self, buf: torch.Tensor) -> torch.Tensor:
        for _, off, nb, _, _, t in self.layout:
            if nb:
                buf[off: off + nb].copy_(t.reshape(-1).view(torch.uint8))
        return buf

    def to_device(self, device, dst: torch.Tensor | None = None) -> dict:
        device = torch.device(device)
        if device.type == "cuda":
            dst = _upload(self._fill, self.nbytes, device, dst)
        else:
            staged = self._fill(torch.empty(self.nbytes, dtype=torch.uint8))
            dst = staged if dst is None else dst.copy_(staged)
        return self.views(dst)

    def views(self, buf: torch.Tensor) -> dict:
        out = {}
        for name, off, nb, dt, shape, _ in self.layout:
            out[name] = buf[off: off + nb].view(dt).view(shape)
        return out
