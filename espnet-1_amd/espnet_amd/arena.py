"""Flat parameter arena: every parameter of the model lives in ONE f32 device buffer
(plus one f32 grad buffer and, in bf16 mode, one bf16 weight shadow).

Why (MI355X-first): the optimizer, grad-norm, zero_grad and the f32->bf16 weight cast
become single launches over 116 M contiguous floats instead of 615 small kernels, and
the data-parallel all-reduce works on large contiguous buckets (bucket = byte range of
the arena).  Groups of parameters that one fused GEMM consumes (q/k/v weights, the six
decoder layers' cross-attention k/v) are laid out adjacently, so the fused weight is a
plain view.

nn.Parameters stay the reference's (same names, shapes, state_dict layout — SURVEY.md
§8b); after `ParamArena(model)` each Parameter's storage IS a view into the arena and
its `.grad` a view into the grad arena, so `state_dict()`, `load_state_dict()` and
`parameters()` keep working unchanged.
"""
from __future__ import annotations

from typing import Dict, List, Sequence

import torch

ALIGN = 64  # elements: keeps every view 256-B aligned in f32 and 128-B aligned in bf16


class ParamArena:
    def __init__(self, model: torch.nn.Module, device, order: Sequence[Sequence[str]] = (),
                 shadow_dtype=None):
        named = dict(model.named_parameters())
        seen = set()
        chunks: List[List[str]] = []  # each chunk is packed back to back, chunk starts aligned
        # registration order, except that an adjacency group is laid out in full where its
        # first-registered member would go: every module's parameters stay in one region of
        # the arena, so a data-parallel bucket (a byte range) is final as soon as the modules
        # in it are, and the front of the arena is the first-registered module (the
        # subsampling front end, whose backward is the last of the step)
        group_of: Dict[str, List[str]] = {}
        for group in order:
            g = [n for n in group if n in named]
            if not g:
                continue
            first = min(g, key=list(named).index)
            group_of.setdefault(first, [])
            group_of[first] += [n for n in g if n not in group_of[first]]
        for n in named:
            if n in seen:
                continue
            g = [m for m in group_of.get(n, [n]) if m not in seen]
            if n not in g:
                g.insert(0, n)
            seen.update(g)
            chunks.append(g)
        self.offsets: Dict[str, int] = {}
        layout: List[str] = []
        off = 0
        for chunk in chunks:
            off = (off + ALIGN - 1) // ALIGN * ALIGN
            for n in chunk:
                self.offsets[n] = off
                off += named[n].numel()
                layout.append(n)
        self.numel = (off + ALIGN - 1) // ALIGN * ALIGN
        self.device = torch.device(device)
        self.data = torch.zeros(self.numel, dtype=torch.float32, device=self.device)
        self.grad = torch.zeros(self.numel, dtype=torch.float32, device=self.device)
        self.shadow = None
        if shadow_dtype is not None and shadow_dtype != torch.float32:
            self.shadow = torch.zeros(self.numel, dtype=shadow_dtype, device=self.device)
        self.names = layout
        self._params = named
        from . import hip_ops  # transposed bf16 copies for the Linear input-gradient GEMMs
        self.tshadow = hip_ops.attach_transposed_shadow(self.shadow)
        self._flatten_buffers(model)
        with torch.no_grad():
            for n in layout:
                p = named[n]
                o = self.offsets[n]
                view = self.data[o:o + p.numel()].view(p.shape)
                view.copy_(p.data.to(self.device, torch.float32))
                p.data = view
                p.grad = self.grad[o:o + p.numel()].view(p.shape)
        self.refresh_shadow()

    def _flatten_buffers(self, model):
        """BatchNorm running stats -> one f32 buffer + one int64 buffer (views keep the
        state_dict keys), so the per-step rank-0 broadcast (DDP broadcast_buffers) is two
        collectives instead of 3 per conv module."""
        fb, ib = [], []
        for m in model.modules():
            for k, v in m._buffers.items():
                if v is None:
                    continue
                (fb if v.is_floating_point() else ib).append((m, k, v))
        self.buf_f32 = torch.zeros(sum(v.numel() for _, _, v in fb), dtype=torch.float32, device=self.device)
        self.buf_i64 = torch.zeros(sum(v.numel() for _, _, v in ib), dtype=torch.long, device=self.device)
        for flat, items in ((self.buf_f32, fb), (self.buf_i64, ib)):
            o = 0
            for m, k, v in items:
                view = flat[o:o + v.numel()].view(v.shape)
                view.copy_(v.to(self.device, flat.dtype))
                m._buffers[k] = view
                o += v.numel()

    # ------------------------------------------------------------------ views
    def contiguous_span(self, names: Sequence[str]):
        o0 = self.offsets[names[0]]
        end = o0
        for n in names:
            if self.offsets[n] != end:
                raise RuntimeError(f"arena: {names} are not adjacent")
            end += self._params[n].numel()
        return o0, end

    def view(self, names: Sequence[str] | str, shape=None, which="data"):
        if isinstance(names, str):
            names = [names]
        o0, end = self.contiguous_span(names)
        buf = {"data": self.data, "grad": self.grad, "shadow": self.shadow}[which]
        if buf is None:
            buf = self.data
        t = buf[o0:end]
        if shape is None:
            shape = self._params[names[0]].shape if len(names) == 1 else (end - o0,)
        return t.view(shape)

    # ------------------------------------------------------------------ housekeeping
    def zero_grad(self):
        self.grad.zero_()

    def refresh_shadow(self):
        if self.shadow is not None:
            from . import hip_ops
            from ._lib import lib
            lib.ea_cast_f32_bf16(self.numel, self.data.data_ptr(), self.shadow.data_ptr(),
                                 hip_ops.stream())
            if self.tshadow is not None:
                self.tshadow.refresh()

    def rebind(self):
        """Re-point Parameters at the arena (after an external .data / .grad reassignment)."""
        for n in self.names:
            p = self._params[n]
            o = self.offsets[n]
            if p.data.data_ptr() != self.data[o:].data_ptr():
                with torch.no_grad():
                    self.data[o:o + p.numel()].view(p.shape).copy_(p.data)
                p.data = self.data[o:o + p.numel()].view(p.shape)
            p.grad = self.grad[o:o + p.numel()].view(p.shape)
