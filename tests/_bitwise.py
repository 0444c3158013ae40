"""Bitwise comparison for the GPU tests that carries its own evidence on failure: which tensor and step differ, how
many elements, by how much, and — for buffers laid out like the flat parameter buffer — the parameter name and
element of the first differing flat offset (VERDICT r04 #1a: a bare ``torch.equal`` records nothing)."""
from __future__ import annotations

import torch


def param_at(layout, off: int) -> str:
    """The state_dict name (and element index) whose view covers flat offset ``off`` of ``layout``."""
    for name, v in sorted(layout.views.items(), key=lambda kv: kv[0].startswith("__")):  # public names first
        lo = v.offset
        hi = lo + sum((n - 1) * s for n, s in zip(v.shape, v.stride))
        if not lo <= off <= hi:
            continue
        rel, idx = off - lo, []
        # views are row-major with positive strides: peel the coordinates from the outermost dimension
        for n, s in zip(v.shape, v.stride):
            i = min(rel // s, n - 1) if s else 0
            idx.append(i)
            rel -= i * s
        if rel == 0:
            return f"{name}{tuple(idx)}"
    return "<padding / outside every view>"


def _mismatch(fa: torch.Tensor, fb: torch.Tensor) -> torch.Tensor:
    ne = fa != fb
    if fa.is_floating_point():
        ne &= ~(torch.isnan(fa) & torch.isnan(fb))  # the same NaN on both sides is the same result
    return ne


def describe(a: torch.Tensor, b: torch.Tensor, layout=None) -> str:
    if a.shape != b.shape or a.dtype != b.dtype:
        return f"shape/dtype {tuple(a.shape)}/{a.dtype} vs {tuple(b.shape)}/{b.dtype}"
    fa, fb = a.reshape(-1), b.reshape(-1)
    ne = _mismatch(fa, fb)
    n = int(ne.sum())
    first = int(ne.nonzero()[0]) if n else -1
    d = (fa.double() - fb.double()).abs()
    d = d[ne]
    msg = (f"{n} of {fa.numel()} elements differ; max |d| {float(d.max()):.3e}, first at flat {first} "
           f"({float(fa[first]):.9g} vs {float(fb[first]):.9g})")
    if layout is not None and a.numel() >= layout.total:
        msg += f" = {param_at(layout, first)}"
        if n <= 64:  # a localised difference: every element (its pattern points at the kernel and tile)
            msg += "; all: " + ", ".join(param_at(layout, int(i)).split(".")[-1] if k else param_at(layout, int(i))
                                          for k, i in enumerate(ne.nonzero().reshape(-1).tolist()))
    return msg


def assert_bitwise(a: torch.Tensor, b: torch.Tensor, what: str, layout=None) -> None:
    a, b = a.detach(), b.detach()
    if a.shape == b.shape and a.dtype == b.dtype and not bool(_mismatch(a.reshape(-1), b.reshape(-1)).any()):
        return
    raise AssertionError(f"{what}: {describe(a, b, layout)}")
