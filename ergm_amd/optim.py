"""FusedAdamW and the polynomial-decay LR schedule of the reference train loop.

``FusedAdamW`` is a ``torch.optim.Optimizer`` with torch.optim.AdamW's hyper-parameters, defaults
and state_dict format (``exp_avg``, ``exp_avg_sq``, ``step`` per parameter), so
``get_polynomial_decay_schedule_with_warmup`` (src/main.py:93-95) drives it unchanged.  Its one
parameter is the model's flat fp32 buffer; ``reference_state_dict()`` / ``load_state_dict()`` convert
to and from the reference's per-tensor ``torch.optim.AdamW`` state over ``model.parameters()``
(src/main.py:68,107,188), so optimizer checkpoints interchange with the reference in both directions
(tests/golden/optim_ref.npz) for every configuration the reference can build (feature width = n_embd).  With the
build-side feature projections of config 5 (feat_dim != n_embd) the state also holds ``visual_proj`` /
``audio_proj`` entries the reference model has no parameters for: such checkpoints load here, not there.
``step()`` is one HIP launch over the flat parameter buffer (``ergm_adamw_step``) that also refreshes the bf16
weight shadow.
"""
from __future__ import annotations

import math

import torch

from . import ops

# torch.optim.AdamW's per-group keys besides the hyper-parameters (a reference-format state dict carries them)
_ADAMW_GROUP_DEFAULTS = {"amsgrad": False, "maximize": False, "foreach": None, "capturable": False,
                         "differentiable": False, "fused": None}


def reference_param_names(layout):
    """``model.parameters()`` order of the reference GPT2LMHeadModel (src/model.py:386-392,270-284,
    599-608: wte, wpe, every block's ln_1, attn, ln_2, crossattention, ln_cross_attn, mlp, then ln_f and
    emotion_head; the tied lm_head.weight is the wte Parameter and is yielded once) — the index order of
    the reference optimizer's state (src/main.py:68).  Pinned by tests/golden/optim_ref.npz."""
    from .params import state_dict_names
    return [n for n in state_dict_names(layout) if n != "lm_head.weight"]


def _view(layout, name: str, t: torch.Tensor) -> torch.Tensor:
    v = layout.views[name]
    return t.as_strided(v.shape, v.stride, v.offset)


def reference_from_flat(layout, exp_avg, exp_avg_sq, step, group) -> dict:
    """Flat AdamW state (moments laid out like the flat parameter buffer) -> the reference's per-tensor
    ``torch.optim.AdamW`` state_dict over ``reference_param_names(layout)``."""
    names = reference_param_names(layout)
    state = {}
    if exp_avg is not None:
        stp = torch.as_tensor(step).detach().clone().float().cpu().reshape(())
        for i, n in enumerate(names):
            state[i] = {"step": stp.clone(), "exp_avg": _view(layout, n, exp_avg).detach().clone(),
                        "exp_avg_sq": _view(layout, n, exp_avg_sq).detach().clone()}
    g = {k: v for k, v in group.items() if k != "params"}
    for k, v in _ADAMW_GROUP_DEFAULTS.items():
        g.setdefault(k, v)
    g["params"] = list(range(len(names)))
    return {"state": state, "param_groups": [g]}


def flat_from_reference(layout, state_dict, like: torch.Tensor):
    """The reference's per-tensor AdamW state_dict -> (exp_avg, exp_avg_sq) flat tensors shaped like
    ``like`` (padding zero), the common step, and the hyper-parameters of its group.  Raises ValueError
    on a parameter count or shape that is not this layout's, or on per-parameter steps that differ."""
    names = reference_param_names(layout)
    grp = state_dict["param_groups"][0]
    if len(grp["params"]) != len(names):
        raise ValueError(f"optimizer state has {len(grp['params'])} parameters, the reference model.parameters() "
                         f"of this configuration has {len(names)}")
    m = torch.zeros_like(like)
    v = torch.zeros_like(like)
    steps = set()
    ents = state_dict.get("state", {})
    for i, pid in enumerate(grp["params"]):
        e = ents.get(pid)
        if not e:
            continue
        n = names[i]
        dst = _view(layout, n, m)
        if tuple(e["exp_avg"].shape) != tuple(dst.shape):
            raise ValueError(f"optimizer state of {n}: shape {tuple(e['exp_avg'].shape)}, expected {tuple(dst.shape)}")
        dst.copy_(e["exp_avg"])
        _view(layout, n, v).copy_(e["exp_avg_sq"])
        steps.add(float(e["step"]))
    if len(steps) > 1:
        raise ValueError(f"per-parameter AdamW steps differ ({sorted(steps)}): one flat step cannot hold them")
    hp = {k: (tuple(grp[k]) if k == "betas" else grp[k]) for k in ("lr", "betas", "eps", "weight_decay", "initial_lr")
          if k in grp}
    return m, v, (steps.pop() if steps else 0.0), hp


class FusedAdamW(torch.optim.Optimizer):
    """torch.optim.AdamW semantics as one HIP kernel over the flat parameter buffer.

    ``overlap=True`` (needs ``model``): the update of each gradient bucket is launched during the
    backward pass, on the side stream, as soon as that bucket is final (after its all-reduce under
    data parallelism) — AdamW's 30 B/param of HBM traffic then overlaps the remaining backward
    instead of following it.  It uses the learning rate in ``param_groups`` at backward time, which
    is the one ``step()`` would use in the reference loop (zero_grad → backward → step → sched.step,
    src/main.py:152-156, no gradient clipping in between), and ``step()`` only advances the step count.  Each backward applies one update, so this mode is for loops that
    call ``backward()`` once per ``step()`` (the reference's); gradient accumulation (a backward onto
    an existing ``.grad``) falls back to updating in ``step()``.
    """

    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 1e-2,
                 model=None, overlap: bool = False, defer: bool = False):
        if not 0.0 <= lr:
            raise ValueError(f"Invalid learning rate: {lr}")
        if not 0.0 <= eps:
            raise ValueError(f"Invalid epsilon value: {eps}")
        if not 0.0 <= betas[0] < 1.0 or not 0.0 <= betas[1] < 1.0:
            raise ValueError(f"Invalid beta parameters: {betas}")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self.model = model  # when given, its bf16 shadow is refreshed in the same pass
        self._applied = set()
        self.overlap_blocks = 0  # grid cap of the overlapped per-bucket update (CUs it may occupy)
        # single process, overlap=True: the block updates run after the backward, overlapping the next
        # forward (which waits for each block's update before that block; ergm_model_optimizer_join)
        self.defer = bool(defer)
        if overlap:
            if model is None:
                raise ValueError("overlap=True needs model=")
            model._overlap_opt = self

    def _state(self, p):
        st = self.state[p]
        if len(st) == 0:
            st["step"] = torch.tensor(0.0)
            st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
        return st

    def _group_of(self, p):
        for g in self.param_groups:
            if any(q is p for q in g["params"]):
                return g
        return None

    def _backward_hook(self, flat, model):
        """Called by the model's backward: returns post(a, b) updating flat[a:b] from the gradient
        buffer, or None when this optimizer does not own ``flat``."""
        group = self._group_of(flat)
        if group is None:
            return None
        st = self._state(flat)
        t = int(st["step"].item()) + 1
        b1, b2 = group["betas"]
        m, v, g, shadow = st["exp_avg"], st["exp_avg_sq"], model.grad_buf, model.flat_b16
        lr, eps, wd = group["lr"], group["eps"], group["weight_decay"]
        self._applied.add(id(flat))
        nb = self.overlap_blocks

        def post(a, b, rows=None, shadow_out=None):
            # shadow_out: where the updated bf16 copy of flat[a:b] goes instead of the shadow (ZeRO-1: this
            # rank's all-gather slot, from which the exchange writes every rank's chunk into the shadow)
            if rows is None:
                ops.adamw_step(flat.data[a:b], g[a:b], m[a:b], v[a:b], shadow[a:b] if shadow_out is None else shadow_out,
                               lr, b1, b2, eps, wd, t, nb)
            else:  # (row_len, row_flag, select): only the selected rows of the [.., row_len] block
                row_len, flags, select = rows
                ops.adamw_rows(flat.data[a:b], g[a:b], m[a:b], v[a:b], shadow[a:b], row_len, flags, select, lr, b1,
                               b2, eps, wd, t, nb)
        # what a fused native exchange (dist.DPSync, ergm_dp_sum_adamw) needs to apply the same update itself
        post.native = dict(p=flat.data, m=m, v=v, lr=lr, beta1=b1, beta2=b2, eps=eps, weight_decay=wd,
                           step_size=lr / (1 - b1 ** t), bc2_sqrt=math.sqrt(1 - b2 ** t), max_blocks=nb)
        return post

    def _native_desc(self, flat, model):
        """Single process: the same per-bucket schedule run by the native executor
        (ergm_model_set_optimizer) instead of Python hooks — an ergm_adamw_desc for this step, or None
        when this optimizer does not own ``flat``."""
        import ctypes as C
        import math
        from . import _lib as L
        from .params import dp_buckets
        group = self._group_of(flat)
        if group is None:
            return None
        st = self._state(flat)
        t = int(st["step"].item()) + 1
        b1, b2 = group["betas"]
        lay = model.layout
        key = (id(model), lay.total)
        if getattr(self, "_ranges_key", None) != key:
            rs = dp_buckets(lay)[:lay.L] + [lay.seg["capwpe"]]
            self._ranges = (C.c_int64 * (2 * len(rs)))(*[x for ab in rs for x in ab])
            self._ranges_key = key
        d = L.AdamWDesc()
        d.param, d.grad = flat.data.data_ptr(), model.grad_buf.data_ptr()
        d.exp_avg, d.exp_avg_sq = st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr()
        d.param_bf16 = model.flat_b16.data_ptr()
        d.ranges, d.n_ranges = self._ranges, lay.L + 1
        d.wte_begin = lay.seg["wte"][0]
        d.lr, d.beta1, d.beta2, d.eps, d.weight_decay = group["lr"], b1, b2, group["eps"], group["weight_decay"]
        d.step_size = group["lr"] / (1 - b1 ** t)
        d.bc2_sqrt = math.sqrt(1 - b2 ** t)
        d.max_blocks = int(self.overlap_blocks)
        d.defer = int(self.defer)
        self._applied.add(id(flat))
        return d

    # ---- checkpoint interchange with the reference's per-tensor torch.optim.AdamW state ----------------
    def reference_state_dict(self) -> dict:
        """The optimizer state in the reference's format (src/main.py:68,188): ``torch.optim.AdamW``
        over ``model.parameters()`` of the reference GPT2LMHeadModel — one entry per parameter in that
        order (the tied lm_head dropped), ``exp_avg`` / ``exp_avg_sq`` shaped like the parameter (wte
        without its padding rows), ``step`` a float tensor.  ``torch.optim.AdamW(...).load_state_dict``
        of the reference (and ``FusedAdamW.load_state_dict``) accept it."""
        if self.model is None:
            raise ValueError("reference_state_dict needs FusedAdamW(..., model=)")
        self.state_dict()  # flushes deferred updates, refuses sharded moments
        flat = self.model.flat
        st = self.state.get(flat, {})
        return reference_from_flat(self.model.layout, st.get("exp_avg"), st.get("exp_avg_sq"), st.get("step"),
                                   self._group_of(flat))

    def load_state_dict(self, state_dict):
        """Either format: this optimizer's own (one flat parameter) or the reference's per-tensor
        ``torch.optim.AdamW`` state over ``model.parameters()`` (a reference checkpoint's
        ``optim_state_dict``), which is scattered into the flat moments through the layout views."""
        if self.model is not None:
            # deferred block updates may still be writing the moments this replaces
            self.model.flush_deferred_()
        groups = state_dict.get("param_groups", [])
        flat = self.model.flat if self.model is not None else None
        if flat is not None and len(groups) == 1 and len(groups[0]["params"]) != 1:
            m, v, step, hp = flat_from_reference(self.model.layout, state_dict, flat.data)
            grp = self._group_of(flat)
            grp.update(hp)
            self.state[flat] = {"step": torch.tensor(step), "exp_avg": m, "exp_avg_sq": v}
            for r in self.model._runners.values():  # every rank now holds the full moments
                r.dp.sharded.clear()
            return
        super().load_state_dict(state_dict)
        # a checkpoint read with map_location=<gpu> (Trainer.load) puts the step count on the device, and every
        # step's host read of it (the bias corrections) would then wait for the GPU: keep it on the host
        for st in self.state.values():
            if torch.is_tensor(st.get("step")) and st["step"].device.type != "cpu":
                st["step"] = st["step"].detach().to("cpu", torch.float32)

    def state_dict(self):
        if self.model is not None:
            self.model.flush_deferred_()  # the moments of deferred block updates
            if self.model.sharded:
                raise RuntimeError("the sharded optimizer update (ZeRO-1) left this rank's AdamW moments valid only "
                                   "in its own chunks: call model.consolidate_() on EVERY rank first")
        return super().state_dict()

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            b1, b2 = group["betas"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                if not p.is_cuda or p.dtype != torch.float32 or not p.is_contiguous():
                    raise ValueError("FusedAdamW needs contiguous fp32 GPU parameters")
                st = self._state(p)
                st["step"] += 1
                if id(p) in self._applied:   # already updated bucket by bucket during backward
                    self._applied.discard(id(p))
                    if self.model is not None and p is self.model.flat:
                        self.model._b16_version = p._version
                    continue
                if self.model is not None and p is self.model.flat:
                    self.model.flush_deferred_()  # pending deferred block updates first
                    if self.model.sharded:
                        self.model.consolidate_()  # the full update needs every rank's master and moments
                t = int(st["step"].item())
                shadow = None
                if self.model is not None and p is self.model.flat:
                    shadow = self.model.flat_b16
                ops.adamw_step(p.data, p.grad, st["exp_avg"], st["exp_avg_sq"], shadow, group["lr"], b1, b2,
                               group["eps"], group["weight_decay"], t)
                if shadow is not None:
                    self.model._b16_version = p._version
        return loss


def polynomial_decay_lr_lambda(num_warmup_steps: int, num_training_steps: int, lr_init: float,
                               lr_end: float = 1e-7, power: float = 2.0):
    """The LR multiplier of ``get_polynomial_decay_schedule_with_warmup`` (power=2 in the reference,
    src/main.py:93-95), restated so training does not depend on transformers."""
    if not lr_init > lr_end:
        raise ValueError(f"lr_end ({lr_end}) must be smaller than initial lr ({lr_init})")

    def f(step: int) -> float:
        if step < num_warmup_steps:
            return float(step) / float(max(1, num_warmup_steps))
        if step > num_training_steps:
            return lr_end / lr_init
        decay_steps = num_training_steps - num_warmup_steps
        pct_remaining = 1 - (step - num_warmup_steps) / decay_steps
        return (( lr_init - lr_end) * pct_remaining ** power + lr_end) / lr_init
    return f


def get_polynomial_decay_schedule_with_warmup(optimizer, num_warmup_steps: int, num_training_steps: int,
                                              lr_end: float = 1e-7, power: float = 1.0, last_epoch: int = -1):
    lr_init = optimizer.defaults["lr"]
    return torch.optim.lr_scheduler.LambdaLR(
        optimizer, polynomial_decay_lr_lambda(num_warmup_steps, num_training_steps, lr_init, lr_end, power), last_epoch)
