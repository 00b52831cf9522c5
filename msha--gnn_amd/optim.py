"""``Adam``: train.py's optimizer (train.py:207 ``optim.Adam(model.parameters(), lr,
weight_decay)``, stepped at :232) as one HIP launch over every parameter
(``msha_adam_step``, csrc/optim.hip).

Same update as ``torch.optim.Adam`` (L2 weight decay; no amsgrad / maximize), same
constructor and ``state_dict`` layout (``step``, ``exp_avg``, ``exp_avg_sq`` per
parameter; the moments in the parameter's dtype).  The step counts live on the device,
so a captured HIP graph (step.GraphedStep) replays the update with the right bias
corrections.

``fuse_dropout_grad(param)``: the parameter's only consumer is the models' feature
dropout (``Sfeatures``, Ablation.py:296 / Ours.py:161).  Its backward then hands the
dropout's OUTPUT gradient and mask seed to this optimizer instead of materialising the
parameter's gradient, and ``step()`` folds the mask into its gradient read: the 5M-float
gradient is never written or re-read, and every parameter still updates in ONE launch
at ``step()``.  The parameter's ``.grad`` stays None.  (One backward per step for a fused
parameter: a second backward before ``step()`` raises, as accumulation would need the
gradient this path never forms.)
"""
from __future__ import annotations

import ctypes
import weakref

import torch

from . import _lib

_DT = {torch.float32: 0, torch.bfloat16: 1}


class Adam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0,
                 amsgrad=False, *, maximize=False, foreach=None, capturable=True,
                 differentiable=False, fused=None):
        if amsgrad or maximize or differentiable:
            raise NotImplementedError("msha Adam: amsgrad / maximize / differentiable")
        if not 0.0 <= lr or not 0.0 <= eps or not 0.0 <= weight_decay:
            raise ValueError("msha Adam: lr, eps and weight_decay must be >= 0")
        if not (0.0 <= betas[0] < 1.0 and 0.0 <= betas[1] < 1.0):
            raise ValueError("msha Adam: betas must be in [0, 1)")
        # capturable / fused in the defaults: torch's load_state_dict then moves every
        # loaded 'step' to the parameter's device as fp32 (a CPU step from a
        # map_location='cpu' checkpoint or a torch.optim.Adam state_dict would otherwise
        # stay on the host, and the kernel reads it through a device pointer)
        super().__init__(params, dict(lr=lr, betas=tuple(betas), eps=eps,
                                      weight_decay=weight_decay, amsgrad=False,
                                      maximize=False, foreach=None, capturable=True,
                                      differentiable=False, fused=False))
        self._ws = {}  # device -> the launches' per-tensor scalars (stream-ordered reuse)

    def _workspace(self, dev):
        ws = self._ws.get(dev)
        if ws is None:
            nb = int(_lib.load().msha_adam_workspace_size())
            ws = self._ws[dev] = torch.zeros(nb, dtype=torch.uint8, device=dev)
        return ws

    def _state_of(self, p):
        st = self.state[p]
        if not st:
            st["step"] = torch.zeros((), dtype=torch.float32, device=p.device)
            st["exp_avg"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
            st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
            return st
        # state loaded from elsewhere: the kernel reads 'step' (fp32) and the moments (the
        # parameter's dtype, contiguous) through device pointers
        stp = st["step"]
        if not (torch.is_tensor(stp) and stp.device == p.device and stp.dtype == torch.float32
                and stp.numel() == 1):
            st["step"] = torch.as_tensor(float(stp), dtype=torch.float32,
                                         device=p.device).reshape(())
        for k in ("exp_avg", "exp_avg_sq"):
            m = st[k]
            if m.device != p.device or m.dtype != p.dtype or not m.is_contiguous():
                st[k] = m.to(device=p.device, dtype=p.dtype).contiguous()
        return st

    def _group_of(self, p):
        for g in self.param_groups:
            if any(q is p for q in g["params"]):
                return g
        raise ValueError("parameter is not in this optimizer")

    @staticmethod
    def _check(p, g):
        _lib.require_cuda(p, g)
        if p.dtype not in _DT or g.dtype != p.dtype:
            raise TypeError(f"msha Adam: fp32 / bf16 parameters with same-dtype gradients "
                            f"(got {p.dtype} / {g.dtype})")
        if not (p.is_contiguous() and g.is_contiguous()):
            raise ValueError("msha Adam: contiguous parameters and gradients")

    def _desc(self, p, grad, drop_p=0.0, drop_seed=0):
        st = self._state_of(p)
        d = _lib.MshaAdamTensor()
        d.param, d.grad = p.data_ptr(), grad.data_ptr()
        d.exp_avg, d.exp_avg_sq = st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr()
        d.step, d.n, d.dtype = st["step"].data_ptr(), p.numel(), _DT[p.dtype]
        d.drop_p, d.drop_seed, d.drop_offset = float(drop_p), int(drop_seed), 0
        return d

    def _launch(self, group, descs, dev):
        b1, b2 = group["betas"]
        for lo in range(0, len(descs), _lib.MAX_ADAM):
            part = descs[lo:lo + _lib.MAX_ADAM]
            arr = (_lib.MshaAdamTensor * len(part))(*part)
            _lib.call("msha_adam_step", len(part), ctypes.byref(arr), float(group["lr"]),
                      float(b1), float(b2), float(group["eps"]), float(group["weight_decay"]),
                      self._workspace(dev).data_ptr(), _lib.stream_handle(dev))

    def _check_groups(self):
        # a loaded torch.optim.Adam state_dict may carry flags this kernel does not run
        for g in self.param_groups:
            bad = [k for k in ("amsgrad", "maximize", "differentiable") if g.get(k)]
            if bad:
                raise NotImplementedError(f"msha Adam: {', '.join(bad)} set in a parameter "
                                          "group (loaded state_dict?)")

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        self._check_groups()

    @torch.no_grad()
    def step(self, closure=None):
        self._check_groups()
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            by_dev = {}
            for p in group["params"]:
                stash = getattr(p, "_msha_dropout_grad", None)
                if stash is not None:  # fused: the dropout's output gradient + its mask
                    if p.grad is not None:
                        # a second consumer of the fused parameter put a gradient in .grad:
                        # the fused update would silently drop it
                        raise RuntimeError(
                            "msha Adam: a fuse_dropout_grad parameter also has a .grad (it has "
                            "another consumer besides its feature dropout): do not fuse it")
                    dout, drop_p, seed = stash
                    p._msha_dropout_grad = None
                    self._check(p, dout)
                    by_dev.setdefault(p.device, []).append(self._desc(p, dout, drop_p, seed))
                    continue
                if p.grad is None:
                    continue
                g = p.grad
                if g.is_sparse:
                    raise NotImplementedError("msha Adam: sparse gradients")
                self._check(p, g)
                by_dev.setdefault(p.device, []).append(self._desc(p, g))
            for dev, descs in by_dev.items():
                self._launch(group, descs, dev)
        return loss

    def zero_grad(self, set_to_none: bool = True):
        super().zero_grad(set_to_none)
        for group in self.param_groups:
            for p in group["params"]:
                if getattr(p, "_msha_dropout_grad", None) is not None:
                    p._msha_dropout_grad = None

    # ---------------------------------------------- fused dropout-backward updates
    def fuse_dropout_grad(self, param):
        """Update ``param`` inside its feature dropout's backward (functional.feature_dropout
        checks for this registration); returns ``param``."""
        self._group_of(param)  # must be ours
        param._msha_fused_adam = weakref.ref(self)
        return param

    def stash_dropout_grad(self, param, dout, p: float, seed: int):
        """Called from the feature dropout's backward: keep the dropout's output gradient
        ``dout`` and its mask (p, seed) for ``step()`` in place of ``param.grad``."""
        if getattr(param, "_msha_dropout_grad", None) is not None:
            raise RuntimeError("msha Adam: a fused parameter got a second backward before "
                               "step(); gradient accumulation needs its .grad (do not fuse)")
        dout = dout.contiguous()
        self._check(param, dout)
        param._msha_dropout_grad = (dout, float(p), int(seed))


def fused_optimizer_of(param):
    """The msha Adam registered by ``fuse_dropout_grad`` for ``param`` (or None)."""
    ref = getattr(param, "_msha_fused_adam", None)
    return ref() if ref is not None else None
