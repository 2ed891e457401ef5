"""The rest of train.py's closure around the teacher-forced step (code_src/train.py:63,197-219; models/model_factory.py:71):
``CrossEntropyLoss`` on the packed scores and the ``Adam`` step, each one HIP launch chain through
the C-ABI (``aa_cross_entropy_*``, ``aa_adam_step`` in adaptive_amd/csrc/aa_optim.hip) instead of
PyTorch's per-op kernels (softmax + nll forward and backward; nine foreach passes for Adam).

Drop-ins with the same constructor arguments, numerics (torch's op order, fp32) and state layout:

    criterion = adaptive_amd.optim.CrossEntropyLoss()           # nn.CrossEntropyLoss()
    optimizer = adaptive_amd.optim.Adam(params, lr=cf.lr)       # torch.optim.Adam(..., betas, weight_decay)

``Adam.state_dict()`` has torch's keys (``step`` as a CPU float32 tensor, ``exp_avg``,
``exp_avg_sq``), so a checkpoint moves between the two optimizers.  There is no CPU fallback: CPU
tensors raise ``RuntimeError``.
"""
from __future__ import annotations

import torch

from . import _lib


def _require_hip(t: torch.Tensor, what: str) -> None:
    if not t.is_cuda:
        raise RuntimeError(f"adaptive_amd.optim: {what} must be a GPU tensor (the HIP kernels have no CPU path)")
    if t.dtype != torch.float32:
        raise TypeError(f"adaptive_amd.optim: {what} must be float32, got {t.dtype}")


class Adam(torch.optim.Optimizer):
    """torch.optim.Adam (model_factory.py:71: ``Adam(params, lr, betas, weight_decay)``) for fp32 GPU parameters:
    amsgrad=False, maximize=False, L2 ``weight_decay`` added to the gradient.  Every parameter with a
    gradient is updated by one ``aa_adam_step`` launch (per 24 tensors) in torch's foreach op order."""

    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0, amsgrad: bool = False):
        if not 0.0 <= lr:
            raise ValueError(f"Invalid learning rate: {lr}")
        if not 0.0 <= eps:
            raise ValueError(f"Invalid epsilon value: {eps}")
        if not 0.0 <= betas[0] < 1.0 or not 0.0 <= betas[1] < 1.0:
            raise ValueError(f"Invalid beta parameters: {betas}")
        if not 0.0 <= weight_decay:
            raise ValueError(f"Invalid weight_decay value: {weight_decay}")
        if amsgrad:
            raise NotImplementedError("adaptive_amd.optim.Adam: amsgrad is not supported (train.py does not use it)")
        super().__init__(params, dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay, amsgrad=False,
                                      maximize=False, foreach=None, capturable=False, differentiable=False,
                                      fused=None))
        self._tables = {}

    def zero_grad(self, set_to_none: bool = True) -> None:
        """torch.optim.Optimizer.zero_grad (train.py:204); set_to_none=True (the default) as one loop
        over the groups' parameters without the profiler scope, otherwise torch's own."""
        if not set_to_none:
            return super().zero_grad(set_to_none)
        for group in self.param_groups:
            for p in group["params"]:
                if p.grad is not None:
                    p.grad = None

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        lib = _lib.load()
        for gi, group in enumerate(self.param_groups):
            beta1, beta2 = group["betas"]
            live = [p for p in group["params"] if p.grad is not None]
            if not live:
                continue
            # the plan (validated parameters, their state, the launch tables) is reused while the
            # group's live parameters and the state dict are the same objects (load_state_dict replaces
            # the state dict: rebuilt); the gradients are new tensors every step (zero_grad sets them to
            # None and the caching allocator need not hand back the same blocks), so they are checked
            # and their pointers written into the tables on every step
            ident = (id(self.state), tuple(map(id, live)))
            plan = self._tables.get(gi)
            if plan is None or plan[0] != ident:
                plan = self._plan(live, ident)
                if len(self._tables) > 16:
                    self._tables.clear()
                self._tables[gi] = plan
            _, sbuf, calls, gslots = plan
            for p, (arr, i) in zip(live, gslots):
                g = p.grad
                if g.dtype is not torch.float32 or g.is_sparse or not g.is_cuda or not g.is_contiguous() \
                        or g.shape != p.shape or g.device != p.device:
                    self._check_grad(p)
                arr[i].grad = g.data_ptr()
            # the step counts, kept as torch.optim.Adam keeps them (a CPU float32 tensor per parameter),
            # are 0-d views of one buffer: one add per step (a foreach add over 21 CPU scalars cost ~70 us)
            sbuf.add_(1.0)
            for dev, first, arr, n in calls:
                step = float(sbuf[first].item())
                with _lib.on_device(dev):
                    rc = lib.aa_adam_step(arr, n, step, group["lr"], beta1, beta2, group["eps"],
                                          group["weight_decay"], _lib.stream_handle())
                _lib.check(rc, "adam_step")
        return loss

    def _plan(self, live, ident):
        """Validate the group's live parameters (a rejected tensor leaves no parameter with a step
        count for an update that never ran: torch's bias correction would drift), create missing
        state, move the step counts into one buffer (each parameter's state keeps its own 0-d CPU
        float32 ``step`` tensor, a view), and group the tensors that share a device and a step count
        into launch tables."""
        for p in live:
            self._check_grad(p)
        sbuf = torch.zeros(len(live), dtype=torch.float32)
        by_step = {}
        for i, p in enumerate(live):
            st = self.state[p]
            if len(st) == 0:
                st["step"] = torch.tensor(0.0, dtype=torch.float32)
                st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            v = float(st["step"].item())
            sbuf[i] = v
            st["step"] = sbuf[i]
            by_step.setdefault((p.device, v), []).append(
                (i, (p.data_ptr(), p.grad.data_ptr(), st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr(),
                     p.numel())))
        calls, gslots = [], [None] * len(live)
        for (dev, _), rows in by_step.items():
            arr = (_lib.AdamTensor * len(rows))(*[_lib.AdamTensor(*r) for _, r in rows])
            calls.append((dev, rows[0][0], arr, len(rows)))
            for j, (i, _) in enumerate(rows):
                gslots[i] = (arr, j)
        return ident, sbuf, calls, gslots

    @staticmethod
    def _check_grad(p):
        if p.grad.is_sparse:
            raise RuntimeError("adaptive_amd.optim.Adam does not support sparse gradients")
        _require_hip(p, "parameter")
        _require_hip(p.grad, "gradient")
        if not (p.is_contiguous() and p.grad.is_contiguous()):
            raise RuntimeError("adaptive_amd.optim.Adam: parameters and gradients must be contiguous")
        if p.grad.shape != p.shape or p.grad.device != p.device:
            raise RuntimeError("adaptive_amd.optim.Adam: a gradient's shape/device differs from its parameter's")


_clip_cache = {}


def clip_grad_norm_(parameters, max_norm: float, norm_type: float = 2.0, error_if_nonfinite: bool = False,
                    foreach=None) -> torch.Tensor:
    """torch.nn.utils.clip_grad_norm_ with the 2-norm (train.py:213-214: ``clip_grad_norm_(lstm params,
    cf.clip)``) for fp32 contiguous GPU gradients, as one ``aa_clip_grad_norm`` host call (three
    launches per 24 tensors): per-tensor norms, the total over them, every gradient scaled in place by
    ``min(max_norm / (total + 1e-6), 1)``.  Returns the total norm as a 0-d device tensor, as torch
    does.  Other norm types raise ``NotImplementedError``; CPU tensors raise ``RuntimeError``."""
    if isinstance(parameters, torch.Tensor):
        parameters = [parameters]
    grads = [p.grad for p in parameters if p.grad is not None]
    if float(norm_type) != 2.0:
        raise NotImplementedError("adaptive_amd.optim.clip_grad_norm_: only the 2-norm (train.py:213-214)")
    if not grads:
        return torch.tensor(0.0)
    dev = grads[0].device
    for g in grads:
        if g.dtype is not torch.float32 or g.is_sparse or not g.is_cuda or not g.is_contiguous() or g.device != dev:
            _require_hip(g, "gradient")
            if g.is_sparse or not g.is_contiguous() or g.device != dev:
                raise RuntimeError("adaptive_amd.optim.clip_grad_norm_: gradients must be dense, contiguous and "
                                   "on one device")
    lib = _lib.load()
    if len(grads) > _lib.CLIP_MAX_TENSORS:
        raise ValueError(f"adaptive_amd.optim.clip_grad_norm_: at most {_lib.CLIP_MAX_TENSORS} tensors")
    key = (dev, tuple(g.numel() for g in grads))
    ent = _clip_cache.get(key)
    if ent is None:
        arr = (_lib.GradTensor * len(grads))(*[_lib.GradTensor(None, g.numel()) for g in grads])
        nbytes = lib.aa_clip_grad_norm_workspace_bytes(arr, len(grads))
        if nbytes == 0:
            raise RuntimeError("adaptive_amd.optim.clip_grad_norm_: invalid gradient table")
        ent = (arr, nbytes)
        if len(_clip_cache) > 16:
            _clip_cache.clear()
        _clip_cache[key] = ent
    arr, nbytes = ent
    for i, g in enumerate(grads):
        arr[i].grad = g.data_ptr()
    # the workspace comes from the caching allocator on every call (stream-ordered: calls on
    # different streams never share one); the launch table is copied into the kernel arguments
    ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    total = torch.empty((), dtype=torch.float32, device=dev)
    with _lib.on_device(dev):
        rc = lib.aa_clip_grad_norm(arr, len(grads), float(max_norm), total.data_ptr(), ws.data_ptr(), ws.numel(),
                                   _lib.stream_handle())
    _lib.check(rc, "clip_grad_norm")
    if error_if_nonfinite and not bool(torch.isfinite(total)):
        raise RuntimeError(f"The total norm of order {float(norm_type)} for gradients from `parameters` is "
                           "non-finite, so it cannot be clipped.")
    return total


class _CrossEntropy(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, ignore_index):
        lib = _lib.load()
        N, V = logits.shape
        x = logits if logits.stride(1) == 1 else logits.contiguous()
        ws = torch.empty(lib.aa_cross_entropy_workspace_bytes(N), dtype=torch.uint8, device=x.device)
        loss = torch.empty((), dtype=torch.float32, device=x.device)
        count = torch.empty(1, dtype=torch.float32, device=x.device)
        with _lib.on_device(x.device):
            rc = lib.aa_cross_entropy_forward(x.data_ptr(), N, V, x.stride(0), target.data_ptr(), ignore_index,
                                              loss.data_ptr(), count.data_ptr(), ws.data_ptr(), ws.numel(),
                                              _lib.stream_handle())
        _lib.check(rc, "cross_entropy_forward")
        ctx.save_for_backward(x, target, ws, count)
        ctx.ignore_index = ignore_index
        return loss

    @staticmethod
    def backward(ctx, dloss):
        lib = _lib.load()
        x, target, ws, count = ctx.saved_tensors
        N, V = x.shape
        dloss = dloss.contiguous().float()
        dx = torch.empty(N, V, dtype=torch.float32, device=x.device)
        with _lib.on_device(x.device):
            rc = lib.aa_cross_entropy_backward(x.data_ptr(), N, V, x.stride(0), target.data_ptr(), ctx.ignore_index,
                                               dloss.data_ptr(), count.data_ptr(), ws.data_ptr(), ws.numel(),
                                               dx.data_ptr(), dx.stride(0), _lib.stream_handle())
        _lib.check(rc, "cross_entropy_backward")
        return dx, None, None


def cross_entropy(input: torch.Tensor, target: torch.Tensor, ignore_index: int = -100) -> torch.Tensor:
    """F.cross_entropy(input [N, C] fp32, target [N] class indices) with reduction 'mean' on the GPU:
    one read of the scores forward, one read + one write backward (aa_cross_entropy_*)."""
    _require_hip(input, "input")
    if input.dim() != 2:
        raise ValueError(f"adaptive_amd.optim.cross_entropy: input must be [N, C], got {tuple(input.shape)}")
    if target.dim() != 1 or target.size(0) != input.size(0):
        raise ValueError("adaptive_amd.optim.cross_entropy: target must be [N] class indices")
    if target.dtype != torch.int64:
        raise TypeError(f"adaptive_amd.optim.cross_entropy: target must be int64, got {target.dtype}")
    target = target.to(input.device).contiguous()
    if input.size(0) == 0:  # torch: mean over no rows is NaN
        return input.sum() * float("nan")
    return _CrossEntropy.apply(input, target, int(ignore_index))


class CrossEntropyLoss(torch.nn.Module):
    """nn.CrossEntropyLoss() (train.py:63) for [N, C] fp32 GPU scores and int64 targets; reduction
    'mean' with torch's ``ignore_index`` (weights and label smoothing are not used by the reference)."""

    def __init__(self, ignore_index: int = -100, reduction: str = "mean"):
        super().__init__()
        if reduction != "mean":
            raise NotImplementedError("adaptive_amd.optim.CrossEntropyLoss: only reduction='mean' (train.py:63)")
        self.ignore_index = ignore_index

    def forward(self, input, target):
        return cross_entropy(input, target, self.ignore_index)


__all__ = ["Adam", "CrossEntropyLoss", "clip_grad_norm_", "cross_entropy"]
