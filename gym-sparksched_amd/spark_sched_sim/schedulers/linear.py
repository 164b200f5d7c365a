"""nn.Linear for the Decima MLPs whose device forward and backward run on the library's small-layer kernels
(csrc/k_linear.hip: widths <= 64). The PPO learner evaluates ~200 such layers per minibatch over 1e5..3e5 node rows;
through hipBLASLt each GEMM cost ~70 us of host time and the tall-skinny weight gradients ran on a few workgroups
(DESIGN.md §9). Same parameters and state_dict as nn.Linear (reference: schedulers/decima/utils.py:51-70); CPU
tensors take torch's own F.linear (the CPU learner and tests), device tensors always take the kernels (no silent
fallback: a missing library raises)."""

from __future__ import annotations

import torch
import torch.nn.functional as F
from torch import nn

_MAX = 64


_FN = None  # (fwd, wgrad_parts, wgrad, check): bound once (each learner pass makes ~6k calls)
_MLP = None  # (supported, fwd, parts, partial_floats, bwd, check)


def _fns():
    global _FN
    if _FN is None:
        from .. import native

        L = native.lib()
        _FN = (L.ssim_linear_fwd, L.ssim_linear_wgrad_parts, L.ssim_linear_wgrad, native.check)
    return _FN


def _mlp_fns():
    global _MLP
    if _MLP is None:
        from .. import native

        L = native.lib()
        _MLP = (L.ssim_mlp3_supported, L.ssim_mlp3_fwd, L.ssim_mlp3_parts, L.ssim_mlp3_partial_floats,
                L.ssim_mlp3_bwd, native.check)
    return _MLP


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None):
        fwd, _, _, check = _fns()
        x = x.contiguous()
        w = w.contiguous()
        rows, k = x.shape
        n = w.shape[0]
        y = torch.empty((rows, n), dtype=torch.float32, device=x.device)
        check(fwd(x.data_ptr(), w.data_ptr(), None if b is None else b.data_ptr(), y.data_ptr(), rows, k, n, 1,
                  _stream(x)), "ssim_linear_fwd")
        ctx.save_for_backward(x, w)
        ctx.has_bias = b is not None
        return y

    @staticmethod
    def backward(ctx, gy: torch.Tensor):
        fwd, wgrad_parts, wgrad, check = _fns()
        x, w = ctx.saved_tensors
        gy = gy.contiguous()
        rows, k = x.shape
        n = w.shape[0]
        s = _stream(gy)
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            gx = torch.empty((rows, k), dtype=torch.float32, device=gy.device)
            check(fwd(gy.data_ptr(), w.data_ptr(), None, gx.data_ptr(), rows, n, k, 0, s),
                  "ssim_linear_fwd (input gradient)")
        if ctx.needs_input_grad[1] or (ctx.has_bias and ctx.needs_input_grad[2]):
            parts = int(wgrad_parts(rows))
            part = torch.empty((parts, n * (k + 1)), dtype=torch.float32, device=gy.device)
            gw = torch.empty((n, k), dtype=torch.float32, device=gy.device)
            gb = torch.empty((n,), dtype=torch.float32, device=gy.device) if ctx.has_bias else None
            check(wgrad(gy.data_ptr(), x.data_ptr(), gw.data_ptr(), None if gb is None else gb.data_ptr(), rows, k,
                        n, part.data_ptr(), parts, s), "ssim_linear_wgrad")
        return gx, gw, gb


class HipLinear(nn.Linear):
    """nn.Linear (same parameters); f32 device inputs of widths <= 64 run on csrc/k_linear.hip."""

    def _kernel_ok(self, x: torch.Tensor) -> bool:
        """The kernels read raw f32 pointers on x's device: anything else (CPU tensors, other dtypes, parameters on
        another device, widths > 64) takes F.linear, which raises torch's own errors for mismatches."""
        if not x.is_cuda or x.dtype != torch.float32 or self.in_features > _MAX or self.out_features > _MAX:
            return False
        w, b = self.weight, self.bias
        if w.dtype != torch.float32 or w.device != x.device:
            return False
        return b is None or (b.dtype == torch.float32 and b.device == x.device)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if not self._kernel_ok(x):
            return F.linear(x, self.weight, self.bias)
        lead = x.shape[:-1]
        with torch.cuda.device(x.device):
            y = _LinearFn.apply(x.reshape(-1, self.in_features), self.weight, self.bias)
        return y.reshape(*lead, self.out_features)


_ACTS = {nn.LeakyReLU: 0, nn.Tanh: 1}  # include/sparksched.h SSIM_ACT_*


def _ptr(t):
    return None if t is None else t.data_ptr()


def _mlp3_forward(x, params, grid_n: int, act: int, slope: float, keep: bool):
    _, fwd, _, _, _, check = _mlp_fns()
    x = x.contiguous()
    w0, b0, w1, b1, w2, b2 = params
    d1, d0 = w0.shape
    d2, d3 = w1.shape[0], w2.shape[0]
    rows = x.shape[0] * grid_n if grid_n else x.shape[0]
    dev = x.device
    h1 = torch.empty((rows, d1), dtype=torch.float32, device=dev) if keep else None
    h2 = torch.empty((rows, d2), dtype=torch.float32, device=dev) if keep else None
    y = torch.empty((rows, d3), dtype=torch.float32, device=dev)
    check(fwd(None if grid_n else x.data_ptr(), x.data_ptr() if grid_n else None, grid_n, w0.data_ptr(),
              b0.data_ptr(), w1.data_ptr(), b1.data_ptr(), w2.data_ptr(), b2.data_ptr(), _ptr(h1), _ptr(h2),
              y.data_ptr(), rows, d0, d1, d2, d3, act, slope, _stream(x)), "ssim_mlp3_fwd")
    return y, h1, h2


def _mlp3(x, params, grid_n: int, act: int, slope: float):
    """Autograd when a gradient can flow (the learner), else the forward alone without the hidden-row stores."""
    with torch.cuda.device(x.device):
        if torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in params)):
            return _Mlp3Fn.apply(x, *params, grid_n, act, slope)
        return _mlp3_forward(x, params, grid_n, act, slope, keep=False)[0]


class _Mlp3Fn(torch.autograd.Function):
    """The whole Linear-act-Linear-act-Linear chain (csrc/k_linear.hip ssim_mlp3_*). x: [rows, d0], or with grid_n > 0
    the exec-score grid's base rows [decisions, d0 - 1] (rows = decisions * grid_n, last input column = action / N)."""

    @staticmethod
    def forward(ctx, x, w0, b0, w1, b1, w2, b2, grid_n: int, act: int, slope: float):
        _, fwd, _, _, _, check = _mlp_fns()
        x = x.contiguous()
        d1, d0 = w0.shape
        d2, d3 = w1.shape[0], w2.shape[0]
        y, h1, h2 = _mlp3_forward(x, (w0, b0, w1, b1, w2, b2), grid_n, act, slope, keep=True)
        ctx.save_for_backward(x, w0, w1, w2, h1, h2)
        ctx.cfg = (grid_n, act, slope, y.shape[0])
        return y

    @staticmethod
    def backward(ctx, gy):
        _, _, parts_fn, floats_fn, bwd, check = _mlp_fns()
        x, w0, w1, w2, h1, h2 = ctx.saved_tensors
        grid_n, act, slope, rows = ctx.cfg
        gy = gy.contiguous()
        d1, d0 = w0.shape
        d2, d3 = w1.shape[0], w2.shape[0]
        dev = gy.device
        e = lambda *s: torch.empty(s, dtype=torch.float32, device=dev)  # noqa: E731
        g1, g2 = e(rows, d1), e(rows, d2)
        gx = e(*x.shape) if ctx.needs_input_grad[0] else None
        gw0, gb0, gw1, gb1, gw2, gb2 = e(d1, d0), e(d1), e(d2, d1), e(d2), e(d3, d2), e(d3)
        parts = int(parts_fn(rows))
        part = e(int(floats_fn(rows, d0, d1, d2, d3)))
        check(bwd(gy.data_ptr(), None if grid_n else x.data_ptr(), x.data_ptr() if grid_n else None, grid_n,
                  w0.data_ptr(), w1.data_ptr(), w2.data_ptr(), h1.data_ptr(), h2.data_ptr(), g1.data_ptr(),
                  g2.data_ptr(), _ptr(gx), gw0.data_ptr(), gb0.data_ptr(), gw1.data_ptr(), gb1.data_ptr(),
                  gw2.data_ptr(), gb2.data_ptr(), rows, d0, d1, d2, d3, act, slope, part.data_ptr(), parts,
                  _stream(gy)), "ssim_mlp3_bwd")
        return gx, gw0, gb0, gw1, gb1, gw2, gb2, None, None, None


class HipMlp3(nn.Sequential):
    """make_mlp's nn.Sequential (same modules, same state_dict keys 0.*, 2.*, 4.*) whose device forward runs the
    whole Linear-act-Linear-act-Linear chain as one fused kernel (1 forward + 4 backward launches instead of 5 + ~11)
    when its shape is one the library fuses (the decima_tpch.yaml GNN and score MLPs: ssim_mlp3_supported); anything
    else (CPU tensors, other widths or activations) runs the modules one by one."""

    def _fused(self, x: torch.Tensor, d0: int):
        if len(self) != 5 or not x.is_cuda or x.dtype != torch.float32:
            return None
        l0, a0, l1, a1, l2 = self
        act = _ACTS.get(type(a0))
        if act is None or type(a1) is not type(a0) or not all(isinstance(m, nn.Linear) for m in (l0, l1, l2)):
            return None
        slope = float(getattr(a0, "negative_slope", 0.0))
        if act == 0 and float(a1.negative_slope) != slope:
            return None
        params = [l0.weight, l0.bias, l1.weight, l1.bias, l2.weight, l2.bias]
        if any(p is None or p.dtype != torch.float32 or p.device != x.device for p in params):
            return None
        if l0.in_features != d0 or not _mlp_fns()[0](d0, l0.out_features, l1.out_features, l2.out_features, act):
            return None
        return params, act, slope

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        f = self._fused(x, x.shape[-1])
        if f is None:
            return super().forward(x)
        params, act, slope = f
        lead = x.shape[:-1]
        y = _mlp3(x.reshape(-1, x.shape[-1]), params, 0, act, slope)
        return y.reshape(*lead, y.shape[-1])

    def grid(self, base: torch.Tensor, n: int) -> torch.Tensor:
        """The MLP over every (base row k, action a < n) pair with input [base[k], a / n] (the exec-score grid,
        scheduler.py:355-367): [K * n, out]. Same values as self(cat([base expanded, arange(n) / n])) without
        materialising that [K * n, d0] input on the device."""
        K, db = base.shape
        f = self._fused(base, db + 1) if n > 0 and K > 0 else None
        if f is None:
            acts = torch.arange(n, device=base.device) / n
            inp = torch.cat([base[:, None, :].expand(K, n, db), acts[None, :, None].expand(K, n, 1)], dim=2)
            return super().forward(inp.reshape(K * n, db + 1))
        params, act, slope = f
        return _mlp3(base, params, n, act, slope)
