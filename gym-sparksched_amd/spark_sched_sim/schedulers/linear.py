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


def _fns():
    global _FN
    if _FN is None:
        from .. import native

        L = native.lib()
        _FN = (L.ssim_linear_fwd, L.ssim_linear_wgrad_parts, L.ssim_linear_wgrad, native.check)
    return _FN


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
