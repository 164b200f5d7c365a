"""Returns and baselines on device tensors (trainers/utils/returns_calculator.py, baselines.py).

Trajectories are padded rows: times [R, T+1] (wall time before each decision, then the final wall time),
rewards [R, T], lengths [R] (valid decisions per row).
"""

from __future__ import annotations

import torch


class ReturnsCalculator:
    """returns_calculator.py:23-89. `beta`: continuously discounted returns (R_k = r_k + exp(-beta 1e-3 dt_k)
    R_{k+1}); `buff_cap`: differential returns against a moving-average number of jobs."""

    def __init__(self, buff_cap: int | None = None, beta: float | None = None):
        assert bool(buff_cap) ^ bool(beta), "exactly one of `buff_cap` and `beta` must be specified"
        self.buff_cap, self.beta = buff_cap, beta
        self.avg_num_jobs = None
        self._buf = None  # [n, 2] (dt, reward) rows, most recent last (CircularArray, :5-20)

    def __call__(self, times: torch.Tensor, rewards: torch.Tensor, lengths: torch.Tensor) -> torch.Tensor:
        T = rewards.shape[1]
        valid = torch.arange(T, device=rewards.device)[None, :] < lengths[:, None]
        dt = torch.where(valid, times[:, 1:] - times[:, :-1], torch.zeros_like(rewards))
        r = torch.where(valid, rewards, torch.zeros_like(rewards))
        if self.beta:
            return self._discounted(dt, r)
        return self._differential(dt, r, valid)

    def _discounted(self, dt: torch.Tensor, r: torch.Tensor) -> torch.Tensor:
        # R_k = sum_{j>=k} r_j exp(-b (t_j - t_k)) with t_j - t_k = sum_{i=k}^{j-1} dt_i; the backward
        # recursion is evaluated exactly as the reference does, one step per column (vectorised over rows).
        decay = torch.exp(-self.beta * 1e-3 * dt)
        if r.is_cuda and r.dtype in (torch.float64, torch.float32) and decay.dtype == r.dtype:
            # the same recursion and roundings in one launch (csrc/k_linear.hip) instead of 3 launches per column
            from .. import native

            r, decay = r.contiguous(), decay.contiguous()
            out = torch.empty_like(r)
            with torch.cuda.device(r.device):
                native.check(native.lib().ssim_discounted_returns(
                    r.data_ptr(), decay.data_ptr(), out.data_ptr(), r.shape[0], r.shape[1],
                    int(r.dtype == torch.float64), torch.cuda.current_stream(r.device).cuda_stream),
                    "ssim_discounted_returns")
            return out
        out = torch.zeros_like(r)
        R = torch.zeros_like(r[:, 0])
        for k in range(r.shape[1] - 1, -1, -1):
            R = r[:, k] + decay[:, k] * R
            out[:, k] = R
        return out

    def _differential(self, dt: torch.Tensor, r: torch.Tensor, valid: torch.Tensor) -> torch.Tensor:
        new = torch.stack([dt[valid], r[valid]], dim=1)
        new = new[new[:, 0] > 0]  # filter zero-duration steps (:82)
        self._buf = new if self._buf is None else torch.cat([self._buf, new])
        self._buf = self._buf[-self.buff_cap:]
        total_time, rew_sum = self._buf.sum(0)
        self.avg_num_jobs = float(-rew_sum / total_time)
        step = -(-r - dt * self.avg_num_jobs)
        step = torch.where(valid, step, torch.zeros_like(step))
        return torch.flip(torch.cumsum(torch.flip(step, [1]), 1), [1])


def interp(x: torch.Tensor, xp: torch.Tensor, fp: torch.Tensor, n: torch.Tensor) -> torch.Tensor:
    """np.interp row-wise: x [R, M] at rows' (xp [R, T], fp [R, T], first n[r] points valid). With repeated xp
    values numpy lands on the last of the repeats (binary search of the last xp <= x), as here."""
    R, T = xp.shape
    big = torch.finfo(xp.dtype).max
    col = torch.arange(T, device=xp.device)[None, :]
    xpv = torch.where(col < n[:, None], xp, torch.full_like(xp, big))
    j = torch.searchsorted(xpv.contiguous(), x.contiguous(), right=True) - 1  # last index with xp <= x
    last = (n - 1)[:, None]
    jc = j.clamp(min=0)
    jc = torch.minimum(jc, last)
    j1 = torch.minimum(jc + 1, last)
    x0, x1 = torch.gather(xpv, 1, jc), torch.gather(xpv, 1, j1)
    f0, f1 = torch.gather(fp, 1, jc), torch.gather(fp, 1, j1)
    slope = torch.where(x1 > x0, (f1 - f0) / (x1 - x0), torch.zeros_like(f0))
    y = f0 + slope * (x - x0)
    y = torch.where(j < 0, fp[:, :1].expand_as(y), y)
    y = torch.where(j >= last, torch.gather(fp, 1, last.expand(R, 1)).expand_as(y), y)
    return y


class Baseline:
    """baselines.py:4-43: per job sequence, the mean over its rollouts of each rollout's returns linearly
    interpolated at the query time (np.interp semantics, clamped at the ends)."""

    def __init__(self, num_sequences: int, num_rollouts: int):
        self.num_sequences, self.num_rollouts = num_sequences, num_rollouts

    def __call__(self, times: torch.Tensor, returns: torch.Tensor, lengths: torch.Tensor) -> torch.Tensor:
        """times/returns [S*R, T] (rows of a sequence contiguous), lengths [S*R] -> baselines [S*R, T]."""
        Sq, Rr = self.num_sequences, self.num_rollouts
        T = times.shape[1]
        # every (sequence s, rollout r, curve r2) row at once: rollout r2's curve evaluated at rollout r's times
        # (interp is row-independent), then summed over r2 in the reference's order
        ts, ys, n = times.view(Sq, Rr, T), returns.view(Sq, Rr, T), lengths.view(Sq, Rr)
        q = ts[:, :, None, :].expand(Sq, Rr, Rr, T).reshape(-1, T)
        xp = ts[:, None, :, :].expand(Sq, Rr, Rr, T).reshape(-1, T)
        fp = ys[:, None, :, :].expand(Sq, Rr, Rr, T).reshape(-1, T)
        nn_ = n[:, None, :].expand(Sq, Rr, Rr).reshape(-1)
        v = interp(q, xp, fp, nn_).view(Sq, Rr, Rr, T)
        acc = torch.zeros_like(v[:, :, 0])
        for r2 in range(Rr):
            acc += v[:, :, r2]
        return (acc / Rr).reshape(Sq * Rr, T)
