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
        out = torch.zeros_like(returns)
        for s in range(Sq):
            rows = slice(s * Rr, (s + 1) * Rr)
            ts, ys, n = times[rows], returns[rows], lengths[rows]
            acc = torch.zeros_like(ys)
            for r2 in range(Rr):  # evaluate rollout r2's curve at every rollout's own times
                acc += interp(ts, ts[r2:r2 + 1].expand(Rr, T), ys[r2:r2 + 1].expand(Rr, T), n[r2:r2 + 1].expand(Rr))
            out[rows] = acc / Rr
        return out
