"""TEST INFRASTRUCTURE ONLY — numpy restatement of trainers/utils/returns_calculator.py (discounted and
differential returns, CircularArray) and trainers/utils/baselines.py (Baseline.average), the checker for the
device-tensor versions in spark_sched_sim/trainers/returns.py. Only tests/ may import it."""

from __future__ import annotations

from itertools import chain

import numpy as np


def discounted_returns(times_list, rewards_list, beta):
    """returns_calculator.py:53-62 (dt from consecutive wall times, :44)."""
    out = []
    for ts, rs in zip(times_list, rewards_list):
        dts = np.array(ts[1:]) - np.array(ts[:-1])
        ret = np.zeros(len(rs))
        R = 0
        for k, (dt, r) in reversed(list(enumerate(zip(dts, rs)))):
            R = r + np.exp(-beta * 1e-3 * dt) * R
            ret[k] = R
        out.append(ret)
    return out


class DifferentialReturns:
    """returns_calculator.py:5-20, 40-51, 64-89."""

    def __init__(self, cap):
        self.cap = cap
        self.data = np.zeros((cap, 2))
        self.avg_num_jobs = None

    def __call__(self, times_list, rewards_list):
        dt_list = [np.array(ts[1:]) - np.array(ts[:-1]) for ts in times_list]
        new = np.array(list(zip(chain(*dt_list), chain(*rewards_list))))
        new = new[new[:, 0] > 0]
        n = new.shape[0]
        if n > self.cap:
            new, n = new[-self.cap:], self.cap
        keep = self.cap - n
        if keep > 0:
            self.data[:keep] = self.data[-keep:]
        self.data[keep:] = new
        total_time, rew_sum = self.data.sum(0)
        self.avg_num_jobs = -rew_sum / total_time
        out = []
        for dts, rs in zip(dt_list, rewards_list):
            ret = np.zeros(len(rs))
            R = 0
            for k, (dt, r) in reversed(list(enumerate(zip(dts, rs)))):
                R = -(-r - dt * self.avg_num_jobs) + R
                ret[k] = R
            out.append(ret)
        return out


def baseline_average(ts_list, ys_list, num_sequences, num_rollouts):
    """baselines.py:12-43."""
    out = []
    for j in range(num_sequences):
        ts_l = ts_list[j * num_rollouts:(j + 1) * num_rollouts]
        ys_l = ys_list[j * num_rollouts:(j + 1) * num_rollouts]
        ts_unique = np.unique(np.hstack(ts_l))
        y_hats = np.vstack([np.interp(ts_unique, ts, ys) for ts, ys in zip(ts_l, ys_l)])
        base = {t: y.mean() for t, y in zip(ts_unique, y_hats.T)}
        out += [np.array([base[t] for t in ts]) for ts in ts_l]
    return out
