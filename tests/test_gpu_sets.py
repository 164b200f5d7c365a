"""Known-answer tests of the device's CPython-set code against CPython itself (ssim_debug_set_trace).

The reference chooses executors by set iteration order (spark_sched_sim.py:714-743: set(gen) over pool.copy(), then
pop / list), over ExecutorTracker pools that see add / remove churn (executor_tracker.py:186-220), so the engine keeps
an exact model of each pool's CPython table. Random traces of add / remove / idle-order operations run on one pool
through the engine's own set code on the GPU and on real `set` objects of this interpreter (CPython 3.10, the
reference's), compared after every operation: the iteration order after an add or remove (= the table layout), and
the idle order. Executor counts cover each path the layout selects: one-page lane sets (<= 15 executors), paged
tables (16..127: 64 < capacity <= 512, configs[2]'s 50 and configs[3]'s 100) up to their largest table.
The CPU-suite half checks the trace generator and CPython reference against the serial host model (pyset.h)."""

import numpy as np
import pytest

# (executors, traces, ops per trace)
CASES = [(10, 12, 400), (16, 8, 400), (50, 12, 600), (100, 12, 900), (127, 6, 900)]


def random_ops(rng, n_exec: int, n_ops: int):
    """Phases that fill a pool (tables grow to their largest size), churn it (dummies, off-home keys via the
    last-dummy rule) and drain it, with idle-order queries under random busy masks throughout."""
    s, ops = set(), []
    phases = [0.95, 0.6, 0.2, 0.75, 0.5, 0.05, 0.8]
    for k in range(n_ops):
        p_add = phases[(k * len(phases)) // n_ops]
        r = rng.random()
        if r < 0.12:
            busy = rng.random(n_exec) < rng.choice([0.0, 0.3, 0.7, 0.95])
            ops.append((2, 0, busy))
        elif not s or rng.random() < p_add:
            out = [e for e in range(n_exec) if e not in s]
            key = int(rng.choice(out)) if out and rng.random() < 0.85 else int(rng.integers(n_exec))
            ops.append((0, key, None))
            s.add(key)
        else:
            key = int(rng.choice(sorted(s)))
            ops.append((1, key, None))
            s.discard(key)
    return ops


def cpython_orders(ops):
    s, out = set(), []
    for code, key, busy in ops:
        if code == 0:
            s.add(key)
            out.append(list(s))
        elif code == 1:
            s.remove(key)
            out.append(list(s))
        else:  # _get_idle_source_executors (spark_sched_sim.py:714-728) over get_pool's copy()
            out.append(list(set(e for e in s.copy() if not busy[e])))
    return out


def encode(ops, n_exec: int) -> np.ndarray:
    a = np.zeros((len(ops), 6), dtype=np.int32)
    for i, (code, key, busy) in enumerate(ops):
        a[i, 0], a[i, 1] = code, key
        if busy is not None:
            words = np.zeros(4, dtype=np.uint32)
            for e in np.flatnonzero(busy):
                words[e >> 5] |= np.uint32(1 << (int(e) & 31))
            a[i, 2:6] = words.view(np.int32)
    return a


def test_trace_encoding_round_trip():
    rng = np.random.default_rng(3)
    ops = random_ops(rng, 100, 300)
    enc = encode(ops, 100)
    for (code, key, busy), row in zip(ops, enc):
        assert row[0] == code and row[1] == key
        if busy is not None:
            words = row[2:6].view(np.uint32)
            got = [(int(words[e >> 5]) >> (e & 31)) & 1 for e in range(100)]
            assert got == busy.astype(int).tolist()


def test_cpython_reference_grows_and_churns_tables():
    """The traces reach the table sizes the paged path must handle (sets of 77+ keys: 512 slots) and mix removals
    in (dummies), so the GPU comparison covers resizes, dummy reuse and every copy / set(gen) regime."""
    rng = np.random.default_rng(0)
    ops = random_ops(rng, 100, 900)
    sizes, s = [], set()
    for code, key, _ in ops:
        if code == 0:
            s.add(key)
        elif code == 1:
            s.remove(key)
        sizes.append(len(s))
    assert max(sizes) >= 77 and sum(1 for c, _, _ in ops if c == 1) > 200 and sum(1 for c, _, _ in ops if c == 2) > 50


@pytest.mark.gpu
@pytest.mark.parametrize("n_exec,traces,n_ops", CASES)
def test_device_sets_match_cpython(gpu_device, dataset, n_exec, traces, n_ops):
    import torch

    from spark_sched_sim import native
    from spark_sched_sim.engine import DeviceEngine

    cfg = dict(num_executors=n_exec, job_arrival_cap=2, job_arrival_rate=4.0e-5, moving_delay=2000.0,
               warmup_delay=1000.0)
    eng = DeviceEngine(cfg, 1, dataset, device=gpu_device)
    width = n_exec + 1
    for t in range(traces):
        rng = np.random.default_rng([n_exec, t])
        ops = random_ops(rng, n_exec, n_ops)
        want = cpython_orders(ops)
        dev_ops = torch.from_numpy(encode(ops, n_exec)).to(eng.device)
        orders = torch.full((len(ops), width), -2, dtype=torch.int32, device=eng.device)
        native.check(native.lib().ssim_debug_set_trace(eng.handle, dev_ops.data_ptr(), len(ops), width,
                                                       orders.data_ptr(), eng._stream()), "ssim_debug_set_trace")
        got = orders.cpu().numpy()
        for k, w in enumerate(want):
            row = got[k]
            g = row[row >= 0].tolist()
            assert g == w, (f"N={n_exec} trace {t} op {k} {ops[k][:2]}: device {g} vs CPython {w}")
    eng.close()
