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


# The shipped shape-specialised instantiations (ssim_debug_set_trace_ex runs the KAT through the engine template
# instantiation of the translation unit a launch on the handle selects, compiled there with that unit's flags): the
# configs[1] LDS-resident kernel (stage cap 900), its HBM-resident form for large batches, the configs[2] / [4] engine
# and Decima rollout units (N = 50) and the configs[3] unit (N = 100), where round 4's ROCm i64 miscompile hid from the
# generic kernel. (executors, job cap, config flags, variant, expected unit, traces, ops per trace)
_HBM, _ENG, _DEC = 1, 0, 1  # _abi.SSIM_CFG_FORCE_HBM, SSIM_DEBUG_ENGINE, SSIM_DEBUG_DECIMA
SHIPPED = [(10, 50, 0, _ENG, "bench900", 8, 400), (10, 50, _HBM, _ENG, "hbm_n10", 8, 400),
           (50, 200, _HBM, _ENG, "hbm_n50", 10, 600), (50, 200, _HBM, _DEC, "dr_hbm50", 10, 600),
           (100, 200, _HBM, _ENG, "hbm_n100", 12, 900), (50, 200, 0, _DEC, "dr_lds50", 10, 600)]


def _run_traces(eng, n_exec, traces, n_ops, variant, stop_at_first=False):
    """Runs `traces` random traces through `variant`; returns the mismatches (trace, op, device, CPython)."""
    import torch

    from spark_sched_sim import native

    width, bad = n_exec + 1, []
    for t in range(traces):
        rng = np.random.default_rng([n_exec, t])
        ops = random_ops(rng, n_exec, n_ops)
        want = cpython_orders(ops)
        dev_ops = torch.from_numpy(encode(ops, n_exec)).to(eng.device)
        orders = torch.full((len(ops), width), -2, dtype=torch.int32, device=eng.device)
        native.check(native.lib().ssim_debug_set_trace_ex(eng.handle, dev_ops.data_ptr(), len(ops), width,
                                                          orders.data_ptr(), variant, eng._stream()),
                     "ssim_debug_set_trace_ex")
        got = orders.cpu().numpy()
        for k, w in enumerate(want):
            row = got[k]
            g = row[row >= 0].tolist()
            if g != w:
                bad.append((t, k, g, w))
                if stop_at_first:
                    return bad
    return bad


@pytest.mark.gpu
@pytest.mark.parametrize("n_exec,traces,n_ops", CASES)
def test_device_sets_match_cpython(gpu_device, dataset, n_exec, traces, n_ops):
    """Small-batch layouts (job cap 2, one env): the generic LDS-resident unit."""
    from spark_sched_sim.engine import DeviceEngine

    cfg = dict(num_executors=n_exec, job_arrival_cap=2, job_arrival_rate=4.0e-5, moving_delay=2000.0,
               warmup_delay=1000.0)
    eng = DeviceEngine(cfg, 1, dataset, device=gpu_device)
    bad = _run_traces(eng, n_exec, traces, n_ops, _ENG, stop_at_first=True)
    assert not bad, f"N={n_exec} trace {bad[0][0]} op {bad[0][1]}: device {bad[0][2]} vs CPython {bad[0][3]}"
    eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize("n_exec,job_cap,flags,variant,unit,traces,n_ops", SHIPPED)
def test_shipped_instantiations_sets_match_cpython(gpu_device, dataset, n_exec, job_cap, flags, variant, unit, traces,
                                                   n_ops):
    from spark_sched_sim import native
    from spark_sched_sim.engine import DeviceEngine

    cfg = dict(num_executors=n_exec, job_arrival_cap=job_cap, job_arrival_rate=4.0e-5, moving_delay=2000.0,
               warmup_delay=1000.0)
    eng = DeviceEngine(cfg, 1, dataset, device=gpu_device, config_flags=flags)
    ran = native.lib().ssim_debug_kernel_name(eng.handle, variant).decode()
    assert ran == unit, f"the layout selects {ran!r}, expected the shipped unit {unit!r}"
    bad = _run_traces(eng, n_exec, traces, n_ops, variant, stop_at_first=True)
    assert not bad, f"{unit} N={n_exec} trace {bad[0][0]} op {bad[0][1]}: device {bad[0][2]} vs CPython {bad[0][3]}"
    eng.close()


@pytest.mark.gpu
def test_known_bad_page_assembly_fails_the_kat(gpu_device, dataset):
    """Regression guard: the N = 100 instantiation on a test-only wave type that reproduces round 4's miscompile
    (engine.h KatBadPage: a clean-insert table rebuilt with key 0 in slot 256) must fail the same KAT
    the shipped unit passes, so the KAT has the power to catch that class of error."""
    from spark_sched_sim import native
    from spark_sched_sim.engine import DeviceEngine

    cfg = dict(num_executors=100, job_arrival_cap=200, job_arrival_rate=4.0e-5, moving_delay=2000.0,
               warmup_delay=1000.0)
    eng = DeviceEngine(cfg, 1, dataset, device=gpu_device, config_flags=_HBM)
    assert native.lib().ssim_debug_kernel_name(eng.handle, 2).decode() == "kat_bad_page"
    bad = _run_traces(eng, 100, 4, 900, 2, stop_at_first=True)
    assert bad, "the known-bad page assembly passed the KAT: the KAT cannot see the miscompile it guards against"
    eng.close()

