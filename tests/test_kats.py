"""Known-answer tests pinning the third-party arithmetic the reference depends on:

  * numpy Generator(PCG64) stream consumption (Appendix C): the device model (csrc/pcg64.h, exercised
    through the test-only host build) vs real numpy for mixed random()/integers()/choice() sequences.
  * CPython 3.10 set iteration/pop order (Appendix B): the device model (csrc/pyset.h) vs real `set`
    over random add/remove/copy/set(gen)/pop traces.
  * choice(<7 sizes>) consumes the stream exactly like integers(0, 7) (used by the host reset sampler).
  * executor_intervals (tpch.py:237-262): product table vs the oracle's restatement.
"""

import random

import numpy as np
import pytest

from hostsim.driver import lib
from oracle import restatement as R
from spark_sched_sim.data_samplers.tpch_pack import executor_intervals

QUERY_SIZES = ["2g", "5g", "10g", "20g", "50g", "80g", "100g"]


def _words(rng):
    st = rng.bit_generator.state
    s, inc = st["state"]["state"], st["state"]["inc"]
    m = (1 << 64) - 1
    return np.array([s >> 64, s & m, inc >> 64, inc & m, st["has_uint32"], st["uinteger"]], dtype=np.uint64)


@pytest.mark.parametrize("seed", [0, 1, 1234, 2**31 - 1, 98765432101])
def test_pcg64_model_matches_numpy(seed):
    rs = random.Random(seed)
    rng = np.random.Generator(np.random.PCG64(np.random.SeedSequence(seed)))
    # advance a little with reset-style draws so the buffered uint32 state is exercised
    for _ in range(rs.randrange(0, 5)):
        rng.integers(22)
    ops, ref = [], []
    w = _words(rng)
    for _ in range(5000):
        r = rs.random()
        if r < 0.35:
            ops.append(0)
            ref.append(rng.random())
        elif r < 0.7:
            n = rs.choice([1, 2, 3, 5, 7, 22, 64, 1000, 65537, 2**31 - 19])
            ops.append(n)
            ref.append(float(rng.choice(n) if rs.random() < 0.5 else rng.integers(0, n)))
        else:
            n = rs.randrange(1, 40)
            lst = [float(x) for x in range(n)]
            ops.append(n)
            ref.append(float(rng.choice(lst)))
    out = np.zeros(len(ops))
    ops_a = np.asarray(ops, dtype=np.int64)
    assert ops_a.max() < 2**31, "op codes are int32 lengths"
    ops32 = ops_a.astype(np.int32)
    lib().hs_pcg_run(w.ctypes.data, ops32.ctypes.data, len(ops), out.ctypes.data)
    assert np.array_equal(out, np.asarray(ref, dtype=np.float64))
    assert list(map(int, w)) == list(map(int, _words(rng)))


def test_choice_of_sizes_consumes_like_integers():
    for seed in range(50):
        a, b = (np.random.Generator(np.random.PCG64(np.random.SeedSequence(seed))) for _ in range(2))
        for _ in range(30):
            assert a.integers(22) == b.integers(22)
            assert QUERY_SIZES.index(str(a.choice(QUERY_SIZES))) == b.integers(0, 7)
            assert a.exponential(25000.0) == b.exponential(25000.0)
        assert a.bit_generator.state == b.bit_generator.state


def _real_trace(ops):
    s, orders = set(), []
    for code, key in ops:
        if code == 0:
            s.add(key)
        elif code == 1:
            s.remove(key)
        elif code == 2:
            s = s.copy()
        elif code == 3:
            s = set(x for x in s if (key >> (x % 31)) & 1)
        elif code == 4:
            s.pop()
        orders.append(list(s))
    return orders


@pytest.mark.parametrize("n_keys", [4, 10, 50, 100, 250])
def test_pyset_model_matches_cpython(n_keys):
    rs = random.Random(n_keys)
    for trial in range(150):
        ops, live = [], set()
        for _ in range(rs.randrange(1, 250)):
            r = rs.random()
            if r < 0.45 or not live:
                k = rs.randrange(n_keys)
                ops.append((0, k))
                live.add(k)
            elif r < 0.8:
                k = rs.choice(sorted(live))
                ops.append((1, k))
                live.discard(k)
            elif r < 0.88:
                ops.append((2, 0))
            elif r < 0.95:
                mask = rs.getrandbits(31)
                ops.append((3, mask))
                live = set(x for x in live if (mask >> (x % 31)) & 1)
            else:
                ops.append((4, 0))
                live = None  # recomputed below from the real set
            if live is None:
                live = set(_real_trace(ops)[-1])
        ref = _real_trace(ops)
        width = 256
        flat = np.asarray(ops, dtype=np.int32).reshape(-1)
        out = np.full((len(ops), width), -1, dtype=np.int32)
        rc = lib().hs_pyset_trace(flat.ctypes.data, len(ops), width, out.ctypes.data)
        assert rc == 0
        for k, order in enumerate(ref):
            got = [x for x in out[k] if x >= 0]
            assert got == order, f"trial {trial} op {k} {ops[k]}"


@pytest.mark.parametrize("n", [1, 3, 5, 7, 10, 16, 50, 64, 99, 100, 150])
def test_executor_intervals_match_oracle(n):
    assert np.array_equal(executor_intervals(n), R.executor_intervals(n))


@pytest.mark.parametrize("seeds", [list(range(64)), [2**32 - 1, 2**32, 2**40 + 7, 2**63 + 5, 98765432101]])
def test_seedsequence_pcg64_seeding(seeds):
    """Pcg64::from_seed == Generator(PCG64(SeedSequence(seed))) (gymnasium reset(seed), spark_sched_sim.py:130)."""
    out = np.zeros(4, dtype=np.uint64)
    for s in seeds:
        lib().hs_seed_words(s, out.ctypes.data)
        st = np.random.PCG64(np.random.SeedSequence(s)).state["state"]
        m = (1 << 64) - 1
        assert [int(x) for x in out] == [st["state"] >> 64, st["state"] & m, st["inc"] >> 64, st["inc"] & m], s


@pytest.mark.parametrize("seed,pre", [(3, 0), (2024, 1), (77, 3)])
def test_std_exponential_matches_numpy(seed, pre):
    """Pcg64::std_exponential (ziggurat tables from csrc/ziggurat.h, tail via fd_log1p) == numpy's
    Generator.standard_exponential over 300k draws, after `pre` integers() so the buffered uint32 is live."""
    rng = np.random.Generator(np.random.PCG64(seed))
    for _ in range(pre):
        rng.integers(22)
    w = _words(rng)
    n = 300000
    got = np.zeros(n)
    lib().hs_std_exponential(w.ctypes.data, n, got.ctypes.data)
    ref = rng.standard_exponential(n)
    assert np.array_equal(got.view(np.uint64), ref.view(np.uint64))
    assert (int(w[0]) << 64 | int(w[1])) == rng.bit_generator.state["state"]["state"]


def test_log1p_matches_libm():
    """fd_log1p (csrc/fdlibm.h) == the host libm's log1p numpy calls, on the ziggurat tail's inputs
    x = -u, u a 53-bit uniform, plus small-|x| and branch-boundary inputs."""
    import math

    rs = np.random.default_rng(5)
    u = rs.integers(0, 2**53, size=400000, dtype=np.int64).astype(np.float64) * (1.0 / 9007199254740992.0)
    small = np.ldexp(u[:50000], -rs.integers(1, 60, size=50000))
    edge = -(float.fromhex("-0x1.2bec4p-2") + np.ldexp(rs.integers(-10**6, 10**6, size=50000).astype(np.float64), -60))
    x = np.concatenate([-u, -small, -edge, [-0.0, 0.0, -0.5, -1e-300, -(1 - 2**-53)]])
    got = np.zeros_like(x)
    lib().hs_log1p(x.ctypes.data, len(x), got.ctypes.data)
    ref = np.array([math.log1p(v) for v in x])
    assert np.array_equal(got.view(np.uint64), ref.view(np.uint64))
