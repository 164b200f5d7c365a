"""CPU tests of the host-side product pieces around the kernels:

  * the dataset packer (precomputed tpch.py:135-206 per template) vs the oracle's per-job preprocessing;
  * the host reset sampler (tpch.py:54-73 RNG consumption) vs the oracle's job_sequence;
  * the C-ABI library (in-tree gfx950 build) loads and exports every symbol include/sparksched.h declares
    (no compute call: there is no GPU in the CPU suite).
"""

import copy
import os
import re

import numpy as np
import pytest

from oracle import restatement as R
from spark_sched_sim._abi import DATASET_ARRAYS, SsimDataset, SsimLayout
from spark_sched_sim.data_samplers import job_sequence as js
from spark_sched_sim.data_samplers.synthetic_tpch import EXEC_LEVELS, QUERY_SIZES
from spark_sched_sim.data_samplers.tpch_pack import pack

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WAVES = ("fresh_durations", "first_wave", "rest_wave")


def test_packer_matches_oracle_preprocessing(dataset):
    P = pack(dataset, 10)
    for tid in range(P.num_templates):
        q, size = tid // 7 + 1, QUERY_SIZES[tid % 7]
        adj, tds = dataset[(q, size)]
        base = int(P.tpl_stage_base[tid])
        assert int(P.tpl_stage_base[tid + 1]) - base == adj.shape[0]
        for sid in range(adj.shape[0]):
            ts = base + sid
            d = copy.deepcopy(tds[sid])
            k0 = next(iter(d["first_wave"]))
            nt = len(d["first_wave"][k0]) + len(d["rest_wave"][k0])
            R.preprocess_durations(d)
            assert int(P.ts_num_tasks[ts]) == nt
            assert P.ts_rough[ts] == R.rough_duration(d)  # bit-exact numpy pairwise mean
            mask = sum(1 << EXEC_LEVELS.index(k) for k in d["first_wave"])
            assert int(P.ts_fw_keymask[ts]) == mask
            assert EXEC_LEVELS[int(P.ts_fw_maxlevel[ts])] == max(d["first_wave"])
            for w, wave in enumerate(WAVES):
                for lvl, key in enumerate(EXEC_LEVELS):
                    i = (ts * 3 + w) * 8 + lvl
                    if key not in d[wave]:
                        assert P.dur_len[i] == -1
                    else:
                        o, n = int(P.dur_off[i]), int(P.dur_len[i])
                        assert n == len(d[wave][key])
                        assert np.array_equal(P.durations[o: o + n], np.asarray(d[wave][key], dtype=np.float64))
            kids = list(P.ts_children[P.ts_child_base[ts]: P.ts_child_base[ts + 1]])
            pars = sorted(P.ts_parents[P.ts_parent_base[ts]: P.ts_parent_base[ts + 1]])
            assert kids == list(np.nonzero(adj[sid])[0])
            assert pars == list(np.nonzero(adj[:, sid])[0])


@pytest.mark.parametrize("seed", [0, 1234, 77])
@pytest.mark.parametrize("cap,limit", [(50, np.inf), (200, np.inf), (None, 3e6), (200, 2e6)])
def test_reset_sampler_matches_oracle_job_sequence(dataset, seed, cap, limit):
    cfg = dict(num_executors=10, job_arrival_cap=cap, job_arrival_rate=4e-5, warmup_delay=1000.0)
    s = R.TpchSamplerOracle(cfg, dataset)
    s.rng = js.make_rng(seed)
    ref = s.job_sequence(limit)
    rng = js.make_rng(seed)
    tpl, arr = js.sample_jobs(rng, cap, 4e-5, limit)
    assert len(tpl) == len(ref)
    for (t, job), tid, a in zip(ref, tpl, arr):
        assert float(t) == a
        assert tid == (job.query - 1) * 7 + QUERY_SIZES.index(job.size)
    assert rng.bit_generator.state == s.rng.bit_generator.state


def _declared_functions():
    src = open(os.path.join(REPO, "include", "sparksched.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ssim_[a-z0-9_]+)\s*\(", src)))


def test_c_abi_library_exports_every_declared_symbol():
    import ctypes

    from spark_sched_sim import native

    if not os.path.exists(native.LIB_PATH):
        import __graft_entry__

        __graft_entry__.build_lib()
    lib = ctypes.CDLL(native.LIB_PATH)
    names = _declared_functions()
    assert "ssim_step" in names and "ssim_reset" in names and len(names) >= 9
    for n in names:
        assert hasattr(lib, n), f"{n} not exported"
    assert set(names) == set(native.EXPORTED_SYMBOLS)


def test_layout_structs_match_header():
    import ctypes

    from spark_sched_sim import native

    lib = native.lib()
    from spark_sched_sim._abi import SsimConfig

    cfg = SsimConfig(num_envs=3, num_executors=10, job_cap=50, max_stages=18, max_edges=20, trace_cap=7,
                     moving_delay=2000.0, warmup_delay=1000.0, beta=0.0)
    L = SsimLayout()
    assert lib.ssim_layout_for(ctypes.byref(cfg), ctypes.byref(L)) == 0
    assert (L.num_envs, L.num_executors, L.job_cap, L.stage_cap) == (3, 10, 50, 900)
    assert L.set_cap == 64  # smallest power of two > 4N
    offs = [L.ob_nodes, L.ob_edge_links, L.ob_dag_ptr, L.ob_supplies, L.ob_frontier, L.ob_sched_rank,
            L.ob_counts, L.ob_reward, L.ob_wall_time, L.ob_acc, L.ob_trace]
    assert offs == sorted(offs) and all(o % 16 == 0 for o in offs) and L.obs_bytes >= offs[-1]
    assert len(SsimDataset._fields_) == 2 + len(DATASET_ARRAYS)
    # the bench shape (BASELINE configs[1]) runs its 1024 single-wave workgroups one per SIMD: four envs' LDS (hot
    # block + scratch) must fit a CU's 160 KB, or a quarter of the batch waits for a second round
    assert L.lds_resident == 1 and 4 * L.lds_bytes <= 160 * 1024, L.lds_bytes
    # HBM-resident shapes run 4 one-wave workgroups per SIMD: 16 per CU must share its LDS. With the LDS copy of the
    # executor records (sc_execs, 32 B per executor) neither J=200 shard fits the stage->row map too: configs[3]'s
    # (N=100) and configs[2]'s (N=50) keep it in the cold block.
    for n_exec, row_map_in_lds in ((100, False), (50, False)):
        big = SsimConfig(num_envs=4096, num_executors=n_exec, job_cap=200, max_stages=18, max_edges=20,
                         moving_delay=2000.0, warmup_delay=1000.0, beta=0.0)
        assert lib.ssim_layout_for(ctypes.byref(big), ctypes.byref(L)) == 0
        assert L.lds_resident == 0 and 16 * L.lds_bytes <= 160 * 1024, (n_exec, L.lds_bytes)
        assert (L.lds_bytes == L.scratch_bytes) == row_map_in_lds, (n_exec, L.lds_bytes, L.scratch_bytes)
    # batches past 1.5x the LDS-resident kernel's concurrency (4 configs[1] envs per CU, 1024 on the chip) run on
    # the 4-wave HBM-resident kernels (layout.h lds_concurrent_envs)
    # (thresholds from the CU count the library reports: a partitioned device has fewer than the MI355X's 256)
    cfg.num_envs = 1
    assert lib.ssim_layout_for(ctypes.byref(cfg), ctypes.byref(L)) == 0
    cus = int(L.chip_cus)
    assert cus > 0
    conc = 4 * cus  # 4 configs[1] envs per CU
    for envs, resident in ((conc, 1), (conc * 3 // 2, 1), (conc * 3 // 2 + 1, 0), (4 * conc, 0)):
        cfg.num_envs = envs
        assert lib.ssim_layout_for(ctypes.byref(cfg), ctypes.byref(L)) == 0
        assert L.lds_resident == resident, (envs, L.lds_resident)
        if not resident:
            assert 16 * L.lds_bytes <= 160 * 1024, L.lds_bytes
            assert L.lds_share == 160 * 1024 // 16
        else:  # 4 envs per CU: each may hold a quarter of the CU's LDS
            assert L.lds_share == 160 * 1024 // 4 and L.lds_bytes <= L.lds_share
    # at most one env per CU: the whole CU
    cfg.num_envs = cus
    assert lib.ssim_layout_for(ctypes.byref(cfg), ctypes.byref(L)) == 0
    assert L.lds_resident == 1 and L.lds_share == 160 * 1024
    cfg.num_executors = 0
    assert lib.ssim_layout_for(ctypes.byref(cfg), ctypes.byref(L)) != 0


def test_topology_bit_sets_match_csr(dataset):
    """ts_topo (parents in bits 0-31, children in bits 32-63 of each template stage) holds exactly the CSR's DAG."""
    from spark_sched_sim.data_samplers.tpch_pack import pack

    p = pack(dataset, 10)
    assert p.max_stages <= 32 and p.ts_topo.dtype == np.uint64 and p.ts_topo.shape == (p.num_template_stages,)
    for ts in range(p.num_template_stages):
        par = p.ts_parents[p.ts_parent_base[ts]: p.ts_parent_base[ts + 1]]
        kid = p.ts_children[p.ts_child_base[ts]: p.ts_child_base[ts + 1]]
        w = int(p.ts_topo[ts])
        assert [b for b in range(32) if (w >> b) & 1] == sorted(par.tolist())
        assert [b for b in range(32) if (w >> (32 + b)) & 1] == kid.tolist()  # CSR children are ascending
