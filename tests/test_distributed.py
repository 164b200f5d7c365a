"""Multi-rank path on CPU: world_size-2 `gloo` process group, the same sharding, timing
reduction and per-env statistics gather bench.py runs over RCCL (spark_sched_sim.distributed), each rank
stepping its own env block through the test-only host build of the engine."""

import multiprocessing as mp
import os
import socket
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CFG = dict(num_executors=10, job_arrival_cap=50, job_arrival_rate=4.0e-5, moving_delay=2000.0, warmup_delay=1000.0)
B_LOCAL, STEPS = 3, 40


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _local_run(rank):
    from hostsim.driver import HostEngine
    from spark_sched_sim import _abi
    from spark_sched_sim.data_samplers.synthetic_tpch import generate
    from spark_sched_sim.distributed import shard_seeds

    eng = HostEngine(CFG, B_LOCAL, generate(0))
    eng.reset(seeds=shard_seeds(rank, B_LOCAL, 100))
    eng.rollout(_abi.SSIM_POLICY_RANDOM, 7, STEPS)
    c = eng.host_views()["counts"]
    return np.array(c[:, [_abi.OC_NUM_COMPLETED, _abi.OC_NUM_ARRIVED, _abi.OC_DECISIONS, _abi.OC_EVENTS]])


def _worker(rank, world, port, q):
    for p in (HERE, REPO, os.path.join(REPO, "gym-sparksched_amd")):
        sys.path.insert(0, p)
    import torch
    import torch.distributed as dist

    from spark_sched_sim.distributed import gather_env_stats, reduce_timing

    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        mine = _local_run(rank)
        g = gather_env_stats(torch.tensor(mine, dtype=torch.int64), world)
        st = reduce_timing(torch.tensor([0.5 + rank, float(mine[:, 2].sum()), 1.0], dtype=torch.float64), world)
        q.put((rank, mine, g.numpy(), st.numpy()))
    finally:
        dist.destroy_process_group()


def test_two_rank_gloo_shards_gather_and_reduce():
    from hostsim.driver import build

    build()  # compile the host build once, before the ranks import it
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, mine, g, st = q.get(timeout=240)
        res[r] = (mine, g, st)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    full = np.concatenate([res[r][0] for r in range(world)])
    for r in range(world):
        mine, g, st = res[r]
        assert np.array_equal(g, full)  # global env order: rank-major contiguous blocks
        assert st[0] == 0.5 + (world - 1)  # max elapsed over ranks
        assert st[1] == float(full[:, 2].sum()) and st[2] == world  # summed counters
    assert (full[:, 2] == STEPS).all()  # every env made STEPS decisions
    # the two shards simulate different envs (disjoint seeds), and the same shard replays identically
    assert not np.array_equal(res[0][0], res[1][0])
    assert np.array_equal(_local_run(1), res[1][0])
