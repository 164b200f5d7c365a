import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
for p in (REPO, os.path.join(REPO, "gym-sparksched_amd"), HERE):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the gfx950 kernels through the C ABI)")


ENV_CFG_SMALL = dict(num_executors=10, job_arrival_cap=50, job_arrival_rate=4.0e-5, moving_delay=2000.0,
                     warmup_delay=1000.0)  # examples.py:15-23 (render_mode dropped)


@pytest.fixture(scope="session")
def dataset():
    from spark_sched_sim.data_samplers.synthetic_tpch import generate

    return generate(0)


@pytest.fixture(scope="session")
def env_cfg():
    return dict(ENV_CFG_SMALL)


@pytest.fixture(scope="session")
def gpu_device():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return "cuda:0"
