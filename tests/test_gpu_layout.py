"""LDS sizing of the persistent Decima rollout against the layout's per-env share (ssim_layout.lds_share).

compute_layout decides LDS residency assuming a number of envs per CU; the Decima rollout's policy plan grows into
whatever LDS room it is given, so it must stay within the env's share or a many-env launch silently drops to fewer
workgroups per CU than the layout counted on."""

import pytest

from conftest import ENV_CFG_SMALL

J200_N50 = dict(num_executors=50, job_arrival_cap=200, job_arrival_rate=4.0e-5, moving_delay=2000.0,
                warmup_delay=1000.0)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,B,resident,share", [
    (ENV_CFG_SMALL, 1024, 1, 160 * 1024 // 4),  # configs[1] env, many envs: 4 per CU
    (ENV_CFG_SMALL, 4096, 0, 160 * 1024 // 16),  # HBM-resident: 16 one-wave workgroups per CU
    (J200_N50, 16, 1, 160 * 1024),  # the PPO collect's 16 envs: one env per CU, the whole CU
    (J200_N50, 4096, 0, 160 * 1024 // 16),  # configs[2]
])
def test_decima_rollout_lds_within_share(gpu_device, dataset, cfg, B, resident, share):
    from spark_sched_sim import native
    from spark_sched_sim.engine import DeviceEngine

    eng = DeviceEngine(cfg, B, dataset, device=gpu_device)
    L = eng.layout
    cus = int(L.chip_cus)
    if B > cus and B <= 4 * cus and cfg is J200_N50:
        pytest.skip("partitioned device")
    assert int(L.lds_resident) == resident
    if resident and B > cus:
        share = 160 * 1024 // 4
    assert int(L.lds_share) == share
    lds = int(native.lib().ssim_decima_rollout_lds_bytes(eng.handle))
    assert int(L.lds_bytes) <= lds <= int(L.lds_share), (lds, int(L.lds_bytes), int(L.lds_share))
