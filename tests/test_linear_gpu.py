"""The learner's small dense layers on csrc/k_linear.hip (schedulers/linear.py HipLinear) against torch's fp32
nn.Linear: forward, input, weight and bias gradients over the Decima MLP widths, including empty and ragged row
counts and multi-chunk weight-gradient reductions. Tolerance: 1e-5 relative to the output scale (fp32, a different
summation order)."""

import pytest
import torch


def _close(a, b):
    if b.numel() == 0:
        return a.shape == b.shape
    scale = max(1.0, float(b.abs().max()))
    return float((a - b).abs().max()) <= 1e-5 * scale


def test_hiplinear_on_cpu_is_nn_linear():
    """CPU tensors (the CPU learner and tests) take torch's own path: bit-identical to nn.Linear."""
    from spark_sched_sim.schedulers.linear import HipLinear

    torch.manual_seed(0)
    a = HipLinear(21, 32)
    b = torch.nn.Linear(21, 32)
    b.load_state_dict(a.state_dict())
    x = torch.randn(17, 21)
    assert torch.equal(a(x), b(x))


@pytest.mark.gpu
@pytest.mark.parametrize("rows", [0, 1, 37, 1000, 100003])
@pytest.mark.parametrize("k,n", [(5, 32), (32, 16), (21, 32), (53, 64), (64, 64), (64, 1), (36, 64), (16, 16)])
def test_hiplinear_matches_torch(gpu_device, rows, k, n):
    from spark_sched_sim.schedulers.linear import HipLinear

    torch.manual_seed(rows * 131 + k * 7 + n)
    dev = torch.device(gpu_device)
    ref = torch.nn.Linear(k, n).to(dev)
    hip = HipLinear(k, n).to(dev)
    hip.load_state_dict(ref.state_dict())
    x0 = torch.randn(rows, k, device=dev)
    g = torch.randn(rows, n, device=dev)
    xa = x0.clone().requires_grad_(True)
    xb = x0.clone().requires_grad_(True)
    ya, yb = ref(xa), hip(xb)
    assert _close(yb, ya), "forward"
    ya.backward(g)
    yb.backward(g)
    assert _close(xb.grad, xa.grad), "input gradient"
    assert _close(hip.weight.grad, ref.weight.grad), "weight gradient"
    assert _close(hip.bias.grad, ref.bias.grad), "bias gradient"


@pytest.mark.gpu
def test_hiplinear_wgrad_is_deterministic(gpu_device):
    """The weight gradient sums per-chunk partials in chunk order: two runs agree bit for bit."""
    from spark_sched_sim.schedulers.linear import HipLinear

    dev = torch.device(gpu_device)
    torch.manual_seed(3)
    m = HipLinear(53, 64).to(dev)
    x = torch.randn(250000, 53, device=dev)
    g = torch.randn(250000, 64, device=dev)
    out = []
    for _ in range(2):
        m.zero_grad()
        m(x).backward(g)
        out.append((m.weight.grad.clone(), m.bias.grad.clone()))
    assert torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1])
