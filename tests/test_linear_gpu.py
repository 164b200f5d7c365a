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


# ---- fused three-layer MLPs (HipMlp3: csrc/k_linear.hip ssim_mlp3_*) against the same nn.Sequential in torch fp32

_MLP_SHAPES = [  # (d0, hidden, out, act): the decima_tpch.yaml GNN MLPs (prep, msg/update/glob, dag) and score MLPs
    (5, [32, 16], 16, "LeakyReLU"), (16, [32, 16], 16, "LeakyReLU"), (21, [32, 16], 16, "LeakyReLU"),
    (53, [64, 64], 1, "Tanh"), (36, [64, 64], 1, "Tanh")]


def _mlp_pair(d0, hid, out, act, dev):
    from spark_sched_sim.schedulers.decima import make_mlp

    kw = {"act_kwargs": {"inplace": True, "negative_slope": 0.2}} if act == "LeakyReLU" else {}
    fused = make_mlp(d0, hid, out, act, **kw).to(dev)
    a = getattr(torch.nn, act)
    ref = torch.nn.Sequential(torch.nn.Linear(d0, hid[0]), a(**kw.get("act_kwargs", {})),
                              torch.nn.Linear(hid[0], hid[1]), a(**kw.get("act_kwargs", {})),
                              torch.nn.Linear(hid[1], out)).to(dev)
    ref.load_state_dict(fused.state_dict())
    return fused, ref


def test_hipmlp3_on_cpu_is_the_sequential():
    """CPU tensors run the modules one by one: bit-identical to nn.Sequential, and grid() to the expanded input."""
    torch.manual_seed(1)
    for d0, hid, out, act in _MLP_SHAPES:
        fused, ref = _mlp_pair(d0, hid, out, act, "cpu")
        x = torch.randn(29, d0)
        assert torch.equal(fused(x), ref(x))
    fused, ref = _mlp_pair(36, [64, 64], 1, "Tanh", "cpu")
    base = torch.randn(7, 35)
    acts = torch.arange(10) / 10
    inp = torch.cat([base[:, None, :].expand(7, 10, 35), acts[None, :, None].expand(7, 10, 1)], dim=2)
    assert torch.equal(fused.grid(base, 10), ref(inp.reshape(70, 36)))


def _kinks_masked(ref, x, g):
    """The upstream gradient with the rows zeroed whose hidden pre-activations lie within 2e-5 of LeakyReLU's kink:
    there a different fp32 summation order can pick the other slope (1 vs 0.2), a legitimate difference that says
    nothing about the kernel. Zeroed rows contribute to no gradient in either implementation."""
    if not isinstance(ref[1], torch.nn.LeakyReLU) or x.shape[0] == 0:
        return g
    with torch.no_grad():
        pre1 = ref[0](x)
        pre2 = ref[2](torch.nn.functional.leaky_relu(pre1, ref[1].negative_slope))
        kink = (pre1.abs() < 2e-5).any(1) | (pre2.abs() < 2e-5).any(1)
    assert float(kink.float().mean()) < 5e-2
    return g.masked_fill(kink[:, None], 0.0)


def _grads(m):
    return [p.grad for p in m.parameters()]


@pytest.mark.gpu
@pytest.mark.parametrize("rows", [0, 1, 37, 1000, 100003])
@pytest.mark.parametrize("shape", _MLP_SHAPES, ids=lambda s: f"{s[0]}-{s[1][0]}-{s[2]}-{s[3]}")
def test_hipmlp3_matches_torch(gpu_device, rows, shape):
    """Forward, input gradient and all six parameter gradients of the fused chain vs torch (1e-5 of the scale)."""
    d0, hid, out, act = shape
    dev = torch.device(gpu_device)
    torch.manual_seed(rows * 7 + d0)
    fused, ref = _mlp_pair(d0, hid, out, act, dev)
    x0 = torch.randn(rows, d0, device=dev)
    g = _kinks_masked(ref, x0, torch.randn(rows, out, device=dev))
    xa, xb = x0.clone().requires_grad_(True), x0.clone().requires_grad_(True)
    ya, yb = ref(xa), fused(xb)
    assert _close(yb, ya), "forward"
    ya.backward(g)
    yb.backward(g)
    assert _close(xb.grad, xa.grad), "input gradient"
    for k, (gb, ga) in enumerate(zip(_grads(fused), _grads(ref))):
        assert _close(gb, ga), f"parameter {k} gradient"
    with torch.no_grad():  # inference: no hidden rows kept, same output
        assert torch.equal(fused(x0), yb.detach())


@pytest.mark.gpu
@pytest.mark.parametrize("K,n", [(0, 50), (1, 1), (3, 50), (4099, 50), (600, 10)])
def test_hipmlp3_exec_grid_matches_expanded_input(gpu_device, K, n):
    """grid(base, n) (the exec-score MLP over every decision x action, scheduler.py:355-367) vs the expanded
    [K * n, d0] input through torch: output, base gradient (summed over each decision's actions) and weights."""
    dev = torch.device(gpu_device)
    torch.manual_seed(K + n)
    fused, ref = _mlp_pair(36, [64, 64], 1, "Tanh", dev)
    b0 = torch.randn(K, 35, device=dev)
    ba, bb = b0.clone().requires_grad_(True), b0.clone().requires_grad_(True)
    acts = torch.arange(n, device=dev) / n
    inp = torch.cat([ba[:, None, :].expand(K, n, 35), acts[None, :, None].expand(K, n, 1)], dim=2)
    ya = ref(inp.reshape(K * n, 36))
    yb = fused.grid(bb, n)
    assert yb.shape == ya.shape and _close(yb, ya), "forward"
    g = torch.randn(K * n, 1, device=dev)
    ya.backward(g)
    yb.backward(g)
    assert _close(bb.grad, ba.grad), "base gradient"
    for k, (gb, ga) in enumerate(zip(_grads(fused), _grads(ref))):
        assert _close(gb, ga), f"parameter {k} gradient"


@pytest.mark.gpu
def test_hipmlp3_backward_is_deterministic(gpu_device):
    dev = torch.device(gpu_device)
    torch.manual_seed(5)
    fused, _ = _mlp_pair(53, [64, 64], 1, "Tanh", dev)
    x = torch.randn(250000, 53, device=dev, requires_grad=True)
    g = torch.randn(250000, 1, device=dev)
    out = []
    for _ in range(2):
        fused.zero_grad()
        x.grad = None
        fused(x).backward(g)
        out.append([x.grad.clone()] + [p.grad.clone() for p in fused.parameters()])
    assert all(torch.equal(a, b) for a, b in zip(out[0], out[1]))
