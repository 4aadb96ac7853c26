"""GPU: the MNIST CNN (Gaia Exp. 6 workload) on MI355X — the whole-step hipGraph learns and removes
the launch overhead of the eager step; the capturable AdamW inside a captured graph matches eager."""
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _train(*extra):
    e = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    p = subprocess.run([sys.executable, "-m", "gpu_topology_on_k8s_amd.models.train", "--model", "mnist-cnn", "--batch", "64",
                        "--steps", "150", "--warmup", "5", "--gemm-tuning", "off", *extra],
                       capture_output=True, text=True, timeout=600, cwd=REPO, env=e)
    assert p.returncode == 0, p.stderr[-4000:]
    return json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])


def test_mnist_graph_step_learns_and_beats_eager():
    eager = _train("--graph", "off")
    graph = _train("--graph", "on")
    print(json.dumps({"eager_images_per_s": eager["images_per_s"], "graph_images_per_s": graph["images_per_s"],
                      "eager_ms": eager["ms_per_step"], "graph_ms": graph["ms_per_step"], "graph_epoch_s": graph["epoch_s"]}))
    assert graph["graph"] and not eager["graph"]
    for r in (eager, graph):
        assert r["loss_last"] < 0.5 * r["loss_first"], r["losses"][:3] + r["losses"][-3:]
    assert graph["images_per_s"] > eager["images_per_s"], (graph["ms_per_step"], eager["ms_per_step"])


def test_capturable_adamw_in_graph_matches_eager():
    from gpu_topology_on_k8s_amd.models import FlatAdamW
    from gpu_topology_on_k8s_amd.models.mnist import MnistCNN

    a, b = MnistCNN(device="cuda", seed=2), MnistCNN(device="cuda", seed=2)
    oa, ob = FlatAdamW(a.flat, lr=1e-3), FlatAdamW(b.flat, lr=1e-3, capturable=True)
    g = torch.Generator(device="cuda").manual_seed(4)
    grads = [(torch.randn(a.flat.numel, generator=g, device="cuda") * 0.1).to(torch.bfloat16) for _ in range(4)]
    src = torch.empty_like(grads[0])
    b.flat.grad.copy_(grads[0])
    ob.step(grad_scale=0.5)  # eager first step (warm-up), then capture one and replay it
    oa.flat.grad.copy_(grads[0])
    oa.step(grad_scale=0.5)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        b.flat.grad.copy_(src)
        ob.step(grad_scale=0.5)
    assert ob.t == 1  # capture does not run the step
    for gr in grads[1:]:
        src.copy_(gr)
        graph.replay()
        ob.note_replay()
        a.flat.grad.copy_(gr)
        oa.step(grad_scale=0.5)
    torch.cuda.synchronize()
    assert ob.t == oa.t == 4 and float(ob.t_dev.item()) == 4.0
    assert torch.allclose(oa.master, ob.master, atol=1e-6)
    assert torch.allclose(a.flat.data.float(), b.flat.data.float(), rtol=8e-3, atol=1e-6)


def test_mnist_synth_kernel_matches_reference():
    from gpu_topology_on_k8s_amd.models.mnist import MnistCNN, synth_reference

    m = MnistCNN(device="cuda", seed=0)
    step = torch.tensor([7.0], device="cuda")
    x, y = m.synthetic_batch_dev(96, step, seed=1234)
    xr, yr = synth_reference(m.prototypes, 96, 7, 1234)
    assert torch.equal(y.cpu(), yr)
    err = ((x.float().cpu() - xr).abs() - 8e-3 * xr.abs()).max().item()  # bf16 rounding + transcendental ulps
    assert err < 1e-2, err
    assert x.shape == (96, 1, 28, 28) and x.dtype == torch.bfloat16
    x2, y2 = m.synthetic_batch_dev(96, step + 1, seed=1234)
    assert not torch.equal(x, x2)
    assert len(set(y.tolist())) == 10 and abs(float(x.float().mean()) - float(xr.mean())) < 1e-2


def test_fused_dev_optimizer_matches_host_optimizer():
    from gpu_topology_on_k8s_amd.models import FlatAdamW
    from gpu_topology_on_k8s_amd.models.mnist import MnistCNN

    a, b = MnistCNN(device="cuda", seed=5), MnistCNN(device="cuda", seed=5)
    oa, ob = FlatAdamW(a.flat, lr=1e-3, clip_norm=0.05), FlatAdamW(b.flat, lr=1e-3, clip_norm=0.05, capturable=True)
    g = torch.Generator(device="cuda").manual_seed(9)
    for _ in range(3):  # norm ~ 0.1 * sqrt(1.2M) >> clip: the clipping factor matters
        gr = (torch.randn(a.flat.numel, generator=g, device="cuda") * 0.1).to(torch.bfloat16)
        a.flat.grad.copy_(gr)
        b.flat.grad.copy_(gr)
        oa.step(grad_scale=0.5)
        ob.step(grad_scale=0.5)
    torch.cuda.synchronize()
    assert ob.t == 3 and float(ob.t_dev.item()) == 3.0
    assert torch.allclose(oa.master, ob.master, rtol=1e-4, atol=1e-6)


def _reference_features(m, x, dropout_keep=None):
    """fp32 conv1 -> ReLU -> conv2 -> ReLU -> pool on the same bf16 weights, NHWC-flattened.  The
    kernels store h1 in bf16, so the reference rounds it too (straight-through in backward): otherwise
    near-tied pooling windows pick different argmaxes and route gradients to different pixels."""
    import torch.nn.functional as F

    P = {n: m.flat.params[n].detach().float().clone().requires_grad_(True) for n in ("conv1.w", "conv1.b", "conv2.w", "conv2.b")}
    h = F.relu(F.conv2d(x.float(), P["conv1.w"].permute(0, 3, 1, 2), P["conv1.b"]))
    h = h + (h.to(torch.bfloat16).float() - h).detach()
    h = F.relu(F.conv2d(h, P["conv2.w"].permute(0, 3, 1, 2), P["conv2.b"]))
    h = F.max_pool2d(h, 2).permute(0, 2, 3, 1).reshape(x.shape[0], -1)
    return h, P


def test_hip_conv_stack_matches_fp32_reference():
    from gpu_topology_on_k8s_amd.models.mnist import MnistCNN

    m = MnistCNN(device="cuda", seed=3)
    m.eval()  # no dropout: compare the deterministic function
    x, _ = m.synthetic_batch(20, torch.Generator(device="cuda").manual_seed(1))
    feats = m.conv_features(x)
    ref, P = _reference_features(m, x)
    assert feats.shape == ref.shape == (20, 9216)
    err = (feats.float() - ref).norm() / ref.norm()
    assert err < 1e-2, float(err)
    dp = (torch.randn(feats.shape, device="cuda", generator=torch.Generator(device="cuda").manual_seed(2)) * 0.01).to(torch.bfloat16)
    m.flat.zero_grad()
    feats.backward(dp)
    ref.backward(dp.float())
    for n, t in P.items():
        got, want = m.flat.params[n].grad.float(), t.grad
        e = (got - want).norm() / want.norm()
        print(n, float(e))
        assert e < 2e-2, (n, float(e))
    # a second backward without zero_grad accumulates into the flat buffer
    g1 = m.flat.params["conv2.w"].grad.float().clone()
    m.conv_features(x).backward(dp)
    assert torch.allclose(m.flat.params["conv2.w"].grad.float(), 2 * g1, rtol=2e-2, atol=1e-3)


def test_hip_conv_dropout_keeps_three_quarters():
    from gpu_topology_on_k8s_amd.models.mnist import MnistCNN

    m = MnistCNN(device="cuda", seed=4)
    x, _ = m.synthetic_batch(64, torch.Generator(device="cuda").manual_seed(3))
    m.step_counter = torch.tensor([5.0], device="cuda")
    m.eval()
    full = m.conv_features(x).float()
    m.train()
    a = m.conv_features(x).float()
    b = m.conv_features(x).float()
    assert torch.equal(a, b)  # same step counter -> same mask
    live = full > 0
    kept = (a > 0) & live
    frac = float(kept.sum() / live.sum())
    assert 0.72 < frac < 0.78, frac
    assert torch.allclose(a[kept], full[kept] / 0.75, rtol=1e-2)
    m.step_counter.add_(1.0)
    assert not torch.equal(m.conv_features(x).float(), a)


def test_hip_conv_training_beats_library_conv():
    torch_conv = _train("--graph", "on", "--conv", "torch")
    hip_conv = _train("--graph", "on", "--conv", "hip")
    print(json.dumps({"torch_conv_ms": torch_conv["ms_per_step"], "hip_conv_ms": hip_conv["ms_per_step"]}))
    assert hip_conv["conv"] == "hip" and torch_conv["conv"] == "torch"
    assert hip_conv["loss_last"] < 0.5 * hip_conv["loss_first"]
    assert hip_conv["ms_per_step"] < torch_conv["ms_per_step"]


def test_hip_head_matches_fp32_reference():
    """fc1 -> ReLU -> fc2 -> cross-entropy through the HIP head (eval: no dropout) against fp32."""
    import torch.nn.functional as F

    from gpu_topology_on_k8s_amd.models.mnist import MnistCNN

    m = MnistCNN(device="cuda", seed=6)
    m.eval()
    x, y = m.synthetic_batch(48, torch.Generator(device="cuda").manual_seed(7))
    m.flat.zero_grad()
    loss = m(x, y)
    loss.backward()
    P = {n: m.flat.params[n].detach().float().clone().requires_grad_(True) for n in ("fc1.w", "fc1.b", "fc2.w", "fc2.b")}
    feats = m.conv_features(x).detach().float()
    h = F.relu(feats @ P["fc1.w"].t() + P["fc1.b"])
    ref = F.cross_entropy(h @ P["fc2.w"].t() + P["fc2.b"], y)
    ref.backward()
    assert abs(float(loss) - float(ref)) < 2e-2 * max(1.0, float(ref)), (float(loss), float(ref))
    for n, t in P.items():
        e = (m.flat.params[n].grad.float() - t.grad).norm() / t.grad.norm()
        print(n, float(e))
        assert e < 3e-2, (n, float(e))
    # conv gradients flowed through the head's dfeats
    assert m.flat.params["conv2.w"].grad.float().abs().sum() > 0
