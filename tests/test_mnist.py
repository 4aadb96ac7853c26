"""MNIST CNN — the Gaia paper's Exp. 6 workload (paper p.7 Figs. 11-12) on CPU: architecture size,
learnable synthetic data, the capturable AdamW against the eager one, and the best-vs-worst harness
with two 2-rank gloo jobs on a fake 8-device node."""
import json
import os
import socket
import subprocess
import sys

import torch

from gpu_topology_on_k8s_amd.models import FlatAdamW
from gpu_topology_on_k8s_amd.models.mnist import MnistCNN, MnistConfig

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_architecture_matches_the_pytorch_example():
    cfg = MnistConfig.named("mnist-cnn")
    assert cfg.num_params() == 1_199_882  # torchvision/examples mnist/main.py Net
    assert cfg.pooled == 9216
    m = MnistCNN(cfg, device="cpu")
    x, y = m.synthetic_batch(4, torch.Generator().manual_seed(0))
    assert x.shape == (4, 1, 28, 28) and x.dtype == torch.bfloat16 and x.is_contiguous(memory_format=torch.channels_last)
    assert m(x).shape == (4, 10) and 0 <= int(y.min()) and int(y.max()) < 10
    # identical replicas from the same seed (DP ranks), different data per generator seed
    assert torch.equal(MnistCNN(cfg, device="cpu").flat.data, m.flat.data)
    x2, _ = m.synthetic_batch(4, torch.Generator().manual_seed(1))
    assert not torch.equal(x, x2)


def test_capturable_adamw_matches_eager_on_cpu():
    cfg = MnistConfig()
    a, b = MnistCNN(cfg, device="cpu", seed=1), MnistCNN(cfg, device="cpu", seed=1)
    oa, ob = FlatAdamW(a.flat, lr=1e-3), FlatAdamW(b.flat, lr=1e-3, capturable=True)
    g = torch.Generator().manual_seed(3)
    for _ in range(3):
        grad = (torch.randn(a.flat.numel, generator=g) * 0.1).to(torch.bfloat16)
        a.flat.grad.copy_(grad)
        b.flat.grad.copy_(grad)
        oa.step(grad_scale=0.5)
        ob.step(grad_scale=0.5)
    assert oa.t == ob.t == 3 and float(ob.t_dev) == 3.0
    # bias corrections in fp32 on the device vs double on the host: master agrees to fp32 rounding,
    # the bf16 weights to at most one ulp at rounding boundaries
    assert torch.allclose(oa.master, ob.master, atol=1e-6)
    assert torch.allclose(a.flat.data.float(), b.flat.data.float(), rtol=8e-3, atol=1e-6)
    ob.t = 7  # checkpoint restore sets the device counter too
    assert float(ob.t_dev) == 7.0


def test_mnist_training_learns_on_cpu():
    from gpu_topology_on_k8s_amd.models.train import train

    env = {k: os.environ.get(k) for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    try:
        with socket.socket() as sk:  # a fixed port collides with other tests under pytest -n
            sk.bind(("127.0.0.1", 0))
            os.environ["MASTER_PORT"] = str(sk.getsockname()[1])
        out = train("mnist-cnn", batch=32, steps=25, warmup=1, device_kind="cpu", log=False, lr=1e-3)
    finally:
        import torch.distributed as dist

        if dist.is_initialized():
            dist.destroy_process_group()
        for k, v in env.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    assert out["throughput_unit"] == "images/s" and out["images_per_s"] > 0 and out["tokens_per_s"] is None
    assert out["epoch_s"] == 60000 / out["images_per_s"] and out["graph"] is False
    assert out["loss_first"] > 2.0 and out["loss_last"] < 0.5 * out["loss_first"]


def test_mnist_best_vs_worst_harness_cpu(tmp_path):
    out = tmp_path / "r.json"
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench", "train_llama.py"), "--gpus", "2", "--device", "cpu",
                        "--discovery", "fake", "--model", "mnist-cnn", "--batch", "16", "--steps", "3", "--warmup", "1",
                        "--out", str(out)], capture_output=True, text=True, timeout=600, cwd=REPO, env=dict(env, GTK_FAKE_GPUS="8"))
    assert p.returncode == 0, p.stderr[-4000:]
    s = json.loads(out.read_text())["summary"]
    assert s["throughput_unit"] == "images/s" and s["best_throughput"] > 0 and s["worst_throughput"] > 0
    assert s["best_devices"] != s["worst_devices"] and s["best_epoch_s"] > 0 and s["seq_len"] is None
