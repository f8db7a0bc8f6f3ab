"""The fused HIP MNIST Net (csrc/mnist_ops.hip, engine/native_mnist.py) against the fp32 torch Net:
forward log-probabilities, and the gradients of a training step whose Dropout2d / dropout masks the
reference reproduces from the same Philox streams (ops/reference.py philox_u32)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from dbx_distributed_pytorch_examples_amd.models.mnist import Net
from dbx_distributed_pytorch_examples_amd.ops import reference as R

pytestmark = pytest.mark.gpu


def _mask(n, width, seed, offset):
    u = R.philox_u32(np.arange(n * width, dtype=np.uint64), seed, offset)
    return torch.from_numpy((u < np.uint64(0x80000000)).astype(np.float32) * 2.0).view(n, width)


def test_native_mnist_forward_and_grads_match_fp32_torch():
    from dbx_distributed_pytorch_examples_amd.engine.native_mnist import NativeMNIST
    torch.manual_seed(0)
    ref = Net()
    net = Net()
    net.load_state_dict(ref.state_dict())
    nm = NativeMNIST(net, torch.device("cuda"))
    N = 37
    x = torch.randn(N, 1, 28, 28)
    y = torch.randint(0, 10, (N,))
    # eval: no dropout
    nm.eval()
    ref.eval()
    with torch.no_grad():
        lo = nm(x.cuda()).cpu()
        lr = ref(x)
    assert (lo - lr).abs().max() < 1e-4
    # training step with the kernel's masks
    nm.train()
    seed, off = nm._seed, nm._offset
    out = nm(x.cuda())
    F.nll_loss(out, y.cuda()).backward()
    m2 = _mask(N, 20, seed, off).view(N, 20, 1, 1)
    m1 = _mask(N, 50, seed, off + 1)
    r = ref
    h = F.relu(F.max_pool2d(r.conv1(x), 2))
    h = F.relu(F.max_pool2d(r.conv2(h) * m2, 2))
    h = F.relu(r.fc1(h.view(-1, 320))) * m1
    lp = F.log_softmax(r.fc2(h), dim=1)
    assert (out.detach().cpu() - lp.detach()).abs().max() < 1e-4
    F.nll_loss(lp, y).backward()
    for (name, p), (_, q) in zip(ref.named_parameters(), net.named_parameters()):
        assert q.grad is not None, name
        err = (q.grad.cpu() - p.grad).abs().max() / p.grad.abs().max().clamp_min(1e-12)
        assert err < 1e-4, (name, err.item())


def test_native_mnist_trains():
    from dbx_distributed_pytorch_examples_amd.engine.native_mnist import native_mnist
    torch.manual_seed(1)
    nm = native_mnist(Net(), torch.device("cuda"))
    opt = torch.optim.SGD(nm.parameters(), lr=0.05, momentum=0.5)
    protos = torch.randn(10, 1, 28, 28, device="cuda")
    y = torch.randint(0, 10, (100,), device="cuda")
    x = protos[y] + 0.5 * torch.randn(100, 1, 28, 28, device="cuda")  # learnable: class prototypes + noise
    losses = []
    for _ in range(60):
        opt.zero_grad()
        loss = F.nll_loss(nm(x), y)
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert losses[-1] < 0.5 * losses[0], losses[::10]


def test_native_mnist_two_forwards_and_accumulation():
    """Torch autograd semantics: two training forwards, then their backwards, give the sum of the
    two single-step gradients (each forward keeps its own saved activations; the second backward
    adds into the un-zeroed gradients)."""
    from dbx_distributed_pytorch_examples_amd.engine.native_mnist import NativeMNIST
    torch.manual_seed(4)
    nm = NativeMNIST(Net(), torch.device("cuda")).train()
    xa, xb = torch.randn(16, 1, 28, 28, device="cuda"), torch.randn(8, 1, 28, 28, device="cuda")
    ya, yb = torch.randint(0, 10, (16,), device="cuda"), torch.randint(0, 10, (8,), device="cuda")

    def grads():
        return torch.cat([p.grad.reshape(-1).clone() for p in nm.parameters()])

    s0, o0 = nm._seed, nm._offset
    F.nll_loss(nm(xa), ya).backward()
    ga = grads()
    for p in nm.parameters():
        p.grad = None
    F.nll_loss(nm(xb), yb).backward()
    gb = grads()
    for p in nm.parameters():
        p.grad = None
    nm._offset = o0  # the same dropout streams as above
    la = F.nll_loss(nm(xa), ya)
    lb = F.nll_loss(nm(xb), yb)  # second forward before the first backward
    la.backward()
    lb.backward()  # accumulates
    assert torch.allclose(grads(), ga + gb, rtol=1e-5, atol=1e-6)
