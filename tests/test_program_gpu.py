"""End-to-end numerics of the native ResNet program vs a PyTorch fp32 autograd reference.

The native path runs bf16 activations / fp32 accumulation, so per-tensor gradients are compared
by cosine similarity and relative norm error against fp32 autograd on the same (bf16-rounded)
input, same weights, same labels.
"""
import copy
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
dev = torch.device("cuda")


def _cos(a, b):
    a = a.float().flatten()
    b = b.float().flatten()
    return (a @ b / (a.norm() * b.norm() + 1e-20)).item()


@pytest.mark.parametrize("arch,size,batch,fold", [("resnet50", 64, 8, 0), ("resnet50", 64, 8, 1 << 40),
                                                  ("resnet18", 32, 16, 0), ("cifar_resnet18", 32, 8, 0)])
def test_program_matches_autograd(arch, size, batch, fold, monkeypatch, engine):
    # fold: fold_min_elems -- 0 folds every foldable BN-backward apply into its dgrad, 2^40 none
    engine(fold_min_elems=str(fold))
    from dbx_distributed_pytorch_examples_amd.engine.native_trainer import NativeTrainer, OptimConfig
    from dbx_distributed_pytorch_examples_amd.models import build_model

    torch.manual_seed(0)
    model = build_model(arch, num_classes=10 if "cifar" in arch else 100)
    # Damp the residual branches (last BN gamma = 0.2): a random-init ResNet-50 at kaiming init
    # is in the gradient-explosion regime where bf16-vs-fp32 rounding alone decorrelates the
    # backward (cos ~0.2 even with the CPU reference ops); damped, it is well conditioned.
    for n_, m_ in model.named_modules():
        if n_.endswith("bn3") or (n_.endswith("bn2") and "layer" in n_ and arch != "resnet50"):
            torch.nn.init.constant_(m_.weight, 0.2)
    ref = copy.deepcopy(model).to(dev).train()
    tr = NativeTrainer(model, batch, (size, size), dev, optim=OptimConfig(lr=0.0, momentum=0.0, weight_decay=0.0),
                       use_graphs=False)
    p = tr.prog
    g = torch.Generator().manual_seed(1)
    img = torch.randint(0, 256, (batch, size, size, 3), dtype=torch.uint8, generator=g).to(dev)
    lab = torch.randint(0, p.num_classes, (batch,), generator=g).to(dev)
    tr.step(img, lab)
    torch.cuda.synchronize()
    loss_native = p.metrics[0].item() / batch
    x = p.x4[..., :3].float().permute(0, 3, 1, 2).contiguous()
    out = ref(x)
    loss = F.cross_entropy(out, lab)
    loss.backward()
    assert abs(loss_native - loss.item()) / loss.item() < 3e-2, (loss_native, loss.item())
    # gradients (lr = 0: master params unchanged, grads left in the flat buffer)
    named_ref = dict(ref.named_parameters())
    worst = 1.0
    for name, prm in model.named_parameters():
        rg = named_ref[name].grad
        off_ranges = [r for r in p.param_ranges]
        # locate the flat-grad view of this parameter through its storage offset in master
        off = (prm.data_ptr() - p.master.data_ptr()) // 4
        n = prm.numel()
        gflat = p.grad[off:off + n]
        if prm.dim() == 4:
            gn = gflat.view(prm.shape[0], prm.shape[2], prm.shape[3], prm.shape[1]).permute(0, 3, 1, 2)
        else:
            gn = gflat.view(prm.shape)
        c = _cos(gn, rg)
        worst = min(worst, c)
        assert c > (0.9 if prm.dim() > 1 else 0.75), (name, c)
    # BN running stats updated like torch
    for (n1, b1), (n2, b2) in zip(model.named_buffers(), ref.named_buffers()):
        if "running_mean" in n1:
            assert _cos(b1, b2) > 0.99 or b2.abs().max() < 1e-3, n1


class _Q(torch.autograd.Function):
    """bf16 rounding of a stored activation (forward) and of a stored gradient (backward)."""

    @staticmethod
    def forward(ctx, x):
        return x.bfloat16().float()

    @staticmethod
    def backward(ctx, g):
        return g.bfloat16().float()


def _bf16_emulating(model):
    """fp32 reference that rounds where the native program stores bf16: every conv / fc operand
    (input, weight), every conv output, and every dgrad result flowing back into a conv input."""
    def wrap(mod):
        f = mod.forward

        def fwd(x):
            w0 = mod.weight.data
            mod.weight.data = w0.bfloat16().float()
            try:
                y = f(_Q.apply(x))
            finally:
                mod.weight.data = w0
            return _Q.apply(y) if isinstance(mod, torch.nn.Conv2d) else y
        mod.forward = fwd
    for m in model.modules():
        if isinstance(m, (torch.nn.Conv2d, torch.nn.Linear)):
            wrap(m)
    return model


@pytest.mark.parametrize("arch,size,batch", [("resnet50", 64, 8), ("resnet18", 32, 16)])
def test_program_grads_match_bf16_emulating_reference(arch, size, batch):
    """Tight end-to-end check: every parameter gradient of one native step against autograd of a
    reference that rounds to bf16 at the program's storage points (BN gamma / beta included), held to
    the rounding noise floor of the network itself: the native program must agree with the emulating
    reference at least as well as plain fp32 autograd does (per tensor, within 0.03, capped at 0.99),
    and at the median within 0.01. A fixed cosine bound cannot do this for ResNet-50: at b8 the
    fp32-vs-emulating cosine of some BN biases is 0.87-0.91 (near-cancelling pixel sums), while the
    native program sits at or above that floor on every tensor (tools/grad_noise.py,
    profiles/r3s2_gradnoise/). A wrong-but-correlated BN-backward term drops below the floor."""
    from dbx_distributed_pytorch_examples_amd.engine.native_trainer import NativeTrainer, OptimConfig
    from dbx_distributed_pytorch_examples_amd.models import build_model
    torch.manual_seed(0)
    model = build_model(arch, num_classes=100)
    for n_, m_ in model.named_modules():
        if n_.endswith("bn3") or (n_.endswith("bn2") and "layer" in n_ and arch != "resnet50"):
            torch.nn.init.constant_(m_.weight, 0.2)
    ref32 = copy.deepcopy(model).to(dev).train()
    ref = _bf16_emulating(copy.deepcopy(model).to(dev).train())
    tr = NativeTrainer(model, batch, (size, size), dev, optim=OptimConfig(lr=0.0, momentum=0.0, weight_decay=0.0),
                       use_graphs=False)
    p = tr.prog
    g = torch.Generator().manual_seed(1)
    img = torch.randint(0, 256, (batch, size, size, 3), dtype=torch.uint8, generator=g).to(dev)
    lab = torch.randint(0, p.num_classes, (batch,), generator=g).to(dev)
    tr.step(img, lab)
    torch.cuda.synchronize()
    x = p.x4[..., :3].float().permute(0, 3, 1, 2).contiguous()
    F.cross_entropy(ref(x), lab).backward()
    F.cross_entropy(ref32(x), lab).backward()
    named_ref, named32 = dict(ref.named_parameters()), dict(ref32.named_parameters())
    cs, floor = {}, {}
    for name, prm in model.named_parameters():
        off = (prm.data_ptr() - p.master.data_ptr()) // 4
        gflat = p.grad[off:off + prm.numel()]
        gn = (gflat.view(prm.shape[0], prm.shape[2], prm.shape[3], prm.shape[1]).permute(0, 3, 1, 2)
              if prm.dim() == 4 else gflat.view(prm.shape))
        cs[name] = _cos(gn, named_ref[name].grad)
        floor[name] = _cos(named32[name].grad, named_ref[name].grad)
    bad = sorted(((n, c, floor[n]) for n, c in cs.items() if c < min(0.99, floor[n]) - 0.03), key=lambda t: t[1])
    med, med_floor = (sorted(d.values())[len(d) // 2] for d in (cs, floor))
    print(f"[grad-cos] {arch}: median {med:.4f} (floor {med_floor:.4f}), worst "
          f"{sorted(cs.items(), key=lambda kv: kv[1])[:3]}")
    assert not bad, bad[:5]
    assert med >= min(0.99, med_floor) - 0.01, (med, med_floor)


def test_program_trains_and_graph_replay():
    """Loss decreases on a fixed batch; graph replay reproduces eager training bit for bit (every
    reduction in the step is order-independent: fp64 statistics atomics, fixed-order split-K and
    shard sums), and so does a second eager run with the wgrad side stream disabled."""
    from dbx_distributed_pytorch_examples_amd.engine.native_trainer import NativeTrainer, OptimConfig
    from dbx_distributed_pytorch_examples_amd.models import build_model

    torch.manual_seed(0)
    size, batch = 32, 32
    m1 = build_model("resnet18", num_classes=10)
    m2 = copy.deepcopy(m1)
    m3 = copy.deepcopy(m1)
    t1 = NativeTrainer(m1, batch, (size, size), dev, optim=OptimConfig(lr=0.05), use_graphs=True)
    t2 = NativeTrainer(m2, batch, (size, size), dev, optim=OptimConfig(lr=0.05), use_graphs=False)
    t3 = NativeTrainer(m3, batch, (size, size), dev, optim=OptimConfig(lr=0.05), use_graphs=False)
    t3.prog.overlap_wgrad = False
    g = torch.Generator().manual_seed(2)
    img = torch.randint(0, 256, (batch, size, size, 3), dtype=torch.uint8, generator=g).to(dev)
    lab = torch.randint(0, 10, (batch,), generator=g).to(dev)
    losses = []
    for i in range(12):
        for t in (t1, t2, t3):
            t.step(img, lab)
        (l1, _), (l2, _), (l3, _) = t1.read_metrics(), t2.read_metrics(), t3.read_metrics()
        losses.append(l1 / batch)
        assert l1 == l2 == l3, (i, l1, l2, l3)
    assert losses[-1] < 0.5 * losses[0], losses
    assert torch.equal(t1.prog.master, t2.prog.master)
    assert torch.equal(t1.prog.master, t3.prog.master)


def test_train_entrypoint_native_engine(tmp_path, monkeypatch):
    """train() picks the graph-captured native engine on the GPU and runs loader + aug + eval + ckpt."""
    monkeypatch.setenv("DBX_MLRUNS", str(tmp_path / "mlruns"))
    from dbx_distributed_pytorch_examples_amd.config import TrainConfig
    from dbx_distributed_pytorch_examples_amd.data.datasets import SyntheticImages
    from dbx_distributed_pytorch_examples_amd.train.engine import train
    cfg = TrainConfig(model="resnet18", num_classes=10, batch_size=32, epochs=2, log_every=0)
    cfg.data.image_size = 32
    cfg.optim.lr = 0.02
    cfg.checkpoint_dir = str(tmp_path / "ck")
    res = train(cfg, train_dataset=SyntheticImages(128, 32, 3, 10), eval_dataset=SyntheticImages(64, 32, 3, 10, seed=9))
    assert res.engine == "native"
    assert all(h["train_loss"] == h["train_loss"] for h in res.history)
    assert "val_accuracy" in res.history[-1]
    assert (tmp_path / "ck" / "checkpoint-2.pth.tar").exists()


@pytest.mark.gpu
def test_frozen_backbone_native_gpu():
    """Reference workload shape (frozen ResNet-50 backbone, new head, 64x64 TinyImageNet): native
    inference-mode backbone on the HIP kernels + autograd head."""
    from dbx_distributed_pytorch_examples_amd.config import OptimizerConfig
    from dbx_distributed_pytorch_examples_amd.engine.frozen_trainer import FrozenFeatureTrainer
    from dbx_distributed_pytorch_examples_amd.models import FrozenBackboneClassifier
    torch.manual_seed(0)
    m = FrozenBackboneClassifier("resnet50", num_classes=200)
    m.eval()
    img = torch.randint(0, 256, (16, 64, 64, 3), dtype=torch.uint8)
    lab = torch.randint(0, 200, (16,))
    x = (img.permute(0, 3, 1, 2).float() / 255 - torch.tensor([0.485, 0.456, 0.406]).view(1, 3, 1, 1)) \
        / torch.tensor([0.229, 0.224, 0.225]).view(1, 3, 1, 1)
    with torch.no_grad():
        r = m.resnet
        f = r.maxpool(r.relu(r.bn1(r.conv1(x))))
        ref = torch.flatten(r.avgpool(r.layer4(r.layer3(r.layer2(r.layer1(f))))), 1)
    tr = FrozenFeatureTrainer(m, 16, (64, 64), torch.device("cuda"), OptimizerConfig(name="adam", lr=1e-3))
    feats = tr._features(img.cuda(), lab.cuda(), None, None).float().cpu()
    cos = torch.nn.functional.cosine_similarity(feats.flatten(), ref.flatten(), dim=0)
    assert cos > 0.98, cos
    w0 = m.resnet.fc[1].weight.detach().clone()
    for _ in range(3):
        tr.step(img.cuda(), lab.cuda())
    torch.cuda.synchronize()
    assert not torch.equal(w0, m.resnet.fc[1].weight.detach())
    loss, _ = tr.read_metrics()
    assert math.isfinite(loss) and loss > 0


@pytest.mark.gpu
def test_frozen_backbone_graph_replay_matches_eager():
    """the graph-captured backbone forward (after two eager calls) follows new inputs every replay and
    gives bit-identical features to the eager program, including a short final batch"""
    from dbx_distributed_pytorch_examples_amd.config import OptimizerConfig
    from dbx_distributed_pytorch_examples_amd.engine.frozen_trainer import FrozenFeatureTrainer
    from dbx_distributed_pytorch_examples_amd.models import FrozenBackboneClassifier
    torch.manual_seed(1)
    m = FrozenBackboneClassifier("resnet18", num_classes=10)
    dev = torch.device("cuda")
    g = FrozenFeatureTrainer(m, 32, (32, 32), dev, OptimizerConfig(name="adam", lr=1e-3))
    e = FrozenFeatureTrainer(m, 32, (32, 32), dev, OptimizerConfig(name="adam", lr=1e-3), use_graphs=False)
    imgs = [torch.randint(0, 256, (32, 32, 32, 3), dtype=torch.uint8, device=dev) for _ in range(5)]
    lab = torch.randint(0, 10, (32,), device=dev)
    for i, x in enumerate(imgs + [imgs[0][:20]]):
        fg = g._features(x, lab[:x.shape[0]], None, None).clone()
        fe = e._features(x, lab[:x.shape[0]], None, None).clone()
        assert torch.equal(fg, fe), i
    assert g._graph is not None and e._graph is None
    for _ in range(3):
        g.step(imgs[1], lab)
    torch.cuda.synchronize()
    loss, _ = g.read_metrics()
    assert math.isfinite(loss) and loss > 0


@pytest.mark.gpu
def test_frozen_whole_step_graph_matches_eager():
    """world-1 Adam: the whole frozen step (backbone + autograd head + capturable Adam + metrics) as one
    graph tracks the eager step over 6 steps with a changing learning rate (dropout off: p=0)"""
    import copy
    from dbx_distributed_pytorch_examples_amd.config import OptimizerConfig
    from dbx_distributed_pytorch_examples_amd.engine.frozen_trainer import FrozenFeatureTrainer
    from dbx_distributed_pytorch_examples_amd.models import FrozenBackboneClassifier
    torch.manual_seed(2)
    m = FrozenBackboneClassifier("resnet18", num_classes=10, dropout=0.0)
    m2 = copy.deepcopy(m)
    dev = torch.device("cuda")
    oc = OptimizerConfig(name="adam", lr=1e-2)
    g = FrozenFeatureTrainer(m, 32, (32, 32), dev, oc)
    e = FrozenFeatureTrainer(m2, 32, (32, 32), dev, OptimizerConfig(name="adam", lr=1e-2), use_graphs=False)
    assert g.full_graph and not e.full_graph
    gen = torch.Generator(device="cpu").manual_seed(3)
    for i in range(6):
        x = torch.randint(0, 256, (32, 32, 32, 3), dtype=torch.uint8, generator=gen).to(dev)
        y = torch.randint(0, 10, (32,), generator=gen).to(dev)
        lr = 1e-2 * (i + 1) / 6
        g.set_lr(lr)
        e.set_lr(lr)
        g.step(x, y)
        e.step(x, y)
    torch.cuda.synchronize()
    assert g._sgraph is not None
    wg, we = m.resnet.fc[1].weight.detach(), m2.resnet.fc[1].weight.detach()
    assert ((wg - we).norm() / we.norm()).item() < 1e-4
    lg, cg = g.read_metrics()
    le, ce = e.read_metrics()
    assert abs(lg - le) / le < 1e-4 and abs(cg - ce) <= 1  # (an argmax near-tie may flip)


# SURVEY.md §7.4 "50-step loss-decrease smoke per BASELINE config": each BASELINE.json config's
# architecture / resolution / optimizer family, at a small per-GPU batch, trained 50 steps on one
# fixed synthetic batch through the graph-captured native step. A correct forward/backward/optimizer
# memorises the batch; a broken kernel anywhere in the chain stalls or diverges.
@pytest.mark.parametrize("arch,size,classes,batch,optim,clip,zero", [
    ("resnet50", 224, 1000, 16, "sgd", 0.0, 0),       # headline ImageNet-1K large-batch (SGD)
    ("resnet50", 224, 1000, 16, "lars", 0.0, 0),      # large-batch LARS variant
    ("resnet50", 224, 1000, 16, "adamw", 0.3, 1),     # DeepSpeed ImageNet config: AdamW, clip 0.3, ZeRO-1
    ("resnet18", 32, 10, 64, "adam", 0.0, 0),         # CIFAR-10 TorchDistributor (Adam 1e-3)
    ("resnet50", 64, 200, 32, "adam", 0.0, 0),        # TinyImageNet TorchDistributor (Adam 1e-3)
])
def test_baseline_config_loss_decreases(arch, size, classes, batch, optim, clip, zero):
    from dbx_distributed_pytorch_examples_amd.engine.native_trainer import NativeTrainer, OptimConfig
    from dbx_distributed_pytorch_examples_amd.models import build_model

    torch.manual_seed(0)
    model = build_model(arch, num_classes=classes)
    # SGD at lr 0.05 memorises this batch chaotically (loss spikes to 15-60 at step ~7 and lands
    # anywhere in 0.5-2.9 at step 50 depending on last-bit rounding: tools/loss_probe.py, with and
    # without the patch kernels); at 0.02 both kernel paths reach ~0.001 -- a clean pass/fail signal
    lr = {"sgd": 0.02, "lars": 9.0, "adamw": 2e-4, "adam": 1e-3}[optim]
    oc = OptimConfig(name=optim, lr=lr, grad_clip=clip, weight_decay=0.0 if optim != "lars" else 5e-5)
    tr = NativeTrainer(model, batch, (size, size), dev, optim=oc, use_graphs=True, zero_stage=zero)
    g = torch.Generator().manual_seed(3)
    img = torch.randint(0, 256, (batch, size, size, 3), dtype=torch.uint8, generator=g).to(dev)
    lab = torch.randint(0, classes, (batch,), generator=g).to(dev)
    losses = []
    for _ in range(50):
        tr.step(img, lab)
        losses.append(tr.read_metrics()[0] / batch)
    print(f"[loss50] {arch} {size} {optim}: " + " ".join(f"{v:.3f}" for v in losses[::7]))
    assert all(math.isfinite(v) for v in losses), losses
    first, last = sum(losses[:3]) / 3, sum(losses[-3:]) / 3
    assert last < 0.5 * first, (arch, optim, losses[:3], losses[-3:])


@pytest.mark.parametrize("optim,clip,zero", [("adamw", 0.3, 1), ("adamw", 0.0, 2), ("sgd", 0.0, 1), ("lars", 0.5, 0)])
def test_graph_matches_eager_with_lr_schedule(optim, clip, zero):
    """A graph-captured step must follow set_lr() and the Adam step count on every replay (the
    optimizer reads lr / bias corrections from a device tensor, never from capture-time host
    scalars) -- also on the ZeRO path, whose optimizer phase is inside the world-1 graph. Graph
    and eager trainers with the same changing LR stay bit-identical over more steps than the
    warm-up + capture (3)."""
    from dbx_distributed_pytorch_examples_amd.engine.native_trainer import NativeTrainer, OptimConfig
    from dbx_distributed_pytorch_examples_amd.models import build_model

    torch.manual_seed(0)
    size, batch = 32, 32
    m1 = build_model("resnet18", num_classes=10)
    m2 = copy.deepcopy(m1)
    lr0 = {"adamw": 1e-3, "sgd": 0.05, "lars": 2.0}[optim]

    def mk(m, graphs):
        oc = OptimConfig(name=optim, lr=lr0, grad_clip=clip, weight_decay=1e-4)
        return NativeTrainer(m, batch, (size, size), dev, optim=oc, use_graphs=graphs, zero_stage=zero)

    t1, t2 = mk(m1, True), mk(m2, False)
    g = torch.Generator().manual_seed(5)
    img = torch.randint(0, 256, (batch, size, size, 3), dtype=torch.uint8, generator=g).to(dev)
    lab = torch.randint(0, 10, (batch,), generator=g).to(dev)
    for i in range(8):
        lr = lr0 * (0.5 ** i)  # halved every step: a stale captured lr shows up at once
        for t in (t1, t2):
            t.set_lr(lr)
            t.step(img, lab)
        (l1, _), (l2, _) = t1.read_metrics(), t2.read_metrics()
        assert l1 == l2, (i, l1, l2)
    assert torch.equal(t1.prog.master, t2.prog.master)
    if zero:
        assert t1.zero.step_count == t2.zero.step_count == 8


def test_native_module_gpu_matches_autograd():
    """engine.native_module on the HIP kernels inside a plain autograd loop: loss and per-parameter
    gradients vs fp32 autograd of the same module (soft targets + label smoothing computed by torch)."""
    from dbx_distributed_pytorch_examples_amd.engine.native_module import native_module
    from dbx_distributed_pytorch_examples_amd.models import build_model
    torch.manual_seed(0)
    model = build_model("resnet50", num_classes=100)
    for n_, m_ in model.named_modules():
        if n_.endswith("bn3"):
            torch.nn.init.constant_(m_.weight, 0.2)
    ref = copy.deepcopy(model).to(dev).train()
    nm = native_module(model, 8, (64, 64), dev).train()
    g = torch.Generator().manual_seed(1)
    x = torch.randn(8, 3, 64, 64, generator=g).bfloat16().float().to(dev)
    t = torch.softmax(torch.randn(8, 100, generator=g), 1).to(dev)
    loss_n = F.cross_entropy(nm(x), t, label_smoothing=0.1)
    loss_n.backward()
    loss_r = F.cross_entropy(ref(x), t, label_smoothing=0.1)
    loss_r.backward()
    assert abs(loss_n.item() - loss_r.item()) < 3e-2 * loss_r.item(), (loss_n.item(), loss_r.item())
    nr = dict(ref.named_parameters())
    for name, prm in nm.named_parameters():
        c = _cos(prm.grad, nr[name].grad)
        assert c > (0.9 if prm.dim() > 1 else 0.75), (name, c)
    opt = torch.optim.Adam(nm.parameters(), lr=1e-3)
    y = torch.randint(0, 100, (8,), device=dev)
    losses = []
    for _ in range(8):
        opt.zero_grad()
        loss = F.cross_entropy(nm(x), y)
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert losses[-1] < 0.7 * losses[0], losses


def test_native_module_graph_replay_bit_exact():
    """native_module's captured forward / backward graphs (from the third call on) reproduce the eager
    module bit for bit over 6 steps of a torch Adam loop with changing data."""
    from dbx_distributed_pytorch_examples_amd.engine.native_module import native_module
    from dbx_distributed_pytorch_examples_amd.models import build_model
    torch.manual_seed(0)
    m1 = build_model("resnet18", num_classes=10)
    m2 = copy.deepcopy(m1)
    a = native_module(m1, 16, (32, 32), dev).train()
    b = native_module(m2, 16, (32, 32), dev).train()
    b.use_graphs = False
    oa, ob = torch.optim.Adam(a.parameters(), lr=1e-3), torch.optim.Adam(b.parameters(), lr=1e-3)
    g = torch.Generator().manual_seed(3)
    for i in range(6):
        x = torch.randn(16, 3, 32, 32, generator=g).to(dev)
        y = torch.randint(0, 10, (16,), generator=g).to(dev)
        for m, o in ((a, oa), (b, ob)):
            o.zero_grad()
            F.cross_entropy(m(x), y, label_smoothing=0.1).backward()
            o.step()
        assert torch.equal(a.prog.master, b.prog.master), i
    assert set(a._graphs) == {"fwd_train", "bwd"} and not b._graphs
    a.eval()
    b.eval()
    with torch.no_grad():
        for _ in range(3):
            assert torch.equal(a(x), b(x))


def test_composer_trainer_runs_on_native_module():
    """frontends.composer.Trainer on one GPU: ComposerResNet50 wrapped by native_module (CutMix soft targets
    + label smoothing through autograd) trains 3 epochs and evaluates; the short final batch takes the
    torch-module path."""
    from torch.utils.data import DataLoader, TensorDataset
    from dbx_distributed_pytorch_examples_amd.frontends.composer import CutMix, LabelSmoothing, Trainer
    from dbx_distributed_pytorch_examples_amd.models import ComposerResNet50
    torch.manual_seed(0)
    n, nc = 200, 10
    protos = torch.randn(nc, 3, 32, 32)
    y = torch.randint(0, nc, (n,))
    x = protos[y] + 0.3 * torch.randn(n, 3, 32, 32)
    dl = DataLoader(TensorDataset(x, y), batch_size=64, shuffle=True)
    model = ComposerResNet50(num_classes=nc)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    tr = Trainer(model, optimizers=opt, train_dataloader=dl, eval_dataloader=dl, max_duration="3ep",
                 algorithms=[LabelSmoothing(0.1), CutMix(1.0)], device="cuda")
    assert tr.native
    w0 = model.model.model.fc.weight.detach().clone()
    hist = tr.fit()
    assert len(hist) == 3 and all(math.isfinite(h["train/loss"]) for h in hist), hist
    assert not torch.equal(w0, model.model.model.fc.weight.detach())
    assert 0.0 <= hist[-1]["metrics/eval/Accuracy"] <= 1.0


@pytest.mark.parametrize("mode", ["2", "3", "2+tail2", "2+defer", "2+tail2+defer", "2+lazy", "2+tail2+defer+lazy",
                                  "3+defer+lazy", "3+defer+lazy+dsf", "3+btail2+defer+lazy", "3+btail2+defer+lazy+dsf"])
@pytest.mark.parametrize("arch,size,batch", [("resnet50", 64, 32), ("resnet18", 32, 64)])
def test_batched_side_stream_bit_identical(arch, size, batch, mode, monkeypatch, engine):
    """overlap_wgrad=2 (weight gradients forked once per backward segment, joined one segment
    later) and =3 (forked once per block, joined at the segment's end) train bit-identically to the
    in-order schedule, eager and graph-replayed."""
    from dbx_distributed_pytorch_examples_amd.engine.native_trainer import NativeTrainer, OptimConfig
    from dbx_distributed_pytorch_examples_amd.models import build_model
    torch.manual_seed(0)
    m1 = build_model(arch, num_classes=10)
    m2 = copy.deepcopy(m1)
    # the same BN-backward fold schedule on both sides (without the side stream it defaults to fold-all)
    engine(fold_min_elems=str(1 << 25))
    engine(fold_max_ratio="1")
    # "2+tail2": the last batch's two last weight gradients on the main stream's tail (tail_main),
    # the stem weight gradient on the main stream (the batched default)
    engine(overlap_wgrad=mode[0])
    engine(tail_main="2" if "tail2" in mode.split("+") else "0")
    # "defer": each side batch launched after the main stream's next kernel (side_defer)
    engine(side_defer="1" if "defer" in mode else "0")
    # "lazy": no intermediate joins of the side stream (lazy_join)
    engine(lazy_join="1" if "lazy" in mode else "0")
    opts = mode.split("+")
    # "btail2": per-block forks, the last block's last two weight gradients on the main stream (block_tail_main)
    engine(block_tail_main="2" if "btail2" in opts else "0")
    # "dsf": the downsample conv's forward on the side stream beside conv2 / conv3 (ds_fwd_side)
    engine(ds_fwd_side="1" if "dsf" in opts else "0")
    t1 = NativeTrainer(m1, batch, (size, size), dev, optim=OptimConfig(lr=0.05))
    engine(overlap_wgrad="0")
    t2 = NativeTrainer(m2, batch, (size, size), dev, optim=OptimConfig(lr=0.05))
    assert (t1.prog.side_batch if mode[0] == "2" else t1.prog.side_block) and t1.prog.overlap_wgrad
    assert t1.prog.tail_main == (2 if "tail2" in mode.split("+") else 0)
    assert t1.prog.side_defer == ("defer" in mode)
    assert not t2.prog.overlap_wgrad
    g = torch.Generator().manual_seed(3)
    for i in range(5):
        img = torch.randint(0, 256, (batch, size, size, 3), dtype=torch.uint8, generator=g).to(dev)
        lab = torch.randint(0, 10, (batch,), generator=g).to(dev)
        t1.step(img, lab)
        t2.step(img, lab)
    torch.cuda.synchronize()
    assert torch.equal(t1.prog.master, t2.prog.master)
    assert torch.equal(t1.prog.grad, t2.prog.grad)


@pytest.mark.parametrize("arch,size,batch,optim", [("resnet50", 64, 32, "sgd"), ("resnet18", 32, 64, "sgd"),
                                                   ("resnet50", 64, 32, "adamw")])
def test_optimizer_in_backward_bit_identical(arch, size, batch, optim, engine):
    """overlap_optimizer (opt-in): each segment's update runs on the side stream behind its last block
    batch, inside the captured step -- bit-identical to the end-of-step optimizer over graph replays."""
    from dbx_distributed_pytorch_examples_amd.engine.native_trainer import NativeTrainer, OptimConfig
    from dbx_distributed_pytorch_examples_amd.models import build_model
    o = OptimConfig(lr=0.05) if optim == "sgd" else OptimConfig(name="adamw", lr=1e-3, weight_decay=0.01)
    torch.manual_seed(0)
    m1 = build_model(arch, num_classes=10)
    m2 = copy.deepcopy(m1)
    engine(overlap_optimizer=-1)
    t1 = NativeTrainer(m1, batch, (size, size), dev, optim=o)
    engine(overlap_optimizer=0)
    t2 = NativeTrainer(m2, batch, (size, size), dev, optim=o)
    assert t1.opt_ranges is not None and t2.opt_ranges is None
    g = torch.Generator().manual_seed(5)
    for i in range(6):
        img = torch.randint(0, 256, (batch, size, size, 3), dtype=torch.uint8, generator=g).to(dev)
        lab = torch.randint(0, 10, (batch,), generator=g).to(dev)
        t1.step(img, lab)
        t2.step(img, lab)
        assert t1.read_metrics()[0] == t2.read_metrics()[0], i
    torch.cuda.synchronize()
    assert torch.equal(t1.prog.master, t2.prog.master) and torch.equal(t1.mom, t2.mom)
