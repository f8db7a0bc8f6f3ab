"""Per-parameter gradient agreement of the native program vs fp32 autograd (debug aid)."""
import copy, sys, os, torch, torch.nn.functional as F
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dbx_distributed_pytorch_examples_amd.engine.native_trainer import NativeTrainer, OptimConfig
from dbx_distributed_pytorch_examples_amd.models import build_model
dev = torch.device(sys.argv[1] if len(sys.argv) > 1 else "cuda")
arch, size, batch = (sys.argv[2], int(sys.argv[3]), int(sys.argv[4])) if len(sys.argv) > 4 else ("resnet50", 64, 8)
torch.manual_seed(0)
model = build_model(arch, num_classes=100)
import os as _os
if _os.environ.get("DAMP"):
    for _n, _m in model.named_modules():
        if _n.endswith("bn3") or (_n.endswith("bn2") and arch != "resnet50"):
            torch.nn.init.constant_(_m.weight, float(_os.environ["DAMP"]))
ref = copy.deepcopy(model).to(dev).train()
tr = NativeTrainer(model, batch, (size, size), dev, optim=OptimConfig(lr=0.0, momentum=0.0, weight_decay=0.0), use_graphs=False)
p = tr.prog
g = torch.Generator().manual_seed(1)
img = torch.randint(0, 256, (batch, size, size, 3), dtype=torch.uint8, generator=g).to(dev)
lab = torch.randint(0, 100, (batch,), generator=g).to(dev)
tr.step(img, lab)
x = p.x4[..., :3].float().permute(0, 3, 1, 2).contiguous()
loss = F.cross_entropy(ref(x), lab); loss.backward()
print("loss", p.metrics[0].item() / batch, loss.item())
nr = dict(ref.named_parameters())
for name, prm in model.named_parameters():
    off = (prm.data_ptr() - p.master.data_ptr()) // 4; n = prm.numel()
    gf = p.grad[off:off + n]
    gn = gf.view(prm.shape[0], prm.shape[2], prm.shape[3], prm.shape[1]).permute(0, 3, 1, 2) if prm.dim() == 4 else gf.view(prm.shape)
    a = gn.flatten().float(); b = nr[name].grad.flatten().float()
    c = (a @ b / (a.norm() * b.norm() + 1e-20)).item()
    print(f"{name:40s} cos {c:8.4f} |n| {a.norm().item():10.4e} |r| {b.norm().item():10.4e}")
