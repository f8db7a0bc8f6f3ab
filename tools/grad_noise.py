"""Per-parameter gradient agreement of one native step against two autograd references -- plain fp32
and a reference that rounds to bf16 where the program stores bf16 (tests/test_program_gpu.py) -- so a
low native-vs-reference cosine can be read against the rounding noise floor (fp32 vs bf16-emulating).

usage: python tools/grad_noise.py ARCH SIZE BATCH [DAMP]
"""
import copy
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from dbx_distributed_pytorch_examples_amd.engine.native_trainer import NativeTrainer, OptimConfig  # noqa: E402
from dbx_distributed_pytorch_examples_amd.models import build_model  # noqa: E402
from test_program_gpu import _bf16_emulating, _cos  # noqa: E402

dev = torch.device("cuda")
arch, size, batch = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
damp = float(sys.argv[4]) if len(sys.argv) > 4 else 0.2
torch.manual_seed(0)
model = build_model(arch, num_classes=100)
for n_, m_ in model.named_modules():
    if n_.endswith("bn3") or (n_.endswith("bn2") and "layer" in n_ and arch != "resnet50"):
        torch.nn.init.constant_(m_.weight, damp)
ref32 = copy.deepcopy(model).to(dev).train()
ref16 = _bf16_emulating(copy.deepcopy(model).to(dev).train())
tr = NativeTrainer(model, batch, (size, size), dev, optim=OptimConfig(lr=0.0, momentum=0.0, weight_decay=0.0),
                   use_graphs=False)
p = tr.prog
g = torch.Generator().manual_seed(1)
img = torch.randint(0, 256, (batch, size, size, 3), dtype=torch.uint8, generator=g).to(dev)
lab = torch.randint(0, p.num_classes, (batch,), generator=g).to(dev)
tr.step(img, lab)
torch.cuda.synchronize()
x = p.x4[..., :3].float().permute(0, 3, 1, 2).contiguous()
for r in (ref32, ref16):
    F.cross_entropy(r(x), lab).backward()
n32, n16 = dict(ref32.named_parameters()), dict(ref16.named_parameters())
rows = []
for name, prm in model.named_parameters():
    off = (prm.data_ptr() - p.master.data_ptr()) // 4
    gf = p.grad[off:off + prm.numel()]
    gn = gf.view(prm.shape[0], prm.shape[2], prm.shape[3], prm.shape[1]).permute(0, 3, 1, 2) if prm.dim() == 4 \
        else gf.view(prm.shape)
    rows.append((name, _cos(gn, n16[name].grad), _cos(gn, n32[name].grad), _cos(n32[name].grad, n16[name].grad),
                 (n16[name].grad.sum() / (n16[name].grad.abs().sum() + 1e-30)).item()))
rows.sort(key=lambda r: r[1])
print(f"[grad-noise] {arch} {size} b{batch} damp {damp}: native-vs-emu, native-vs-fp32, fp32-vs-emu, sum/abs")
for r in rows[:12]:
    print(f"  {r[0]:32s} {r[1]:.4f} {r[2]:.4f} {r[3]:.4f} {r[4]:+.3f}")
print(f"  median native-vs-emu {sorted(r[1] for r in rows)[len(rows) // 2]:.4f}  "
      f"worst fp32-vs-emu {min(r[3] for r in rows):.4f}")
