import copy, torch, torch.nn.functional as F, sys
sys.path.insert(0, "/root/repo")
from dbx_distributed_pytorch_examples_amd.engine.native_trainer import NativeTrainer, OptimConfig
from dbx_distributed_pytorch_examples_amd.models import build_model
torch.manual_seed(0)
size, batch = 32, 32
m1 = build_model("resnet18", num_classes=10)
ref = copy.deepcopy(m1)
dev = torch.device(sys.argv[1] if len(sys.argv) > 1 else "cpu")
t1 = NativeTrainer(m1, batch, (size, size), dev, optim=OptimConfig(lr=0.05), use_graphs=False)
ref = ref.to(dev)
opt = torch.optim.SGD(ref.parameters(), lr=0.05, momentum=0.9, weight_decay=5e-5)
g = torch.Generator().manual_seed(2)
img = torch.randint(0, 256, (batch, size, size, 3), dtype=torch.uint8, generator=g).to(dev)
lab = torch.randint(0, 10, (batch,), generator=g).to(dev)
for i in range(8):
    t1.step(img, lab)
    l1, _ = t1.read_metrics()
    x = t1.prog.x4[..., :3].float().permute(0, 3, 1, 2).contiguous()
    loss = F.cross_entropy(ref(x), lab); opt.zero_grad(); loss.backward(); opt.step()
    print(i, l1 / batch, loss.item())
