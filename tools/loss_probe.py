import sys, os, math, torch
sys.path.insert(0, '/root/repo')
from dbx_distributed_pytorch_examples_amd.engine.native_trainer import NativeTrainer, OptimConfig
from dbx_distributed_pytorch_examples_amd.models import build_model
from dbx_distributed_pytorch_examples_amd.ops import kernels as K
dev=torch.device('cuda')
for patch in (1, 0):
    os.environ["DBX_ENGINE"] = f"patch3={'all' if patch else '0'},stem_patch={int(patch)}"
    for lr, steps in ((0.05, 80), (0.02, 50), (0.1, 50)):
        torch.manual_seed(0)
        model=build_model('resnet50', num_classes=1000)
        tr=NativeTrainer(model,16,(224,224),dev,optim=OptimConfig(name='sgd',lr=lr,weight_decay=0.0),use_graphs=True)
        g=torch.Generator().manual_seed(3)
        img=torch.randint(0,256,(16,224,224,3),dtype=torch.uint8,generator=g).to(dev)
        lab=torch.randint(0,1000,(16,),generator=g).to(dev)
        L=[]
        for _ in range(steps):
            tr.step(img,lab); L.append(tr.read_metrics()[0]/16)
        print(f"patch={patch} lr={lr} steps={steps}: " + " ".join(f"{v:.2f}" for v in L[::8]) + f" | last3 {sum(L[-3:])/3:.3f} first3 {sum(L[:3])/3:.3f}", flush=True)
