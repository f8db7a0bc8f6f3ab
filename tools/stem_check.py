import torch, torch.nn.functional as F, sys
sys.path.insert(0, '/root/repo')
from dbx_distributed_pytorch_examples_amd.ops import kernels as k
dev='cuda'
torch.manual_seed(10)
N,H,W=2,224,224
img=torch.randn(N,H,W,3,device=dev)
x4=torch.zeros(N,H,W,4,device=dev); x4[...,:3]=img; x4=x4.bfloat16()
w=torch.randn(64,7,7,3,device=dev)*0.05
ws_=torch.zeros(64,8,8,4,device=dev); ws_[:,:7,:7,:3]=w
w16s=ws_.bfloat16().view(64,256)
OH,OW=k.conv_out_hw(H,W,7,7,2,3)
ref=F.conv2d(x4[...,:3].float().permute(0,3,1,2), ws_.bfloat16().float()[:,:7,:7,:3].permute(0,3,1,2), stride=2, padding=3).permute(0,2,3,1)
for patch in (True, False):
    out=torch.empty(N,OH,OW,64,device=dev,dtype=torch.bfloat16)
    k.conv_stem_fwd(x4,w16s,out,patch=patch)
    torch.cuda.synchronize()
    rb=ref.bfloat16().float()
    d=(out.float()-rb).abs()
    ulp=(rb.abs()*2**-7).clamp_min(1e-30)
    frac=(d>ulp*1.01).float().mean().item()
    print('patch' if patch else 'igemm', 'max abs', d.max().item(), 'frac > 1ulp', frac, 'frac !=', (d>0).float().mean().item())
    # where are the worst errors
    idx=torch.nonzero(d > 4*ulp)
    print('  count >4ulp', idx.shape[0], idx[:5].tolist())
