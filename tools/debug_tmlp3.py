import torch as th, numpy as np, sys
sys.path.insert(0, '.')
from imitation_amd.ops import mlp as M
dev = th.device('cuda')
def run(dims, act, B, mask_rows=None, tag=''):
    g = th.Generator().manual_seed(0)
    ws = [(th.randn(dims[i+1], dims[i], generator=g)/np.sqrt(dims[i])).to(dev).requires_grad_(True) for i in range(len(dims)-1)]
    bs = [(0.1*th.randn(dims[i+1], generator=g)).to(dev).requires_grad_(True) for i in range(len(dims)-1)]
    x = th.randn(B, dims[0], generator=g).to(dev).requires_grad_(True)
    y = M.tmlp(x, ws, bs, act, 0)
    wr = [w.detach().clone().requires_grad_(True) for w in ws]; br = [b.detach().clone().requires_grad_(True) for b in bs]
    xr = x.detach().clone().requires_grad_(True)
    yr = M.tmlp_reference(xr, wr, br, act, 0)
    gy = th.randn(y.shape, generator=g).to(dev)
    if mask_rows is not None:
        m = th.zeros(B, 1, device=dev); m[mask_rows] = 1; gy = gy * m
    (y*gy).sum().backward(); (yr*gy).sum().backward()
    e = (x.grad - xr.grad).abs().max(dim=1).values / (xr.grad.abs().max() + 1e-9)
    per_wave = [round(e[i*16:(i+1)*16].max().item(), 3) for i in range((B+15)//16)]
    gb = [(b.grad - bb.grad).abs().max().item()/(bb.grad.abs().max().item()+1e-9) for b, bb in zip(bs, br)]
    gw = [(w.grad - ww.grad).abs().max().item()/(ww.grad.abs().max().item()+1e-9) for w, ww in zip(ws, wr)]
    print(tag, dims, act, B, 'xerr/wave', per_wave, 'db', [round(v,3) for v in gb], 'dW', [round(v,3) for v in gw], flush=True)
for act in [0, 1]:
    run([4,16,16,1], act, 64, tag='all')
    for k in range(4):
        run([4,16,16,1], act, 64, mask_rows=list(range(16*k, 16*k+16)), tag=f'only{k}')
run([23,32,32,1], 1, 64, tag='all')
for k in range(4):
    run([23,32,32,1], 1, 64, mask_rows=list(range(16*k, 16*k+16)), tag=f'only{k}')
run([4,16,16,16,1], 0, 64, tag='L4')
