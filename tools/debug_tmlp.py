import torch as th, numpy as np, sys
sys.path.insert(0, '.')
from imitation_amd.ops import mlp as M
dev = th.device('cuda')
def run(dims, act, B, norm=False):
    g = th.Generator().manual_seed(0)
    ws = [(th.randn(dims[i+1], dims[i], generator=g)/np.sqrt(dims[i])).to(dev).requires_grad_(True) for i in range(len(dims)-1)]
    bs = [(0.1*th.randn(dims[i+1], generator=g)).to(dev).requires_grad_(True) for i in range(len(dims)-1)]
    x = th.randn(B, dims[0], device=dev).mul_(2.0).add_(0.5).requires_grad_(True)
    y = M.tmlp(x, ws, bs, act, 0)
    wr = [w.detach().clone().requires_grad_(True) for w in ws]; br = [b.detach().clone().requires_grad_(True) for b in bs]
    xr = x.detach().clone().requires_grad_(True)
    yr = M.tmlp_reference(xr, wr, br, act, 0)
    gy = th.randn_like(y)
    (y*gy).sum().backward(); (yr*gy).sum().backward()
    print(dims, act, B, 'y err', (y-yr).abs().max().item(), yr.abs().max().item())
    names = [f'W{i}' for i in range(len(ws))] + [f'b{i}' for i in range(len(bs))] + ['x']
    for n, a, b in zip(names, ws+bs+[x], wr+br+[xr]):
        e = (a.grad-b.grad).abs()
        print(f'  {n}: maxerr {e.max().item():.4g} ref {b.grad.abs().max().item():.4g} argmax {np.unravel_index(e.argmax().item(), e.shape)}')
for B in [16, 64, 65, 128, 16384]:
    run([23,32,32,1], 1, B)
run([17,32,32,6], 2, 64)
