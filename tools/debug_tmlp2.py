import torch as th, numpy as np, sys
sys.path.insert(0, '.')
from imitation_amd.ops import mlp as M
dev = th.device('cuda')
def run(dims, act, B):
    g = th.Generator().manual_seed(0)
    ws = [(th.randn(dims[i+1], dims[i], generator=g)/np.sqrt(dims[i])).to(dev).requires_grad_(True) for i in range(len(dims)-1)]
    bs = [(0.1*th.randn(dims[i+1], generator=g)).to(dev).requires_grad_(True) for i in range(len(dims)-1)]
    x = th.randn(B, dims[0], generator=g).to(dev).requires_grad_(True)
    y = M.tmlp(x, ws, bs, act, 0)
    wr = [w.detach().clone().requires_grad_(True) for w in ws]; br = [b.detach().clone().requires_grad_(True) for b in bs]
    xr = x.detach().clone().requires_grad_(True)
    yr = M.tmlp_reference(xr, wr, br, act, 0)
    gy = th.randn(y.shape, generator=g).to(dev)
    (y*gy).sum().backward(); (yr*gy).sum().backward()
    names = [f'W{i}' for i in range(len(ws))] + [f'b{i}' for i in range(len(bs))] + ['x']
    out = []
    for n, a, b in zip(names, ws+bs+[x], wr+br+[xr]):
        e = (a.grad-b.grad).abs().max().item() / (b.grad.abs().max().item()+1e-6)
        out.append(f'{n}:{e:.3f}')
    if 'x' in names:
        e = (x.grad - xr.grad).abs().max(dim=1).values
        bad = th.nonzero(e > 0.05 * xr.grad.abs().max()).flatten().tolist()
        out.append(f'badrows:{bad[:20]}')
    print(dims, act, B, ' '.join(out), flush=True)
for dims in [[4,1],[4,16,1],[4,16,16,1],[32,32,1]]:
    for act in [0,1]:
        for B in [16,32,48,64]:
            run(dims, act, B)
