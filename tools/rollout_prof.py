import os, sys, time, numpy as np, torch as th
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.engine.test_device_engine import _setup
tr, venv, gen, rn = _setup(n_envs=8, n_steps=512, batch=64, n_epochs=5)
prof = th.zeros(8, 4, dtype=th.int64, device='cuda')
pprof = th.zeros(16, dtype=th.int64, device='cuda')
orig = tr._C.engine_rollout
orig2 = tr._C.engine_ppo_update
def wrapped(d):
    d['prof'] = prof
    return orig(d)
def wrapped2(d):
    d['prof'] = pprof
    return orig2(d)
tr._C.engine_rollout = wrapped
tr._C.engine_ppo_update = wrapped2
for i in range(3):
    th.cuda.synchronize(); t = time.perf_counter(); tr._rollout(); th.cuda.synchronize(); dt = time.perf_counter() - t
    p = prof.cpu().numpy().astype(np.float64)
    print(f'rollout {dt*1e3:.2f} ms; cycles/step per env: policy {p[:,0].mean()/512:.0f} env {p[:,1].mean()/512:.0f} reward {p[:,2].mean()/512:.0f} total {p[:,3].mean()/512:.0f}', flush=True)
for allow_rc in (1, 0):
    tr._ppo_static['allow_rc'] = allow_rc
    path = tr._C.engine_ppo_path(tr._ppo_static)
    names = ['fwd+loss+bwd', 'dW+exchange', 'adam'] if path.startswith('rc') else ['rows', 'prep', 'fwd', 'loss', 'bwd', 'adam']
    for i in range(3):
        pprof.zero_()
        th.cuda.synchronize(); t = time.perf_counter(); tr._ppo_update(); th.cuda.synchronize(); dt = time.perf_counter() - t
        pp = pprof.cpu().numpy() / 320
        print(f'ppo update [{path}] {dt*1e3:.2f} ms; cycles/minibatch: ' + ' '.join(f'{n}={v:.0f}' for n, v in zip(names, pp)), flush=True)
        if path.startswith('rc'):
            print('   actor wave: rows %.0f fwd %.0f loss %.0f bwd %.0f | critic wave: rows %.0f fwd %.0f loss %.0f bwd %.0f' % tuple(pp[3:11]), flush=True)
tr._ppo_static['allow_rc'] = 1
tr._ep_lens_running[:] = 0
