"""The rollout chain's phase-clock instance (``prof``, rollout.hip ``PROF = true``) and its LDS
split-form actor (``lds_actor``, the form before the row form) compute exactly what the production
instance does: same env state in, bitwise the same transitions out, plus the per-phase cycle
counters (tools/rollout_breakdown.py reads them)."""

import pytest
import torch as th


@pytest.mark.gpu
def test_phase_clock_instance_is_bitwise_the_production_chain():
    from imitation_amd import models

    b = models.build("gail_halfcheetah", device="cuda", env_id="HalfCheetah-v4")
    tr = b.trainer
    tr.train(tr.gen_train_timesteps)
    keys = ("state", "env_rng", "elapsed", "ep_ret", "cur_obs", "cur_start")
    snap = {k: getattr(tr, k).clone() for k in keys}
    step0 = tr._step0

    def run(prof, lds_actor=0):
        for k in keys:
            getattr(tr, k).copy_(snap[k])
        tr._step0 = step0
        C = tr._C

        class P:
            def __getattr__(self, k):
                return getattr(C, k)

            def engine_rollout(self, d):
                return C.engine_rollout(dict(d, prof=prof, lds_actor=lds_actor))

        tr._C = P()
        try:
            tr._launch_chain()
        finally:
            tr._C = C
        th.cuda.synchronize()
        return {k: tr.buf[k].clone() for k in tr._CHAIN_OUT}, {k: getattr(tr, k).clone() for k in keys}

    ref, ref_state = run(None)
    assert ref["obs_buf"].abs().sum() > 0 and ref["act_raw"].abs().sum() > 0
    for prof_on, lds_actor in ((True, 0), (False, 1), (True, 1)):
        prof = th.zeros(tr.N, 5, dtype=th.int64, device="cuda") if prof_on else None
        got, got_state = run(prof, lds_actor)
        for k in ref:
            assert th.equal(ref[k], got[k]), (k, prof_on, lds_actor)
        for k in ref_state:
            assert th.equal(ref_state[k], got_state[k]), (k, prof_on, lds_actor)
        if prof_on:
            p = prof.cpu()
            assert (p[:, 4] == tr.T).all()
            assert (p[:, :4] > 0).all()
