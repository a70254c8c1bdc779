"""Per-step phase breakdown of the bench's rollout chain.

Runs the bench trainer (``gail_halfcheetah``) and, for a few rounds, launches the rollout chain's
phase-clock instance (``prof`` argument, rollout.hip ``PROF = true``): every wave accumulates the
core-clock cycles of each step phase -- actor + sampling, env physics, observation, step tail.
Prints cycles / step per phase, their shares, and the chain kernel's time with and without the
stamps (events around the launch; the stamps' own cost shows as the difference), for the
production row-form actor and the LDS split form it replaced (``lds_actor``).

    python tools/rollout_breakdown.py
"""

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PHASES = ("actor_sampling", "physics", "observation", "tail")


class _Proxy:
    def __init__(self, C):
        self._C = C
        self.prof = None
        self.lds_actor = 0

    def __getattr__(self, k):
        return getattr(self._C, k)

    def engine_rollout(self, d):
        return self._C.engine_rollout(dict(d, prof=self.prof, lds_actor=self.lds_actor))


def main():
    import torch as th

    from imitation_amd import models

    b = models.build("gail_halfcheetah", device="cuda", env_id="HalfCheetah-v4")
    tr = b.trainer
    spr = tr.gen_train_timesteps
    tr.train(3 * spr)
    eng = tr
    px = _Proxy(eng._C)
    eng._C = px
    N, T = eng.N, eng.T
    for form in ("row", "lds"):
        px.lds_actor = int(form == "lds")
        measure(eng, px, N, T, form)


def measure(eng, px, N, T, form):
    import torch as th

    res = {"actor_form": form, "N": N, "T": T}
    for mode in ("plain", "stamped", "plain"):
        px.prof = th.zeros(N, 5, dtype=th.int64, device="cuda") if mode == "stamped" else None
        times = []
        for _ in range(10):
            e0, e1 = th.cuda.Event(enable_timing=True), th.cuda.Event(enable_timing=True)
            e0.record()
            eng._launch_chain()
            e1.record()
            th.cuda.synchronize()
            times.append(e0.elapsed_time(e1) * 1000)
        times.sort()
        res.setdefault(f"chain_us_{mode}", []).append(times[len(times) // 2])
        if mode == "stamped":
            p = px.prof.cpu().double()
            steps = p[:, 4]
            per = (p[:, :4] / steps[:, None]).mean(0)
            tot = float(per.sum())
            res["cycles_per_step"] = {k: round(float(v), 1) for k, v in zip(PHASES, per)}
            res["share"] = {k: round(float(v) / tot, 3) for k, v in zip(PHASES, per)}
            res["cycles_per_step_total"] = round(tot, 1)
            res["steps_per_wave"] = int(steps[0])
    res["us_per_step_plain"] = round(min(res["chain_us_plain"]) / T, 3)
    res["us_per_step_stamped"] = round(res["chain_us_stamped"][0] / T, 3)
    res["implied_clock_ghz_stamped"] = round(res["cycles_per_step_total"] / (res["us_per_step_stamped"] * 1000), 3)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
