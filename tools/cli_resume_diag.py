"""Where does a device-engine CLI resume diverge? (train_adversarial, full checkpoints every 2 rounds)

Runs: A = 8 rounds, B = 8 rounds again (run-to-run determinism), C = 4 rounds, D = resume C for 8.
Compares the full-checkpoint states field by field: A vs B at every step, C vs A at 2 / 4, D vs A
at 6 / 8. One line per differing field.

    python tools/cli_resume_diag.py [gail|airl]
"""

import glob
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch as th  # noqa: E402


def run(root, cmd, total, **kw):
    from imitation_amd.scripts.train_adversarial import train_adversarial_ex

    upd = dict(environment=dict(gym_id="seals/Hopper-v1", num_vec=8, parallel=False),
               expert=dict(policy_type="zero", loader_kwargs={}),
               rl=dict(batch_size=1024, rl_kwargs=dict(batch_size=64, n_epochs=1)), engine="device",
               algorithm_kwargs=dict(demo_batch_size=256, n_disc_updates_per_round=2), checkpoint_interval=0,
               full_checkpoint_interval=2, full_checkpoint_keep=10, total_timesteps=total * 1024, seed=0,
               logging={"log_root": root})
    upd.update(kw)
    from imitation_amd.algorithms.adversarial import common

    seen = {}
    orig = common.AdversarialTrainer.train

    def spy(self, *a, **k):
        seen.setdefault("fused", (getattr(self, "_fused_disc", None), getattr(self, "_fused_disc_why", None),
                                  type(self).__name__))
        return orig(self, *a, **k)

    common.AdversarialTrainer.train = spy
    try:
        r = train_adversarial_ex.run(cmd, named_configs=["demonstrations.fast", "policy_evaluation.fast"], config_updates=upd)
    finally:
        common.AdversarialTrainer.train = orig
    print(f"{root}: trainer {seen.get('fused')}", flush=True)
    assert r.status == "COMPLETED"
    cks = sorted(glob.glob(os.path.join(root, "**", "full_checkpoints", "ckpt-*"), recursive=True))
    return {int(os.path.basename(c)[5:]): th.load(os.path.join(c, "state.pt"), weights_only=True) for c in cks}, cks


def _trace_reward_training():
    """Print, per reward-model training call, the path taken, the dataset size, the epochs and the
    optimizer's step counter before / after."""
    from imitation_amd.algorithms import preference_comparisons as pcm

    if getattr(pcm, "_diag_traced", False):
        return
    pcm._diag_traced = True
    orig_fast, orig_fused = pcm.BasicRewardTrainer._train_fast, pcm.BasicRewardTrainer._train_fused_epochs

    def step_of(self):
        f = getattr(self.optim, "_flat", None)
        return float(f[0]["step"]) if f else None

    def fast(self, dataset, epoch_multiplier):
        s0 = step_of(self)
        r = orig_fast(self, dataset, epoch_multiplier)
        print(f"  reward _train_fast: P={len(dataset)} mult={epoch_multiplier} step {s0} -> {step_of(self)} "
              f"optim={type(self.optim).__name__}", flush=True)
        return r

    def fused(self, store, index_loader, epochs, P, dev):
        print(f"  reward fused epochs: P={P} epochs={epochs}", flush=True)
        return orig_fused(self, store, index_loader, epochs, P, dev)

    pcm.BasicRewardTrainer._train_fast = fast
    pcm.BasicRewardTrainer._train_fused_epochs = fused


def run_pref(root, iters_total=3, **kw):
    """train_preference_comparisons on the device agent (full checkpoint per iteration)."""
    from imitation_amd.scripts.train_preference_comparisons import train_preference_comparisons_ex

    _trace_reward_training()
    print(f"== run {root} {kw}", flush=True)

    upd = dict(environment=dict(gym_id="seals/Hopper-v1", num_vec=8, parallel=False),
               rl=dict(batch_size=1024, rl_kwargs=dict(batch_size=64, n_epochs=1)), engine="device",
               total_timesteps=4 * 1024, total_comparisons=16, num_iterations=iters_total, fragment_length=4,
               reward_trainer_kwargs=dict(epochs=1), checkpoint_interval=0, full_checkpoint_interval=1,
               full_checkpoint_keep=10, seed=0, logging={"log_root": root}, **kw)
    r = train_preference_comparisons_ex.run(named_configs=["fast", "rl.fast", "environment.fast", "policy_evaluation.fast"],
                                            config_updates=upd)
    assert r.status == "COMPLETED"
    cks = sorted(glob.glob(os.path.join(root, "**", "full_checkpoints", "ckpt-*"), recursive=True))
    return {int(os.path.basename(c)[5:]): th.load(os.path.join(c, "state.pt"), weights_only=True) for c in cks}, cks


def cmp(tag, a, b, path=""):
    n = 0
    if isinstance(a, th.Tensor):
        if not (isinstance(b, th.Tensor) and a.shape == b.shape and th.equal(a, b)):
            extra = f" {a.flatten()[:4].tolist()} != {b.flatten()[:4].tolist()}" if isinstance(b, th.Tensor) and a.numel() <= 4 else ""
            print(f"{tag}: DIFF {path}{extra}", flush=True)
            return 1
        return 0
    if isinstance(a, dict):
        for k in a:
            n += cmp(tag, a[k], b.get(k) if isinstance(b, dict) else None, f"{path}.{k}")
        return n
    if isinstance(a, (list, tuple)):
        for i, (x, y) in enumerate(zip(a, b)):
            n += cmp(tag, x, y, f"{path}[{i}]")
        return n
    if a != b:
        print(f"{tag}: DIFF {path} {str(a)[:60]} != {str(b)[:60]}", flush=True)
        return 1
    return 0


def final_params(root):
    """The final reward_train.pt state and the generator's policy parameters of a run."""
    from imitation_amd.rewards import serialize as reward_serialize
    from imitation_amd.rl.save_util import load_from_zip_file

    (rew,) = glob.glob(os.path.join(root, "**", "checkpoints", "final", "reward_train.pt"), recursive=True)
    out = {"reward": reward_serialize.load_reward_net(rew, device="cpu").state_dict()}
    (zp,) = glob.glob(os.path.join(root, "**", "checkpoints", "final", "gen_policy", "model.zip"), recursive=True)
    out["gen"] = load_from_zip_file(zp, device="cpu")[1]
    return out


def chunk_check(tmp, cmd):
    """Does chunking train() at the full-checkpoint interval (or the saving itself) change an
    uninterrupted run? E: one train() call; A: interval 2 with saves; F: interval 2, saves skipped."""
    from imitation_amd.utils import checkpoint

    run(os.path.join(tmp, "E"), cmd, 8, full_checkpoint_interval=0)
    run(os.path.join(tmp, "A"), cmd, 8)
    orig = checkpoint.CheckpointManager.save
    checkpoint.CheckpointManager.save = lambda self, *a, **k: None
    try:
        run(os.path.join(tmp, "F"), cmd, 8)
    finally:
        checkpoint.CheckpointManager.save = orig
    E, A, F = (final_params(os.path.join(tmp, x)) for x in "EAF")
    print(f"{cmd}: E (one call) vs A (chunks + saves): {cmp('E/A', E, A)} differing fields", flush=True)
    print(f"{cmd}: E (one call) vs F (chunks, no saves): {cmp('E/F', E, F)} differing fields", flush=True)


def main():
    cmd = sys.argv[1] if len(sys.argv) > 1 else "gail"
    if "--deterministic" in sys.argv:
        from imitation_amd.utils import determinism

        determinism.set_deterministic(True)
        print("torch deterministic algorithms on", flush=True)
    tmp = tempfile.mkdtemp()
    os.chdir(tmp)
    if cmd == "pref":
        A, _ = run_pref(os.path.join(tmp, "A"))
        B, _ = run_pref(os.path.join(tmp, "B"))
        for s in sorted(A):
            print(f"pref A vs B iteration {s}: {cmp(f'A/B@{s}', A[s], B[s])} differing fields", flush=True)
        import shutil

        _, cks = run_pref(os.path.join(tmp, "C0"))
        ck2 = [c for c in cks if c.endswith("ckpt-0000000002")][0]
        killed = os.path.join(tmp, "killed")
        shutil.copytree(ck2, os.path.join(killed, os.path.basename(ck2)))
        D, _ = run_pref(os.path.join(tmp, "D"), resume_from=killed)
        for s in sorted(D):
            print(f"pref D (resumed after 2) vs A iteration {s}: {cmp(f'D/A@{s}', D[s], A[s])} differing fields",
                  flush=True)
        return
    if "--chunks" in sys.argv:
        chunk_check(tmp, cmd)
        return
    A, _ = run(os.path.join(tmp, "A"), cmd, 8)
    B, _ = run(os.path.join(tmp, "B"), cmd, 8)
    for s in sorted(A):
        print(f"A vs B step {s}: {cmp(f'A/B@{s}', A[s], B[s])} differing fields", flush=True)
    C, ck = run(os.path.join(tmp, "C"), cmd, 4)
    for s in sorted(C):
        print(f"C vs A step {s}: {cmp(f'C/A@{s}', C[s], A[s])} differing fields", flush=True)
    D, _ = run(os.path.join(tmp, "D"), cmd, 8, resume_from=os.path.dirname(ck[-1]))
    for s in sorted(D):
        print(f"D vs A step {s}: {cmp(f'D/A@{s}', D[s], A[s])} differing fields", flush=True)


if __name__ == "__main__":
    main()
