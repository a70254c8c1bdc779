"""Trial parallelism pins GPUs correctly: every trial is a fresh process
started with a free slot's ``HIP_VISIBLE_DEVICES``, and no slot ever hosts two running trials
(reference: Ray Tune per-trial GPU resources, ``src/imitation/scripts/parallel.py:114-148``)."""

from imitation_amd.scripts import parallel

FAKE = "imitation_amd.testing.distributed:fake_gpu_trial"


def test_trials_never_share_a_slot_and_run_in_fresh_processes(tmp_path):
    slots = ["0,1", "2,3"]
    # unequal durations: completion order differs from submission order
    trials = [dict(config_updates={"sleep": s}) for s in (0.6, 0.1, 0.3, 0.1, 0.4, 0.2)]
    recs = parallel.run_trials(FAKE, trials, str(tmp_path), "t", {"gpu": 2}, gpu_slots=slots)
    assert len(recs) == 6 and all(r["status"] == "COMPLETED" for r in recs)
    res = [r["result"] for r in recs]
    assert all(r["hip"] in slots for r in res)
    assert len({r["pid"] for r in res}) == 6  # one fresh process per trial
    for slot in slots:
        iv = sorted((r["t0"], r["t1"]) for r in res if r["hip"] == slot)
        assert all(a[1] <= b[0] for a, b in zip(iv, iv[1:])), f"slot {slot} held by two running trials: {iv}"
    # both slots were used (process start-up time under load decides how much they overlap)
    assert {r["hip"] for r in res} == set(slots)
    assert all(r["metric"] == 1.0 for r in recs)


def test_failed_trial_frees_its_slot(tmp_path):
    trials = [dict(config_updates={"sleep": 0.05, "fail": i == 1}) for i in range(4)]
    recs = parallel.run_trials(FAKE, trials, str(tmp_path), "t", {"gpu": 1}, gpu_slots=["0"])
    assert [r["status"] for r in recs] == ["COMPLETED", "FAILED", "COMPLETED", "COMPLETED"]
    assert "failed on purpose" in recs[1]["error"]
