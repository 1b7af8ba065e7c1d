"""Synchronous HyperBand, BOHB, PBT policy logs + replay and ResourceChangingScheduler restarts
(reference: tune/tests/test_trial_scheduler.py HyperBand tests, test_trial_scheduler_pbt.py
replay tests, test_resource_changing_scheduler.py)."""
import json
import os
import tempfile

import pytest

import ray_community_amd as ray
from ray_community_amd import tune
from ray_community_amd.train import Checkpoint, RunConfig


@pytest.fixture(scope="module")
def ray4():
    ray.init(num_cpus=4, include_dashboard=False, log_to_driver=False)
    yield
    ray.shutdown()


def _ckpt_trainable(config):
    """Reports q * iteration; checkpoints every step so paused trials resume where they were."""
    start = 0
    ck = tune.get_checkpoint()
    if ck:
        start = int(open(os.path.join(ck.path, "it")).read())
    for it in range(start + 1, 30):
        with tempfile.TemporaryDirectory() as d:
            open(os.path.join(d, "it"), "w").write(str(it))
            tune.report({"acc": config["q"] * it, "it": it}, checkpoint=Checkpoint.from_directory(d))


def test_sync_hyperband_halving(ray4, tmp_path):
    hb = tune.schedulers.HyperBandScheduler(metric="acc", mode="max", max_t=9, reduction_factor=3)
    assert hb.s_max == 2
    qs = [0.1 * (i + 1) for i in range(9)]
    grid = tune.Tuner(_ckpt_trainable, param_space={"q": tune.grid_search(qs)},
                      tune_config=tune.TuneConfig(scheduler=hb, max_concurrent_trials=4),
                      run_config=RunConfig(storage_path=str(tmp_path))).fit()
    assert grid.num_errors == 0
    # one bracket of n=9 trials at milestone 1: keep 3, then 1 at milestone 3, which runs to max_t
    assert [(m, len(k), len(c)) for _, m, k, c in hb.decisions] == [(1.0, 3, 6), (3.0, 1, 2)]
    its = {round(r.config["q"], 1): r.metrics["it"] for r in grid}
    assert its[0.9] == 9
    assert sorted(its.values()) == [1] * 6 + [3, 3, 9]
    # resumed trials continued from their checkpoint, not from iteration 1
    best = next(r for r in grid if round(r.config["q"], 1) == 0.9)
    assert [m["it"] for m in best.metrics_history] == list(range(1, 10))


def test_bohb_models_largest_budget(ray4, tmp_path):
    from ray_community_amd.tune.search import TuneBOHB

    def f(config):
        for it in range(1, 10):
            tune.report({"loss": (config["x"] - 2.0) ** 2 / it})

    bohb = TuneBOHB(metric="loss", mode="min", seed=0, min_points_in_model=3, random_fraction=0.0)
    hb = tune.schedulers.HyperBandForBOHB(metric="loss", mode="min", max_t=9, reduction_factor=3)
    grid = tune.Tuner(f, param_space={"x": tune.uniform(-5, 5)},
                      tune_config=tune.TuneConfig(search_alg=bohb, scheduler=hb, num_samples=14,
                                                  max_concurrent_trials=3),
                      run_config=RunConfig(storage_path=str(tmp_path))).fit()
    assert grid.num_errors == 0 and len(grid) == 14
    modelled = [b for b in bohb.model_budgets if b is not None]
    assert modelled, "BOHB never fitted a model"
    assert max(modelled) >= 2.0  # it moved to a larger budget once one had enough observations
    assert abs(grid.get_best_result("loss", "min").config["x"] - 2.0) < 1.5


def _pbt_trainable(config):
    v = 0.0
    ck = tune.get_checkpoint()
    if ck:
        v = float(open(os.path.join(ck.path, "v")).read())
    for _ in range(12):
        v += config["lr"]
        with tempfile.TemporaryDirectory() as d:
            open(os.path.join(d, "v"), "w").write(str(v))
            tune.report({"v": v, "lr": config["lr"]}, checkpoint=Checkpoint.from_directory(d))


def test_pbt_policy_log_and_replay(ray4, tmp_path):
    pbt = tune.PopulationBasedTraining(metric="v", mode="max", perturbation_interval=3,
                                       hyperparam_mutations={"lr": tune.uniform(0.0, 1.0)}, seed=0)
    grid = tune.Tuner(_pbt_trainable, param_space={"lr": tune.grid_search([0.01, 0.02, 0.5, 1.0])},
                      tune_config=tune.TuneConfig(scheduler=pbt, max_concurrent_trials=4),
                      run_config=RunConfig(name="pbt", storage_path=str(tmp_path))).fit()
    assert pbt.num_perturbations > 0
    logs = [p for p in os.listdir(tmp_path / "pbt") if p.startswith("pbt_policy_")]
    assert logs
    policy = str(tmp_path / "pbt" / logs[0])
    rows = [json.loads(l) for l in open(policy)]
    assert all(len(r) == 6 and "lr" in r[5] for r in rows)

    replay = tune.schedulers.PopulationBasedTrainingReplay(policy)
    g2 = tune.Tuner(_pbt_trainable, param_space={"lr": 0.0},
                    tune_config=tune.TuneConfig(scheduler=replay),
                    run_config=RunConfig(name="replay", storage_path=str(tmp_path))).fit()
    assert g2.num_errors == 0
    assert len(replay.applied) == len(rows)
    hist = g2[0].metrics_history
    assert hist[0]["lr"] == pytest.approx(rows[0][4]["lr"])  # starts from the first logged config
    assert hist[-1]["lr"] == pytest.approx(rows[-1][5]["lr"])  # ends on the last change


def _res_trainable(config):
    start = 0
    ck = tune.get_checkpoint()
    if ck:
        start = int(open(os.path.join(ck.path, "it")).read())
    for it in range(start + 1, 5):
        cpus = ray.get_runtime_context().get_assigned_resources().get("CPU", 0)
        with tempfile.TemporaryDirectory() as d:
            open(os.path.join(d, "it"), "w").write(str(it))
            tune.report({"it": it, "cpus": cpus}, checkpoint=Checkpoint.from_directory(d))


def test_resource_changing_scheduler_restarts_with_new_resources(ray4, tmp_path):
    from ray_community_amd.tune.schedulers import FIFOScheduler, ResourceChangingScheduler

    def alloc(controller, trial, result, scheduler):
        return {"CPU": 2} if result.get("training_iteration", 0) >= 2 else None

    sched = ResourceChangingScheduler(FIFOScheduler(), resources_allocation_function=alloc)
    grid = tune.Tuner(_res_trainable, param_space={"x": tune.grid_search([1, 2])},
                      tune_config=tune.TuneConfig(scheduler=sched),
                      run_config=RunConfig(storage_path=str(tmp_path))).fit()
    assert grid.num_errors == 0
    for r in grid:
        hist = r.metrics_history
        assert [m["it"] for m in hist] == [1, 2, 3, 4]  # resumed from the checkpoint
        assert hist[0]["cpus"] == 1 and hist[-1]["cpus"] == 2  # the new trial actor is bigger
    assert len(sched.changes) == 2
