"""Tune edge cases (reference test models: python/ray/tune/tests/test_tuner.py (grid x num_samples
expansion, ResultGrid errors / best result), test_api.py (stop criteria, max_concurrent_trials),
test_sample.py (seeded sampling domains))."""
import pytest

import ray_community_amd as ray
from ray_community_amd import tune
from ray_community_amd.train import RunConfig


@pytest.fixture(scope="module")
def session():
    ray.init(num_cpus=4)
    yield
    ray.shutdown()


def _quadratic(config):
    for i in range(5):
        tune.report({"score": -(config["x"] - 3) ** 2 - i * 0.01, "it": i})


def test_grid_times_samples_expansion_and_best(session, tmp_path):
    tuner = tune.Tuner(_quadratic,
                       param_space={"x": tune.grid_search([1, 2, 3, 4]), "y": tune.uniform(0, 1)},
                       tune_config=tune.TuneConfig(num_samples=2, metric="score", mode="max"),
                       run_config=RunConfig(storage_path=str(tmp_path), name="grid"))
    grid = tuner.fit()
    assert len(grid) == 8                                 # 4 grid points x 2 samples
    xs = sorted(r.config["x"] for r in grid)
    assert xs == [1, 1, 2, 2, 3, 3, 4, 4]
    best = grid.get_best_result()
    assert best.config["x"] == 3
    assert grid.get_best_result(metric="score", mode="min").config["x"] in (1,)
    assert not grid.errors


def test_trial_errors_are_collected(session, tmp_path):
    def sometimes(config):
        if config["x"] == 2:
            raise ValueError("bad x")
        tune.report({"v": config["x"]})

    grid = tune.Tuner(sometimes, param_space={"x": tune.grid_search([1, 2, 3])},
                      run_config=RunConfig(storage_path=str(tmp_path), name="errs")).fit()
    assert len(grid) == 3 and len(grid.errors) == 1
    assert "bad x" in str(grid.errors[0])
    ok = sorted(r.metrics["v"] for r in grid if r.error is None)
    assert ok == [1, 3]


def test_stop_criteria_dict(session, tmp_path):
    def forever(config):
        i = 0
        while True:
            tune.report({"it": i})
            i += 1

    grid = tune.Tuner(forever, param_space={},
                      run_config=RunConfig(storage_path=str(tmp_path), name="stop", stop={"it": 4})).fit()
    assert grid[0].metrics["it"] == 4


def test_seeded_search_space_is_reproducible(session, tmp_path):
    def echo(config):
        tune.report({"a": config["a"], "b": config["b"]})

    def run(name):
        space = {"a": tune.uniform(-1, 1), "b": tune.choice(["p", "q", "r"])}
        from ray_community_amd.tune.search import BasicVariantGenerator

        g = tune.Tuner(echo, param_space=space,
                       tune_config=tune.TuneConfig(num_samples=5, search_alg=BasicVariantGenerator(random_state=123)),
                       run_config=RunConfig(storage_path=str(tmp_path), name=name)).fit()
        return sorted((r.metrics["a"], r.metrics["b"]) for r in g)

    first, second = run("s1"), run("s2")
    assert first == second
    assert all(-1 <= a <= 1 and b in "pqr" for a, b in first)
