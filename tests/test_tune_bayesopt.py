"""BayesOptSearch (reference: python/ray/tune/search/bayesopt/bayesopt_search.py; reference test
python/ray/tune/tests/test_searchers.py::testBayesOpt): a native GP searcher over continuous
spaces -- random warm-up, then acquisition-driven suggestions that home in on the optimum."""
import numpy as np
import pytest

import ray_community_amd as ray
from ray_community_amd import tune
from ray_community_amd.tune.registry import create_searcher
from ray_community_amd.tune.search import Searcher
from ray_community_amd.tune.search.bayesopt import BayesOptSearch


def _drive(s, f, n):
    best = None
    for i in range(n):
        cfg = s.suggest(f"t{i}")
        if cfg is None or cfg == Searcher.FINISHED:
            continue
        v = f(cfg)
        s.on_trial_complete(f"t{i}", {"loss": v})
        best = v if best is None else min(best, v)
    return best


@pytest.mark.parametrize("kind", ["ucb", "ei", "poi"])
def test_converges_on_a_quadratic_faster_than_random(kind):
    f = lambda c: (c["x"] - 0.3) ** 2 + (c["nested"]["y"] + 1.2) ** 2  # noqa: E731
    space = {"x": (-2.0, 2.0), "nested": {"y": tune.uniform(-2.0, 2.0)}, "fixed": 7}
    s = BayesOptSearch(space, metric="loss", mode="min", random_search_steps=5, random_state=0,
                       utility_kwargs={"kind": kind, "kappa": 1.0, "xi": 0.01}, patience=None)
    best = _drive(s, f, 30)
    rng = np.random.RandomState(0)
    rand_best = min(f({"x": rng.uniform(-2, 2), "nested": {"y": rng.uniform(-2, 2)}}) for _ in range(30))
    assert best < 0.02 and best < rand_best
    cfg = s.suggest("last")
    assert cfg["fixed"] == 7 and set(cfg) == {"x", "nested", "fixed"}


def test_waits_for_random_phase_log_space_duplicates_and_state(tmp_path):
    s = BayesOptSearch({"lr": tune.loguniform(1e-5, 1e-1)}, metric="acc", mode="max", random_search_steps=2,
                       points_to_evaluate=[{"lr": 1e-3}], patience=2)
    a, b, c = s.suggest("a"), s.suggest("b"), s.suggest("c")
    assert a == {"lr": 1e-3} and 1e-5 <= b["lr"] <= 1e-1
    assert c is None  # both warm-up trials (the given point and one random) issued, none finished: wait
    s.on_trial_complete("a", {"acc": 0.5})
    s.on_trial_complete("b", {"acc": 0.1})
    d = s.suggest("d")
    assert 1e-5 <= d["lr"] <= 1e-1
    # a repeated configuration is skipped, and more than `patience` repeats end the search
    s2 = BayesOptSearch({"x": (0.0, 1.0)}, metric="m", mode="max", points_to_evaluate=[{"x": 0.5}] * 4,
                        patience=2, random_search_steps=0)
    assert s2.suggest("1") == {"x": 0.5} and s2.suggest("2") is None and s2.suggest("3") == Searcher.FINISHED
    s.save(str(tmp_path / "s.pkl"))
    r = BayesOptSearch({"lr": tune.loguniform(1e-5, 1e-1)}, metric="acc", mode="max")
    r.restore(str(tmp_path / "s.pkl"))
    assert len(r._y) == 2 and set(r._live) == {"d"}
    r.on_trial_complete("d", {"acc": 0.3})  # the restored searcher keeps the in-flight trial
    assert len(r._y) == 3 and r.suggest("e") is not None
    with pytest.raises(ValueError, match="continuous"):
        BayesOptSearch({"k": tune.choice([1, 2])}, metric="m", mode="max")
    assert isinstance(create_searcher("bayesopt", space={"x": (0, 1)}, metric="m", mode="min"), BayesOptSearch)


def test_with_tuner(shutdown_only, tmp_path):
    ray.init(num_cpus=2)

    def objective(config):
        tune.report({"score": -(config["a"] - 2.0) ** 2})

    searcher = BayesOptSearch(random_search_steps=4, random_state=1)
    grid = tune.Tuner(objective, param_space={"a": tune.uniform(0.0, 5.0)},
                      tune_config=tune.TuneConfig(search_alg=searcher, metric="score", mode="max", num_samples=12,
                                                  max_concurrent_trials=2),
                      run_config=tune.RunConfig(storage_path=str(tmp_path), name="bo")).fit()
    best = grid.get_best_result()
    assert len(grid) == 12 and best.metrics["score"] > -0.05
