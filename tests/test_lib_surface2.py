"""Preprocessors beyond the basic scalers/encoders, TorchCheckpoint / TorchPredictor, Tune
SearchGenerator and ResourceChangingScheduler (reference: data/tests/preprocessors/*,
train/tests/test_torch_predictor.py, tune/tests/test_resource_changing_scheduler.py)."""
import numpy as np
import pandas as pd
import pytest
import torch

import ray_community_amd as ray
from ray_community_amd import data as rd
from ray_community_amd import tune
from ray_community_amd.data import preprocessors as P


@pytest.fixture(scope="module")
def ray4():
    ray.init(num_cpus=4, include_dashboard=False, log_to_driver=False)
    yield
    ray.shutdown()


def _df(ds):
    return ds.to_pandas().reset_index(drop=True)


def test_numeric_preprocessors(ray4):
    ds = rd.from_pandas(pd.DataFrame({"a": [1.0, 2.0, 3.0, 4.0, 100.0], "b": [3.0, 0.0, 4.0, 0.0, 0.0]}))
    r = _df(P.RobustScaler(["a"]).fit_transform(ds))
    assert np.allclose(r["a"], (np.array([1, 2, 3, 4, 100.0]) - 3.0) / 2.0)
    n = _df(P.Normalizer(["a", "b"], norm="l2").transform(ds))
    assert np.allclose(n["a"] ** 2 + n["b"] ** 2, 1.0)
    p = _df(P.PowerTransformer(["b"], power=0.5).transform(ds))
    assert np.allclose(p["b"], (np.sqrt(np.array([3.0, 0, 4, 0, 0]) + 1) - 1) / 0.5)
    u = _df(P.UniformKBinsDiscretizer(["a"], bins=4, include_lowest=True).fit_transform(ds))
    assert list(u["a"]) == [0, 0, 0, 0, 3]
    c = _df(P.CustomKBinsDiscretizer(["b"], [-1, 1, 5]).transform(ds))
    assert list(c["b"]) == [1, 0, 1, 0, 0]


def test_categorical_and_text_preprocessors(ray4):
    ds = rd.from_pandas(pd.DataFrame({"c": ["x", "y", "x", "z"], "tags": [["a", "b"], ["b"], [], ["a", "a"]],
                                      "t": ["the cat", "the dog the", "cat", "dog dog"]}))
    cat = _df(P.Categorizer(["c"]).fit_transform(ds))
    assert str(cat["c"].dtype) == "category" and list(cat["c"].cat.categories) == ["x", "y", "z"]
    mh = _df(P.MultiHotEncoder(["tags"]).fit_transform(ds))
    assert [list(v) for v in mh["tags"]] == [[1, 1], [0, 1], [0, 0], [2, 0]]
    tok = _df(P.Tokenizer(["t"]).transform(ds))
    assert list(tok["t"][1]) == ["the", "dog", "the"]
    cv = _df(P.CountVectorizer(["t"]).fit_transform(ds))
    assert cv["t_the"].tolist() == [1, 2, 0, 0] and cv["t_dog"].tolist() == [0, 1, 0, 2]
    hv = _df(P.HashingVectorizer(["t"], num_features=8).transform(ds))
    assert hv[[f"hash_t_{j}" for j in range(8)]].to_numpy().sum(1).tolist() == [2, 3, 1, 2]
    fh = _df(P.FeatureHasher(["x1", "x2"], num_features=4).transform(
        rd.from_pandas(pd.DataFrame({"x1": [1, 0], "x2": [2, 5]}))))
    assert fh[[f"hash_{j}" for j in range(4)]].to_numpy().sum(1).tolist() == [3, 5]


def test_torchvision_preprocessor(ray4):
    ds = rd.from_numpy(np.ones((6, 4, 4), dtype=np.float32))
    tv = P.TorchVisionPreprocessor(["data"], transform=lambda t: t * 2 + 1, batched=True)
    out = tv.transform(ds).take_all()
    assert all(float(r["data"].max()) == 3.0 for r in out)


def test_torch_checkpoint_and_predictor(tmp_path):
    from ray_community_amd.train.torch import TorchCheckpoint, TorchPredictor

    torch.manual_seed(0)
    net = torch.nn.Linear(3, 2)
    x = np.random.RandomState(0).randn(5, 3).astype(np.float32)
    want = net(torch.as_tensor(x)).detach().numpy()
    ck = TorchCheckpoint.from_model(net)
    got = TorchPredictor.from_checkpoint(ck).predict(x)["predictions"]
    assert np.allclose(got, want, atol=1e-6)
    ck2 = TorchCheckpoint.from_state_dict(net.state_dict())
    got2 = TorchPredictor.from_checkpoint(ck2, model=torch.nn.Linear(3, 2)).predict({"x": x})["predictions"]
    assert np.allclose(got2, want, atol=1e-6)
    with pytest.raises(ValueError):
        ck2.get_model()


def _trainable(config):
    for i in range(4):
        tune.report({"score": config["x"] + i})


def test_search_generator_and_resource_changing_scheduler(ray4, tmp_path):
    from ray_community_amd.tune.schedulers import FIFOScheduler, ResourceChangingScheduler
    from ray_community_amd.tune.search import BasicVariantGenerator, SearchGenerator

    gen = SearchGenerator(BasicVariantGenerator())
    gen.set_search_properties("score", "max", {"x": tune.grid_search([1, 2])})
    assert gen.next_trial() is not None

    def alloc(controller, trial, result, scheduler):
        return {"CPU": 2} if result.get("training_iteration", 0) >= 2 else None

    sched = ResourceChangingScheduler(FIFOScheduler(), resources_allocation_function=alloc)
    grid = tune.Tuner(_trainable, param_space={"x": tune.grid_search([1, 5])},
                      tune_config=tune.TuneConfig(metric="score", mode="max", scheduler=sched),
                      run_config=ray.train.RunConfig(storage_path=str(tmp_path))).fit()
    assert grid.get_best_result().config["x"] == 5
    assert sched.changes and all(r == {"CPU": 2} for _, r in sched.changes)


def _noisy(config):
    import sys

    print("trial-stdout", config["x"])
    print("trial-stderr", config["x"], file=sys.stderr)
    tune.report({"score": config["x"]})


def test_run_config_log_to_file(ray4, tmp_path):
    import glob
    import os

    grid = tune.Tuner(_noisy, param_space={"x": tune.grid_search([1, 2])},
                      run_config=ray.train.RunConfig(storage_path=str(tmp_path), name="ltf", log_to_file=True)).fit()
    assert len(grid) == 2
    outs = sorted(glob.glob(os.path.join(str(tmp_path), "ltf", "*", "stdout")))
    errs = sorted(glob.glob(os.path.join(str(tmp_path), "ltf", "*", "stderr")))
    assert len(outs) == 2 and len(errs) == 2
    text = "".join(open(p).read() for p in outs)
    assert "trial-stdout 1" in text and "trial-stdout 2" in text
    assert "trial-stderr" in "".join(open(p).read() for p in errs)


def _named(config):
    tune.report({"name": tune.get_context().get_trial_name(), "score": config["x"]})


def test_trial_name_creator(ray4, tmp_path):
    grid = tune.Tuner(_named, param_space={"x": tune.grid_search([3, 4])},
                      tune_config=tune.TuneConfig(trial_name_creator=lambda t: f"xval_{t.config['x']}"),
                      run_config=ray.train.RunConfig(storage_path=str(tmp_path))).fit()
    assert sorted(r.metrics["name"] for r in grid) == ["xval_3", "xval_4"]


class _NoisyTrainable(tune.Trainable):
    def setup(self, config):
        import os as _os

        _os.write(1, f"fd-level {self.trial_name}\n".encode())  # bypasses sys.stdout
        self.x = config["x"]

    def step(self):
        print("class-trial", self.x, flush=True)
        return {"score": self.x, "name": self.trial_name, "done": True}


def test_class_trainable_log_to_file_and_trial_name(ray4, tmp_path):
    """RunConfig(log_to_file) and TuneConfig.trial_name_creator apply to class trainables too;
    the redirect is at the descriptor level, so raw fd writes land in the file."""
    import glob
    import os

    grid = tune.Tuner(_NoisyTrainable, param_space={"x": tune.grid_search([5, 6])},
                      tune_config=tune.TuneConfig(trial_name_creator=lambda t: f"cls_{t.config['x']}"),
                      run_config=ray.train.RunConfig(storage_path=str(tmp_path), name="cltf",
                                                     log_to_file=True)).fit()
    assert sorted(r.metrics["name"] for r in grid) == ["cls_5", "cls_6"]
    text = "".join(open(p).read() for p in glob.glob(os.path.join(str(tmp_path), "cltf", "*", "stdout")))
    assert "class-trial 5" in text and "class-trial 6" in text
    assert "fd-level cls_5" in text and "fd-level cls_6" in text
