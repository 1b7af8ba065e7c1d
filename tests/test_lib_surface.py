"""Library API pieces beyond the core flows: Tune registry / Experiment / reporters / factories,
Train DataConfig, Data ReadTask + file datasinks, Serve HTTPOptions (reference: tune/tests/
test_api.py, test_progress_reporter.py, train/tests/test_data_parallel_trainer.py,
data/tests/test_datasink.py)."""
import io
import os

import numpy as np
import pytest

import ray_community_amd as ray
from ray_community_amd import data as rd
from ray_community_amd import tune


@pytest.fixture
def ray4():
    ray.init(num_cpus=4, include_dashboard=False, log_to_driver=False)
    yield
    ray.shutdown()


def _obj(config):
    for i in range(3):
        tune.report({"score": config["x"] * (i + 1)})


def test_register_trainable_run_experiments_and_cli_reporter(ray4, tmp_path):
    tune.register_trainable("quad", _obj)
    out = io.StringIO()
    rep = tune.CLIReporter(metric_columns=["score"], parameter_columns=["x"], max_report_frequency=0, out=out)
    ana = tune.run("quad", config={"x": tune.grid_search([1, 2, 3])}, metric="score", mode="max",
                   storage_path=str(tmp_path), progress_reporter=rep)
    assert ana.best_config == {"x": 3}
    text = out.getvalue()
    assert "Final status" in text and "TERMINATED" in text and "score" in text and "| 9 " in text
    trials = tune.run_experiments({"exp_a": {"run": "quad", "config": {"x": 5}, "storage_path": str(tmp_path)}})
    assert len(trials) == 1 and trials[0].metrics["score"] == 15
    exp = tune.Experiment("exp_b", _obj, config={"x": 1}, storage_path=str(tmp_path))
    assert tune.run_experiments(exp)[0].metrics["score"] == 3
    grid = tune.Tuner("quad", param_space={"x": 4},
                      run_config=ray.train.RunConfig(storage_path=str(tmp_path))).fit()
    assert grid[0].metrics["score"] == 12


def test_factories_pgf_resume_config():
    assert isinstance(tune.create_scheduler("asha", metric="m", mode="max"), tune.ASHAScheduler)
    assert isinstance(tune.create_scheduler("fifo"), tune.FIFOScheduler)
    assert tune.create_searcher("variant_generator") is not None
    with pytest.raises(ValueError):
        tune.create_scheduler("nope")
    pgf = tune.PlacementGroupFactory([{"CPU": 1}, {"CPU": 2, "GPU": 1}])
    assert pgf.required_resources == {"CPU": 3.0, "GPU": 1.0}
    wrapped = tune.with_resources(_obj, pgf)
    assert wrapped._rca_resources == {"CPU": 3.0, "GPU": 1.0}
    assert tune.ResumeConfig().errored == "skip"


def test_register_env_reaches_rllib():
    from ray_community_amd.rllib.env import envs

    tune.register_env("my-cartpole", lambda cfg: envs.CartPoleVec(num_envs=cfg.get("n", 2)))
    assert "my-cartpole" in envs._REGISTRY


def test_train_data_config_splits_only_named_datasets(ray4):
    from ray_community_amd.train import DataConfig, ScalingConfig, TRAIN_DATASET_KEY
    from ray_community_amd.train.data_parallel_trainer import DataParallelTrainer

    assert TRAIN_DATASET_KEY == "train"

    def loop():
        from ray_community_amd import train

        tr = sum(1 for _ in train.get_dataset_shard("train").iter_rows())
        ev = sum(1 for _ in train.get_dataset_shard("eval").iter_rows())
        train.report({"tr": tr, "ev": ev})

    t = DataParallelTrainer(loop, scaling_config=ScalingConfig(num_workers=2),
                            datasets={"train": rd.range(40), "eval": rd.range(10)},
                            dataset_config=DataConfig(datasets_to_split=["train"]))
    m = t.fit().metrics
    assert m["tr"] == 20 and m["ev"] == 10
    with pytest.raises(TypeError):
        DataConfig(datasets_to_split="train")


class _NpySink(rd.BlockBasedFileDatasink):
    def __init__(self, path):
        super().__init__(path, file_format="npy")

    def write_block_to_file(self, block, file):
        np.save(file, block.to_numpy()["id"])


class _TxtRowSink(rd.RowBasedFileDatasink):
    def __init__(self, path):
        super().__init__(path, file_format="txt")

    def write_row_to_file(self, row, file):
        file.write(str(row["id"]).encode())


class _Squares(rd.Datasource):
    def get_read_tasks(self, parallelism, **kw):
        return [rd.ReadTask(lambda i=i: [{"sq": np.arange(i * 5, i * 5 + 5) ** 2}]) for i in range(parallelism)]


def test_read_task_and_file_datasinks(ray4, tmp_path):
    ds = rd.read_datasource(_Squares(), parallelism=3)
    assert sorted(r["sq"] for r in ds.take_all()) == [i * i for i in range(15)]
    rd.range(12, override_num_blocks=3).write_datasink(_NpySink(str(tmp_path / "npy")))
    got = sorted(int(x) for f in os.listdir(tmp_path / "npy") for x in np.load(tmp_path / "npy" / f))
    assert got == list(range(12))
    rd.range(5).write_datasink(_TxtRowSink(str(tmp_path / "txt")))
    assert sorted(int(open(tmp_path / "txt" / f).read()) for f in os.listdir(tmp_path / "txt")) == list(range(5))
    assert rd.set_progress_bars(False) in (True, False)
    with pytest.raises(ImportError):
        rd.from_dask(None)


def test_serve_http_options_object():
    from ray_community_amd import serve

    o = serve.HTTPOptions(host="0.0.0.0", port=8123)
    assert (o.host, o.port, o.location) == ("0.0.0.0", 8123, "HeadOnly")
