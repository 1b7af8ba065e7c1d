"""Tune result loggers (reference: python/ray/tune/tests/test_logger.py -- CSV / JSON outputs
per trial, custom LoggerCallback hooks, legacy Logger classes)."""
import csv
import json
import os

import pytest

import ray_community_amd as ray
from ray_community_amd import tune
from ray_community_amd.train import RunConfig
from ray_community_amd.tune.logger import (CSVLoggerCallback, JsonLoggerCallback, LegacyLoggerCallback, Logger,
                                           LoggerCallback)


@pytest.fixture
def ray4():
    ray.init(num_cpus=4, log_to_driver=False)
    yield
    ray.shutdown()


def _train(config):
    for i in range(3):
        tune.report({"score": config["x"] * (i + 1), "nested": {"a": i}})


def test_default_csv_and_json_loggers(ray4, tmp_path):
    grid = tune.Tuner(_train, param_space={"x": tune.grid_search([1, 2])},
                      run_config=RunConfig(name="lg", storage_path=str(tmp_path))).fit()
    assert len(grid) == 2
    for r in grid:
        d = r.path
        params = json.load(open(os.path.join(d, "params.json")))
        rows = list(csv.DictReader(open(os.path.join(d, "progress.csv"))))
        assert [float(row["score"]) for row in rows] == [params["x"] * k for k in (1, 2, 3)]
        assert "nested/a" in rows[0] and "config/x" not in rows[0]
        assert len(open(os.path.join(d, "result.json")).read().strip().splitlines()) == 3


def test_custom_logger_callback_and_legacy_logger(ray4, tmp_path, monkeypatch):
    events = []

    class Rec(LoggerCallback):
        def log_trial_start(self, trial):
            events.append(("start", trial.config["x"]))

        def log_trial_result(self, iteration, trial, result):
            events.append(("result", result["score"]))

        def log_trial_end(self, trial, failed=False):
            events.append(("end", failed))

    seen = []

    class MyLogger(Logger):
        def on_result(self, result):
            seen.append((os.path.basename(self.logdir) != "", result["score"]))

    monkeypatch.setenv("TUNE_DISABLE_AUTO_CALLBACK_LOGGERS", "1")
    grid = tune.Tuner(_train, param_space={"x": 5},
                      run_config=RunConfig(name="lg2", storage_path=str(tmp_path),
                                           callbacks=[Rec(), LegacyLoggerCallback([MyLogger])])).fit()
    assert events == [("start", 5), ("result", 5), ("result", 10), ("result", 15), ("end", False)]
    assert seen == [(True, 5), (True, 10), (True, 15)]
    d = next(iter(grid)).path
    assert not os.path.exists(os.path.join(d, "progress.csv"))  # defaults disabled


def test_explicit_default_loggers_are_not_duplicated(ray4, tmp_path):
    grid = tune.Tuner(_train, param_space={"x": 1},
                      run_config=RunConfig(name="lg3", storage_path=str(tmp_path),
                                           callbacks=[CSVLoggerCallback(), JsonLoggerCallback()])).fit()
    d = next(iter(grid)).path
    rows = list(csv.DictReader(open(os.path.join(d, "progress.csv"))))
    assert len(rows) == 3  # one writer, not two


def _read_tfevents(path):
    """Minimal tfevents reader: TFRecord frames -> (step, tag, value) of scalar Events."""
    import struct

    from ray_community_amd.data.datasource import _masked_crc

    def varint(b, i):
        n = s = 0
        while True:
            c = b[i]
            i += 1
            n |= (c & 0x7F) << s
            s += 7
            if c < 0x80:
                return n, i

    def fields(b):
        i, out = 0, []
        while i < len(b):
            key, i = varint(b, i)
            num, wire = key >> 3, key & 7
            if wire == 0:
                v, i = varint(b, i)
            elif wire == 1:
                v, i = b[i:i + 8], i + 8
            elif wire == 5:
                v, i = b[i:i + 4], i + 4
            else:
                n, i = varint(b, i)
                v, i = b[i:i + n], i + n
            out.append((num, v))
        return out

    out, data = [], open(path, "rb").read()
    i = 0
    while i < len(data):
        (n,) = struct.unpack("<Q", data[i:i + 8])
        assert struct.unpack("<I", data[i + 8:i + 12])[0] == _masked_crc(data[i:i + 8])
        payload = data[i + 12:i + 12 + n]
        assert struct.unpack("<I", data[i + 12 + n:i + 16 + n])[0] == _masked_crc(payload)
        i += 16 + n
        ev = dict(fields(payload))
        if 5 in ev:
            val = dict(fields(dict(fields(ev[5]))[1]))
            out.append((ev.get(2, 0), val[1].decode(), struct.unpack("<f", val[2])[0]))
    return out


def test_tbx_logger_writes_tfevents_scalars(ray4, tmp_path):
    from ray_community_amd.tune.logger import TBXLoggerCallback

    grid = tune.Tuner(_train, param_space={"x": 2},
                      run_config=RunConfig(name="tb", storage_path=str(tmp_path),
                                           callbacks=[TBXLoggerCallback()])).fit()
    d = next(iter(grid)).path
    files = [f for f in os.listdir(d) if f.startswith("events.out.tfevents.")]
    assert len(files) == 1
    ev = _read_tfevents(os.path.join(d, files[0]))
    score = [(s, v) for s, t, v in ev if t == "ray/tune/score"]
    assert score == [(1, 2.0), (2, 4.0), (3, 6.0)]
    assert any(t == "ray/tune/nested/a" for _, t, _ in ev)
