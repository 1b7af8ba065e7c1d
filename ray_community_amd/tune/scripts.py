"""The ``tune`` command line (reference: ``python/ray/tune/cli/scripts.py`` and ``commands.py``).

    python -m ray_community_amd.tune ls EXPERIMENT_PATH [--sort K ...] [--desc] [--filter "COL OP VAL"]
        [--columns a,b] [--limit N] [--output F.csv|F.pkl]
    python -m ray_community_amd.tune lsx PROJECT_PATH [same options]
    python -m ray_community_amd.tune add-note PATH [--filename note.txt]

``ls`` tabulates one row per trial of an experiment directory (its last result: trial id,
iteration, time, episode return, ``config/*`` columns, ``logdir`` relative to the experiment);
``lsx`` one row per experiment under a storage path (name, trials, last update). ``--filter``
takes ``"<column> <op> <value>"`` with ``op`` one of ``< <= == != >= >``. ``add-note`` opens
``$EDITOR`` (``vim`` by default) on ``PATH/<filename>``.
"""
from __future__ import annotations

import argparse
import operator
import os
import shutil
import subprocess
import sys
import time
from typing import List, Optional

DEFAULT_TRIAL_KEYS = ("trial_id", "training_iteration", "time_total_s", "timesteps_total", "episode_reward_mean",
                      "mean_accuracy", "mean_loss", "timestamp")
DEFAULT_PROJECT_KEYS = ("name", "total_trials", "last_updated")
OPERATORS = {"<": operator.lt, "<=": operator.le, "==": operator.eq, "!=": operator.ne, ">=": operator.ge,
             ">": operator.gt}
TIMESTAMP_FORMAT = "%Y-%m-%d %H:%M:%S (%A)"


class CLIError(Exception):
    pass


def print_table(df) -> tuple:
    """Print ``df`` fitted to the terminal width; returns (dropped columns, empty columns)."""
    from tabulate import tabulate

    width = shutil.get_terminal_size(fallback=(160, 100)).columns
    empty = [c for c in df.columns if df[c].isnull().all()]
    shown = df[[c for c in df.columns if c not in empty]]
    dropped: List[str] = []
    while len(shown.columns) > 1:
        first_line = tabulate(shown, headers="keys", tablefmt="psql", showindex="never").split("\n", 1)[0]
        if len(first_line) <= width:
            break
        dropped.insert(0, shown.columns[-1])
        shown = shown[shown.columns[:-1]]
    print(tabulate(shown, headers="keys", tablefmt="psql", showindex="never"))
    if dropped:
        print(f"Dropped columns: {dropped}\nWiden the terminal to see the remaining columns.")
    if empty:
        print(f"Empty columns: {empty}")
    return dropped, empty


def _filter_sort_limit(df, filter_op, sort, desc, limit):
    from pandas.api.types import is_numeric_dtype, is_string_dtype

    if filter_op:
        try:
            col, op, val = filter_op.split(" ", 2)
        except ValueError:
            raise CLIError(f"--filter takes '<column> <op> <value>', got {filter_op!r}")
        if col not in df:
            raise CLIError(f"{col} not in: {list(df)}")
        if op not in OPERATORS:
            raise CLIError(f"operator must be one of {list(OPERATORS)}, got {op!r}")
        if is_numeric_dtype(df[col].dtype):
            val = float(val)
        elif is_string_dtype(df[col].dtype) or df[col].dtype == object:
            val = str(val)
        else:
            raise CLIError(f"Unsupported dtype for {col}: {df[col].dtype}")
        df = df[OPERATORS[op](df[col], val)]
    if sort:
        for k in sort:
            if k not in df:
                raise CLIError(f"{k} not in: {list(df)}")
        df = df.sort_values(by=list(sort), ascending=not desc)
    if limit:
        df = df[:limit]
    return df


def _save(df, output):
    if not output:
        return
    ext = os.path.splitext(output)[1].lower()
    if ext in (".p", ".pkl", ".pickle"):
        df.to_pickle(output)
    elif ext == ".csv":
        df.to_csv(output, index=False)
    else:
        raise CLIError(f"Unsupported filetype: {output}")
    print(f"Output saved at {output}")


def list_trials(experiment_path: str, sort: Optional[List[str]] = None, output: Optional[str] = None,
                filter_op: Optional[str] = None, info_keys: Optional[List[str]] = None, limit: Optional[int] = None,
                desc: bool = False):
    """Table of the trials of one experiment directory; returns the DataFrame printed."""
    from datetime import datetime

    from .analysis import ExperimentAnalysis

    path = os.path.expanduser(experiment_path)
    try:
        df = ExperimentAnalysis(path).dataframe()
    except ValueError as e:
        raise CLIError(f"No trial data found under {path}") from e
    if info_keys:
        bad = [k for k in info_keys if k not in df.columns]
        if bad:
            raise CLIError(f"Provided key(s) invalid: {bad}. Available keys: {list(df.columns)}")
        cols = list(info_keys)
    else:
        cols = [k for k in DEFAULT_TRIAL_KEYS if k in df] + [k for k in df.columns if k.startswith("config/")] + \
            (["logdir"] if "logdir" in df else [])
    if not cols:
        raise CLIError("No columns to output.")
    df = df[cols].copy()
    if "timestamp" in df:
        df["timestamp"] = df["timestamp"].apply(
            lambda t: datetime.fromtimestamp(float(t)).strftime(TIMESTAMP_FORMAT) if t == t and t is not None else t)
    if "logdir" in df:
        df["logdir"] = df["logdir"].astype(str).str.replace(path.rstrip("/") + "/", "", regex=False)
    df = _filter_sort_limit(df, filter_op, sort, desc, limit)
    print_table(df)
    _save(df, output)
    return df


def list_experiments(project_path: str, sort: Optional[List[str]] = None, output: Optional[str] = None,
                     filter_op: Optional[str] = None, info_keys: Optional[List[str]] = None,
                     limit: Optional[int] = None, desc: bool = False):
    """Table of the experiments under a storage path (name, trial count, last update)."""
    import pandas as pd

    base = os.path.expanduser(project_path)
    if not os.path.isdir(base):
        raise CLIError(f"{base} is not a directory")
    rows = []
    for name in sorted(os.listdir(base)):
        d = os.path.join(base, name)
        if not os.path.isdir(d):
            continue
        results = [os.path.join(r, "result.json") for r, _, files in os.walk(d) if "result.json" in files]
        if not results and not os.path.exists(os.path.join(d, "experiment_state.json")):
            continue
        mtime = max([os.path.getmtime(p) for p in results] or [os.path.getmtime(d)])
        rows.append({"name": name, "total_trials": len(results),
                     "last_updated": time.strftime("%Y-%m-%d %H:%M:%S", time.localtime(mtime))})
    if not rows:
        raise CLIError("No experiments found!")
    df = pd.DataFrame(rows)
    keys = [k for k in (info_keys or DEFAULT_PROJECT_KEYS) if k in df]
    if not keys:
        raise CLIError(f"None of keys {info_keys} in experiment data!")
    df = _filter_sort_limit(df[keys], filter_op, sort, desc, limit)
    print_table(df)
    _save(df, output)
    return df


def add_note(path: str, filename: str = "note.txt") -> str:
    p = os.path.expanduser(path)
    if not os.path.isdir(p):
        raise CLIError(f"{p} is not a valid directory.")
    fp = os.path.join(p, filename)
    existed = os.path.exists(fp)
    try:
        subprocess.call([os.environ.get("EDITOR", "vim"), fp])
    except OSError as e:
        print(f"Editing note failed: {e}")
    if os.path.exists(fp):
        print(("Note updated at: " if existed else "Note created at: ") + fp)
    return fp


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="tune", description="Tune experiment browser")
    sub = ap.add_subparsers(dest="cmd", required=True)
    for name, arg in (("ls", "experiment_path"), ("lsx", "project_path")):
        p = sub.add_parser(name, help="list trials of an experiment" if name == "ls" else "list experiments")
        p.add_argument(arg)
        p.add_argument("--sort", nargs="+", default=None)
        p.add_argument("--output", "-o", default=None)
        p.add_argument("--filter", dest="filter_op", default=None)
        p.add_argument("--columns", default=None, help="comma-separated columns to show")
        p.add_argument("--limit", type=int, default=None)
        p.add_argument("--desc", action="store_true")
    n = sub.add_parser("add-note", help="write a note into a trial / experiment directory with $EDITOR")
    n.add_argument("path")
    n.add_argument("--filename", default="note.txt")
    return ap


def main(argv: Optional[List[str]] = None) -> int:
    args = build_parser().parse_args(argv)
    try:
        if args.cmd == "add-note":
            add_note(args.path, args.filename)
            return 0
        cols = args.columns.split(",") if args.columns else None
        fn = list_trials if args.cmd == "ls" else list_experiments
        path = args.experiment_path if args.cmd == "ls" else args.project_path
        fn(path, sort=args.sort, output=args.output, filter_op=args.filter_op, info_keys=cols, limit=args.limit,
           desc=args.desc)
        return 0
    except CLIError as e:
        print(f"Error: {e}", file=sys.stderr)
        return 1


if __name__ == "__main__":
    sys.exit(main())
