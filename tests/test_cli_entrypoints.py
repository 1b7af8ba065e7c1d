"""``python -m`` entry points of the library CLIs (reference console scripts: ``ray``, ``serve``,
``rllib``, ``tune``): each starts, parses its subcommands and exits cleanly."""
import subprocess
import sys

import pytest


@pytest.mark.parametrize("mod,args,expect", [
    ("ray_community_amd", ["--help"], "microbenchmark"),
    ("ray_community_amd.serve", ["--help"], "deploy"),
    ("ray_community_amd.rllib", ["example", "list"], "cartpole-ppo"),
    ("ray_community_amd.tune", ["--help"], "lsx"),
])
def test_entrypoint(mod, args, expect):
    p = subprocess.run([sys.executable, "-m", mod, *args], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-2000:]
    assert expect in p.stdout
