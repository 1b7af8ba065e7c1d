"""``python -m ray_community_amd.serve <command>``: the ``serve`` CLI (reference:
``python/ray/serve/scripts.py``) -- the same commands as ``python -m ray_community_amd serve``."""
import sys

from ..scripts.scripts import main

sys.exit(main(["serve", *sys.argv[1:]]))
