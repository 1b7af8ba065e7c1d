"""``python -m ray_community_amd <command>``: the CLI (scripts/scripts.py)."""
import sys

from .scripts.scripts import main

sys.exit(main())
