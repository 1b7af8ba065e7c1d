"""``python -m ray_community_amd.tune``: the ``tune`` command line (see ``tune/scripts.py``)."""
import sys

from .scripts import main

sys.exit(main())
