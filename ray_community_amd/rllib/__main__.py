"""``python -m ray_community_amd.rllib``: the ``rllib`` command line (see ``rllib/scripts.py``)."""
import sys

from .scripts import main

sys.exit(main())
