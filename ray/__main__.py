"""``python -m ray <command>``: the ray_community_amd CLI."""
import sys

from ray_community_amd.scripts.scripts import main

sys.exit(main())
