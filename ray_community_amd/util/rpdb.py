"""``ray.util.rpdb`` import path: the remote debugger lives in ``util/pdb.py``."""
from .pdb import *  # noqa: F401,F403
from .pdb import set_trace  # noqa: F401
