"""Reference module layout (/root/reference/dataset.py) for a drop-in switch:
put `dropin/` ahead of the reference directory on sys.path and the
reference's own `from dataset import ...` lines bind the MI355X path."""
import os as _os
import sys as _sys

_REPO = _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__)))
if _REPO not in _sys.path:
    _sys.path.insert(0, _REPO)

from image_segmentation_project_amd.dataset import *  # noqa: E402,F401,F403
