"""Importable alias of the ``image-segmentation-project_amd`` package (whose
directory name carries hyphens): ``import image_segmentation_project_amd as amd``
and ``from image_segmentation_project_amd.ddp import enable_data_parallel``
resolve to the very same module objects (one copy, one loaded library)."""
import importlib
import sys

_real = importlib.import_module("image-segmentation-project_amd")
for _name, _mod in list(sys.modules.items()):
    if _name.startswith("image-segmentation-project_amd."):
        sys.modules["image_segmentation_project_amd." + _name.split(".", 1)[1]] = _mod
sys.modules[__name__] = _real
