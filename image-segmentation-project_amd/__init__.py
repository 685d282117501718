"""image-segmentation-project_amd — MI355X-native U-Net segmentation training path.

Drop-in for the hot path of SwagMag1213/image-segmentation-project
(``advanced_models.UNetWithBackbone`` resnet34/no-attention, ``losses``
bce/dice/combo, ``utils.calculate_metrics``, ``train.train_epoch/evaluate``),
computed by hand-written gfx950 HIP kernels in ``libunet_hip.so`` (C ABI:
``include/unet_hip.h``).  The directory name carries hyphens, so import it with
``importlib.import_module("image-segmentation-project_amd")``.
"""
from .advanced_models import UNetWithBackbone  # noqa: F401
from .losses import BCELoss, ComboLoss, DiceLoss, get_loss_function  # noqa: F401
from .utils import (EarlyStopping, calculate_metrics, calculate_metrics_from_logits,  # noqa: F401
                    get_device)
from .train import (evaluate, quick_train, train_epoch, train_model, TensorLoader,  # noqa: F401
                    GraphedTrainStep)
from .synthetic import random_batch, synthetic_cells  # noqa: F401
from . import dataset  # noqa: F401
from .dataset import CellAugmenter, CellSegmentationDataset, prepare_data, preprocess  # noqa: F401
from . import ddp  # noqa: F401
from . import optim  # noqa: F401
from .optim import Adam  # noqa: F401
from .ddp import enable_data_parallel  # noqa: F401
from ._lib import LIB_PATH  # noqa: F401

__version__ = "0.1.0"
