"""MI355X-native DAD (Dynamic Asymmetric Distillation) train step.

Drop-in for the hot path of the reference's DAD-train-{IEMOCAP,CASIA,EMODB} trainers:
`SSRLModel` (I/model.py) and the train_epoch loop body (I/train.py:484-492), backed by
hand-written HIP kernels for gfx950 behind the C ABI in include/dad.h (libdad_hip.so).

The package directory name is not a Python identifier; it is importable with
`importlib.import_module(...)` and registers the alias `dad_amd` on import.
"""
import sys as _sys

from . import _build, _lib
from .config import FLAVOR_DEFAULTS, ConfigView, dad_config_for
from .model import EmotionClassifier, Emotion2VecEncoder, SSRLModel
from .step import DADStep
from .dist import DPComm, ProcessGroupComm
from .data import DeviceLoader, FeatureStore
from .utils import DACPManager, DataAugmentation, ECDALoss
from . import checkpoint, evaluate, pretrain

__all__ = ["SSRLModel", "Emotion2VecEncoder", "EmotionClassifier", "DADStep", "DPComm", "ProcessGroupComm", "ConfigView",
           "dad_config_for", "FLAVOR_DEFAULTS", "FeatureStore", "DeviceLoader", "DataAugmentation", "DACPManager", "ECDALoss", "build", "lib"]


def build(verbose=True):
    """Compile libdad_hip.so for gfx950 (in-tree)."""
    return _build.build(verbose=verbose)


def lib():
    return _lib.lib()


_sys.modules.setdefault("dad_amd", _sys.modules[__name__])
for _m in ("_build", "_lib", "config", "model", "step", "dist", "data", "utils", "evaluate", "checkpoint", "pretrain"):
    _sys.modules.setdefault("dad_amd." + _m, _sys.modules[__name__ + "." + _m])
