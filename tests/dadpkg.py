"""Import helper: the package directory name is not a Python identifier."""
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_NAME = "robust-speech-emotion-recognition-via-dynamic-asymmetric-distillation-in-noisy-environments_amd"
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pkg():
    return importlib.import_module(PKG_NAME)


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
