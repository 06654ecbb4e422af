"""Build the encoder floor variants (diagnostic libraries lib/libdad_hip_fl_*.so) for
tools/gpu_ws_floor.sh.  Never loaded by the product path."""
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
pkg = importlib.import_module("robust-speech-emotion-recognition-via-dynamic-asymmetric-distillation-in-noisy-environments_amd")

VARIANTS = {
    "fl_norng": ["-DWS_FLOOR_NO_RNG=1"],
    "fl_noxs": ["-DWS_FLOOR_NO_XS=1"],
    "fl_nomfma": ["-DWS_FLOOR_NO_MFMA=1"],
    "fl_nodma": ["-DWS_FLOOR_NO_DMA=1"],
    # compute skeleton: MFMA, conversion without RNG, epilogue, barriers; no row DMA, no copies
    "fl_skeleton": ["-DWS_FLOOR_NO_RNG=1", "-DWS_FLOOR_NO_XS=1", "-DWS_FLOOR_NO_DMA=1"],
    # data movement: row DMA, conversion without RNG, bf16 copies; no MFMA
    "fl_data": ["-DWS_FLOOR_NO_RNG=1", "-DWS_FLOOR_NO_MFMA=1"],
}

if __name__ == "__main__":
    for name, flags in VARIANTS.items():
        pkg._build.build(variant=name, extra=flags)
