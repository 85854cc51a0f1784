"""Packaged data assets.

bsdf_256_256.bin: the split-sum FG LUT the reference loads at scene/NVDIFFREC/light.py:41
(float32 [1, 256, 256, 2]; rows = roughness, columns = NdotV).  Shipped as a hashed asset
because /root/reference does not exist on the GPU box.
"""
import hashlib
import os

import numpy as np

ASSET_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "assets")
FG_LUT_PATH = os.path.join(ASSET_DIR, "bsdf_256_256.bin")
FG_LUT_SHA256 = "aee514f7c7e561a357e529567222da99e84886c31c46a32fe767a5b066bbe196"


def load_fg_lut(check=True):
    raw = open(FG_LUT_PATH, "rb").read()
    if check and hashlib.sha256(raw).hexdigest() != FG_LUT_SHA256:
        raise RuntimeError(f"FG LUT {FG_LUT_PATH} sha256 mismatch")
    return np.frombuffer(raw, dtype=np.float32).reshape(256, 256, 2).copy()
