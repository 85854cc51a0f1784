"""Prints test_relit_features_match_composition's relative errors per gradient (the margin
to its 2e-5 bar) for the library GSR_LIB_PATH selects."""
import sys
import torch
import os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "tests"), os.path.join(ROOT, "relightable3dgaussians-w_amd"), ROOT):
    sys.path.insert(0, p)
import test_gpu_relit as t

captured = []
orig = t._rel
def rel(a, b):
    v = orig(a, b)
    captured.append(float(v))
    return v
t._rel = rel
for sp, fs in [(True, False), (False, False), (True, True)]:
    captured.clear()
    try:
        t.test_relit_features_match_composition(sp, fs)
        ok = "ok"
    except AssertionError as e:
        ok = f"FAIL {e}"
    print(sp, fs, ["%.2e" % v for v in captured], ok)
