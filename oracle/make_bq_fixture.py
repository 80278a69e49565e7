"""Copies the reference's B-matrix statistics (dataset/bq_info_lr/*.npy: data, not code) into the committed fixture
tests/golden/bq_info_lr.npz, so the sc4dvar parity tests run where /root/reference is absent (the GPU box).
Loaded with allow_pickle=False. Usage: python -B oracle/make_bq_fixture.py"""
import os
import sys

import numpy as np

SRC = "/root/reference/dataset/bq_info_lr"
DST = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", "bq_info_lr.npz")
KEYS = ("len_scale", "reg_coeff", "std_sur", "vert_eig_value", "vert_eig_vec")

if __name__ == "__main__":
    if not os.path.isdir(SRC):
        sys.exit(f"{SRC} not found")
    np.savez(DST, **{k: np.load(os.path.join(SRC, k + ".npy"), allow_pickle=False) for k in KEYS})
    print("wrote", DST)
