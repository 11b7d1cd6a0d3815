"""Helpers shared by the golden-vector tests (load fixtures, rebuild their inputs)."""
import os

import numpy as np

import pcs_amd.data as pdata
import pointnet_oracle as orc

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = ["eval_c2_bnrand", "train_c2", "train_c3_ragged_bnrand", "train_c2_nodrop_small"]


def load(name):
    z = np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False)
    return {k: z[k] for k in z.files}


def inputs(g):
    """Rebuild (state_dict, points, labels, mask, masks) exactly as make_golden.py did."""
    C = int(g["C"]); seed = int(g["seed"])
    sd = orc.init_params(C, seed, bn_affine_random=bool(g["bn_rand"]))
    pts, lab, msk = pdata.synthetic_batch(seed + 1, [int(n) for n in g["n_points"]], C,
                                          grid=int(g["grid"]))
    M = pts.shape[0] * pts.shape[1]
    if bool(g["dropout"]):
        masks = orc.dropout_masks(seed + 2, M)
    else:
        masks = (np.ones((M, 512), np.uint8), np.ones((M, 256), np.uint8))
    return sd, pts, lab, msk, masks


def rel_err(a, b):
    a = np.asarray(a, np.float64); b = np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))
