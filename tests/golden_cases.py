"""Shared helpers to rebuild a golden case's inputs/config/weights (tests only)."""
import ast

import numpy as np
import torch

from conftest import load_golden

CASES = ["c1", "c2", "c3", "c4s", "c5s", "pool_mean", "pool_max", "pool_sum",
         "act_relu", "act_leakyrelu", "act_elu", "act_gelu", "evidential", "noedges", "stereo", "stereo_pc",
         "nm0", "nm3"]
FEATURE_KEYS = ("atom_type", "hydrogen_count", "degree", "hybridization")


def case_config(z):
    cfg = dict(ast.literal_eval(str(z["cfg_json"])))
    return cfg


def case_inputs(z, device="cpu"):
    feats = torch.from_numpy(z["feats"].astype(np.int64))
    af = {k: feats[:, i].contiguous().to(device) for i, k in enumerate(FEATURE_KEYS)}
    edges = torch.from_numpy(z["edges"].astype(np.int64)).reshape(-1, 2).to(device)
    batch = torch.from_numpy(z["batch"].astype(np.int64)).to(device)
    tc = torch.from_numpy(z["total_charges"]).to(device)
    return af, edges, batch, tc


def case_stereo(z, device="cpu"):
    """The collated (tetrahedral [M,4], cis [C,2], trans [T,2]) tensors of a case (empty if none)."""
    def get(k, w):
        if k in z.files:
            return torch.from_numpy(z[k].astype(np.int64)).reshape(-1, w).to(device)
        return torch.empty(0, w, dtype=torch.long, device=device)
    return get("tet", 4), get("cis", 2), get("trans", 2)


def load_case(name, device="cpu"):
    z = load_golden(name)
    return z, case_config(z), case_inputs(z, device)
