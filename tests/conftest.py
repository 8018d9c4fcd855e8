import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "aimnet-x2d_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running")


def load_golden(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)


def norm_rel(a, b):
    """max|a-b| / max|b| — the per-tensor norm-relative metric the north star's 1e-5 refers to."""
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    if a.shape != b.shape:
        raise AssertionError(f"shape {a.shape} != {b.shape}")
    den = np.abs(b).max() if b.size else 0.0
    num = np.abs(a - b).max() if a.size else 0.0
    return num / den if den > 0 else num


@pytest.fixture
def golden():
    return load_golden


def _scale_for(key, ref64):
    """Gradients whose exact value is 0 (softmax shift invariance: d/db_h of the attention bias,
    pooling.py:136-145) are pure rounding noise; judge them against their sibling weight's scale."""
    if ".attention_weights." in key and key.startswith("grad.") and key.endswith(".bias"):
        w = key[:-len("bias")] + "weight"
        if w in ref64:
            return float(np.abs(ref64[w]).max())
    return 0.0


def parity_failures(ours, ref32, ref64, atol_rel=1e-5, factor=3.0):
    """North-star tolerance, per tensor: err(ours vs fp64) <= max(1e-5, factor * err(ref fp32 vs fp64)).

    1e-5 norm-relative is the contract (BASELINE.json north_star). Where the reference's own fp32
    result is further than that from the exact (fp64) value — measured per tensor, e.g. c3's
    attention / partial charges at ~6e-5..9e-5 (tools/noise_floor.py) — the bound is `factor` times
    the reference's own fp32 error instead: no fp32 implementation can be closer to the reference
    than the reference is to the exact answer.
    """
    bad = []
    for k, v64 in ref64.items():
        if k not in ours:
            continue
        sc = _scale_for(k, ref64)
        a = np.asarray(ours[k], np.float64)
        b = np.asarray(v64, np.float64)
        den = max(np.abs(b).max() if b.size else 0.0, sc)
        err = (np.abs(a - b).max() / den) if (b.size and den > 0) else 0.0
        floor = 0.0
        if ref32 is not None and k in ref32:
            r = np.asarray(ref32[k], np.float64)
            floor = (np.abs(r - b).max() / den) if (b.size and den > 0) else 0.0
        tol = max(atol_rel, factor * floor)
        if not err <= tol:
            bad.append((k, err, tol))
    return bad


SKETCH_K = 32


def sketch(key, g):
    """g @ P, P a seeded Gaussian [cols, 32] keyed by the tensor name — the same summary
    tests/golden/make_golden.py stores (as 'sketch.<key>') for gradients too large to commit."""
    import zlib
    rng = np.random.default_rng([77, zlib.crc32(key.encode())])
    P = rng.standard_normal((np.asarray(g).shape[1], SKETCH_K))
    return np.asarray(g, np.float64) @ P


def add_sketches(res, z):
    """For every 'sketch.<key>' in fixture z, add res['sketch.<key>'] = sketch(key, res[key])."""
    for k in z.files:
        if k.startswith("sketch.") and k[len("sketch."):] in res:
            res[k] = sketch(k[len("sketch."):], res[k[len("sketch."):]])
    return res


def fixture_refs(z):
    """The reference fp32 tensors a model-case fixture stores (outputs, gradients, sketches)."""
    return {k: z[k] for k in z.files if k in ("out", "attn", "q") or k.startswith("grad.") or k.startswith("sketch.")}
