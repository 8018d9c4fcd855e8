import numpy as np


def err(a, b, sc=0.0):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    den = max(np.abs(b).max() if b.size else 0, sc)
    return np.abs(a - b).max() / den if den > 0 else 0.0
