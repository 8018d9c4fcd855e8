"""RDKit-free SMILES -> molecular graph featuriser (QM9 subset).

Restates what the reference obtains from RDKit in ``compute_all``
(reference: src/datasets/features.py:153-334) for the organic subset QM9 uses:

* ``Chem.MolFromSmiles`` + ``Chem.AddHs`` atom order: heavy atoms in SMILES order,
  then each heavy atom's hydrogens appended in heavy-atom order (features.py:166-170).
* ``Chem.GetAdjacencyMatrix`` (features.py:178) -> symmetric 0/1 matrix.
* atom feature indices (features.py:289-319): atom_type = Z-1, hydrogen_count capped at 8,
  degree 0..5 else 6, hybridization index 0..5 else 6.

Chemical fidelity to RDKit (aromatic perception, hybridization) is approximate; the graph
topology and atom ordering are what the hot path consumes, and both the reference and this
framework are fed the same featurised tensors, so parity holds by construction.
"""
from __future__ import annotations

import numpy as np

_Z = {"H": 1, "B": 5, "C": 6, "N": 7, "O": 8, "F": 9, "P": 15, "S": 16, "Cl": 17, "Br": 35, "I": 53}
_VALENCE = {1: 1, 5: 3, 6: 4, 7: 3, 8: 2, 9: 1, 15: 3, 16: 2, 17: 1, 35: 1, 53: 1}
_BOND = {"-": 1.0, "=": 2.0, "#": 3.0, ":": 1.5, "/": 1.0, "\\": 1.0}


class SmilesError(ValueError):
    pass


def _parse_bracket(s: str):
    # [isotope]symbol[chirality][Hcount][charge][:class]
    i = 0
    while i < len(s) and s[i].isdigit():
        i += 1
    arom = False
    if s[i:i + 2] in ("Cl", "Br"):
        sym, i = s[i:i + 2], i + 2
    elif s[i].islower():
        sym, arom, i = s[i].upper(), True, i + 1
    else:
        sym, i = s[i], i + 1
    while i < len(s) and s[i] == "@":
        i += 1
    nh = 0
    if i < len(s) and s[i] == "H":
        i += 1
        nh = 1
        j = i
        while i < len(s) and s[i].isdigit():
            i += 1
        if i > j:
            nh = int(s[j:i])
    charge = 0
    while i < len(s) and s[i] in "+-":
        sign = 1 if s[i] == "+" else -1
        i += 1
        j = i
        while i < len(s) and s[i].isdigit():
            i += 1
        charge += sign * (int(s[j:i]) if i > j else 1)
    if sym not in _Z:
        raise SmilesError(f"unsupported element {sym}")
    return _Z[sym], arom, nh, charge


def parse_smiles(smi: str):
    """Return (Z[n], bonds[(i,j,order)], explicit_h[n] or -1, charge[n], aromatic[n]) heavy atoms."""
    Z, arom, hcnt, chg = [], [], [], []
    bonds = []
    stack = []
    prev = -1
    pending_bond = None
    rings = {}
    i = 0
    while i < len(smi):
        c = smi[i]
        if c == "(":
            stack.append(prev)
            i += 1
            continue
        if c == ")":
            prev = stack.pop()
            i += 1
            continue
        if c in _BOND:
            pending_bond = _BOND[c]
            i += 1
            continue
        if c == ".":
            prev = -1
            i += 1
            continue
        if c.isdigit() or c == "%":
            if c == "%":
                num, i = int(smi[i + 1:i + 3]), i + 3
            else:
                num, i = int(c), i + 1
            if num in rings:
                j, bo = rings.pop(num)
                order = pending_bond or bo
                if order is None:
                    order = 1.5 if (arom[j] and arom[prev]) else 1.0
                bonds.append((j, prev, order))
            else:
                rings[num] = (prev, pending_bond)
            pending_bond = None
            continue
        # atom
        if c == "[":
            k = smi.index("]", i)
            z, a, nh, ch = _parse_bracket(smi[i + 1:k])
            i = k + 1
        else:
            if smi[i:i + 2] in ("Cl", "Br"):
                sym, i = smi[i:i + 2], i + 2
                a = False
            elif c.islower():
                sym, a, i = c.upper(), True, i + 1
            else:
                sym, a, i = c, False, i + 1
            if sym not in _Z:
                raise SmilesError(f"unsupported element {sym}")
            z, nh, ch = _Z[sym], -1, 0
        idx = len(Z)
        Z.append(z)
        arom.append(a)
        hcnt.append(nh)
        chg.append(ch)
        if prev >= 0:
            order = pending_bond
            if order is None:
                order = 1.5 if (arom[prev] and a) else 1.0
            bonds.append((prev, idx, order))
        pending_bond = None
        prev = idx
    if rings:
        raise SmilesError("unclosed ring")
    return Z, bonds, hcnt, chg, arom


def featurize(smi: str):
    """SMILES -> dict(adj (bool [n,n]), atom feature index arrays (int8), total_charge, Z).

    Atom order follows RDKit AddHs: heavy atoms first, then hydrogens grouped by heavy atom.
    """
    Z, bonds, hcnt, chg, arom = parse_smiles(smi)
    nh_atoms = len(Z)
    bo_sum = [0.0] * nh_atoms
    for a, b, o in bonds:
        bo_sum[a] += o
        bo_sum[b] += o
    n_h = []
    for k in range(nh_atoms):
        if hcnt[k] >= 0:
            n_h.append(hcnt[k])
        else:
            v = _VALENCE.get(Z[k], 0)
            n_h.append(max(0, v - int(np.floor(bo_sum[k] + 0.5))))
    n = nh_atoms + sum(n_h)
    adj = np.zeros((n, n), dtype=np.int32)
    maxo = [0.0] * nh_atoms
    ndouble = [0] * nh_atoms
    for a, b, o in bonds:
        adj[a, b] = adj[b, a] = 1
        maxo[a] = max(maxo[a], o)
        maxo[b] = max(maxo[b], o)
        if o == 2.0:
            ndouble[a] += 1
            ndouble[b] += 1
    Zall = list(Z)
    nxt = nh_atoms
    for k in range(nh_atoms):
        for _ in range(n_h[k]):
            adj[k, nxt] = adj[nxt, k] = 1
            Zall.append(1)
            nxt += 1
    deg = adj.sum(1)
    atom_type = np.array([z - 1 for z in Zall], dtype=np.int8)
    hydrogen = np.zeros(n, dtype=np.int8)
    hydrogen[:nh_atoms] = np.minimum(np.array(n_h, dtype=np.int64), 8)
    degree = np.array([d if d < 6 else 6 for d in deg], dtype=np.int8)
    hyb = np.zeros(n, dtype=np.int8)  # H -> S (index 0)
    for k in range(nh_atoms):
        if maxo[k] == 3.0 or ndouble[k] >= 2:
            hyb[k] = 1  # SP
        elif maxo[k] >= 1.5 or arom[k]:
            hyb[k] = 2  # SP2
        else:
            hyb[k] = 3  # SP3
    return {
        "adj": adj,
        "atom_type": atom_type,
        "hydrogen_count": hydrogen,
        "degree": degree,
        "hybridization": hyb,
        "total_charge": float(sum(chg)),
        "atomic_numbers": np.array(Zall, dtype=np.int32),
    }
