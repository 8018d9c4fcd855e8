"""RDKit-free SMILES -> molecular graph featuriser (QM9 subset).

Restates what the reference obtains from RDKit in ``compute_all``
(reference: src/datasets/features.py:153-334) for the organic subset QM9 uses:

* ``Chem.MolFromSmiles`` + ``Chem.AddHs`` atom order: heavy atoms in SMILES order,
  then each heavy atom's hydrogens appended in heavy-atom order (features.py:166-170).
* ``Chem.GetAdjacencyMatrix`` (features.py:178) -> symmetric 0/1 matrix.
* atom feature indices (features.py:289-319): atom_type = Z-1, hydrogen_count capped at 8,
  degree 0..5 else 6, hybridization index into [S, SP, SP2, SP3, SP3D, SP3D2] else 6
  (datasets/constants.py:9-18).
* hybridization (``atom.GetHybridization()``, features.py:190): RDKit's rule restated. Bonds are
  conjugated when aromatic, or when they leave an atom that carries a multiple bond and has 2-3
  substituents towards a neighbour with at most 3 substituents. An atom's orbital count is its
  total degree plus its lone pairs ((outer electrons - total valence - charge) / 2): 1 -> S,
  2 -> SP, 3 -> SP2, 4 -> SP2 when the atom has at most 3 neighbours and a conjugated bond (amide
  N, ester O, phenol O, aniline N) else SP3, 5 -> SP3D, 6 -> SP3D2.
* potential tetrahedral centres (``Chem.FindMolChiralCenters(includeUnassigned=True)``,
  features.py:212-217): atoms with 4 neighbours (or an N with 3 in a 3-membered ring) whose
  neighbours all fall in different symmetry classes (iterative neighbour-class refinement, the
  legacy perception's rank refinement restated); each centre's neighbour list is in bond order.
* cis/trans (features.py:220-283) needs E/Z-specified double bonds. QM9 SMILES carry no ``/`` or
  backslash marks, so the lists are empty (marked bonds are read as plain single bonds).

Parity unpinned: RDKit is not installed offline and the reference holds no featurised fixtures,
so these rules are restated, not checked against RDKit output. Known gaps: ring
pseudo-asymmetric centres (e.g. cis/trans-1,3-dimethylcyclobutane) are not reported; the
neighbour order around a ring-closure atom follows bond creation order (closure bonds when the
ring closes). The graph topology and atom ordering, which the hot path consumes, are exact.
"""
from __future__ import annotations

import numpy as np

_Z = {"H": 1, "B": 5, "C": 6, "N": 7, "O": 8, "F": 9, "P": 15, "S": 16, "Cl": 17, "Br": 35, "I": 53}
_VALENCE = {1: 1, 5: 3, 6: 4, 7: 3, 8: 2, 9: 1, 15: 3, 16: 2, 17: 1, 35: 1, 53: 1}
_BOND = {"-": 1.0, "=": 2.0, "#": 3.0, ":": 1.5, "/": 1.0, "\\": 1.0}
_NOUTER = {1: 1, 5: 3, 6: 4, 7: 5, 8: 6, 9: 7, 15: 5, 16: 6, 17: 7, 35: 7, 53: 7}
# largest valence RDKit's sanitisation accepts per element (a charged atom takes the valences of its
# isoelectronic neighbour: N+ as C, O- as F, ...); more and MolFromSmiles returns None, which
# compute_all turns into a dropped molecule (features.py:165-167)
_MAX_VALENCE = {1: 1, 5: 3, 6: 4, 7: 3, 8: 2, 9: 1, 15: 7, 16: 6, 17: 1, 35: 1, 53: 5}
_BY_NOUTER = {3: 5, 4: 6, 5: 7, 6: 8, 7: 9}


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


def _conjugated_bonds(Z, deg, chg, bonds, nbr_bonds):
    """Per-bond conjugation flags (RDKit setConjugation / markConjAtomBonds, restated): aromatic
    bonds, plus, for every atom with a multiple bond, 2-3 substituents and electrons to share,
    that bond and each other bond to a neighbour with at most 3 substituents."""
    conj = [o == 1.5 for _, _, o in bonds]

    def cand(a):  # first-row atoms, or heavier ones outside groups 15/16 (or a terminal chalcogen)
        no = _NOUTER.get(Z[a], 0)
        return Z[a] <= 10 or (no != 5 and no != 6) or (no == 6 and deg[a] < 2)

    for a in range(len(Z)):
        if _NOUTER.get(Z[a], 0) < 4:
            continue
        dv = _VALENCE.get(Z[a], 0)
        if dv <= 1 or deg[a] > 3:  # countAtomElec < 0: univalent, or more than 3 neighbours
            continue
        nlp = max(_NOUTER[Z[a]] - dv - chg[a], 0)
        if (dv - deg[a]) + nlp <= 0 or not cand(a) or not 2 <= deg[a] <= 3:
            continue
        for b1 in nbr_bonds[a]:
            if bonds[b1][2] < 1.5:
                continue
            for b2 in nbr_bonds[a]:
                if b2 == b1:
                    continue
                i, j, _ = bonds[b2]
                other = j if i == a else i
                if deg[other] <= 3 and cand(other):
                    conj[b1] = conj[b2] = True
    return conj


def _hybridization(Z, deg, chg, bonds, nbr_bonds, conj):
    """RDKit setHybridization restated: index into [S, SP, SP2, SP3, SP3D, SP3D2], else 6."""
    hyb = np.zeros(len(Z), dtype=np.int8)
    for a in range(len(Z)):
        if Z[a] <= 1:
            norbs = deg[a]
        else:
            tv = int(np.floor(sum(bonds[b][2] for b in nbr_bonds[a]) + 0.5))
            norbs = deg[a] + max(0, _NOUTER.get(Z[a], 0) - (tv + chg[a])) // 2
        if norbs <= 1:
            h = 0
        elif norbs == 2:
            h = 1
        elif norbs == 3:
            h = 2
        elif norbs == 4:
            h = 2 if deg[a] <= 3 and any(conj[b] for b in nbr_bonds[a]) else 3
        elif norbs in (5, 6):
            h = norbs - 1
        else:
            h = 6
        hyb[a] = h
    return hyb


def _symmetry_classes(Z, chg, bonds, nbr_bonds):
    """Atom classes by iterative refinement of (element, charge) with the multiset of
    (bond order, neighbour class), until the partition stops splitting."""
    cls = [(Z[a], chg[a]) for a in range(len(Z))]
    keys = sorted(set(cls))
    cls = [keys.index(c) for c in cls]
    n_cls = len(keys)
    while True:
        sig = []
        for a in range(len(Z)):
            nb = []
            for b in nbr_bonds[a]:
                i, j, o = bonds[b]
                nb.append((o, cls[j if i == a else i]))
            sig.append((cls[a], tuple(sorted(nb))))
        keys = sorted(set(sig))
        new = [keys.index(x) for x in sig]
        if len(keys) == n_cls:
            return new
        cls, n_cls = new, len(keys)


def _in_ring_of_3(a, nbrs):
    return any(c in nbrs[b] for b in nbrs[a] for c in nbrs[a] if b < c)


def featurize(smi: str):
    """SMILES -> dict(adj (int32 [n,n]), atom feature index arrays (int8), total_charge, Z,
    chiral_tensors (neighbour lists of potential tetrahedral centres), cis/trans pairs).

    Atom order follows RDKit AddHs: heavy atoms first, then hydrogens grouped by heavy atom.
    """
    Z, hbonds, hcnt, chg, arom = parse_smiles(smi)
    nh_atoms = len(Z)
    bo_sum = [0.0] * nh_atoms
    for a, b, o in hbonds:
        bo_sum[a] += o
        bo_sum[b] += o
    n_h = []
    for k in range(nh_atoms):
        if hcnt[k] >= 0:
            n_h.append(hcnt[k])
        else:
            v = _VALENCE.get(Z[k], 0)
            n_h.append(max(0, v - int(np.floor(bo_sum[k] + 0.5))))
    for k in range(nh_atoms):
        if arom[k]:
            continue  # aromatic bonds count 1.5 here; RDKit checks the Kekule valence
        tv = int(np.floor(bo_sum[k] + 0.5)) + n_h[k]
        z_eff = _BY_NOUTER.get(_NOUTER.get(Z[k], 0) - chg[k], Z[k]) if chg[k] else Z[k]
        if Z[k] <= 9 and tv > _MAX_VALENCE.get(z_eff, 8):
            raise SmilesError(f"explicit valence {tv} of atom {k} (Z={Z[k]}, charge {chg[k]}) exceeds what RDKit accepts")
    n = nh_atoms + sum(n_h)
    Zall = list(Z)
    chg_all = list(chg) + [0] * (n - nh_atoms)
    bonds = list(hbonds)
    nxt = nh_atoms
    for k in range(nh_atoms):  # AddHs: each heavy atom's hydrogens, appended in heavy-atom order
        for _ in range(n_h[k]):
            bonds.append((k, nxt, 1.0))
            Zall.append(1)
            nxt += 1
    adj = np.zeros((n, n), dtype=np.int32)
    nbr_bonds = [[] for _ in range(n)]  # bond indices per atom, in bond creation order
    for bi, (a, b, _) in enumerate(bonds):
        adj[a, b] = adj[b, a] = 1
        nbr_bonds[a].append(bi)
        nbr_bonds[b].append(bi)
    nbrs = [[(j if i == a else i) for i, j, _ in (bonds[b] for b in nbr_bonds[a])] for a in range(n)]
    deg = [len(x) for x in nbrs]
    conj = _conjugated_bonds(Zall, deg, chg_all, bonds, nbr_bonds)
    hyb = _hybridization(Zall, deg, chg_all, bonds, nbr_bonds, conj)
    cls = _symmetry_classes(Zall, chg_all, bonds, nbr_bonds)
    chiral = []
    for a in range(nh_atoms):
        if deg[a] == 4 or (Zall[a] == 7 and deg[a] == 3 and _in_ring_of_3(a, nbrs)):
            if len({cls[b] for b in nbrs[a]}) == deg[a]:
                chiral.append(np.array(nbrs[a], dtype=np.int32))
    atom_type = np.array([z - 1 for z in Zall], dtype=np.int8)
    hydrogen = np.zeros(n, dtype=np.int8)
    hydrogen[:nh_atoms] = np.minimum(np.array(n_h, dtype=np.int64), 8)
    degree = np.array([d if d < 6 else 6 for d in deg], dtype=np.int8)
    return {
        "adj": adj,
        "atom_type": atom_type,
        "hydrogen_count": hydrogen,
        "degree": degree,
        "hybridization": hyb,
        "total_charge": float(sum(chg)),
        "atomic_numbers": np.array(Zall, dtype=np.int32),
        "chiral_tensors": chiral,
        "cis_bonds_tensors": [],
        "trans_bonds_tensors": [],
    }
