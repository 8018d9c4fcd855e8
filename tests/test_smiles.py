"""The RDKit-free featuriser (aimx/smiles.py) on known answers: RDKit's hybridization rule with
conjugation (reference features.py:186-196 via atom.GetHybridization()), potential tetrahedral
centres (features.py:212-217, FindMolChiralCenters(includeUnassigned=True)), AddHs atom order and
the sanitisation rejects that make compute_all return None (features.py:165-167).
Parity unpinned: RDKit is absent offline; the expectations are textbook chemistry (amide N,
ester O and phenol O are SP2 in RDKit's model), not RDKit output."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "aimnet-x2d_amd"))
from aimx.smiles import SmilesError, featurize  # noqa: E402

S, SP, SP2, SP3 = 0, 1, 2, 3


def heavy_hyb(smi):
    f = featurize(smi)
    nh = int((f["atomic_numbers"] > 1).sum())
    return f["hybridization"][:nh].tolist(), f


@pytest.mark.parametrize("smi,want", [
    ("CC(=O)N", [SP3, SP2, SP2, SP2]),            # acetamide: the amide N is conjugated
    ("COC=O", [SP3, SP2, SP2, SP2]),              # methyl formate: the ester O too
    ("CC#N", [SP3, SP, SP]),
    ("C=C=C", [SP2, SP, SP2]),
    ("c1ccncc1", [SP2] * 6),
    ("c1cc[nH]c1", [SP2] * 5),
    ("c1ccoc1", [SP2] * 5),
    ("Oc1ccccc1", [SP2] * 7),
    ("CN", [SP3, SP3]),
    ("CO", [SP3, SP3]),
    ("C=CN", [SP2, SP2, SP2]),
    ("[NH3+]CC([O-])=O", [SP3, SP3, SP2, SP2, SP2]),
    ("C[N+](=O)[O-]", [SP3, SP2, SP2, SP2]),
    ("CS(=O)(=O)C", [SP3, SP3, SP2, SP2, SP3]),
])
def test_hybridization_known_answers(smi, want):
    got, f = heavy_hyb(smi)
    assert got == want
    assert (f["hybridization"][len(want):] == S).all()  # hydrogens


@pytest.mark.parametrize("smi,centres", [
    ("CC(O)CC", [[0, 2, 3, 8]]),        # 2-butanol: C1 with C0, O2, C3 and its H (index 8)
    ("CC(C)O", []),
    ("OC1CCCC1", []),                   # the two ring branches are the same
    ("CC(C)(C)C", []),
    ("C1CC1", []),
    ("NC(C)C(=O)O", [[0, 2, 3, 8]]),    # alanine
    ("FC(Cl)Br", [[0, 2, 3, 4]]),
    ("CC1CCCC1O", [[0, 2, 5, 10], [4, 1, 6, 17]]),  # ring closure bond listed when the ring closes
])
def test_potential_tetrahedral_centres(smi, centres):
    f = featurize(smi)
    assert [c.tolist() for c in f["chiral_tensors"]] == centres
    assert f["cis_bonds_tensors"] == [] and f["trans_bonds_tensors"] == []


def test_addhs_order_degree_and_h_count():
    f = featurize("CC(=O)O")  # heavy atoms in SMILES order, then H of C0 (3), then H of O3 (1)
    assert f["atomic_numbers"].tolist() == [6, 6, 8, 8, 1, 1, 1, 1]
    assert f["hydrogen_count"].tolist() == [3, 0, 0, 1, 0, 0, 0, 0]
    assert f["degree"].tolist() == [4, 3, 1, 2, 1, 1, 1, 1]
    assert f["adj"][0, 4:7].tolist() == [1, 1, 1] and f["adj"][3, 7] == 1
    assert (f["adj"] == f["adj"].T).all()


@pytest.mark.parametrize("smi", ["CN(=O)=O", "C(C)(C)(C)(C)C", "CO(C)C"])
def test_rdkit_sanitisation_rejects(smi):
    with pytest.raises(SmilesError):
        featurize(smi)
