"""CPU-side checks: the C-ABI library loads and exports every symbol include/aimx.h declares, the
module API mirrors the reference (names, signatures, state_dict keys), and the product path fails
loudly without a HIP device (no CPU fallback)."""
import inspect
import os
import re

import pytest
import torch

from conftest import ROOT


def _header_symbols():
    src = open(os.path.join(ROOT, "include", "aimx.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|size_t|const char\*)\s+(aimx_\w+)\s*\(", src, re.M)))


def test_library_exports_every_header_symbol():
    import ctypes

    from aimx import _lib
    lib = _lib.load()
    syms = _header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), s
        assert s in _lib.EXPORTED_SYMBOLS, f"{s} not bound in aimx/_lib.py"
    assert lib.aimx_version().startswith(b"aimx/")
    assert isinstance(lib.aimx_csr_workspace_bytes(100, 10), int)
    del ctypes


def test_struct_layouts_match_header():
    """ctypes mirrors of the C structs: field names in header order."""
    from aimx import _lib
    src = open(os.path.join(ROOT, "include", "aimx.h")).read()
    for cname, py in (("AimxGemmArgs", _lib.GemmArgs), ("AimxShellStack", _lib.ShellStack),
                      ("AimxShellStackGrad", _lib.ShellStackGrad), ("AimxEmbeddingTables", _lib.EmbeddingTables),
                      ("AimxHead", _lib.Head), ("AimxHeadGrad", _lib.HeadGrad), ("AimxAdamTensor", _lib.AdamTensor),
                      ("AimxAdamHyper", _lib.AdamHyper), ("AimxLossAccum", _lib.LossAccum),
                      ("AimxPadBatch", _lib.PadBatch)):
        body = re.search(r"typedef struct (?:%s )?\{([^{}]*)\} %s;" % (cname, cname), src, re.S).group(1)
        body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
        names = re.findall(r"\**\s*(\w+)\s*(?:\[[^\]]*\])?\s*[;,]", body)
        assert names == [f[0] for f in py._fields_], (cname, names)


def test_module_api_and_state_dict_keys():
    from models import GNN, ShellConvolutionLayer
    from models.pooling import MultiHeadAttentionPoolingLayer, create_pooling_layer
    from oracle.model import default_config, param_shapes
    fs = {"atom_type": 119, "hydrogen_count": 9, "degree": 7, "hybridization": 7}
    sig = inspect.signature(GNN.__init__)
    assert list(sig.parameters)[1:] == [
        "feature_sizes", "hidden_dim", "output_dim", "num_shells", "num_message_passing_layers", "dropout",
        "ffn_hidden_dim", "ffn_num_layers", "pooling_type", "task_type", "embedding_dim", "use_partial_charges",
        "use_stereochemistry", "ffn_dropout", "activation_type", "shell_conv_num_mlp_layers", "shell_conv_dropout",
        "attention_num_heads", "attention_temperature", "loss_function"]
    assert list(inspect.signature(GNN.forward).parameters)[1:] == [
        "atom_features", "multi_hop_edge_indices", "batch_indices", "total_charges", "tetrahedral_indices",
        "cis_indices", "trans_indices"]
    for kw in (dict(hidden_dim=256), dict(hidden_dim=128, pooling_type="sum"),
               dict(hidden_dim=256, num_shells=4, use_partial_charges=True, output_dim=12)):
        cfg = default_config(**kw)
        m = GNN(fs, cfg["hidden_dim"], cfg["output_dim"], num_shells=cfg["num_shells"],
                pooling_type=cfg["pooling_type"], use_partial_charges=cfg["use_partial_charges"])
        sd = m.state_dict()
        assert [k for k, _ in param_shapes(cfg)] == list(sd)
        assert isinstance(m.concat_self_other, torch.nn.Linear)
        assert m.get_model_info()["hidden_dim"] == cfg["hidden_dim"]
    assert len(GNN(fs, 512, 1).state_dict()) == 73
    layer = ShellConvolutionLayer(38, 38, num_hops=3)
    assert [n for n, _ in layer.named_parameters()][:2] == ["input_proj.weight", "input_proj.bias"]
    assert isinstance(create_pooling_layer("attention", 64), MultiHeadAttentionPoolingLayer)
    with pytest.raises(ValueError):
        create_pooling_layer("nope", 64)


def test_no_cpu_fallback():
    from aimx import AimxError
    from models import GNN
    fs = {"atom_type": 119, "hydrogen_count": 9, "degree": 7, "hybridization": 7}
    m = GNN(fs, 128, 1)
    n = 5
    af = {k: torch.zeros(n, dtype=torch.long) for k in fs}
    e = torch.tensor([[0, 1], [1, 0]])
    with pytest.raises(AimxError):
        m(af, e, torch.zeros(n, dtype=torch.long), torch.zeros(1), torch.empty(0, 4, dtype=torch.long),
          torch.empty(0, 2, dtype=torch.long), torch.empty(0, 2, dtype=torch.long))


def test_pad_collated_keeps_real_molecules():
    import numpy as np

    from aimx import data as adata
    from aimx.synth import QM9Asset
    col = adata.collate(QM9Asset().molecules(range(8)), 3)
    n, e = col["batch"].shape[0], col["edges"].shape[0]
    pc = adata.pad_collated(col, n + 10, e + 25, 8, n_pad_mols=4)
    assert np.array_equal(pc["edges"][:e], col["edges"]) and np.array_equal(pc["batch"][:n], col["batch"])
    assert (pc["batch"][n:] >= 8).all() and (pc["batch"][n:] < 12).all() and pc["n_atoms"].sum() == n + 10
    assert list(pc["n_atoms"][8:]) == [3, 3, 2, 2] and (np.diff(pc["batch"]) >= 0).all()
    assert (pc["edges"][e:] >= n).all() and (pc["edges"][e:] < n + 10).all()


def test_fused_adam_has_no_cpu_path():
    import pytest
    import torch

    from aimx import AimxError
    from aimx.optim import FusedAdam
    p = torch.zeros(4, requires_grad=True)
    p.grad = torch.ones(4)
    with pytest.raises(AimxError):
        FusedAdam([p], lr=1e-3, max_grad_norm=1.0).step()


def test_head_cluster_rule(monkeypatch):
    """Clustered head launches: a lone process and data parallelism with one GPU per rank keep them;
    ranks sharing a GPU and an unknown launcher layout drop to 1 workgroup per tile
    (aimx/_lib.py head_cluster_allowed); HEAD_CLUSTER_FORCE overrides."""
    import torch.distributed as dist

    from aimx import _lib
    for k in ("LOCAL_WORLD_SIZE", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setattr(_lib, "HEAD_CLUSTER_FORCE", None)
    assert _lib.head_cluster(256) == 2 and _lib.head_cluster(512) == 4  # lone process
    monkeypatch.setattr(dist, "is_initialized", lambda: True)
    monkeypatch.setattr(dist, "get_world_size", lambda group=None: 8)
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 8)
    monkeypatch.setattr(torch.cuda, "current_device", lambda: 3)
    assert _lib.head_cluster(256) == 1  # no LOCAL_WORLD_SIZE: layout unknown
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    monkeypatch.setenv("LOCAL_RANK", "3")
    assert _lib.head_cluster(256) == 2 and _lib.head_cluster(512) == 4  # torchrun, one GPU per rank
    monkeypatch.setenv("LOCAL_RANK", "0")
    assert _lib.head_cluster(256) == 1  # this rank is not on its own device
    monkeypatch.setenv("LOCAL_RANK", "3")
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    assert _lib.head_cluster(256) == 1  # 8 ranks share one GPU (rehearsal)
    monkeypatch.setattr(_lib, "HEAD_CLUSTER_FORCE", 4)
    assert _lib.head_cluster(256) == 4  # explicit override


def test_product_library_switches_are_the_documented_options():
    """The product library reads no environment variable (getenv only in the tuning build's branch
    of version.hip), and the only AIMX_* names compiled into it are the path options include/aimx.h
    documents (tune_i64 knobs compile to their defaults: their names must not be in libaimx.so)."""
    csrc = os.path.join(ROOT, "aimnet-x2d_amd", "csrc")
    header = open(os.path.join(ROOT, "include", "aimx.h")).read()
    block = header[header.index("/* Path options"):header.index("int aimx_set_option")]
    documented = set(re.findall(r'"(AIMX_[A-Z0-9_]+)"', block))
    used = set()
    for dirpath, _, files in os.walk(csrc):
        for f in files:
            if not f.endswith((".hip", ".h", ".cpp")):
                continue
            src = open(os.path.join(dirpath, f)).read()
            used |= set(re.findall(r'opt_i64\("(AIMX_[A-Z0-9_]+)"', src))
            if "getenv" in src:
                assert f == "version.hip", f
                i = src.index("getenv")
                assert src.rfind("#ifdef AIMX_TUNING", 0, i) > src.rfind("#endif", 0, i), "getenv outside the tuning branch"
    assert used == documented, (sorted(used - documented), sorted(documented - used))
    assert len(documented) < 10
    lib = os.path.join(ROOT, "aimnet-x2d_amd", "lib", "libaimx.so")
    if os.path.exists(lib):
        names = set(re.findall(rb"AIMX_[A-Z0-9_]{2,}", open(lib, "rb").read()))
        names = {n.decode() for n in names if not n.decode().startswith(("AIMX_PREC", "AIMX_ACT", "AIMX_OK", "AIMX_EARG"))}
        assert names <= documented, sorted(names - documented)
