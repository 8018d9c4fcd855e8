"""ORACLE — test infrastructure only. NOT part of the product.

CPU restatement of the reference AIMNet-X2D hot path (mahdi-shafiei/AIMNet-X2D,
src/models/{gnn,layers,pooling}.py, src/datasets/{features,molecular}.py), used as the
checker for the MI355X/HIP implementation in aimnet-x2d_amd/.

Who may import this package: tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg,
and only as the checker / the timed CPU baseline ("kind": "port"). The product path
(aimnet-x2d_amd/) never imports it and fails loudly if its HIP library is missing.

Pinning: the restatement is checked against golden fixtures under tests/golden/ produced in the
development container by importing the reference itself (tests/golden/make_golden.py) — see
tests/test_oracle_golden.py. One boundary stays "parity unpinned": torch_scatter 2.1.2 is not
installed offline, so the scatter_* semantics are restated from its published source (the
reference's own call sites use scatter_add / scatter_softmax / scatter_sum / scatter_mean /
scatter_max, layers.py:158, pooling.py:33,56,79,145,159).

Modules:
  graph.py  multi-hop BFS (features.py:82-150), collate (molecular.py:339-458), stable CSR (numpy)
  model.py  functional fp32 torch-CPU GNN forward (gnn.py:197-308, 622-658; layers.py:63-267;
            pooling.py:15-172); autograd supplies the backward.
"""
