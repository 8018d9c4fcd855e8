"""bench.py with the fused post-pool head switched off (models.gnn.FUSED_HEAD = False: the module
path, each Linear on aimx_gemm) — an A/B of the two head paths on the same step.

usage: python tools/ab_module_head.py [bench.py arguments]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aimnet-x2d_amd")]
import models.gnn as gnn  # noqa: E402

gnn.FUSED_HEAD = False
import bench  # noqa: E402

sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[1:]
bench.main()
