"""Diagnostic: gradient accumulation under aimx.autograph vs eager, per parameter."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aimnet-x2d_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402
import test_gpu_autograph as T  # noqa: E402
from aimx import autograph  # noqa: E402

b = T._batches(1, 31)[0]
m0, m1, m2 = T._model(), T._model(), T._model()
m1.load_state_dict(m0.state_dict())
m2.load_state_dict(m0.state_dict())
autograph.enable(m2)
out, _, _ = m0(*b.model_args())
out.sum().backward()  # single fresh gradient
for m in (m1, m2):
    for _ in range(2):
        out, _, _ = m(*b.model_args())
        out.sum().backward()
names = [k for k, _ in m0.named_parameters()]
P0, P1, P2 = list(m0.parameters()), list(m1.parameters()), list(m2.parameters())
print("part1 (2x accumulate): rel(m1, 2*m0), rel(m2, 2*m0)")
for k, a, c, d in zip(names, P0, P1, P2):
    if a.grad is not None:
        print(f"  {k:45s} {T._rel(c.grad, 2 * a.grad):.2e} {T._rel(d.grad, 2 * a.grad):.2e}")
for m in (m1, m2):
    m.zero_grad(set_to_none=False)
    out, _, _ = m(*b.model_args())
    out.sum().backward()
print("part2 (zeroed in place, 1x): rel(m1, m0), rel(m2, m0)")
for k, a, c, d in zip(names, P0, P1, P2):
    if a.grad is not None:
        print(f"  {k:45s} {T._rel(c.grad, a.grad):.2e} {T._rel(d.grad, a.grad):.2e}")
