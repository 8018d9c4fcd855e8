"""Port/reference CPU ratio (SURVEY.md §8c "what the build's CPU counterpart must reproduce" (ii)).

Times the same c2 train step (forward + L1 loss + backward + clip(1.0) + Adam, dropout on, 512
QM9-shaped molecules, hidden 256, 3 hops) on this host's CPU twice, on identical inputs and weights:
  * the oracle's CPU restatement (oracle/model.py, the `cpu_baseline` leg bench.py times on the GPU
    box, kind "port");
  * the reference's own GNN imported from /root/reference/src (with the torch_scatter 2.1.2
    stand-in tests/golden/_shim, as tests/golden/make_golden.py does).
Each runs in its own child process (the reference's `models` package must not meet the build's).
Runs ONLY in the development container (the reference is not on the GPU box); the committed result
(profiles/port_vs_reference.json) is what bench.py reports as `cpu_baseline.port_vs_reference`.

usage: python tools/port_vs_reference.py [--threads 8] [--steps 12] [--out profiles/port_vs_reference.json]
"""
import argparse
import json
import os
import platform
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference/src"
FS = {"atom_type": 119, "hydrogen_count": 9, "degree": 7, "hybridization": 7}
KEYS = ("atom_type", "hydrogen_count", "degree", "hybridization")


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def make_inputs(path):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "aimnet-x2d_amd")]
    import numpy as np
    import bench
    col, tg, q = bench.make_collated(bench.CONFIGS["c2"], 1, 4321)[0]
    np.savez(path, edges=col["edges"], batch=col["batch"], targets=tg, total_charges=q,
             **{k: col["feats"][:, i].copy() for i, k in enumerate(KEYS)})


def child(which, path, threads, steps, seed=0):
    import numpy as np
    import torch
    torch.set_num_threads(threads)
    torch.manual_seed(0)
    z = np.load(path)
    af = {k: torch.from_numpy(z[k]).long() for k in KEYS}
    edges, batch = torch.from_numpy(z["edges"]).long(), torch.from_numpy(z["batch"]).long()
    tc, tg = torch.from_numpy(z["total_charges"]), torch.from_numpy(z["targets"])
    sys.path.insert(0, ROOT)
    from oracle import model as om
    cfg = om.default_config(hidden_dim=256, num_shells=3, output_dim=1)
    params = om.seeded_params(cfg, seed)
    if which == "oracle":
        p = {k: v.requires_grad_() for k, v in params.items()}
        plist = list(p.values())

        def fwd():
            return om.gnn_forward(p, cfg, af, edges, batch, tc, training=True)[0]
    else:
        sys.dont_write_bytecode = True
        os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
        sys.path.insert(0, REF)
        sys.path.insert(0, os.path.join(ROOT, "tests", "golden", "_shim"))
        for m in [m for m in sys.modules if m == "models" or m.startswith("models.")]:
            del sys.modules[m]
        from models.gnn import GNN
        assert GNN.__module__ == "models.gnn" and sys.modules["models.gnn"].__file__.startswith(REF)
        model = GNN(FS, 256, 1, num_shells=3)
        model.load_state_dict(params)
        model.train()
        plist = list(model.parameters())
        e0 = torch.empty(0, 2, dtype=torch.long)

        def fwd():
            return model(af, edges, batch, tc, torch.empty(0, 4, dtype=torch.long), e0, e0)[0]
    opt = torch.optim.Adam(plist, lr=2.5e-4)

    def step():
        opt.zero_grad(set_to_none=True)
        loss = torch.nn.functional.l1_loss(fwd(), tg)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(plist, 1.0)
        opt.step()

    for _ in range(2):
        step()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    dt = time.perf_counter() - t0
    print(json.dumps({"which": which, "mol_per_s": 512 * steps / dt, "s_per_step": dt / steps}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "port_vs_reference.json"))
    ap.add_argument("--child", nargs=2)
    a = ap.parse_args()
    if a.child:
        child(a.child[0], a.child[1], a.threads, a.steps)
        return
    res, samples = {}, {}
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "c2_inputs.npz")
        make_inputs(path)
        for which in ("oracle", "reference") * 3:  # interleaved, best of three each (this host is shared)
            out = subprocess.run([sys.executable, __file__, "--threads", str(a.threads), "--steps", str(a.steps),
                                  "--child", which, path], check=True, capture_output=True, text=True,
                                 env={**os.environ, "PYTHONDONTWRITEBYTECODE": "1"}).stdout
            r = json.loads(out.strip().splitlines()[-1])
            res[which] = max(res.get(which, 0.0), r["mol_per_s"])
            samples.setdefault(which, []).append(round(r["mol_per_s"], 1))
    rec = {"config": "c2 (512 QM9-shaped molecules, hidden 256, 3 hops, train step fwd+L1+bwd+clip+Adam, "
                     "dropout on)",
           "threads": a.threads, "cpu_model": cpu_model(), "cpu_count": os.cpu_count(),
           "oracle_mol_per_s": round(res["oracle"], 1), "reference_mol_per_s": round(res["reference"], 1),
           "ratio_port_over_reference": round(res["oracle"] / res["reference"], 3),
           "samples_mol_per_s": samples, "steps": a.steps, "measured": "development container (reference importable here only)",
           "script": "tools/port_vs_reference.py"}
    print(json.dumps(rec))
    with open(a.out, "w") as f:
        json.dump(rec, f, indent=1)


if __name__ == "__main__":
    main()
