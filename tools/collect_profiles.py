"""Copy the round's profile summaries from gpurun_out/round/ into profiles/ (tracked).

usage: python tools/collect_profiles.py <round tag, e.g. r01>
"""
import glob
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1]
src = os.path.join(ROOT, "gpurun_out", "round")
dst = os.path.join(ROOT, "profiles")
os.makedirs(dst, exist_ok=True)


def one(pattern):
    """The newest match (gpurun_out/ accumulates the run directories of earlier calls)."""
    hits = glob.glob(os.path.join(src, pattern), recursive=True)
    if not hits:
        raise SystemExit(f"missing {pattern}")
    return max(hits, key=os.path.getmtime)


shutil.copy(one("bench/**/*kernel_stats.csv"), os.path.join(dst, f"{tag}_bench_kernel_stats.csv"))
shutil.copy(one("roof/**/*kernel_stats.csv"), os.path.join(dst, f"{tag}_hop_roofline_kernel_stats.csv"))
with open(os.path.join(dst, f"{tag}_step_breakdown.txt"), "w") as f:
    f.write(subprocess.run([sys.executable, os.path.join(ROOT, "tools", "step_kernels.py"), os.path.join(src, "bench")],
                           capture_output=True, text=True, check=True).stdout)
subprocess.run([sys.executable, os.path.join(ROOT, "tools", "hop_traffic.py"), os.path.join(src, "pmc_fetch"),
                os.path.join(src, "pmc_write"), os.path.join(src, "pmc_fetch.log"),
                os.path.join(dst, "hop_traffic.json")], check=True)
for name in ("bench_plain.log", "roof.log"):
    lines = [ln for ln in open(os.path.join(src, name)) if ln.startswith("{")]
    with open(os.path.join(dst, f"{tag}_{name.replace('.log', '.json')}"), "w") as f:
        f.write(lines[-1])
print(json.dumps(json.load(open(os.path.join(dst, "hop_traffic.json"))), indent=1))

# extra configs (c3/c4/c5 bench lines), the c4 step breakdown and its MFMA utilisation
for cfgname in ("c3", "c4", "c5", "c2_amp", "c4_amp", "c5_amp", "c5_stream"):
    p = os.path.join(src, f"bench_{cfgname}.log")
    if os.path.exists(p):
        lines = [ln for ln in open(p) if ln.startswith("{")]
        with open(os.path.join(dst, f"{tag}_bench_{cfgname}.json"), "w") as f:
            f.write(lines[-1])
if os.path.isdir(os.path.join(src, "c4_trace")):
    with open(os.path.join(dst, f"{tag}_c4_step_breakdown.txt"), "w") as f:
        f.write(subprocess.run([sys.executable, os.path.join(ROOT, "tools", "step_kernels.py"),
                                os.path.join(src, "c4_trace")], capture_output=True, text=True, check=True).stdout)
for cfgname in ("c2", "c4", "c5"):
    if os.path.isdir(os.path.join(src, f"{cfgname}_mfma")):
        with open(os.path.join(dst, f"{tag}_{cfgname}_mfma_util.json"), "w") as f:
            f.write(subprocess.run([sys.executable, os.path.join(ROOT, "tools", "mfma_summary.py"),
                                    os.path.join(src, f"{cfgname}_mfma"), "15"], capture_output=True, text=True,
                                   check=True).stdout)
# step kernel sequences (default bench command = c2, c4, c5), the parity report, the DDP lines,
# the k_mlps phase stamps and the GPU suite's summary (part c)
for name, out in (("c2_trace_step_seq.txt", "c2_step_seq.txt"), ("c4_trace_step_seq.txt", "c4_step_seq.txt"),
                  ("c5_trace_step_seq.txt", "c5_step_seq.txt"), ("parity.json", "parity.json"),
                  ("mlps_trace_c4.log", "mlps_trace_c4.txt"), ("mlps_trace_c5.log", "mlps_trace_c5.txt")):
    p = os.path.join(src, name)
    if os.path.exists(p):
        with open(p) as fi, open(os.path.join(dst, f"{tag}_{out}"), "w") as fo:
            fo.write("".join(ln for ln in fi if "amdgpu.ids" not in ln))
for name in ("bench_ddp_world1", "bench_dp2_gloo"):
    p = os.path.join(src, f"{name}.log")
    if os.path.exists(p):
        lines = [ln for ln in open(p) if ln.startswith("{")]
        if lines:
            with open(os.path.join(dst, f"{tag}_{name}.json"), "w") as f:
                f.write(lines[-1])
p = os.path.join(src, "tests.log")
if os.path.exists(p):
    tail = [ln for ln in open(p) if "passed" in ln or "failed" in ln or ln.startswith("FAILED")]
    with open(os.path.join(dst, f"{tag}_gpu_tests.txt"), "w") as f:
        f.write("".join(tail[-20:]))

# the hop roofline's forward / backward launches separated (same kernel instance at c2), and the
# c5 stream feed's own rate
for name in ("roof_split_c2.json", "roof_split_c5.json"):
    p = os.path.join(src, name)
    if os.path.exists(p):
        shutil.copy(p, os.path.join(dst, f"{tag}_{name}"))
p = os.path.join(src, "feed_rate_c5.log")
if os.path.exists(p):
    lines = [ln for ln in open(p) if ln.startswith("{")]
    if lines:
        with open(os.path.join(dst, f"{tag}_feed_rate_c5.json"), "w") as f:
            f.write(lines[-1])
