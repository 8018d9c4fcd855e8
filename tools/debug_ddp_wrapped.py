"""Two gloo ranks on one GPU running the reference's unchanged DDP wrapping over the autograph's
replay (tests/test_gpu_ddp.py::test_ddp_wrapped_drop_in_equals_full_batch[ddp_wrapped]) with a
progress line per phase, every warning with its stack, a stack dump of every thread every 20 s and
on a crash, into gpurun_out/ddp_rank<r>.log; then (rank "held") one process without DDP whose
parameters' gradient accumulators are made up front on the default stream and held, as DDP's
reducer holds them.

usage: python tools/debug_ddp_wrapped.py
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aimnet-x2d_amd"), os.path.join(ROOT, "tests")]


def rank_main(rank, world, port):
    import faulthandler
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    log = open(os.path.join(ROOT, "gpurun_out", f"ddp_rank{rank}.log"), "w", buffering=1)
    faulthandler.enable(file=log, all_threads=True)
    faulthandler.dump_traceback_later(20, repeat=True, file=log)

    def say(msg):
        log.write(f"{time.strftime('%T')} rank {rank}: {msg}\n")
        log.flush()

    import traceback
    import warnings
    warnings.simplefilter("always")

    def show(message, category, filename, lineno, file=None, line=None):
        say(f"WARNING {category.__name__}: {str(message)[:160]}\n" + "".join(traceback.format_stack()[-12:-1]))
    warnings.showwarning = show

    import numpy as np
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    from aimx import autograph
    from models import L1Loss
    import test_gpu_ddp as T
    held = str(rank).startswith("held")
    if rank == "heldold":  # the capture before stand-ins: gradients taken at the parameters themselves
        class _Same:
            def __init__(self, model, live):
                self.live = live

            def __enter__(self):
                return {id(p): p for p in self.live}

            def __exit__(self, *exc):
                return False
        autograph._aliased = _Same
    b = T._qm9_batch(np.arange(0 if held else rank * T.B_HALF, (1 if held else rank + 1) * T.B_HALF))
    m = T._model()
    autograph.enable(m, True)
    if held:
        accs = [p.view_as(p).grad_fn.next_functions[0][0] for p in m.parameters()]
        say(f"{len(accs)} accumulators held")
        ddp = m
    else:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        say("pg up")
        from torch.nn.parallel import DistributedDataParallel as DDP
        ddp = DDP(m, device_ids=[0], find_unused_parameters=True)
        say("ddp built")
    for it in range(2):
        for p in m.parameters():
            p.grad = None
        out, _, _ = ddp(*b.model_args())
        torch.cuda.synchronize()
        say(f"iter {it} forward done")
        loss = L1Loss()(out, b.targets)
        loss.backward()
        say(f"iter {it} backward returned")
        torch.cuda.synchronize()
        say(f"iter {it} synced")
    g = {n: float(p.grad.norm()) for n, p in m.named_parameters() if p.grad is not None}
    say(f"done, {len(g)} grads, buckets {len(autograph._state(m).buckets)}")
    if not held:
        dist.destroy_process_group()
    faulthandler.cancel_dump_traceback_later()


def main():
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = [subprocess.Popen([sys.executable, __file__, "--rank", str(r), str(port)]) for r in range(2)]
    t0 = time.time()
    while any(p.poll() is None for p in procs) and time.time() - t0 < 150:
        time.sleep(1)
    for p in procs:
        if p.poll() is None:
            p.kill()
    print("exit codes", [p.wait() for p in procs])
    for r in range(2):
        print(open(os.path.join(ROOT, "gpurun_out", f"ddp_rank{r}.log")).read()[-6000:])
    for v in ("held", "heldold"):
        p = subprocess.Popen([sys.executable, __file__, "--rank", v, "0"])
        try:
            print(v, "exit code", p.wait(timeout=120))
        except subprocess.TimeoutExpired:
            p.kill()
            print(v, "killed after 120 s", p.wait())
        print(open(os.path.join(ROOT, "gpurun_out", f"ddp_rank{v}.log")).read()[-6000:])


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--rank":
        rank_main(sys.argv[2] if sys.argv[2].startswith("held") else int(sys.argv[2]), 2, int(sys.argv[3]))
    else:
        main()
