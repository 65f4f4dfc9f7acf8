"""Diagnostic: the grouped RCCL gather plan captured in two double-buffered graphs at
world 1, in one of three arrangements, with a progress line per stage (which call a
hang is in).

    python tools/rccl_two_graphs.py --variant {one_comm,one_comm_prewarm,two_comms}

one_comm: graph 0 captured, then set 1's eager warm-up + capture on the same comm
(mixed eager / captured RCCL work outstanding on one communicator).
one_comm_prewarm: both sets warmed up eagerly before either graph is captured.
two_comms: one communicator per input set (each graph owns its comm).
"""
import argparse
import os
import sys
import time

sys.path.insert(0, ".")


def log(msg):
    print(f"[{time.strftime('%H:%M:%S')}] {msg}", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", default="one_comm", choices=["one_comm", "one_comm_prewarm", "two_comms"])
    ap.add_argument("--teardown", default="reset", choices=["reset", "del"])
    ap.add_argument("--close", default="abort", choices=["abort", "close"])
    a = ap.parse_args()
    import faulthandler
    faulthandler.dump_traceback_later(45, exit=True)
    import torch

    from triton_client_amd.parallel.rccl import RECV, SEND, NativeComm
    from triton_client_amd.pipelines.graph import GraphRunner

    torch.cuda.set_device(0)
    comms = [NativeComm(0, 1)]
    if a.variant == "two_comms":
        comms.append(NativeComm(0, 1))
    log(f"{a.variant}: {len(comms)} comm(s) up")
    inputs = [torch.zeros(1, device="cuda"), torch.zeros(1, device="cuda")]
    src = [torch.zeros((32, 300, 4), device="cuda"), torch.zeros((32,), dtype=torch.int32, device="cuda")]
    dst = [[torch.empty_like(t) for t in src] for _ in range(2)]

    def step(k):
        comm = comms[k % len(comms)]

        def fn():
            src[0].copy_(inputs[k].expand_as(src[0]))
            src[1].copy_(inputs[k].to(torch.int32).expand_as(src[1]))
            comm.group_p2p([(RECV, d, 0) for d in dst[k]] + [(SEND, s, 0) for s in src])
            return src
        return fn
    runs = [GraphRunner(step(0)), GraphRunner(step(1))]
    if a.variant == "one_comm_prewarm":
        for k in (0, 1):
            step(k)()
        torch.cuda.synchronize()
        log("both sets warmed up eagerly")
    for k, r in enumerate(runs):
        r.capture()
        torch.cuda.synchronize()
        log(f"graph {k} captured")
    ok = True
    for t, v in enumerate((2.0, 5.0, 9.0, 13.0)):
        k = t % 2
        inputs[k].fill_(v)
        runs[k]()
        torch.cuda.synchronize()
        got = float(dst[k][0].reshape(-1)[0])
        log(f"replay {t} (set {k}): got {got} want {v}")
        ok &= got == v and int(dst[k][1][0]) == int(v)
    import gc
    graphs = [r.graph for r in runs]
    del runs
    gc.collect()
    log(f"runners released; graph refcounts {[sys.getrefcount(g) - 2 for g in graphs]}")
    if a.teardown == "reset":
        for g in graphs:
            g.reset()
        log("graphs reset")
    del graphs
    gc.collect()
    torch.cuda.synchronize()
    log("synchronized")
    for i, c in enumerate(comms):
        getattr(c, a.close)()
        log(f"comm {i} {a.close}ed")
    log("OK" if ok else "MISMATCH")
    sys.stdout.flush()
    os._exit(0 if ok else 1)


if __name__ == "__main__":
    main()
