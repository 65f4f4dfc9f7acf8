"""Standalone server: python -m triton_client_amd.server --models YOLOv5nCOCO,pointpillar_kitti"""
import argparse
import logging

from . import KServeServer, ModelRepository


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(description="KServe-v2 (Triton protocol) server on MI355X")
    ap.add_argument("--models", default="YOLOv5nCOCO,pointpillar_kitti")
    ap.add_argument("--model-repository", default=None, help="Triton-style directory of config.pbtxt files")
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=8001)
    ap.add_argument("--metrics-port", type=int, default=8002)
    ap.add_argument("--device", default="auto")
    ap.add_argument("--workers", type=int, default=32)
    ap.add_argument("--procs", type=int, default=1,
                    help="server processes sharing the port (SO_REUSEPORT), each with its own copy of the models on "
                         "the GPU and its own Python interpreter: the kernel spreads client connections over them. "
                         "Repository-control RPCs (load / unload) act on the process that receives them, and so do "
                         "shared-memory registrations (system and device): a client must register its regions and "
                         "infer over the same gRPC channel (connection), which one process serves; after a reconnect "
                         "it registers again.")
    ap.add_argument("--child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--export-repository", default=None, metavar="DIR",
                    help="write a Triton-layout repository for --models into DIR and exit")
    ap.add_argument("--weights", action="append", default=[], metavar="MODEL=URI",
                    help="with --export-repository: weights for MODEL (path, file/http(s)/s3 URI); repeatable")
    ap.add_argument("--weights-sha256", action="append", default=[], metavar="MODEL=HEX",
                    help="with --export-repository: expected sha256 of MODEL's weights (written into config.pbtxt)")
    return ap


def main(argv=None):
    args = build_parser().parse_args(argv)
    logging.basicConfig(level=logging.INFO)
    if args.export_repository:
        from .repository import export_repository

        w = dict(kv.split("=", 1) for kv in args.weights)
        sha = dict(kv.split("=", 1) for kv in args.weights_sha256)
        names = filter(None, (m.strip() for m in args.models.split(",")))
        for d in export_repository(names, args.export_repository, w, sha):
            print(d)
        return
    children = []
    if args.procs > 1 and not args.child:
        if args.port == 0:
            raise SystemExit("--procs > 1 needs a fixed --port (the processes share it)")
        import subprocess
        import sys

        # started before this process touches the GPU; each loads its models, reports LOADED and
        # binds the port on GO, so the kernel spreads the first client connections over all of them
        argv_child = [a for a in (argv if argv is not None else sys.argv[1:])]
        for _ in range(args.procs - 1):
            children.append(subprocess.Popen([sys.executable, "-m", "triton_client_amd.server", *argv_child,
                                              "--child", "--metrics-port", "0"],
                                             stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True))
    # SIGTERM ends the children and writes the stage clock; installed before any child can
    # bind the port, so a request served by a child never races the parent's handler
    from .model import PROFILE
    state = {"srv": None}
    if PROFILE.on or children:
        import os
        import signal

        def _term(*_):
            for c in children:
                c.terminate()
            if PROFILE.on:
                if args.child:  # one stage clock per process
                    PROFILE.path = f"{PROFILE.path}.{os.getpid()}"
                PROFILE.dump()
            if state["srv"] is not None:
                state["srv"].stop(0)
            for c in children:
                c.wait(30)
            __import__("sys").exit(0)
        signal.signal(signal.SIGTERM, _term)
    if args.model_repository:
        repo = ModelRepository.from_directory(args.model_repository, args.device)
    else:
        repo = ModelRepository(args.device)
        for m in filter(None, args.models.split(",")):
            repo.load(m.strip())
    if args.child:
        print("LOADED", flush=True)
        sys_stdin_line = __import__("sys").stdin.readline()
        if sys_stdin_line.strip() != "GO":
            return
    for c in children:
        line = c.stdout.readline()
        if line.strip() != "LOADED":
            for k in children:
                k.kill()
            raise SystemExit(f"a server process failed to load its models ({line!r})")
    for c in children:
        c.stdin.write("GO\n")
        c.stdin.flush()
    srv = KServeServer(repo, f"{args.host}:{args.port}", max_workers=args.workers,
                       metrics_port=args.metrics_port if args.metrics_port > 0 else None).start()
    state["srv"] = srv
    logging.info("KServe-v2 server on %s, models: %s%s", srv.target, [m.name for m in repo.models()],
                 f" ({args.procs} processes)" if children else "")
    srv.wait()


if __name__ == "__main__":
    main()
