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
    if args.model_repository:
        repo = ModelRepository.from_directory(args.model_repository, args.device)
    else:
        repo = ModelRepository(args.device)
        for m in filter(None, args.models.split(",")):
            repo.load(m.strip())
    srv = KServeServer(repo, f"{args.host}:{args.port}", max_workers=args.workers,
                       metrics_port=args.metrics_port if args.metrics_port > 0 else None).start()
    logging.info("KServe-v2 server on %s, models: %s", srv.target, [m.name for m in repo.models()])
    srv.wait()


if __name__ == "__main__":
    main()
