"""Accuracy evaluation (reference ``evaluate.py`` / ``EvaluateInference``):
images + ground-truth Detection2DArray → P/R/AP/F1, exported to Prometheus :7658."""
from __future__ import annotations

import argparse
import json
import os
import sys

from .common import DATA, add_framework_flags, add_reference_flags, load_params, play_bag, setup_logging
from .engines import engine_2d


def parse_args(argv=None):
    p = argparse.ArgumentParser(description=__doc__)
    add_reference_flags(p, "YOLOv5nCROP")
    add_framework_flags(p, os.path.join(DATA, "client_parameter.yaml"))
    p.add_argument("--bag", default=None, help="evaluate this bag offline (images + gt topics)")
    p.add_argument("--eval-port", type=int, default=7658, help="Prometheus port (reference 7658; 0 = off)")
    p.add_argument("--json", default=None, help="write the summary here")
    return p.parse_args(argv)


def main(argv=None) -> int:
    flags = parse_args(argv)
    setup_logging(flags.verbose)
    from ..inference import EvaluateInference
    from ..ros import compat, default_bus

    compat.init_node("ros_evaluate")
    params = load_params(flags.params, flags.server)
    engine, channel, client = engine_2d(flags, params, conf_thres=0.001 if flags.conf_thres == 0.3 else None)
    ev = EvaluateInference(channel, client, engine=engine, params=params,
                           metrics_port=flags.eval_port or None, bus=default_bus())
    if flags.bag:
        s = ev.evaluate_bag(flags.bag, batch=max(1, flags.frames_per_step))
    else:
        if flags.play:
            play_bag(flags.play, default_bus(), topics=[params["sub_topic"], params["gt_topic"]], shutdown=False)
        s = ev.start_inference(spin=True, timeout=flags.spin_timeout)
    out = s.as_dict(getattr(engine, "names", None))
    print(json.dumps(out, indent=1))
    if flags.json:
        with open(flags.json, "w") as f:
            json.dump(out, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
