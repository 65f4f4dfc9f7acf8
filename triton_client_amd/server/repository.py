"""Model repository: name → servable factory, load/unload/index.

Known model names mirror the reference's deployments
(``examples/*/config.pbtxt``, ``docker/server/models/weed_detector``,
``.vscode/launch.json:8-47``).  A Triton-style directory
(``<repo>/<model>/config.pbtxt``) can also be scanned: each config's name
selects the factory and its declared tensor dims (e.g. image size) are
honoured.
"""
from __future__ import annotations

import os
import threading
from pathlib import Path
from typing import Callable, Dict, Iterable, List, Optional, Tuple

from .model import EchoModel, ServedModel

Factory = Callable[..., ServedModel]


def _yolo(name, variant="n", nc=80, img=640):
    def f(device="auto", **kw):
        from .models import YoloV5Model
        return YoloV5Model(name, variant, nc, img, device=device, **kw)
    return f


def _pointpillars(name):
    def f(device="auto", **kw):
        from .models import PointPillarsModel
        return PointPillarsModel(name, device=device, **kw)
    return f


def _family(name: str) -> Optional[str]:
    n = name.lower()
    if "yolov4" in n:
        return "yolov4"
    if "yolo" in n or "weed" in n:
        return "yolo"
    if "pointpillar" in n or "pillar" in n:
        return "pointpillars"
    if "retina" in n or "fcos" in n or "detectron" in n or n == "test_model":
        return "detectron"
    if "centerpoint" in n:
        return "centerpoint"
    if "second" in n:
        return "second_iou"
    if "echo" in n:
        return "echo"
    return None


def _second(name):
    def f(device="auto", **kw):
        from .models import SecondIoUModel
        return SecondIoUModel(name, device=device, **kw)
    return f


def _centerpoint(name):
    def f(device="auto", **kw):
        from .models import CenterPointModel
        return CenterPointModel(name, device=device, **kw)
    return f


def _detectron(name, arch, nc=80):
    def f(device="auto", **kw):
        from .models import DetectronModel
        return DetectronModel(name, arch=arch, nc=nc, device=device, **kw)
    return f


def _yolov4(name, nc=80, img=512):
    def f(device="auto", **kw):
        from .models import YoloV4Model
        return YoloV4Model(name, nc, img, device=device, **kw)
    return f


FACTORIES: Dict[str, Factory] = {
    "YOLOv5nCOCO": _yolo("YOLOv5nCOCO", "n", 80, 640),
    "YOLOv5n": _yolo("YOLOv5n", "n", 80, 640),
    "YOLOv5nCROP": _yolo("YOLOv5nCROP", "n", 2, 512),
    "weed_detector": _yolo("weed_detector", "n", 2, 512),
    "pointpillar_kitti": _pointpillars("pointpillar_kitti"),
    "pointpillar_python": _pointpillars("pointpillar_python"),
    "centerpoint_pp": _centerpoint("centerpoint_pp"),
    "second_iou": _second("second_iou"),  # examples/second_iou/config.pbtxt
    "YOLOv4": _yolov4("YOLOv4"),  # examples/YOLOv4/config.pbtxt
    "test_model": _detectron("test_model", "retinanet"),  # examples/RetinaNet_detectron/config.pbtxt
    "RetinaNet_detectron": _detectron("RetinaNet_detectron", "retinanet"),
    "FCOS_detectron": _detectron("FCOS_detectron", "fcos"),
    "fcos_weed_detector": _detectron("fcos_weed_detector", "fcos", 2),  # main.py:75 (weeds, maize)
    "centerpoint": _centerpoint("centerpoint"),
    "echo": lambda device="auto", **kw: EchoModel("echo"),
}


def register_factory(name: str, factory: Factory) -> None:
    FACTORIES[name] = factory


def _weights_for(model_dir: str, cfg) -> Tuple[Optional[str], Optional[str]]:
    """(weights, sha256) of one repository entry.  Weights: ``parameters { key:
    "weights" }`` (path or file/http(s)/s3 URI, see ``utils/model_store.py``), else
    the highest numeric version directory holding ``model.pt`` (Triton's
    ``<model>/<version>/`` layout).  sha256: ``parameters { key: "weights_sha256" }``
    — checked by the model store before the file is loaded (and before a cached
    download is reused)."""
    sha = cfg.parameters["weights_sha256"].string_value if "weights_sha256" in cfg.parameters else ""
    sha = sha or None
    if "weights" in cfg.parameters and cfg.parameters["weights"].string_value:
        w = cfg.parameters["weights"].string_value
        return (w if "://" in w or os.path.isabs(w) else os.path.join(model_dir, w)), sha
    versions = sorted((int(v) for v in os.listdir(model_dir) if v.isdigit()), reverse=True)
    for v in versions:
        f = os.path.join(model_dir, str(v), "model.pt")
        if os.path.isfile(f):
            return f, sha
    return None, sha


class ModelRepository:
    def __init__(self, device="auto"):
        self.device = device
        self._models: Dict[str, ServedModel] = {}
        self._lock = threading.Lock()

    def add(self, model: ServedModel, load: bool = True) -> ServedModel:
        if load and not model.ready:
            from .model import GPU_PHASE
            GPU_PHASE.acquire_exclusive()  # graphs are captured with no other model executing
            try:
                model.load()
            finally:
                GPU_PHASE.release_exclusive()
        with self._lock:
            self._models[model.name] = model
        return model

    def load(self, name: str, **kw) -> ServedModel:
        with self._lock:
            m = self._models.get(name)
        if m is not None and m.ready:
            return m
        if m is None:
            if name not in FACTORIES:
                raise KeyError(f"no factory for model '{name}'")
            m = FACTORIES[name](device=self.device, **kw)
        return self.add(m)

    def unload(self, name: str) -> None:
        with self._lock:
            m = self._models.get(name)
        if m is not None:
            m.unload()

    def get(self, name: str, version: str = "") -> Optional[ServedModel]:
        with self._lock:
            m = self._models.get(name)
        if m is None or (version and version != m.version):
            return None
        return m

    def models(self, name: Optional[str] = None) -> List[ServedModel]:
        with self._lock:
            ms = list(self._models.values())
        return [m for m in ms if name is None or m.name == name]

    def index(self) -> List[Tuple[str, str]]:
        with self._lock:
            loaded = {n: ("READY" if m.ready else "UNAVAILABLE") for n, m in self._models.items()}
        names = sorted(set(FACTORIES) | set(loaded))
        return [(n, loaded.get(n, "UNLOADED")) for n in names]

    def all_ready(self) -> bool:
        with self._lock:
            return all(m.ready for m in self._models.values())

    @staticmethod
    def from_directory(path: str, device="auto", load: bool = True) -> "ModelRepository":
        """Scan a Triton model repository; each ``config.pbtxt`` picks a family."""
        from ..proto import parse_config_pbtxt

        repo = ModelRepository(device)
        for entry in sorted(os.listdir(path)):
            cfgp = os.path.join(path, entry, "config.pbtxt")
            if not os.path.isfile(cfgp):
                continue
            with open(cfgp) as f:
                cfg = parse_config_pbtxt(f.read())
            name = cfg.name or entry
            fam = _family(name)
            if name in FACTORIES:
                m = FACTORIES[name](device=device)
            elif fam == "yolo":
                dims = list(cfg.input[0].dims)
                out = list(cfg.output[0].dims)
                from .models import YoloV5Model
                m = YoloV5Model(name, "n", out[-1] - 5, dims[-1], device=device)
            elif fam == "yolov4" or (len(cfg.output) == 2 and {o.name for o in cfg.output} == {"confs", "boxes"}):
                from .models import YoloV4Model
                dims = list(cfg.input[0].dims)
                nc = int(list(cfg.output[0].dims)[-1]) if cfg.output[0].name == "confs" else 80
                m = YoloV4Model(name, nc, dims[-1], device=device)
            elif fam == "detectron" or len(cfg.output) == 4:
                from .models import DetectronModel
                dims = list(cfg.input[0].dims)
                m = DetectronModel(name, "fcos" if "fcos" in name.lower() else "retinanet", tuple(dims[-2:]),
                                   device=device)
            elif fam == "pointpillars":
                from .models import PointPillarsModel
                m = PointPillarsModel(name, device=device)
            elif fam == "centerpoint":
                from .models import CenterPointModel
                m = CenterPointModel(name, device=device)
            elif fam == "second_iou":
                from .models import SecondIoUModel
                m = SecondIoUModel(name, device=device)
            else:
                continue
            weights, sha = _weights_for(os.path.join(path, entry), cfg)
            if weights and hasattr(m, "weights"):
                m.weights, m.weights_sha256 = weights, sha
            repo.add(m, load=load)
        return repo


def export_repository(names: Iterable[str], out_dir: str, weights: Optional[Dict[str, str]] = None,
                      weights_sha256: Optional[Dict[str, str]] = None) -> List[str]:
    """Write a Triton-layout model repository (``<name>/config.pbtxt`` plus
    ``<name>/1/model.pt`` when weights are given) for the named served models.
    A local weights file is copied and its sha256 recorded as the
    ``weights_sha256`` parameter; a remote URI is referenced with the sha256
    given in ``weights_sha256`` (strongly advised: without it the server trusts
    whatever the URI serves).

    This is the deploy step of the reference's ``deploy.sh:1-65`` (export the
    model, write its ``config.pbtxt`` into the server's repository), minus the
    ONNX export: the server here runs the native MI355X pipelines, so the
    repository holds the KServe contract and, optionally, a state_dict.
    ``from_directory`` reads it back."""
    import shutil

    from google.protobuf import text_format

    written = []
    for name in names:
        if name not in FACTORIES:
            raise KeyError(f"no factory for model '{name}'")
        from ..utils.model_store import _sha256_file

        m = FACTORIES[name](device="cpu")
        d = os.path.join(out_dir, name)
        os.makedirs(os.path.join(d, "1"), exist_ok=True)
        cfg = m.config()
        w = (weights or {}).get(name)
        sha = (weights_sha256 or {}).get(name)
        if w:
            if "://" in w:  # remote: reference it, the server fetches it at load time
                cfg.parameters["weights"].string_value = w  # text_format escapes it
            else:
                dst = os.path.join(d, "1", "model.pt")
                shutil.copyfile(w, dst)
                got = _sha256_file(Path(dst))
                if sha and sha.lower() != got:
                    raise ValueError(f"{w}: sha256 {got} != expected {sha}")
                sha = got
            if sha:
                cfg.parameters["weights_sha256"].string_value = sha.lower()
        with open(os.path.join(d, "config.pbtxt"), "w") as f:
            f.write(text_format.MessageToString(cfg))
        written.append(d)
    return written
