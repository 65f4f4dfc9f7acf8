"""Box annotation for the published images (reference ``ros_inference.py:149-169``,
``yolov5_postprocess.py:127-169`` ``plot_boxes_cv2``).

OpenCV is not part of this stack: rectangles are drawn with NumPy slice
assignment (O(perimeter) per box, in place), labels with PIL's bitmap font
when PIL is importable.  The colour of a class is a fixed hash of its id.
"""
from __future__ import annotations

from typing import Optional, Sequence

import numpy as np


def class_color(c: int) -> tuple:
    h = (int(c) * 2654435761) & 0xFFFFFF
    return ((h >> 16) & 255, (h >> 8) & 255, h & 255)


def draw_rect(img: np.ndarray, x1: float, y1: float, x2: float, y2: float, color, thickness: int = 2) -> None:
    H, W = img.shape[:2]
    x1, x2 = int(np.clip(round(x1), 0, W - 1)), int(np.clip(round(x2), 0, W - 1))
    y1, y2 = int(np.clip(round(y1), 0, H - 1)), int(np.clip(round(y2), 0, H - 1))
    if x2 < x1 or y2 < y1:
        return
    t = max(1, thickness)
    col = np.asarray(color, img.dtype)[: img.shape[2]]
    img[y1:min(y1 + t, y2 + 1), x1:x2 + 1] = col
    img[max(y2 - t + 1, y1):y2 + 1, x1:x2 + 1] = col
    img[y1:y2 + 1, x1:min(x1 + t, x2 + 1)] = col
    img[y1:y2 + 1, max(x2 - t + 1, x1):x2 + 1] = col


def draw_detections(img: np.ndarray, dets: np.ndarray, names: Optional[Sequence[str]] = None,
                    thickness: int = 2, labels: bool = True, rects: bool = True) -> np.ndarray:
    """img HxWx3 uint8 (modified in place and returned); dets [n, 6] x1,y1,x2,y2,conf,cls
    in img pixels.  rects=False: only the labels (the rectangles were drawn on
    the GPU by ``ops.image.draw_boxes_``)."""
    dets = np.asarray(dets).reshape(-1, 6)
    for d in dets if rects else ():
        draw_rect(img, d[0], d[1], d[2], d[3], class_color(int(d[5])), thickness)
    if labels and len(dets):
        try:
            from PIL import Image, ImageDraw
        except Exception:  # pragma: no cover
            return img
        pil = Image.fromarray(img)
        dr = ImageDraw.Draw(pil)
        for d in dets:
            c = int(d[5])
            name = names[c] if names is not None and 0 <= c < len(names) else str(c)
            dr.text((float(d[0]) + 2, max(float(d[1]) - 11, 0)), f"{name} {d[4]:.2f}", fill=class_color(c))
        img[...] = np.asarray(pil)
    return img
