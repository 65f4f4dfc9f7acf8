"""Box + label annotation for the published images (reference ``ros_inference.py:149-169``,
``yolov5_postprocess.py:127-169`` ``plot_boxes_cv2``).

OpenCV is not part of this stack.  This is the host painter; the GPU painter
(``csrc/kernels/draw.hip``, :func:`triton_client_amd.ops.image.draw_annotations_`)
draws the same pixels on the device, so the two are interchangeable and the
tests compare them pixel for pixel:

* rectangles: round-half-even corners clipped to the frame, ``thickness``-pixel
  bands inside the box, all boxes first in result order (later boxes win);
* labels: ``"<name> <conf:.2f>"`` in the fixed 6x11 cell font of
  :mod:`.font6x11` at ``(x1 + 2, max(y1 - 11, 0))``, after every rectangle,
  again in result order.  Characters outside printable ASCII print as ``?``;
  names are cut to 31 characters.

The colour of a class is a fixed hash of its id.
"""
from __future__ import annotations

from typing import Optional, Sequence

import numpy as np

from . import font6x11

NAME_MAX = 32  # bytes per row of the device names table (31 chars + NUL)


def class_color(c: int) -> tuple:
    h = (int(c) * 2654435761) & 0xFFFFFF
    return ((h >> 16) & 255, (h >> 8) & 255, h & 255)


def _corners(img: np.ndarray, x1, y1, x2, y2):
    H, W = img.shape[:2]
    return (int(np.clip(round(float(x1)), 0, W - 1)), int(np.clip(round(float(y1)), 0, H - 1)),
            int(np.clip(round(float(x2)), 0, W - 1)), int(np.clip(round(float(y2)), 0, H - 1)))


def draw_rect(img: np.ndarray, x1: float, y1: float, x2: float, y2: float, color, thickness: int = 2) -> None:
    x1, y1, x2, y2 = _corners(img, x1, y1, x2, y2)
    if x2 < x1 or y2 < y1:
        return
    t = max(1, thickness)
    col = np.asarray(color, img.dtype)[: img.shape[2]]
    img[y1:min(y1 + t, y2 + 1), x1:x2 + 1] = col
    img[max(y2 - t + 1, y1):y2 + 1, x1:x2 + 1] = col
    img[y1:y2 + 1, x1:min(x1 + t, x2 + 1)] = col
    img[y1:y2 + 1, max(x2 - t + 1, x1):x2 + 1] = col


def _sanitize(name: str) -> str:
    return "".join(ch if 32 <= ord(ch) <= 126 else "?" for ch in name)[:NAME_MAX - 1]


def label_text(c: int, conf: float, names: Optional[Sequence[str]] = None) -> str:
    """The label the painters draw: class name (or id) and the confidence to 2
    decimals, rounded half-even from the exact fp32 value (what ``'{:.2f}'``
    does, computed the way the kernel computes it)."""
    c = int(c)
    name = _sanitize(str(names[c])) if names is not None and 0 <= c < len(names) else str(c)
    p = float(np.rint(np.float64(np.float32(conf)) * 100.0))
    v = (int(p) if p < 1e9 else 999999999) if p > 0 else 0  # NaN -> 0, like the kernel
    return f"{name} {v // 100}.{v % 100:02d}"


def names_table(names: Optional[Sequence[str]]) -> np.ndarray:
    """Class names -> [n, 32] uint8 rows (sanitised, NUL-padded) for the GPU painter."""
    names = list(names or [])
    t = np.zeros((max(len(names), 1), NAME_MAX), np.uint8)
    for i, n in enumerate(names):
        b = _sanitize(str(n)).encode("ascii")
        t[i, :len(b)] = np.frombuffer(b, np.uint8)
    return t[:len(names)] if names else t[:0]


_GLYPHS = None


def _glyphs() -> np.ndarray:
    """[95, 11, 6] bool glyph cells."""
    global _GLYPHS
    if _GLYPHS is None:
        rows = np.asarray(font6x11.ROWS, np.uint8)
        _GLYPHS = ((rows[..., None] >> np.arange(font6x11.W, dtype=np.uint8)) & 1).astype(bool)
    return _GLYPHS


def text_mask(text: str) -> np.ndarray:
    """[11, 6 * len(text)] bool pixels of a label."""
    codes = np.frombuffer(text.encode("ascii", "replace"), np.uint8).astype(np.int64)
    codes = np.where((codes < font6x11.FIRST) | (codes > font6x11.LAST), ord("?"), codes) - font6x11.FIRST
    g = _glyphs()[codes]  # [L, 11, 6]
    return g.transpose(1, 0, 2).reshape(font6x11.H, -1)


def draw_label(img: np.ndarray, x1: float, y1: float, x2: float, y2: float, text: str, color) -> None:
    X1, Y1, X2, Y2 = _corners(img, x1, y1, x2, y2)
    if X2 < X1 or Y2 < Y1:
        return
    H, W = img.shape[:2]
    m = text_mask(text)
    x0, y0 = X1 + 2, max(Y1 - font6x11.H, 0)
    m = m[:max(0, H - y0), :max(0, W - x0)]
    region = img[y0:y0 + m.shape[0], x0:x0 + m.shape[1]]
    region[m] = np.asarray(color, img.dtype)[: img.shape[2]]


def draw_detections(img: np.ndarray, dets: np.ndarray, names: Optional[Sequence[str]] = None,
                    thickness: int = 2, labels: bool = True, rects: bool = True) -> np.ndarray:
    """img HxWx3 uint8 (modified in place and returned); dets [n, 6] x1,y1,x2,y2,conf,cls
    in img pixels.  rects=False: only the labels."""
    dets = np.asarray(dets).reshape(-1, 6)
    for d in dets if rects else ():
        draw_rect(img, d[0], d[1], d[2], d[3], class_color(int(d[5])), thickness)
    if labels:
        for d in dets:
            c = int(d[5])
            draw_label(img, d[0], d[1], d[2], d[3], label_text(c, d[4], names), class_color(c))
    return img
