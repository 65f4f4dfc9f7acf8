"""Inference driver base (reference ``communicator/base_inference.py:6-10``)."""
from __future__ import annotations


class BaseInference:
    """Holds the transport channel and the model-family client.  Drivers add
    an engine (:mod:`.engines`) that does the per-frame work."""

    def __init__(self, channel=None, client=None):
        self.channel = channel
        self.client = client

    @property
    def params(self) -> dict:
        return getattr(self.channel, "params", None) or getattr(self, "_params", {})
