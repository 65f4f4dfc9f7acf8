"""Transport ABC (reference ``communicator/channel/base_channel.py:3-34``)."""
from __future__ import annotations

from abc import ABC, abstractmethod


class BaseChannel(ABC):
    """Holds the client parameters (``client_parameter.yaml`` dict) and the
    parsed CLI flags, and exposes the four operations every transport has."""

    def __init__(self, params: dict, FLAGS):
        self.params = params
        self.FLAGS = FLAGS

    @abstractmethod
    def register_channel(self):
        """Open the connection / stub."""

    @abstractmethod
    def fetch_channel(self):
        """Return the underlying stub."""

    @abstractmethod
    def get_metadata(self) -> dict:
        """{'metadata_request','metadata_response','config_request','config_response'}."""

    @abstractmethod
    def do_inference(self):
        """Run one inference with the channel's current request."""
