"""Serve proxy options (reference: ``python/ray/serve/config.py``: ``HTTPOptions``,
``gRPCOptions``)."""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Callable, List, Union


@dataclass
class HTTPOptions:
    host: str = "127.0.0.1"
    port: int = 8000
    root_path: str = ""


@dataclass
class gRPCOptions:
    """``grpc_servicer_functions``: generated ``add_<Service>Servicer_to_server`` functions (or
    their import paths) whose methods the gRPC proxy serves."""
    port: int = 9000
    host: str = "127.0.0.1"
    grpc_servicer_functions: List[Union[str, Callable]] = field(default_factory=list)
