"""The ``Channel`` plugin interface and the identity (fp32 byte) channel.

``Channel`` has the six-method surface of ``Src/ADFL/Channel/channel.py:10-45``; ``IdentityChannel``
follows ``Src/ADFL/Channel/channel.py:48-133`` (it is what ``USLQChannel`` uses for the uncompressed
direction, quant.py:123-130). Neither touches the GPU.
"""

import time
from abc import ABC, abstractmethod
from typing import Dict, Tuple

import torch

from ..model import (ByteParameter, ByteParameters, CompressedParameters, Parameters, get_parameter_info)


class Channel(ABC):
    """Base Channel interface (channel.py:10-45)."""

    @abstractmethod
    def on_server_send(self, params: Parameters) -> Tuple[CompressedParameters, float]:
        """Server send: returns the parameters to send and the compute time."""

    @abstractmethod
    def on_server_receive(self, c_params: CompressedParameters) -> Tuple[Parameters, float]:
        """Server receive: returns the parameters received and the compute time."""

    @abstractmethod
    def on_client_send(self, params: Parameters) -> Tuple[CompressedParameters, float]:
        """Client send: returns the parameters to send and the compute time."""

    @abstractmethod
    def on_client_receive(self, c_params: CompressedParameters) -> Tuple[Parameters, float]:
        """Client receive: returns the parameters received and the compute time."""

    @abstractmethod
    def simulate_bandwidth(self, params: Parameters, mbps: float) -> float:
        """Sleep for the simulated transfer time of `params` at `mbps`; return that time."""

    @abstractmethod
    def to_json(self) -> Dict:
        """Serialization for the results JSON."""


class IdentityChannel(Channel):
    """Serializes parameters to raw bytes and back (channel.py:48-133)."""

    def __init__(self, no_compute_time: bool) -> None:
        self.no_compute_time = no_compute_time

    def on_server_send(self, params: Parameters) -> Tuple[CompressedParameters, float]:
        s_time = time.time()
        b_params = self._serialize_params(params)
        return b_params, self._finalize_compute_time(s_time)

    def on_server_receive(self, c_params: CompressedParameters) -> Tuple[Parameters, float]:
        assert isinstance(c_params, ByteParameters)
        s_time = time.time()
        params = self._deserialize_params(c_params)
        return params, self._finalize_compute_time(s_time)

    def on_client_send(self, params: Parameters) -> Tuple[CompressedParameters, float]:
        s_time = time.time()
        b_params = self._serialize_params(params)
        return b_params, self._finalize_compute_time(s_time)

    def on_client_receive(self, c_params: CompressedParameters) -> Tuple[Parameters, float]:
        assert isinstance(c_params, ByteParameters)
        s_time = time.time()
        params = self._deserialize_params(c_params)
        return params, self._finalize_compute_time(s_time)

    def simulate_bandwidth(self, params: Parameters, mbps: float) -> float:
        """Every element counted as 32 bits (channel.py:83-93)."""
        p_info = get_parameter_info(params)
        num_bytes = (p_info.num_bias_w + p_info.num_non_bias_w) * 4
        transfer_time = num_bytes / (mbps * 1_000_000 / 8)
        time.sleep(transfer_time)
        return transfer_time

    def to_json(self) -> Dict:
        return {"name": self.__class__.__name__}

    def _serialize_params(self, params: Parameters) -> ByteParameters:
        b_params = ByteParameters({}, 0)
        for name, param in params.items():
            data = param.detach().cpu().numpy().tobytes()
            b_params.params[name] = ByteParameter(data=data, shape=param.shape, dtype=param.dtype)
            b_params.size += len(data)
        return b_params

    def _deserialize_params(self, b_params: ByteParameters) -> Parameters:
        return {name: torch.frombuffer(bytearray(b.data), dtype=b.dtype).reshape(b.shape)
                for name, b in b_params.params.items()}

    def _finalize_compute_time(self, s_time: float) -> float:
        return 0.0 if self.no_compute_time else time.time() - s_time
