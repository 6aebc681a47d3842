"""adfl_amd — MI355X-native (gfx950) SLQ gradient codec for ADFL (Tavonput/AD-FederatedLearning).

Layout mirrors the reference's ``Src/ADFL`` package for the one hot path this repo rebuilds:

* ``adfl_amd.Channel``      ``Channel``, ``IdentityChannel``, ``SLQChannel``, ``USLQChannel``
                            (drop-in for ``ADFL.Channel``; HIP-backed SLQ)
* ``adfl_amd.model``        payload dataclasses + ``get_parameter_info`` (``ADFL.model``)
* ``adfl_amd.compression``  ``quantize_tensor`` / ``dequantize_tensor`` / ``pack_4bit`` / ``unpack_4bit``
                            (``ADFL.compression``'s hot-path functions) on the GPU
* ``adfl_amd.ops``          device-resident codec ops; ``torch.ops.adfl.*`` custom ops
* ``adfl_amd.exchange``     one-client-per-GPU peer exchange: encode -> RCCL all-gather -> mean

The compute lives in ``libadfl_slq.so`` (``ad-federatedlearning_amd/csrc/slq_codec.hip``, C ABI in
``include/adfl_slq.h``). Importing this package loads it and fails loudly if it was not built.
"""

from . import _lib

_lib.load()

from . import compression, model, ops, stoch  # noqa: E402
from .Channel import (Channel, CNATChannel, IdentityChannel, PackedSLQChannel, QSGDChannel,  # noqa: E402
                      RQSGDChannel, SLQChannel, UCNATChannel, UQSGDChannel, URQSGDChannel, USLQChannel)

__all__ = ["Channel", "IdentityChannel", "SLQChannel", "USLQChannel", "PackedSLQChannel", "QSGDChannel",
           "UQSGDChannel", "RQSGDChannel", "URQSGDChannel", "CNATChannel", "UCNATChannel", "compression", "model",
           "ops", "stoch"]
