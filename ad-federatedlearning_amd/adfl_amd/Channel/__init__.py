"""Channel plugin layer (mirror of Src/ADFL/Channel/__init__.py): the SLQ codec on MI355X."""

from .channel import Channel, IdentityChannel
from .quant import HipSLQChannel, HipUSLQChannel, PackedSLQChannel, SLQChannel, USLQChannel

__all__ = ["Channel", "IdentityChannel", "SLQChannel", "USLQChannel", "PackedSLQChannel", "HipSLQChannel",
           "HipUSLQChannel"]
