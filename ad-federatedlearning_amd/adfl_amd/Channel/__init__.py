"""Channel plugin layer (mirror of Src/ADFL/Channel/__init__.py): the SLQ and stochastic codecs on MI355X."""

from .channel import Channel, IdentityChannel
from .quant import (CNATChannel, HipSLQChannel, HipUSLQChannel, PackedSLQChannel, QSGDChannel, RQSGDChannel,
                    SLQChannel, UCNATChannel, UQSGDChannel, URQSGDChannel, USLQChannel)

__all__ = ["Channel", "IdentityChannel", "SLQChannel", "USLQChannel", "PackedSLQChannel", "HipSLQChannel",
           "HipUSLQChannel", "QSGDChannel", "UQSGDChannel", "RQSGDChannel", "URQSGDChannel", "CNATChannel",
           "UCNATChannel"]
