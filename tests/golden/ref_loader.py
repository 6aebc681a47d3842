"""Load the reference ADFL codec modules in place, for golden-vector generation only.

This file is test infrastructure. It is used by ``make_golden.py`` (run in the build container, where
``/root/reference`` exists) and by the optional drop-in test in ``tests/test_dropin_reference.py``
(skipped when the reference tree is absent, e.g. on the GPU box). Nothing in the product package,
``bench.py`` or ``__graft_entry__.smoke()`` imports it.

``import ADFL`` fails in this image: ``Src/ADFL/__init__.py:1-19`` imports ``ray``, ``memray`` and
``torchvision``, which are not installed (an ordinary ``ModuleNotFoundError``). The codec modules
themselves only need ``torch`` plus the names ``Src/ADFL/model.py:8-15`` imports from torchvision and
transformers, so we register a bare ``ADFL`` package, stub those names, and execute exactly the four
reference modules on the hot path:

* ``Src/ADFL/model.py``            payload dataclasses, ``get_parameter_info``
* ``Src/ADFL/Channel/channel.py``  ``Channel`` ABC, ``IdentityChannel``
* ``Src/ADFL/Channel/quant.py``    ``SLQChannel``, ``USLQChannel`` (the north-star codec)
* ``Src/ADFL/compression.py``      ``pack_4bit`` / ``unpack_4bit`` (int4 layout)

No reference source is copied; the files are executed where they lie.
"""

import importlib.util
import os
import sys
import types

REF_ROOT = os.environ.get("ADFL_REFERENCE_ROOT", "/root/reference")
REF_SRC = os.path.join(REF_ROOT, "Src", "ADFL")


def reference_available() -> bool:
    return os.path.isfile(os.path.join(REF_SRC, "Channel", "quant.py"))


def _stub_module(name: str, attrs) -> types.ModuleType:
    mod = types.ModuleType(name)
    for a in attrs:
        setattr(mod, a, type(a, (), {}))
    return mod


def _load(name: str, path: str, package: bool = False) -> types.ModuleType:
    kwargs = {"submodule_search_locations": [os.path.dirname(path)]} if package else {}
    spec = importlib.util.spec_from_file_location(name, path, **kwargs)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def load_reference():
    """Return a namespace with the reference ``model``, ``channel``, ``quant`` and ``compression`` modules."""
    if not reference_available():
        raise FileNotFoundError(f"reference codec not found under {REF_SRC}")
    if "ADFL.Channel.quant" in sys.modules:
        m = sys.modules
        return types.SimpleNamespace(model=m["ADFL.model"], channel=m["ADFL.Channel.channel"],
                                     quant=m["ADFL.Channel.quant"], compression=m["ADFL.compression"])

    # Names imported at Src/ADFL/model.py:8-15; never called on the codec path.
    tv = types.ModuleType("torchvision")
    tv_models = _stub_module("torchvision.models", [
        "mobilenet_v3_small", "MobileNet_V3_Small_Weights", "mobilenet_v3_large",
        "MobileNet_V3_Large_Weights", "resnet50", "ResNet50_Weights", "vit_l_16", "ViT_L_16_Weights"])
    tv.models = tv_models
    sys.modules.setdefault("torchvision", tv)
    sys.modules.setdefault("torchvision.models", tv_models)
    sys.modules.setdefault("transformers", _stub_module("transformers", ["DistilBertForSequenceClassification"]))

    # Bare packages: do not execute Src/ADFL/__init__.py or Src/ADFL/Channel/__init__.py.
    pkg = types.ModuleType("ADFL")
    pkg.__path__ = [REF_SRC]
    sys.modules["ADFL"] = pkg
    chan_pkg = types.ModuleType("ADFL.Channel")
    chan_pkg.__path__ = [os.path.join(REF_SRC, "Channel")]
    sys.modules["ADFL.Channel"] = chan_pkg

    model = _load("ADFL.model", os.path.join(REF_SRC, "model.py"))
    pkg.model = model
    channel = _load("ADFL.Channel.channel", os.path.join(REF_SRC, "Channel", "channel.py"))
    quant = _load("ADFL.Channel.quant", os.path.join(REF_SRC, "Channel", "quant.py"))
    compression = _load("ADFL.compression", os.path.join(REF_SRC, "compression.py"))
    return types.SimpleNamespace(model=model, channel=channel, quant=quant, compression=compression)
