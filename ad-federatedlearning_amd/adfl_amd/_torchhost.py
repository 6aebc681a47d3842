"""Loader of the channels' host-side torch plumbing (csrc/torch_host.cpp -> lib/adfl_torchhost.so): per-tensor
output creation and payload metadata for a whole state dict in one call each (Channel/quant.py). Built
in-tree by _build.build_torch_host (__graft_entry__.build); importing a channel's host path without it
raises."""

import importlib.machinery
import importlib.util
import os

_MOD = None


def get():
    global _MOD
    if _MOD is None:
        from . import _build
        path = _build.TORCH_HOST_PATH
        if not os.path.exists(path):
            raise ImportError(f"adfl_amd: {path} is missing; build it with "
                              "`python -c 'import __graft_entry__ as g; g.build()'`")
        import torch  # noqa: F401  (libc10 / libtorch loaded first)
        stamp = open(_build.TORCH_HOST_STAMP).read().strip() if os.path.exists(_build.TORCH_HOST_STAMP) else None
        if stamp != _build.torch_host_stamp():
            raise ImportError(f"adfl_amd: {path} was built against torch {stamp or '(unknown)'}, this process runs "
                              f"{_build.torch_host_stamp()}; rebuild it with "
                              "`python -c 'import __graft_entry__ as g; g.build()'`")
        loader = importlib.machinery.ExtensionFileLoader("adfl_torchhost", path)
        spec = importlib.util.spec_from_loader("adfl_torchhost", loader)
        mod = importlib.util.module_from_spec(spec)
        loader.exec_module(mod)
        _MOD = mod
    return _MOD
