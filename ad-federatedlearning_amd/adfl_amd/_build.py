"""Build libadfl_slq.so in-tree with hipcc for gfx950 (no JIT cache: the .so travels with the repo)."""

import os
import subprocess

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
SRC_ROOT = os.path.dirname(PKG_DIR)                      # ad-federatedlearning_amd/
REPO_ROOT = os.path.dirname(SRC_ROOT)
CSRC = os.path.join(SRC_ROOT, "csrc", "slq_codec.hip")
SOURCES = [CSRC, os.path.join(SRC_ROOT, "csrc", "stoch_codec.hip"), os.path.join(SRC_ROOT, "csrc", "stoch_dtype.hip"),
           os.path.join(SRC_ROOT, "csrc", "torch_norm.hip"), os.path.join(SRC_ROOT, "csrc", "qerror_ref.hip"),
           os.path.join(SRC_ROOT, "csrc", "bucket_copy.hip"), os.path.join(SRC_ROOT, "csrc", "host_stage.hip"),
           os.path.join(SRC_ROOT, "csrc", "host_copy.cpp")]
DEPENDS = SOURCES + [os.path.join(SRC_ROOT, "csrc", h) for h in ("cnat_log2_table.h", "cnat_log2_dt_table.h", "philox.h", "torch_sum_order.h", "torch_norm_walk.h")]
INCLUDE = os.path.join(REPO_ROOT, "include")
LIB_DIR = os.path.join(PKG_DIR, "lib")
LIB_PATH = os.path.join(LIB_DIR, "libadfl_slq.so")

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# No fast-math, no FMA contraction, default fp32 denormal handling (IEEE): the codec is bit-exact.
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-Wall"]


def build(force: bool = False, verbose: bool = False) -> str:
    os.makedirs(LIB_DIR, exist_ok=True)
    deps = DEPENDS + [os.path.join(INCLUDE, h) for h in ("adfl_slq.h", "adfl_stoch.h", "adfl_host.h", "adfl_qerror.h")]
    stamp = LIB_PATH + ".rounds"
    want = os.environ.get("ADFL_PHILOX_ROUNDS", "7")
    built = open(stamp).read().strip() if os.path.exists(stamp) else "7"
    if (not force and os.path.exists(LIB_PATH) and built == want
            and os.path.getmtime(LIB_PATH) >= max(os.path.getmtime(d) for d in deps)):
        return LIB_PATH
    rounds = int(os.environ.get("ADFL_PHILOX_ROUNDS", "7"))
    if rounds not in (7, 10):
        raise ValueError("ADFL_PHILOX_ROUNDS must be 7 (the product) or 10 (Random123's margin)")
    defs = [] if rounds == 7 else [f"-DADFL_PHILOX_ROUNDS={rounds}"]
    cmd = [HIPCC, *FLAGS, *defs, f"-I{INCLUDE}", "-o", LIB_PATH, *SOURCES]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    with open(stamp, "w") as f:
        f.write(f"{rounds}\n")
    return LIB_PATH


TORCH_HOST_SRC = os.path.join(SRC_ROOT, "csrc", "torch_host.cpp")
TORCH_HOST_PATH = os.path.join(LIB_DIR, "adfl_torchhost.so")
TORCH_HOST_STAMP = TORCH_HOST_PATH + ".torch"   # the torch build it was compiled against


def torch_host_stamp() -> str:
    """The torch version and C++ ABI adfl_torchhost.so links against (libc10 / libtorch symbols)."""
    import torch
    return f"{torch.__version__} cxx11abi={int(torch._C._GLIBCXX_USE_CXX11_ABI)}"


def build_torch_host(force: bool = False, verbose: bool = False) -> str:
    """The channels' host-side torch plumbing (csrc/torch_host.cpp): a CPython extension over ATen, built with
    g++ against this image's torch (headers, libc10 / libtorch, its C++11 ABI), in-tree like the codec."""
    import sysconfig

    import torch
    from torch.utils import cpp_extension as ce
    os.makedirs(LIB_DIR, exist_ok=True)
    stamp = torch_host_stamp()
    built = open(TORCH_HOST_STAMP).read().strip() if os.path.exists(TORCH_HOST_STAMP) else None
    if (not force and os.path.exists(TORCH_HOST_PATH) and built == stamp
            and os.path.getmtime(TORCH_HOST_PATH) >= os.path.getmtime(TORCH_HOST_SRC)):
        return TORCH_HOST_PATH
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    incs = [f"-I{d}" for d in ce.include_paths()] + [f"-I{sysconfig.get_paths()['include']}"]
    libdir = ce.library_paths()[0]
    cmd = [os.environ.get("CXX", "g++"), "-O2", "-std=c++17", "-shared", "-fPIC", "-w",
           f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DTORCH_EXTENSION_NAME=adfl_torchhost", "-DTORCH_API_INCLUDE_EXTENSION_H",
           *incs, TORCH_HOST_SRC, "-o", TORCH_HOST_PATH, f"-L{libdir}", f"-Wl,-rpath,{libdir}",
           "-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python"]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    with open(TORCH_HOST_STAMP, "w") as f:
        f.write(stamp + "\n")
    return TORCH_HOST_PATH


if __name__ == "__main__":
    print(build(force=True, verbose=True))
    print(build_torch_host(force=True, verbose=True))
