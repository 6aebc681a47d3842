"""Build libadfl_slq.so in-tree with hipcc for gfx950 (no JIT cache: the .so travels with the repo)."""

import os
import subprocess

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
SRC_ROOT = os.path.dirname(PKG_DIR)                      # ad-federatedlearning_amd/
REPO_ROOT = os.path.dirname(SRC_ROOT)
CSRC = os.path.join(SRC_ROOT, "csrc", "slq_codec.hip")
SOURCES = [CSRC, os.path.join(SRC_ROOT, "csrc", "stoch_codec.hip"), os.path.join(SRC_ROOT, "csrc", "stoch_dtype.hip"),
           os.path.join(SRC_ROOT, "csrc", "torch_norm.hip"), os.path.join(SRC_ROOT, "csrc", "qerror_ref.hip"),
           os.path.join(SRC_ROOT, "csrc", "bucket_copy.hip"), os.path.join(SRC_ROOT, "csrc", "host_copy.cpp")]
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


if __name__ == "__main__":
    print(build(force=True, verbose=True))
