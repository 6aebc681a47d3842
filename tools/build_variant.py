"""Build an A/B variant of libadfl_slq.so with extra -D flags into tools/_variants/ (git-ignored); select it
at run time with ADFL_LIB_VARIANT=<path> (adfl_amd/_lib.py).

    python tools/build_variant.py stats -DADFL_TN_STATS
"""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ad-federatedlearning_amd"))
from adfl_amd import _build  # noqa: E402

name, defs = sys.argv[1], sys.argv[2:]
out = os.path.join(REPO, "tools", "_variants", f"libadfl_{name}.so")
os.makedirs(os.path.dirname(out), exist_ok=True)
subprocess.run([_build.HIPCC, *_build.FLAGS, *defs, f"-I{_build.INCLUDE}", "-o", out, *_build.SOURCES], check=True)
print(out)
