"""Build an A/B variant of libagx.so whose learner.hip comes from a git
revision (every other object from the current build), for same-box timing:
  python tools/ab_lib.py <rev> <name>     -> ab/libagx_<name>.so
  AGX_LIB=ab/libagx_<name>.so python tools/learn_time.py"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from agilerl_amd import _build  # noqa: E402

rev, name = sys.argv[1], sys.argv[2]
_build.build()
out = os.path.join(ROOT, "ab")
os.makedirs(out, exist_ok=True)
src = os.path.join(_build.CSRC, f"_ab_{name}_learner.hip")  # beside the headers it includes
with open(src, "w") as f:
    f.write(subprocess.check_output(["git", "-C", ROOT, "show", f"{rev}:agilerl_amd/csrc/learner.hip"], text=True))
try:
    obj = os.path.join(out, f"learner_{name}.o")
    subprocess.check_call([_build.HIPCC, *_build.CFLAGS, "-c", src, "-o", obj])
finally:
    os.remove(src)
objs = [os.path.join(_build.OBJDIR, o) for o in sorted(os.listdir(_build.OBJDIR))
        if o.endswith(".o") and o != "learner.hip.o"]
lib = os.path.join(out, f"libagx_{name}.so")
subprocess.check_call([_build.HIPCC, f"--offload-arch={_build.ARCH}", "-shared", "-fPIC", "-o", lib, obj, *objs])
print("built", lib)
