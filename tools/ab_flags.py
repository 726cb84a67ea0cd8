"""Build A/B variants of libagx.so whose learner.hip is compiled with extra
preprocessor flags (shape-only: the config-2 learner instantiations alone,
AGX_BENCH_SHAPE_ONLY), every other object from the current build:
  python tools/ab_flags.py <name> [-DFLAG=V ...]  -> ab/libagx_<name>.so
  AGX_LIB=ab/libagx_<name>.so python tools/learn_time.py"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from agilerl_amd import _build  # noqa: E402

name, flags = sys.argv[1], sys.argv[2:]
_build.build()
out = os.path.join(ROOT, "ab")
os.makedirs(out, exist_ok=True)
obj = os.path.join(out, f"learner_{name}.o")
subprocess.check_call([_build.HIPCC, *_build.CFLAGS, "-DAGX_BENCH_SHAPE_ONLY", *flags, "-c",
                       os.path.join(_build.CSRC, "learner.hip"), "-o", obj])
objs = [os.path.join(_build.OBJDIR, o) for o in sorted(os.listdir(_build.OBJDIR))
        if o.endswith(".o") and o != "learner.hip.o"]
lib = os.path.join(out, f"libagx_{name}.so")
subprocess.check_call([_build.HIPCC, f"--offload-arch={_build.ARCH}", "-shared", "-fPIC", "-o", lib, obj, *objs])
print("built", lib)
