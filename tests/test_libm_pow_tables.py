"""The glibc pow tables the device restatement uses
(agilerl_amd/csrc/libm_pow_tables.h) are exactly what the published recipe
generates (tools/gen_pow_tables.py), and their first entries are the ones
glibc ships (e_pow_log_data.c: A(0x1.6a00000000000p+0,
-0x1.62c82f2b9c800p-2, 0x1.ab42428375680p-48), ...)."""

import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_tables_regenerate_identically():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_pow_tables.py")], capture_output=True,
                         text=True, check=True).stdout
    with open(os.path.join(ROOT, "agilerl_amd", "csrc", "libm_pow_tables.h")) as f:
        assert f.read() == out
    assert "{0x1.6a00000000000p+0, -0x1.62c82f2b9c800p-2, 0x1.ab42428375680p-48}" in out
    assert "{0x1.6800000000000p+0, -0x1.5d1bdbf580800p-2, -0x1.ca508d8e0f720p-46}" in out
