"""The plain-C host program (examples/reduce_copy_c.c, built by __graft_entry__.build() into
xbin/) on MI355X: nexrReduceCopyHost on pageable buffers (fp32 sum K=2, int8 max K=4 M=2) against a C
loop, and the C1 ring all-reduce (2 emulated ranks, 4 MiB fp32) from C."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_c_host_program():
    exe = os.path.join(ROOT, "xbin", "reduce_copy_c")
    if not os.path.exists(exe):
        import __graft_entry__
        exe = __graft_entry__.build_c_example()
    p = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0 and "reduce_copy_c ok" in p.stdout, p.stdout + p.stderr
