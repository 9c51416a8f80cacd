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


@pytest.mark.parametrize("args", [("64", "5", "1"), ("32", "3", "3"), ("256", "20", "1")])
def test_c_multi_device_program(args):
    """C5 from plain C: one independent fp32 sum K=2 reduce-copy per work on every visible GPU from
    one nexrReduceCopyMultiDevice call (several works per device in the second case), every output
    checked against a + b on the host."""
    exe = os.path.join(ROOT, "xbin", "multi_device_c")
    if not os.path.exists(exe):
        import __graft_entry__
        exe = __graft_entry__.build_c_multi_device()
    p = subprocess.run([exe, *args], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0 and "multi_device_c ok" in p.stdout, p.stdout + p.stderr
    print(p.stdout.strip())


@pytest.mark.parametrize("args", [("40", "64"), ("100", "4"), ("9", "1024")])
def test_c_ll_steps_program(args):
    """A run of LL steps with device credits from plain C (nexrReduceCopyLLSteps): 40 steps through 8
    slots of 64 KiB, 100 through 4 KiB slots (one workgroup), 9 through 1 MiB slots (64 workgroups, two
    tiles each); every output element checked against a + b on the host."""
    exe = os.path.join(ROOT, "xbin", "ll_steps_c")
    if not os.path.exists(exe):
        import __graft_entry__
        exe = __graft_entry__.build_c_ll_steps()
    p = subprocess.run([exe, *args], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0 and "ll_steps_c ok" in p.stdout, p.stdout + p.stderr
