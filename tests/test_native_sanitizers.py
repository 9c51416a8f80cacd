"""Host-code sanitizers (CPU only; GPU sanitizers are not available on this pool): the emulated
collectives (nexr_ring.cpp) and the C oracle built from source with g++ under ThreadSanitizer and under
AddressSanitizer + UndefinedBehaviorSanitizer, driven by tests/native/ring_stress.cpp with oracle
steps for the SIMPLE, LL and LL128 protocols, 2-6 rank threads, FIFO wrap-around."""
import os
import subprocess

import pytest

from conftest import ROOT

HIP_INC = "/opt/rocm/include"
HIP_LIB = "/opt/rocm/lib"


@pytest.mark.parametrize("san", ["thread", "address,undefined"])
def test_ring_driver_under_sanitizer(tmp_path, san):
    exe = tmp_path / f"ring_stress_{san.split(',')[0]}"
    cmd = ["g++", "-std=c++17", "-O1", "-g", f"-fsanitize={san}", "-fno-omit-frame-pointer", "-D__HIP_PLATFORM_AMD__",
           f"-I{HIP_INC}", os.path.join(ROOT, "tests", "native", "ring_stress.cpp"),
           os.path.join(ROOT, "nex-nccl_amd", "csrc", "nexr_ring.cpp"),
           "-x", "c", "-std=c11",
           os.path.join(ROOT, "oracle", "nexr_oracle.c"), "-x", "none",
           f"-L{os.path.join(ROOT, 'nex-nccl_amd')}", "-lnexr", f"-Wl,-rpath,{os.path.join(ROOT, 'nex-nccl_amd')}",
           f"-L{HIP_LIB}", "-lamdhip64", f"-Wl,-rpath,{HIP_LIB}", "-lpthread", "-o", str(exe)]
    subprocess.run(cmd, check=True, capture_output=True, text=True, timeout=300)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1",
               ASAN_OPTIONS="detect_leaks=0:halt_on_error=1", UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    p = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600, env=env)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    assert "ring_stress failures=0" in p.stdout
