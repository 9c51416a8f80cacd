"""Host-code sanitizers (CPU only; GPU sanitizers are not available on this pool): the emulated
collectives (nexr_ring.cpp) and the C oracle built from source with g++ under ThreadSanitizer and under
AddressSanitizer + UndefinedBehaviorSanitizer, driven by tests/native/ring_stress.cpp with oracle
steps for the SIMPLE, LL and LL128 protocols, 2-6 rank threads, FIFO wrap-around; and the extras
library's send/recv protocol (nexr_p2p.cpp over nexr_ring.cpp) driven by tests/native/p2p_stress.cpp:
the send and recv halves of every thread rank at once over the shared FIFO counters, SIMPLE chunks and
LL lines, self-sends and ranks without a peer."""
import os
import subprocess

import pytest

from conftest import ROOT

HIP_INC = "/opt/rocm/include"
HIP_LIB = "/opt/rocm/lib"


DRIVERS = {"ring_stress": ["nexr_ring.cpp"], "p2p_stress": ["nexr_ring.cpp", "nexr_p2p.cpp"]}


@pytest.mark.parametrize("driver", sorted(DRIVERS))
@pytest.mark.parametrize("san", ["thread", "address,undefined"])
def test_ring_driver_under_sanitizer(tmp_path, san, driver):
    exe = tmp_path / f"{driver}_{san.split(',')[0]}"
    cmd = ["g++", "-std=c++17", "-O1", "-g", f"-fsanitize={san}", "-fno-omit-frame-pointer", "-D__HIP_PLATFORM_AMD__",
           f"-I{HIP_INC}", os.path.join(ROOT, "tests", "native", f"{driver}.cpp"),
           *[os.path.join(ROOT, "nex-nccl_amd", "csrc", f) for f in DRIVERS[driver]],
           "-x", "c", "-std=c11",
           os.path.join(ROOT, "oracle", "nexr_oracle.c"), "-x", "none",
           f"-L{os.path.join(ROOT, 'nex-nccl_amd')}", "-lnexr", f"-Wl,-rpath,{os.path.join(ROOT, 'nex-nccl_amd')}",
           f"-L{HIP_LIB}", "-lamdhip64", f"-Wl,-rpath,{HIP_LIB}", "-lpthread", "-o", str(exe)]
    subprocess.run(cmd, check=True, capture_output=True, text=True, timeout=300)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1",
               ASAN_OPTIONS="detect_leaks=0:halt_on_error=1", UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    p = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600, env=env)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    assert f"{driver} failures=0" in p.stdout
