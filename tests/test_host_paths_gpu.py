"""nexrReduceCopyHost's two staging paths for pageable buffers, each forced through its knobs in a
child process (the library reads them once) and checked against the oracle on pageable, pinned and
mixed buffers, every datatype family, K = 1..8, M = 1..3, pre/post ops and in place:

  chunk pipeline   the runtime's hipMemcpyAsync into a device ring, two streams (mid-size calls)
  solo             the calling thread memcpys into pinned zero-copy slots, kernel over PCIe (small
                   calls), here with 64 KiB chunks so every call cycles all 3 slots many times
  copy team        a team of host threads does the same copies (large calls), also with small chunks
"""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))

PATHS = {
    "chunk-pipeline": {"NEXR_HOST_COPY_THREADS": "0", "NEXR_HOST_CHUNK_BYTES": "1048576"},
    "solo": {"NEXR_HOST_COPY_THREADS": "1", "NEXR_HOST_MT_MIN_BYTES": str(1 << 60),
             "NEXR_HOST_SOLO_MAX_BYTES": str(1 << 60), "NEXR_HOST_SMALL_CHUNK_BYTES": "65536"},
    "copy-team-3": {"NEXR_HOST_COPY_THREADS": "3", "NEXR_HOST_MT_MIN_BYTES": "0", "NEXR_HOST_MT_CHUNK_BYTES": "65536"},
    "copy-team-8": {"NEXR_HOST_COPY_THREADS": "8", "NEXR_HOST_MT_MIN_BYTES": "0",
                    "NEXR_HOST_MT_CHUNK_BYTES": "4194304"},
}


@pytest.mark.parametrize("path", sorted(PATHS))
def test_host_path_matches_oracle(path):
    env = dict(os.environ, **PATHS[path])
    p = subprocess.run([sys.executable, os.path.join(HERE, "host_path_worker.py"), path], capture_output=True,
                       text=True, timeout=300, env=env)
    assert p.returncode == 0 and "host-path ok" in p.stdout, p.stdout[-2000:] + p.stderr[-2000:]


@pytest.mark.parametrize("path", ["chunk-pipeline", "solo", "copy-team-3"])
def test_host_path_concurrent_callers(path):
    env = dict(os.environ, **PATHS[path])
    p = subprocess.run([sys.executable, os.path.join(HERE, "host_path_worker.py"), path, "concurrent"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode == 0 and "host-path ok concurrent" in p.stdout, p.stdout[-2000:] + p.stderr[-2000:]
