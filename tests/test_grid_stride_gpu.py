"""The kernel's grid-stride loop: a one-shot grid covers every call up to 2^24 workgroups (256 GiB
per buffer), so the stride path only runs beyond that. Forcing a small grid with NEXR_GRID (read
once per process, hence a child process per setting) makes every workgroup stride over many trips;
results must be identical to the oracle under every cache policy."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("grid,policy", [(1, "0"), (7, "1"), (256, "3"), (1000, "0")])
def test_forced_small_grid_strides(grid, policy):
    env = dict(os.environ, NEXR_GRID=str(grid), NEXR_POLICY=policy)
    p = subprocess.run([sys.executable, os.path.join(HERE, "grid_stride_worker.py")], capture_output=True, text=True,
                       timeout=300, env=env)
    assert p.returncode == 0 and "grid-stride ok" in p.stdout, p.stdout[-2000:] + p.stderr[-2000:]
