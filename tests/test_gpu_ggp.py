"""The packed genome-gap path (ggp_kernel.hip, opt-in with GMAPDP_GGP=1) against the oracle and the
reference's golden vectors.  The engine reads GMAPDP_GGP once per process, so these parity checks run
tests/test_gpu_genome_gap.py in a child process with the packed path switched on (one GPU process at
a time: the parent holds no context while the child runs)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("width", ["16", "8"])
def test_gpu_ggp_genome_gaps_bit_exact(width):
    env = dict(os.environ, GMAPDP_GGP="1", GMAPDP_GGP_S=width)
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-m", "gpu", "-p", "no:cacheprovider",
                        os.path.join(HERE, "test_gpu_genome_gap.py")],
                       env=env, capture_output=True, text=True, timeout=600, cwd=os.path.dirname(HERE))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
