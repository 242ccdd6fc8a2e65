"""The drop-in owns all 21 Dynprog_* symbols GMAP imports (the six dynprog*.o objects are the unit
of replacement).  CPU tests, no GPU call:

* oracle/_ref/gmap_gpu_{nosimd,avx2,large} are linked WITHOUT the reference's dynprog objects
  (oracle/ref.mk NODP_V): a string only those objects hold (Dynprog_endalign_string's message,
  dynprog.c:118) is in every unmodified gmap and in no drop-in build;
* the non-DP entry points the shim now defines -- Dynprog_consistent_p's table for every Mode_T and
  genestrand (dynprog.c:895-1197), Dynprog_score (:126), Dynprog_new / _free limits (:606-650) -- print the
  same as the reference's own (oracle/own_check.c linked both ways).
The DP entry points, Dynprog_make_splicejunction_5/3 and Dynprog_end5/3_known run in the owned builds on the
GPU in tests/test_gmap_e2e.py (every end-to-end fixture, -d -s included).
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(ROOT, "oracle", "_ref")
MARK = b"endalign %d not recognized"


@pytest.mark.parametrize("build", ["nosimd", "avx2", "large"])
def test_drop_in_links_without_reference_dynprog_objects(build):
    ref, gpu = os.path.join(REF, "gmap_" + build), os.path.join(REF, "gmap_gpu_" + build)
    if not (os.path.exists(ref) and os.path.exists(gpu)):
        pytest.skip("gmap programs not built (make -C oracle ref)")
    assert MARK in open(ref, "rb").read()
    assert MARK not in open(gpu, "rb").read()


def test_owned_non_dp_entry_points_match_reference():
    a, b = os.path.join(REF, "own_check_ref"), os.path.join(REF, "own_check_shim")
    if not (os.path.exists(a) and os.path.exists(b)):
        pytest.skip("own_check programs not built (make -C oracle ref)")
    ra = subprocess.run([a], capture_output=True, text=True, timeout=60, check=True).stdout
    rb = subprocess.run([b], capture_output=True, text=True, timeout=60, check=True).stdout
    assert ra.count("consistent mode") == 10 and ra.count("score ") == 54 and ra.count("new ") == 5
    assert ra == rb


@pytest.mark.parametrize("fibers", ["1", "0"])
def test_worker_fibers_without_gpu(fibers):
    """The drop-in's worker fibers (pthread_create / _join / _getspecific / _setspecific wrapped as in
    gmap_gpu_*): 300 workers on 5 host threads keep their own pthread-key values, run deep on their own
    stacks and hand their return values to pthread_join; with GMAPDP_SHIM_FIBERS=0 they are OS threads."""
    exe = os.path.join(REF, "fiber_check")
    if not os.path.exists(exe):
        pytest.skip("fiber_check not built (make -C oracle ref)")
    env = dict(os.environ, GMAPDP_SHIM_FIBERS=fibers, GMAPDP_SHIM_FIBER_HOSTS="5")
    r = subprocess.run([exe, "300"], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0 and r.stdout.strip() == "fibers ok 300", (r.stdout, r.stderr[-2000:])
