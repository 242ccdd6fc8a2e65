"""tools/multi_gmap.py (configs[3]'s read sharding across GPUs, one GMAP process per GPU taking the
reads --part=i/N would give it, outputs merged in input order) checked on the CPU with the unmodified reference program:
the merged output of N parts equals the single-process output fixture (tests/golden/e2e_nosimd.sam,
200 synthetic reads).  The GPU run of the same tool is tests/test_gmap_e2e.py::test_gpu_gmap_parts."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
GOLD = os.path.join(ROOT, "tests", "golden")
EXE = os.path.join(ROOT, "oracle", "_ref", "gmap_nosimd")


@pytest.mark.parametrize("parts", [1, 2, 3])
def test_parts_merge_to_single_process_output(parts):
    if not os.path.exists(EXE):
        pytest.skip("reference gmap not built (make -C oracle ref)")
    import multi_gmap
    rc, out, errs, _ = multi_gmap.run(parts, 1, [EXE, "-g", "e2e_genome.fa", "-f", "samse", "--no-sam-headers"],
                                      "e2e_reads.fa", cwd=GOLD)
    assert rc == 0, errs
    assert out == open(os.path.join(GOLD, "e2e_nosimd.sam")).read()


def test_merge_groups_records_by_read():
    import multi_gmap
    a = "r0\t0\n r0\t256\n".replace(" ", "") + "r2\t4\n"
    b = "r1\t16\n"
    assert multi_gmap.merge([a, b]) == "r0\t0\nr0\t256\nr1\t16\nr2\t4\n"
