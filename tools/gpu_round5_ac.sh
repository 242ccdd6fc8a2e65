set -o pipefail
O=gpurun_out/r05ac
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 500 --timeout-method thread tests/test_gpu_oligo.py > $O/t1.log 2>&1 || exit 11
