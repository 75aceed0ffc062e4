set -o pipefail
O=gpurun_out/r5fuzztest; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kryo_fuzz.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
