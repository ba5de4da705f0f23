set -e
mkdir -p gpurun_out/eq
timeout -k 10 300 python -u -m pytest tests/test_gpu_eqnone.py tests/test_gpu_batch.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/eq/tests.log 2>&1
