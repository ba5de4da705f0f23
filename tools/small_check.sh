set -e
mkdir -p gpurun_out/c4
timeout -k 10 120 ipm-zoo_amd/build/kbench 320 small > gpurun_out/kb_small.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/c4/tests.log 2>&1
for b in 1024 128; do
  timeout -k 10 120 python bench.py --workload c4 --batch $b --no-cpu-baseline > gpurun_out/c4/b$b.json 2>gpurun_out/c4/b$b.err
done
