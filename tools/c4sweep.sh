set -e
mkdir -p gpurun_out/c4
for b in 1024 512 256 128; do
  timeout -k 10 120 python bench.py --workload c4 --batch $b --no-cpu-baseline > gpurun_out/c4/b$b.json 2>gpurun_out/c4/b$b.err
  timeout -k 10 120 python bench.py --workload c4 --batch $b --no-cpu-baseline --no-timing > gpurun_out/c4/b${b}_graph.json 2>>gpurun_out/c4/b$b.err
done
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/c4/prof128 -o run --output-format csv -- python bench.py --workload c4 --batch 128 --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/c4/prof128.log 2>&1
echo done
