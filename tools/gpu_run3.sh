set -o pipefail
for c in c3 c2; do
  timeout -k 10 300 python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_${c}_level.json 2> gpurun_out/bench_${c}_level.log || exit $?
  timeout -k 10 300 python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --layout column > gpurun_out/bench_${c}_column.json 2> gpurun_out/bench_${c}_column.log || exit $?
done
