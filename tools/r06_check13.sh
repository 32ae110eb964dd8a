#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
out=gpurun_out/r06_c13
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/c2_kt -o kt --output-format csv -- \
  python3 bench.py --config c2 --steps 10 --warmup 1 --no-cpu-baseline > $out/c2_kt_bench.json 2> $out/c2_kt.log || exit $?
timeout -k 10 600 python3 bench.py --config c3 --gpus 2 --transport host --steps 2 --warmup 1 > $out/c3_n2_host.json 2> $out/c3_n2_host.log
