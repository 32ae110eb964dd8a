#!/bin/bash
# Config 3 (1e7 rows x 40 one-hot fields x 25,000 ids, k = 50, -method vb, one MI355X: "rocprof
# HBM GB/s vs roofline"): rocprofv3 kernel trace of the bench, then FETCH_SIZE and WRITE_SIZE
# in separate --pmc passes on the level kernel (k = 4: a level launch moves the same bytes).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
out=gpurun_out/${1:-prof_c3}
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/kt -o kt --output-format csv -- \
  python3 bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline > $out/bench.json 2> $out/bench.txt || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --kernel-include-regex k_level_lord -d $out/$c -o p \
    --output-format csv -- python3 bench.py --config c3 --k 4 --steps 2 --warmup 0 --no-cpu-baseline \
    > $out/$c.json 2> $out/$c.txt || exit $?
done
exit 0
