#!/bin/bash
# rocprofv3 kernel-trace + PMC (FETCH_SIZE / WRITE_SIZE in separate passes) of one bench step.
# usage: tools/profile_session.sh <config> <tag> [extra bench args]
cd "$GRAFT_REPO_ROOT" || exit 1
cfg=${1:-c3}; tag=${2:-run}; shift 2
export TMPDIR=/tmp
out=gpurun_out/prof_${tag}
mkdir -p $out
B="bench.py --config $cfg --steps 1 --warmup 0 --no-cpu-baseline $*"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $out/kt -o kt --output-format csv -- python3 $B > $out/kt.log 2>&1 || { echo "kt failed $?"; exit 1; }
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $out/fetch -o f --output-format csv -- python3 $B > $out/fetch.log 2>&1 || { echo "fetch failed $?"; exit 1; }
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $out/write -o w --output-format csv -- python3 $B > $out/write.log 2>&1 || { echo "write failed $?"; exit 1; }
find $out -name "*.csv" | head -20
exit 0
