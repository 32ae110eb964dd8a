#!/bin/bash
# Round-3 profile of the DRIVER's bench command on the final tree, in one lease (VERDICT r02
# item 5): rocprofv3 --kernel-trace --stats of `bench.py --gpus 1 --steps 20 --warmup 5` itself
# (its JSON line -- ms_per_step, the HIP-event launch time -- kept beside the summary).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
out=gpurun_out/${1:-prof_r03}
mkdir -p $out
echo "kt start $(date +%T)" >> $out/progress.txt
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $out/kt -o kt --output-format csv -- \
  python3 bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.txt
rc=$?; echo "kt rc=$rc $(date +%T)" >> $out/progress.txt; [ $rc -ne 0 ] && exit $rc
# the PMC passes: tools/profile_r03_pmc.sh (k = 4: counted dispatches of the k = 100 command are
# too slow and the tool's dispatch hook segfaulted after ~8000 of them, profiles/r03_final/)
exit 0
