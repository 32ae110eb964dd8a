cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_split
VBFM_FORCE_SPLIT=1 timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_split -o kt --output-format csv -- python3 bench.py --k 8 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/prof_split/b.json 2> gpurun_out/prof_split/b.log
