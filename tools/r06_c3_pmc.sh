#!/bin/bash
# C3: the level kernel's HBM bytes, one counter per rocprofv3 pass (FETCH_SIZE, then WRITE_SIZE)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
out=gpurun_out/${1:-r06_c3_pmc}
mkdir -p $out
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/fetch -o pmc -- python3 -u bench.py --config c3 --steps 1 --warmup 0 --no-launch-events > $out/b_fetch.json 2> $out/b_fetch.log && \
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/write -o pmc -- python3 -u bench.py --config c3 --steps 1 --warmup 0 --no-launch-events > $out/b_write.json 2> $out/b_write.log
