#!/bin/bash
# probe 22: buffers assembled from scored physical chunks (C4 size, 1 GB chunks, 150 GB scanned)
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-r06_assemble}
mkdir -p $out
timeout -k 10 500 tools/probe_assemble 1e8 1024 150 > $out/assemble.txt 2>&1
