#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/r06_c8
mkdir -p $out
timeout -k 10 400 tools/probe_frag 1e8 8 4 > $out/frag_c4.txt 2>&1 || exit $?
timeout -k 10 300 tools/probe_frag 1.25e7 16 4 > $out/frag_n8.txt 2>&1
