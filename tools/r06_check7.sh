#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/r06_c7
mkdir -p $out
timeout -k 10 300 tools/probe_frag 1e7 6 8 > $out/frag_c3.txt 2>&1 || exit $?
timeout -k 10 300 tools/probe_frag 1.25e7 6 8 > $out/frag_n8.txt 2>&1 || exit $?
timeout -k 10 400 tools/probe_frag 1e8 6 8 > $out/frag_c4.txt 2>&1
