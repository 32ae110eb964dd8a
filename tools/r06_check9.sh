#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/r06_c9
mkdir -p $out
timeout -k 10 300 tools/probe_frag 1e7 pads 6 > $out/pads_c3.txt 2>&1 || exit $?
timeout -k 10 400 tools/probe_frag 1e8 pads 4 > $out/pads_c4.txt 2>&1
