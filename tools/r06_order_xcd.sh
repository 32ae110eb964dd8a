#!/bin/bash
# probe 21: row order inside columns x XCD-contiguous workgroup mapping
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/r06_order_xcd
mkdir -p $out
timeout -k 10 240 tools/probe_order_xcd 1e8 800 6 > $out/c4.txt 2>&1 && timeout -k 10 120 tools/probe_order_xcd 1.25e7 100 8 > $out/n8rank.txt 2>&1
