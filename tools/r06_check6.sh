#!/bin/bash
# probe_frag at C3 and C4 record counts; PMC passes of one N = 8 rank's level, deferred split vs fused
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
out=gpurun_out/r06_c6
mkdir -p $out
timeout -k 10 300 tools/probe_frag 1e7 12 6 > $out/frag_c3.txt 2>&1 || exit $?
echo "frag c3 done $(date +%T)" >> $out/progress.txt
timeout -k 10 400 tools/probe_frag 1e8 8 3 > $out/frag_c4.txt 2>&1 || exit $?
echo "frag c4 done $(date +%T)" >> $out/progress.txt
B="bench.py --rows 12500000 --k 4 --steps 1 --warmup 0 --no-cpu-baseline"
export VBFM_PLACE_TRIES=4
for form in split fused; do
  extra=""; [ $form = split ] && extra="--one-rank-comm"
  i=0
  for pmc in "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" \
             "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $pmc --kernel-trace -d $out/pmc_${form}_$i -o p --output-format csv -- \
      python3 $B $extra > $out/pmc_${form}_$i.json 2> $out/pmc_${form}_$i.log
    rc=$?; echo "pmc $form $i rc=$rc $(date +%T)" >> $out/progress.txt
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
