#!/bin/bash
# online epoch: kernel time vs wall time (launch gaps), C3, one epoch after one warm-up epoch
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r34
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/ovprof -o ov --output-format csv -- \
  python3 bench.py --config c3 --method vb_online --steps 1 --warmup 1 --no-cpu-baseline > $O/online.json 2> $O/online.txt || exit $?
cp /tmp/ovprof/*/ov_kernel_stats.csv $O/ 2>/dev/null || find /tmp/ovprof -name "*kernel_stats.csv" -exec cp {} $O/ \;
python3 - <<'PY' > $O/gaps.txt
import csv, glob
f = glob.glob('/tmp/ovprof/**/*kernel_trace.csv', recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
# the last epoch: the last 45% of the trace by time is enough to see the steady state
t0 = int(rows[0]['Start_Timestamp']); t1 = int(rows[-1]['End_Timestamp'])
cut = t0 + (t1 - t0) * 0.55
sel = [r for r in rows if int(r['Start_Timestamp']) >= cut]
busy = sum(int(r['End_Timestamp']) - int(r['Start_Timestamp']) for r in sel)
span = int(sel[-1]['End_Timestamp']) - int(sel[0]['Start_Timestamp'])
print("kernels %d busy %.1f ms span %.1f ms busy/span %.3f" % (len(sel), busy / 1e6, span / 1e6, busy / span))
from collections import defaultdict
d = defaultdict(lambda: [0, 0])
for r in sel:
    n = r['Kernel_Name'][:60]
    d[n][0] += 1; d[n][1] += int(r['End_Timestamp']) - int(r['Start_Timestamp'])
for n, (c, t) in sorted(d.items(), key=lambda kv: -kv[1][1])[:8]:
    print("%-60s %7d  avg %.2f us" % (n, c, t / c / 1e3))
PY
