#!/bin/bash
# kernel trace + per-(kernel, grid) stats of tools/bench_configs.py --configs "$1"
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/ct -o run -- python3 $R/tools/bench_configs.py --configs "$1" --steps ${STEPS:-4} --warmup 2 > $R/gpurun_out/ct.log 2>&1 || { tail -5 $R/gpurun_out/ct.log; exit 1; }
cd $R && python3 tools/trace_stats.py gpurun_out/ct/run_kernel_trace.csv gpurun_out/ct/stats.csv > gpurun_out/ct/stats.txt && python3 - <<'PY'
import csv, collections
tot = collections.defaultdict(float); cnt = collections.Counter()
for r in csv.DictReader(open('gpurun_out/ct/stats.csv')):
    k = r['Kernel_Name'].split('(')[0].replace('void ', '')
    tot[k] += float(r['Total_us']); cnt[k] += int(r['Calls'])
T = sum(tot.values())
for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[:14]:
    print(f"{k[:40]:40s} {v/1e3:9.2f} ms  {100*v/T:5.1f}%  calls {cnt[k]}")
PY
grep '^{' gpurun_out/ct.log | cut -c1-200
