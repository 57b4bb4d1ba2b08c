#!/bin/bash
cd "$GRAFT_REPO_ROOT"; cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/lv -o run -- python3 $R/tools/ab.py "$@" --rounds 3 > /dev/null 2>&1
#timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/lvpmc -o run -- python3 $R/tools/ab.py "$@" --rounds 1 > /dev/null 2>&1
cd $R && python3 - <<'PY'
import csv, collections
rows = list(csv.DictReader(open('gpurun_out/lv/run_kernel_trace.csv')))
d = collections.defaultdict(list)
for r in rows:
    d[(r['Kernel_Name'][:24], r['Grid_Size_X'], r['Grid_Size_Y'], r['Grid_Size_Z'])].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1000)
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    v.sort(); print(k, len(v), 'median %.1f us' % v[len(v) // 2])
import sys; sys.exit(0)
rows = list(csv.DictReader(open('gpurun_out/lvpmc/run_counter_collection.csv')))
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.defaultdict(set)
for r in rows:
    k = (r['Kernel_Name'][:24], r['Grid_Size'])
    agg[k][r['Counter_Name']] += float(r['Counter_Value']); n[k].add(r['Dispatch_Id'])
for k, c in sorted(agg.items(), key=lambda kv: -kv[1]['SQ_INSTS_VALU']):
    m = len(n[k]); print(k, {x: round(v / m) for x, v in c.items()})
PY
