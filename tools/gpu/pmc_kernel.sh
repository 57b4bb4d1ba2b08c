#!/bin/bash
# SQ counters of one kernel (name substring $1) for a tools/ab.py variant ($2):
#   CTRS="..." bash tools/gpu/pmc_kernel.sh k_pyramid lib.so:streams=1
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
CTRS=${CTRS:-SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE}
timeout -k 10 90 rocprofv3 --pmc $CTRS --output-format csv -d $R/gpurun_out/pmck -o run -- python3 $R/tools/ab.py $2 --rounds 1 --steps 2 > $R/gpurun_out/pmck.log 2>&1 || { tail -5 $R/gpurun_out/pmck.log; exit 1; }
cd $R && python3 - gpurun_out/pmck/run_counter_collection.csv "$1" <<'PY'
import csv, collections, sys
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    if sys.argv[2] not in r['Kernel_Name']:
        continue
    k = (r['Kernel_Name'][:40], int(r['Grid_Size']))
    agg[k][r['Counter_Name']] += float(r['Counter_Value']); n[k].add(r['Dispatch_Id'])
for k, c in agg.items():
    m = len(n[k]); d = {x: v / m for x, v in c.items()}; w = d.get('SQ_WAVES', 1)
    print(k, ' '.join(f"{x}={v:.4g}" for x, v in sorted(d.items())))
    print('   per wave:', ' '.join(f"{x[3:]}={v / w:.0f}" for x, v in sorted(d.items()) if x.startswith('SQ_') and x != 'SQ_WAVES'))
PY
