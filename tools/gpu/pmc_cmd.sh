#!/bin/bash
# SQ counters per (kernel, grid) for any python command of the repo:
#   bash tools/gpu/pmc_cmd.sh tools/bench_configs.py --configs colour
# (CTRS= to override the counter set, TOPK= kernels to print)
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
CTRS=${CTRS:-SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE}
timeout -k 10 120 rocprofv3 --pmc $CTRS --output-format csv -d $R/gpurun_out/pmc_cmd -o run -- python3 $R/"$@" > $R/gpurun_out/pmc_cmd.log 2>&1 || { tail -5 $R/gpurun_out/pmc_cmd.log; exit 1; }
cd $R && python3 - gpurun_out/pmc_cmd/run_counter_collection.csv <<'PY'
import csv, collections, os, sys
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    k = (r['Kernel_Name'][:40], int(r['Grid_Size']))
    agg[k][r['Counter_Name']] += float(r['Counter_Value']); n[k].add(r['Dispatch_Id'])
for k, c in sorted(agg.items(), key=lambda kv: -kv[1]['SQ_INSTS_VALU'])[:int(os.environ.get('TOPK', '4'))]:
    m = len(n[k]); d = {x: v / m for x, v in c.items()}; w = max(d.get('SQ_WAVES', 1), 1)
    print(k, m, 'dispatches;', ' '.join(f"{x}={v:.4g}" for x, v in d.items()))
    print('   per wave: ' + ' '.join(f"{x[3:]}={d[x] / w:.0f}" for x in d if x.startswith('SQ_') and x != 'SQ_WAVES'))
PY
