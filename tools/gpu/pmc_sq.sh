#!/bin/bash
# SQ counters per (kernel, grid) for tools/ab.py "$1" (one variant), top kernels
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
CTRS=${CTRS:-SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE}
k=0
for v in "$@"; do
  k=$((k+1))
  timeout -k 10 90 rocprofv3 --pmc $CTRS --output-format csv -d $R/gpurun_out/pmc_$k -o run -- python3 $R/tools/ab.py $v --rounds 1 --steps 2 > $R/gpurun_out/pmc_$k.log 2>&1 || { tail -5 $R/gpurun_out/pmc_$k.log; exit 1; }
  echo "== $v"
  (cd $R && python3 - gpurun_out/pmc_$k/run_counter_collection.csv <<'PY'
import csv, collections, sys
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    k = (r['Kernel_Name'][:26], int(r['Grid_Size']))
    agg[k][r['Counter_Name']] += float(r['Counter_Value']); n[k].add(r['Dispatch_Id'])
for k, c in sorted(agg.items(), key=lambda kv: -kv[1]['SQ_INSTS_VALU'])[:int(__import__('os').environ.get('TOPK', '3'))]:
    m = len(n[k]); w = c['SQ_WAVES'] / m
    d = {x: v / m for x, v in c.items()}
    print(k, ' '.join(f"{x}={v:.4g}" for x, v in d.items()))
    print('   per wave: VALU %.0f LDS %.0f  wave-cycles %.0f  wait %.0f  bankconf/LDS %.2f' % (
        d["SQ_INSTS_VALU"] / w, d['SQ_INSTS_LDS'] / w, d['SQ_WAVE_CYCLES'] / w,
        d.get('SQ_WAIT_INST_ANY', 0) / w, d.get('SQ_LDS_BANK_CONFLICT', 0) / max(d['SQ_INSTS_LDS'], 1)))
PY
)
done
