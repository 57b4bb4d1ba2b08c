#!/bin/bash
# SQ counters of the finest-level search launch vs iteration count (one stream)
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
LIB=${LIB:-optical-flow-using-dense-inverse-search_amd/disflow/libdis_hip.so}
for it in ${ITERS:-0 25}; do
  timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc$it -o run -- python3 $R/tools/ab.py $LIB:streams=1,iters=$it --rounds 1 --steps 2 > $R/gpurun_out/pmc$it.log 2>&1 || { tail -5 $R/gpurun_out/pmc$it.log; exit 1; }
  echo "iters=$it"
  (cd $R && python3 - gpurun_out/pmc$it/run_counter_collection.csv <<'PY'
import csv, collections, sys
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    k = (r['Kernel_Name'][:26], r['Grid_Size'])
    agg[k][r['Counter_Name']] += float(r['Counter_Value']); n[k].add(r['Dispatch_Id'])
for k, c in sorted(agg.items(), key=lambda kv: -kv[1]['SQ_INSTS_VALU'])[:2]:
    m = len(n[k]); w = c['SQ_WAVES'] / m
    print(k, {x: round(v / m) for x, v in c.items()}, 'VALU/wave %.0f SALU/wave %.0f LDS/wave %.0f VMEM/wave %.0f' % (c['SQ_INSTS_VALU'] / m / w, c['SQ_INSTS_SALU'] / m / w, c['SQ_INSTS_LDS'] / m / w, c['SQ_INSTS_VMEM_RD'] / m / w))
PY
)
done
