#!/bin/bash
# k_pyr12 wave orders: L2 (TCC) counters of the plain order
# and of the XCD order (DIS_PYR12_XCD=1, fewer L2 misses but slower), one PMC
# pass per counter group, tools/ab.py one-stream runs of each library:
#   tools/build_variants.sh pyrxcd:"-DDIS_PYR12_XCD=1"
#   bash tools/gpu/pyr_tcc.sh libdis_hip.so libdis_hip_pyrxcd.so
# Per counter: the mean per dispatch summed over instances, and the spread
# over instances (max / mean: channels or XCDs served unevenly).
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT; D=optical-flow-using-dense-inverse-search_amd/disflow
cd /tmp && export TMPDIR=/tmp
PASSES=("TCC_HIT TCC_MISS GRBM_GUI_ACTIVE" "TCC_EA0_RDREQ TCC_EA0_WRREQ GRBM_GUI_ACTIVE"
        "TCC_EA0_RDREQ_DRAM_CREDIT_STALL TCC_EA0_WRREQ_DRAM_CREDIT_STALL GRBM_GUI_ACTIVE"
        "TCC_EA0_RDREQ_LEVEL TCC_EA0_WRREQ_LEVEL GRBM_GUI_ACTIVE")
k=0
for lib in "$@"; do
  for p in "${PASSES[@]}"; do
    k=$((k+1))
    timeout -s KILL 90 rocprofv3 --pmc $p --output-format csv -d $R/gpurun_out/tcc_$k -o run -- \
      python3 $R/tools/ab.py $D/$lib:streams=1 --rounds 1 --steps 2 > $R/gpurun_out/tcc_$k.log 2>&1 || { tail -5 $R/gpurun_out/tcc_$k.log; exit 1; }
    echo "== $lib: $p"
    (cd $R && python3 - gpurun_out/tcc_$k/run_counter_collection.csv <<'PY'
import csv, collections, sys
vals = collections.defaultdict(list)  # (counter) -> per-dispatch lists of instance values
cur = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    if 'k_pyr12' not in r['Kernel_Name']:
        continue
    cur[r['Dispatch_Id']][r['Counter_Name']].append(float(r['Counter_Value']))
agg = collections.defaultdict(list)
for d, cs in cur.items():
    for c, v in cs.items():
        agg[c].append(v)
for c, runs in sorted(agg.items()):
    tot = sum(sum(v) for v in runs) / len(runs)
    n = len(runs[0])
    spread = max(max(v) / (sum(v) / len(v)) if sum(v) else 0 for v in runs)
    print(f"   {c:36s} per dispatch {tot:.4g}  instances {n}  max/mean {spread:.2f}  ({len(runs)} dispatches)")
PY
)
  done
done
