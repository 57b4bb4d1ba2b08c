#!/bin/bash
# r05 session 6: the fallback search reading its taps through a buffer
# descriptor (libdis_hip_fb.so) -- GPU suite on that build, A/B on the
# fallback-heavy variant 9 and the default; paper-mode output counters.
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
D=$R/optical-flow-using-dense-inverse-search_amd/disflow
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $R/gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v amdgpu.ids $R/gpurun_out/$name.log | tail -${TAILN:-6}; [ $rc -eq 0 ] || exit $rc; }
DISFLOW_LIB=$D/libdis_hip_fb.so run s6_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run s6_ab 300 python3 tools/ab.py $D/libdis_hip.so:variant=9 $D/libdis_hip_fb.so:variant=9 $D/libdis_hip.so $D/libdis_hip_fb.so --rounds 6 --steps 5
cd /tmp && export TMPDIR=/tmp
run s6_sq 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE \
    --output-format csv -d $R/gpurun_out/r05_s6_sq -o run -- python3 $R/tools/ab.py $D/libdis_hip.so:streams=1,paper=1 --rounds 1 --steps 2
run s6_lds 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD TA_BUSY_avr GRBM_GUI_ACTIVE \
    --output-format csv -d $R/gpurun_out/r05_s6_lds -o run -- python3 $R/tools/ab.py $D/libdis_hip.so:streams=1,paper=1 --rounds 1 --steps 2
cd $R
python3 tools/pmc_summary.py gpurun_out/r05_s6_sq/run_counter_collection.csv --match k_output --top 4
python3 - gpurun_out/r05_s6_lds/run_counter_collection.csv <<'PY'
import csv, collections, sys
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    if "k_output" not in r["Kernel_Name"]: continue
    k = (r["Kernel_Name"][:40], r["Grid_Size"]); agg[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[k].add(r["Dispatch_Id"])
for k, d in agg.items():
    m = len(n[k]); print(k, {c: round(v / m) for c, v in d.items()})
PY
echo done
