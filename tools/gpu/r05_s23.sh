#!/bin/bash
# r05 session 23: SOR with 512-thread workgroups (8 waves, 128 x 32 region,
# 14 output rows; two workgroups per CU) against the 1024-thread form:
# config-5 A/B (outputs compared bit for bit), SOR counters.
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
D=$R/optical-flow-using-dense-inverse-search_amd/disflow
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $R/gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v amdgpu.ids $R/gpurun_out/$name.log | tail -${TAILN:-6}; [ $rc -eq 0 ] || exit $rc; }
CFG5="--preset slow --width 3840 --height 2160 --batch 2"
run s23_ab_cfg5 400 python3 tools/ab.py $D/libdis_hip.so $D/libdis_hip_s512.so $CFG5 --rounds 5 --steps 3
cd /tmp && export TMPDIR=/tmp
run s23_tr 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r05_s23 -o run -- python3 $R/tools/ab.py $D/libdis_hip_s512.so $CFG5 --rounds 1 --steps 2
run s23_sq 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE \
    --output-format csv -d $R/gpurun_out/r05_s23_sq -o run -- python3 $R/tools/ab.py $D/libdis_hip_s512.so $CFG5 --rounds 1 --steps 2
cd $R
python3 tools/trace_stats.py gpurun_out/r05_s23/run_kernel_trace.csv /tmp/g.csv | grep "vr_sor" | head -2
python3 tools/pmc_summary.py gpurun_out/r05_s23_sq/run_counter_collection.csv --match k_vr_sor --top 1
echo done
