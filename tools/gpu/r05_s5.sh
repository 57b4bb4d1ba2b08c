#!/bin/bash
# r05 session 5 (= sessions 3 + 4): paper-mode output with the I1 window in
# LDS and refinement v2 -- full GPU suite, A/Bs (paper: against the unstaged
# build; config 5: against the previous refinement), traces and counters.
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
D=$R/optical-flow-using-dense-inverse-search_amd/disflow
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $R/gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v amdgpu.ids $R/gpurun_out/$name.log | tail -${TAILN:-6}; [ $rc -eq 0 ] || exit $rc; }
run s5_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run s5_ab_paper 300 python3 tools/ab.py $D/libdis_hip_base.so:paper=1 $D/libdis_hip.so:paper=1 $D/libdis_hip.so --rounds 6 --steps 10
CFG5="--preset slow --width 3840 --height 2160 --batch 2"
run s5_ab_cfg5 300 python3 tools/ab.py $D/libdis_hip_pstage.so $D/libdis_hip.so $CFG5 --rounds 4 --steps 3
cd /tmp && export TMPDIR=/tmp
run s5_tr_paper 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r05_s5_paper -o run -- python3 $R/tools/ab.py $D/libdis_hip.so:streams=1,paper=1 --rounds 2 --steps 5
run s5_tr_cfg5 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r05_s5_cfg5 -o run -- python3 $R/tools/ab.py $D/libdis_hip.so $CFG5 --rounds 1 --steps 3
run s5_sq 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE \
    --output-format csv -d $R/gpurun_out/r05_s5_sq -o run -- python3 $R/tools/ab.py $D/libdis_hip.so $CFG5 --rounds 1 --steps 2
cd $R
python3 tools/trace_stats.py gpurun_out/r05_s5_paper/run_kernel_trace.csv gpurun_out/r05_s5_paper/grid_stats.csv | head -8
python3 tools/trace_stats.py gpurun_out/r05_s5_cfg5/run_kernel_trace.csv gpurun_out/r05_s5_cfg5/grid_stats.csv | grep -i "vr_\|densify" | head -12
python3 tools/pmc_summary.py gpurun_out/r05_s5_sq/run_counter_collection.csv --match k_vr --top 6
echo done
