#!/bin/bash
# r05 session 2: GPU suite; paper-mode A/B (r04 vs this tree); per-level
# one-stream traces of the auto layout and of 4 lanes per patch everywhere;
# SQ / HBM counters of the config-5 refinement kernels.
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
D=$R/optical-flow-using-dense-inverse-search_amd/disflow
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $R/gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v amdgpu.ids $R/gpurun_out/$name.log | tail -${TAILN:-6}; [ $rc -eq 0 ] || exit $rc; }
run s2_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run s2_ab_paper 300 python3 tools/ab.py $D/libdis_hip_r04.so:paper=1 $D/libdis_hip.so:paper=1 $D/libdis_hip.so --rounds 6 --steps 10
run s2_ab_lds2 300 python3 tools/ab.py $D/libdis_hip.so:fma=1 $D/libdis_hip_lds2.so:fma=1 --rounds 6 --steps 10
cd /tmp && export TMPDIR=/tmp
run s2_lv_lds2 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r05_lv_lds2 -o run -- python3 $R/tools/ab.py $D/libdis_hip.so:streams=1,fma=1 $D/libdis_hip_lds2.so:streams=1,fma=1 --rounds 2 --steps 5
run s2_lv_auto 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r05_lv_auto -o run -- python3 $R/tools/ab.py $D/libdis_hip.so:streams=1 --rounds 2 --steps 5
run s2_lv_lpp4 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r05_lv_lpp4 -o run -- python3 $R/tools/ab.py $D/libdis_hip.so:streams=1,variant=2 --rounds 2 --steps 5
CFG5="--preset slow --width 3840 --height 2160 --batch 2 --rounds 1 --steps 2"
run s2_vr_sq 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE \
    --output-format csv -d $R/gpurun_out/r05_vr_sq -o run -- python3 $R/tools/ab.py $D/libdis_hip.so $CFG5
run s2_vr_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/r05_vr_fetch -o run -- python3 $R/tools/ab.py $D/libdis_hip.so $CFG5
run s2_vr_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/r05_vr_write -o run -- python3 $R/tools/ab.py $D/libdis_hip.so $CFG5
cd $R
python3 tools/trace_stats.py gpurun_out/r05_lv_auto/run_kernel_trace.csv gpurun_out/r05_lv_auto/grid_stats.csv | head -14
python3 tools/trace_stats.py gpurun_out/r05_lv_lpp4/run_kernel_trace.csv gpurun_out/r05_lv_lpp4/grid_stats.csv | head -14
python3 tools/trace_stats.py gpurun_out/r05_lv_lds2/run_kernel_trace.csv gpurun_out/r05_lv_lds2/grid_stats.csv | head -6
python3 tools/pmc_summary.py gpurun_out/r05_vr_sq/run_counter_collection.csv --fetch gpurun_out/r05_vr_fetch/run_counter_collection.csv --write gpurun_out/r05_vr_write/run_counter_collection.csv --top 16
echo done
