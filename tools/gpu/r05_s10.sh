#!/bin/bash
# r05 session 10: paper-mode densify in class-sorted pixel order (_cs), + the
# paper init's votes split over the two lanes of a patch (libdis_hip); A/B of
# the XCD tile order in k_vr_lin (config 5); GPU suite.
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
D=$R/optical-flow-using-dense-inverse-search_amd/disflow
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $R/gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v amdgpu.ids $R/gpurun_out/$name.log | tail -${TAILN:-6}; [ $rc -eq 0 ] || exit $rc; }
run s10_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
TAILN=8 run s10_ab_head 300 python3 tools/ab.py $D/libdis_hip_base.so $D/libdis_hip.so --rounds 8 --steps 20
TAILN=8 run s10_ab_paper 300 python3 tools/ab.py $D/libdis_hip_base.so:paper=1 $D/libdis_hip_cs.so:paper=1 $D/libdis_hip.so:paper=1 --rounds 6 --steps 10
CFG5="--preset slow --width 3840 --height 2160 --batch 2"
run s10_ab_cfg5 300 python3 tools/ab.py $D/libdis_hip_base.so $D/libdis_hip_linnr.so $D/libdis_hip.so $CFG5 --rounds 4 --steps 3
cd /tmp && export TMPDIR=/tmp
run s10_tr_head 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r05_s10_head -o run -- python3 $R/tools/ab.py $D/libdis_hip.so --rounds 2 --steps 5
run s10_tr_paper 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r05_s10_paper -o run -- python3 $R/tools/ab.py $D/libdis_hip.so:streams=1,paper=1 --rounds 2 --steps 5
run s10_sq_paper 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE \
    --output-format csv -d $R/gpurun_out/r05_s10_sqp -o run -- python3 $R/tools/ab.py $D/libdis_hip.so:streams=1,paper=1 --rounds 1 --steps 3
cd $R
python3 tools/trace_stats.py gpurun_out/r05_s10_head/run_kernel_trace.csv gpurun_out/r05_s10_head/grid_stats.csv | head -8
python3 tools/trace_stats.py gpurun_out/r05_s10_paper/run_kernel_trace.csv gpurun_out/r05_s10_paper/grid_stats.csv | head -8
python3 tools/pmc_summary.py gpurun_out/r05_s10_sqp/run_counter_collection.csv --match k_search8 --top 3
python3 tools/pmc_summary.py gpurun_out/r05_s10_sqp/run_counter_collection.csv --match k_output --top 3
echo done
