#!/bin/bash
# r05 session 9: refinement v3 (register-resident SOR with light-cone row
# skipping; XCD-aware tile order in k_vr_lin / k_vr_sor) -- config-5 tests,
# A/B against the committed build, trace + counters of config 5.
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
D=$R/optical-flow-using-dense-inverse-search_amd/disflow
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $R/gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v amdgpu.ids $R/gpurun_out/$name.log | tail -${TAILN:-6}; [ $rc -eq 0 ] || exit $rc; }
run s9_tests 400 python -u -m pytest tests/test_gpu_config5.py -x -q --timeout 300 --timeout-method thread
CFG5="--preset slow --width 3840 --height 2160 --batch 2"
run s9_ab_cfg5 300 python3 tools/ab.py $D/libdis_hip_base.so $D/libdis_hip.so $CFG5 --rounds 4 --steps 3
cd /tmp && export TMPDIR=/tmp
run s9_tr_cfg5 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r05_s9_cfg5 -o run -- python3 $R/tools/ab.py $D/libdis_hip.so $CFG5 --rounds 1 --steps 3
run s9_sq 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE \
    --output-format csv -d $R/gpurun_out/r05_s9_sq -o run -- python3 $R/tools/ab.py $D/libdis_hip.so $CFG5 --rounds 1 --steps 2
run s9_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/r05_s9_fetch -o run -- python3 $R/tools/ab.py $D/libdis_hip.so $CFG5 --rounds 1 --steps 2
run s9_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/r05_s9_write -o run -- python3 $R/tools/ab.py $D/libdis_hip.so $CFG5 --rounds 1 --steps 2
cd $R
python3 tools/trace_stats.py gpurun_out/r05_s9_cfg5/run_kernel_trace.csv gpurun_out/r05_s9_cfg5/grid_stats.csv | grep -i "vr_" | head -12
python3 tools/pmc_summary.py gpurun_out/r05_s9_sq/run_counter_collection.csv --fetch gpurun_out/r05_s9_fetch/run_counter_collection.csv --write gpurun_out/r05_s9_write/run_counter_collection.csv --match k_vr --top 8
echo done
