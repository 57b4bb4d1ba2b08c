#!/bin/bash
# r05 session 29: sor_div behind a wave-uniform ballot test instead of an
# exec-masked branch (SOR and lin): refinement tests, config-5
# A/B against HEAD, SOR counters.
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
D=$R/optical-flow-using-dense-inverse-search_amd/disflow
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $R/gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v amdgpu.ids $R/gpurun_out/$name.log | tail -${TAILN:-6}; [ $rc -eq 0 ] || exit $rc; }
run s29_tests 500 python -u -m pytest tests/test_gpu_config5.py tests/test_gpu_parity.py -m gpu -x -q -k "config5 or refine or vr or paper_mode_batch" --timeout 300 --timeout-method thread
CFG5="--preset slow --width 3840 --height 2160 --batch 2"
run s29_ab_cfg5 400 python3 tools/ab.py $D/libdis_hip_base.so $D/libdis_hip.so $CFG5 --rounds 5 --steps 3
cd /tmp && export TMPDIR=/tmp
run s29_tr 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r05_s29 -o run -- python3 $R/tools/ab.py $D/libdis_hip.so $CFG5 --rounds 1 --steps 2
run s29_sq 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE \
    --output-format csv -d $R/gpurun_out/r05_s29_sq -o run -- python3 $R/tools/ab.py $D/libdis_hip.so $CFG5 --rounds 1 --steps 2
cd $R
python3 tools/trace_stats.py gpurun_out/r05_s29/run_kernel_trace.csv /tmp/g.csv | grep "vr_sor\|vr_lin" | head -4
python3 tools/pmc_summary.py gpurun_out/r05_s29_sq/run_counter_collection.csv --match k_vr_sor --top 1
echo done
