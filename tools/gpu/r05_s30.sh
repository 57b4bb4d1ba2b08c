#!/bin/bash
# r05 session 30: paper-mode densify -- staged/global choice hoisted out of the
# pixel loop, fixed staging row stride (tap addresses by one fma), vote weight
# behind a wave-uniform test: GPU suite, paper / reference A/B, output counters.
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
D=$R/optical-flow-using-dense-inverse-search_amd/disflow
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $R/gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v amdgpu.ids $R/gpurun_out/$name.log | tail -${TAILN:-6}; [ $rc -eq 0 ] || exit $rc; }
run s30_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
TAILN=8 run s30_ab_paper 300 python3 tools/ab.py $D/libdis_hip_base.so:paper=1 $D/libdis_hip.so:paper=1 --rounds 8 --steps 10
TAILN=8 run s30_ab_head 300 python3 tools/ab.py $D/libdis_hip_base.so $D/libdis_hip.so --rounds 6 --steps 10
cd /tmp && export TMPDIR=/tmp
run s30_tr_paper 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r05_s30_paper -o run -- python3 $R/tools/ab.py $D/libdis_hip.so:streams=1,paper=1 --rounds 2 --steps 5
run s30_sq_paper 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE \
    --output-format csv -d $R/gpurun_out/r05_s30_sqp -o run -- python3 $R/tools/ab.py $D/libdis_hip.so:streams=1,paper=1 --rounds 1 --steps 3
cd $R
python3 tools/trace_stats.py gpurun_out/r05_s30_paper/run_kernel_trace.csv /tmp/g.csv | head -8
python3 tools/pmc_summary.py gpurun_out/r05_s30_sqp/run_counter_collection.csv --match k_output --top 3
python3 tools/pmc_summary.py gpurun_out/r05_s30_sqp/run_counter_collection.csv --match k_search8 --top 2
echo done
