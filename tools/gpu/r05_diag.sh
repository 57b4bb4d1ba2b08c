#!/bin/bash
# r05 diagnosis of the search levels (one stream): per-launch SQ counters
# (occupancy, issue rate) and kernel-trace durations at batch 32 and 64 (fixed
# vs per-round cost per launch), plus the config-5 kernel profile (refinement).
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
LIB=optical-flow-using-dense-inverse-search_amd/disflow/${LIB:-libdis_hip.so}
cd /tmp && export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $R/gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/$name.log; exit $rc; }; }
run sq 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE \
    --output-format csv -d $R/gpurun_out/r05_sq -o run -- python3 $R/tools/ab.py $R/$LIB:streams=1 --rounds 1 --steps 2
run tr32 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r05_tr32 -o run -- python3 $R/tools/ab.py $R/$LIB:streams=1 --rounds 2 --steps 5
run tr64 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r05_tr64 -o run -- python3 $R/tools/ab.py $R/$LIB:streams=1 --rounds 2 --steps 5 --batch 64
run cfg5 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r05_cfg5 -o run -- python3 $R/tools/bench_configs.py --configs 5,2p --steps 5
cd $R
python3 tools/trace_stats.py gpurun_out/r05_tr32/run_kernel_trace.csv gpurun_out/r05_tr32/grid_stats.csv > /dev/null
python3 tools/trace_stats.py gpurun_out/r05_tr64/run_kernel_trace.csv gpurun_out/r05_tr64/grid_stats.csv > /dev/null
python3 tools/trace_stats.py gpurun_out/r05_cfg5/run_kernel_trace.csv gpurun_out/r05_cfg5/grid_stats.csv > /dev/null
echo done
