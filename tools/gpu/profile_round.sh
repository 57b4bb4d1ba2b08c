#!/bin/bash
# Round profile: kernel trace + stats, PMC FETCH/WRITE passes -> traffic.json,
# PMC SQ pass, then the bench line (which picks up traffic.json).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${TAG:-r03}
R=$GRAFT_REPO_ROOT
BENCH="$R/bench.py --steps 10 --warmup 5 --warmup-floor 0 --no-cpu-baseline --no-tolerance-mode --no-pipelined"
cd /tmp && export TMPDIR=/tmp
run() { local name=$1; shift; timeout -k 10 400 "$@" > $R/gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/$name.log; exit $rc; }; }
run trace rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_trace -o run -- python3 $BENCH
run fetch rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/${TAG}_fetch -o run -- python3 $BENCH
run write rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/${TAG}_write -o run -- python3 $BENCH
run sq rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/${TAG}_sq -o run -- python3 $BENCH
run marker rocprofv3 --marker-trace --kernel-trace --output-format csv -d $R/gpurun_out/${TAG}_marker -o run -- python3 $R/bench.py --steps 3 --warmup 2 --warmup-floor 0 --no-cpu-baseline --no-tolerance-mode --no-pipelined --no-kernel-timing
cd $R
python3 tools/pmc_traffic.py gpurun_out/${TAG}_fetch/run_counter_collection.csv gpurun_out/${TAG}_write/run_counter_collection.csv --out gpurun_out/traffic.json
python3 tools/trace_stats.py gpurun_out/${TAG}_trace/run_kernel_trace.csv gpurun_out/${TAG}_trace/kernel_grid_stats.csv
timeout -k 10 400 python3 bench.py --traffic-json gpurun_out/traffic.json > gpurun_out/bench_final.log 2>&1; echo "bench rc=$?"; tail -1 gpurun_out/bench_final.log
