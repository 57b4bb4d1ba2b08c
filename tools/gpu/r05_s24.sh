#!/bin/bash
# r05 session 24: SOR knock-outs (timing only, wrong results): sweeps without
# memory (_kpu: no coefficient loads, no vertical LDS reads, no barriers)
# vs the same with every branch gone (_kst: no row skipping, one colour
# branch per half-sweep, no division guard) -- is the issue rate the branches?
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
D=$R/optical-flow-using-dense-inverse-search_amd/disflow
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $R/gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v amdgpu.ids $R/gpurun_out/$name.log | tail -${TAILN:-3}; [ $rc -eq 0 ] || exit $rc; }
CFG5="--preset slow --width 3840 --height 2160 --batch 2 --rounds 1 --steps 2"
cd /tmp && export TMPDIR=/tmp
for v in _kpu _kst; do
  run s24_sq$v 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE \
    --output-format csv -d $R/gpurun_out/r05_s24_sq$v -o run -- python3 $R/tools/ab.py $D/libdis_hip$v.so $CFG5
  run s24_tr$v 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r05_s24$v -o run -- python3 $R/tools/ab.py $D/libdis_hip$v.so $CFG5
done
cd $R
for v in _kpu _kst; do
  echo "-- $v"; python3 tools/trace_stats.py gpurun_out/r05_s24$v/run_kernel_trace.csv /tmp/g.csv | grep "vr_sor" | head -1
  python3 tools/pmc_summary.py gpurun_out/r05_s24_sq$v/run_counter_collection.csv --match k_vr_sor --top 1
done
echo done
