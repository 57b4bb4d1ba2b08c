#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 120 rocprofv3 --pmc $c --output-format csv -d $R/gpurun_out/calib_$c -o run -- $R/tools/pmc_calib > $R/gpurun_out/calib_$c.log 2>&1
  echo "calib $c rc=$?"
done
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc2 -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --streams 1 > $R/gpurun_out/pmc2.log 2>&1
echo "pmc2 rc=$?"
