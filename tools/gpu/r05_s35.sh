#!/bin/bash
# r05 session 35: paper-mode densify reads a pixel's K x K patch flows before
# its first vote (one LDS latency per pixel instead of one per vote): paper
# tests, paper A/B against HEAD, output-kernel trace.
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
D=$R/optical-flow-using-dense-inverse-search_amd/disflow
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $R/gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v amdgpu.ids $R/gpurun_out/$name.log | tail -${TAILN:-6}; [ $rc -eq 0 ] || exit $rc; }
run s35_tests 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "paper or structured" --timeout 300 --timeout-method thread
TAILN=8 run s35_ab_paper 300 python3 tools/ab.py $D/libdis_hip_base.so:paper=1 $D/libdis_hip.so:paper=1 --rounds 8 --steps 10
cd /tmp && export TMPDIR=/tmp
run s35_tr_paper 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r05_s35_paper -o run -- python3 $R/tools/ab.py $D/libdis_hip.so:streams=1,paper=1 --rounds 2 --steps 5
cd $R
python3 tools/trace_stats.py gpurun_out/r05_s35_paper/run_kernel_trace.csv /tmp/g.csv | grep k_output
echo done
