#!/bin/bash
# GPU session script: every GPU step has its own time limit; a crash, abort or
# timeout ends the script (no further GPU work), plain test failures do not.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -25 "gpurun_out/$name.log"
  case $rc in 0|1) ;; *) echo "fatal rc=$rc in $name, stopping"; exit $rc;; esac
}
echo "host cores: $(nproc)"; lscpu | grep "Model name"
step pytest_gpu 900 python -m pytest tests -m gpu -q -rf
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step bench 400 python bench.py --steps 5 --warmup 2 --cpu-seconds 5
