#!/bin/bash
# r03 first GPU session: VALU dependency microbenchmark, GPU tests, smoke, bench.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -25 "gpurun_out/$name.log"
  case $rc in 0|1) ;; *) echo "fatal rc=$rc in $name, stopping"; exit $rc;; esac
}
step valu_dep 120 ./tools/valu_dep
step pytest_gpu 1000 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step bench 400 python bench.py --steps 10 --warmup 3 --cpu-seconds 5
