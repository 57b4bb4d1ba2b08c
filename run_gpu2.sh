#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -${TAILN:-25} "gpurun_out/$name.log"
  case $rc in 0|1) ;; *) echo "fatal rc=$rc in $name, stopping"; exit $rc;; esac
}
step pytest_gpu 900 python -m pytest tests -m gpu -q -rf -x
TAILN=3 step bench 400 python bench.py --steps 10 --warmup 2 --cpu-seconds 5
